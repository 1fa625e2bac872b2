#!/bin/bash
# Round 4: prologue timelines at batch 4 with / without the fused encoder instance norm
# (JR_HALO_NORM A/B), bench A/B, and the raft_small batch-1 breakdown.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_pro
mkdir -p $o
for hn in 1 0; do
  for r in 1 2; do
    JR_HALO_NORM=$hn timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_hn${hn}_$r.json 2> $o/b4_hn${hn}_$r.err || { tail $o/b4_hn${hn}_$r.err; exit 1; }
    echo "halo_norm=$hn b4 r$r $(python -c "import json;d=json.load(open('$o/b4_hn${hn}_$r.json'));print(d['value'],d['ms_per_step'])")"
  done
  JR_HALO_NORM=$hn timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_hn$hn -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof_hn$hn.log 2>&1 || exit 1
  db=$(ls $o/prof_hn$hn/*/run_results.db $o/prof_hn$hn/run_results.db 2>/dev/null | head -1)
  python tools/timeline.py $db --prologue > $o/prologue_hn$hn.txt 2>&1 || exit 1
  python tools/kernel_breakdown.py $db --top 40 > $o/breakdown_hn$hn.txt 2>&1 || exit 1
  rm -rf $o/prof_hn$hn
  head -3 $o/prologue_hn$hn.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_s1 -o run -- python3 bench.py --arch raft_small --batch 1 --steps 5 --warmup 2 --extras off > $o/prof_s1.log 2>&1 || exit 1
db=$(ls $o/prof_s1/*/run_results.db $o/prof_s1/run_results.db 2>/dev/null | head -1)
python tools/kernel_breakdown.py $db --top 30 > $o/breakdown_s1.txt 2>&1 || exit 1
python tools/timeline.py $db --iter 10 > $o/timeline_s1.txt 2>&1 || exit 1
rm -rf $o/prof_s1
head -20 $o/breakdown_s1.txt
cat $o/timeline_s1.txt
