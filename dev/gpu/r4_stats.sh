#!/bin/bash
# Round 4: wider stats-final reductions -- kernel tests + benches + prologue timelines
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_stats
mkdir -p $o
true

for r in 1 2; do
  timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_$r.json 2> $o/b4_$r.err || { tail $o/b4_$r.err; exit 1; }
  timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1_$r.json 2> $o/b1_$r.err || { tail $o/b1_$r.err; exit 1; }
  timeout -k 10 200 python -u bench.py --arch raft_small --batch 1 --extras off --steps 30 > $o/s1_$r.json 2> $o/s1_$r.err || { tail $o/s1_$r.err; exit 1; }
  echo "r$r b4 $(python -c "import json;d=json.load(open('$o/b4_$r.json'));print(d['value'],d['ms_per_step'])") b1 $(python -c "import json;d=json.load(open('$o/b1_$r.json'));print(d['value'],d['ms_per_step'])") small_b1 $(python -c "import json;d=json.load(open('$o/s1_$r.json'));print(d['value'],d['ms_per_step'])")"
done
for t in b4:4 b1:1; do
  n=${t%%:*}; b=${t##*:}
  timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_$n -o run -- python3 bench.py --batch $b --steps 5 --warmup 2 --extras off > $o/prof_$n.log 2>&1 || exit 1
  db=$(ls $o/prof_$n/*/run_results.db $o/prof_$n/run_results.db 2>/dev/null | head -1)
  python tools/kernel_breakdown.py $db --top 40 > $o/breakdown_$n.txt 2>&1 || exit 1
  python tools/timeline.py $db --prologue > $o/prologue_$n.txt 2>&1 || exit 1
  python tools/timeline.py $db --iter 10 > $o/timeline_$n.txt 2>&1 || exit 1
  rm -rf $o/prof_$n
  head -2 $o/prologue_$n.txt
done
