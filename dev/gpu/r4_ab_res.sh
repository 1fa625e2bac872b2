#!/bin/bash
# Round 4: A/B of the residual-block output built inside the next halo conv (JR_HALO_RES) with
# the regenerated tuned table; prologue timelines at batch 4 and 1
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_ab_res
mkdir -p $o
for r in 1 2; do
for hv in 1 0; do
  JR_HALO_RES=$hv timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_h${hv}_$r.json 2> $o/b4_h${hv}_$r.err || { tail $o/b4_h${hv}_$r.err; exit 1; }
  JR_HALO_RES=$hv timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1_h${hv}_$r.json 2> $o/b1_h${hv}_$r.err || { tail $o/b1_h${hv}_$r.err; exit 1; }
  echo "r$r halo_res=$hv b4 $(python -c "import json;d=json.load(open('$o/b4_h${hv}_$r.json'));print(d['value'],d['ms_per_step'],d['autotune']['misses'])") b1 $(python -c "import json;d=json.load(open('$o/b1_h${hv}_$r.json'));print(d['value'],d['ms_per_step'],d['autotune']['misses'])")"
done
done
for hv in 1 0; do
  JR_HALO_RES=$hv timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_$hv -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof_$hv.log 2>&1 || exit 1
  db=$(ls $o/prof_$hv/*/run_results.db $o/prof_$hv/run_results.db 2>/dev/null | head -1)
  python tools/timeline.py $db --prologue > $o/prologue_b4_h$hv.txt 2>&1 || exit 1
  rm -rf $o/prof_$hv
  head -2 $o/prologue_b4_h$hv.txt
done
