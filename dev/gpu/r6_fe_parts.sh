#!/bin/bash
# Round 6: batch-4 prologue: per-image feature-encoder lanes (FE_PARTS=2, default) vs four quarter chains next to the
# context encoder's lane (FE_PARTS=4: quarters).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_fe_parts}
mkdir -p $o
for r in 1 2 3; do
  for v in 2 4; do
    timeout -k 10 300 python -u dev/probes/bench_with.py FE_PARTS=$v -- --extras off --steps 20 > $o/h_$v.json 2> $o/h_$v.err || { tail $o/h_$v.err; exit 1; }
    echo "r$r FE_PARTS=$v $(python -c "import json;d=json.load(open('$o/h_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
