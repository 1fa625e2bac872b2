#!/bin/bash
# Round 6: batch-4 prologue: per-image feature-encoder lanes (FE_SPLIT=1, default) vs one batch-8 chain next to the
# context encoder's lane (FE_SPLIT=0).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_fe_split}
mkdir -p $o
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python -u dev/probes/bench_with.py FE_SPLIT=$v -- --extras off --steps 20 > $o/h_$v.json 2> $o/h_$v.err || { tail $o/h_$v.err; exit 1; }
    echo "r$r FE_SPLIT=$v $(python -c "import json;d=json.load(open('$o/h_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
