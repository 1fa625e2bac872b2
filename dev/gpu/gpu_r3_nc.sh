#!/bin/bash
# Convex-head pixel tiles per wave inside the batch-1 merged grid (JR_CONVEX_NC=1 / 2).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/nc
mkdir -p $o
for r in 1 2; do
  for v in 2 1; do
    JR_CONVEX_NC=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 nc=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
