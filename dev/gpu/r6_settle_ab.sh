#!/bin/bash
# Round 6: does the training step starve the GPU?  A/B of how many steps the host may run ahead.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_settle_ab}
mkdir -p $o
for r in 1 2; do
  for v in 1 2 3; do
    timeout -k 10 300 python -u tools/train_bench.py --steps 20 --settle-lag $v > $o/lag_$v.json 2> $o/lag_$v.err || { tail $o/lag_$v.err; exit 1; }
    echo "r$r lag=$v $(cut -c1-150 $o/lag_$v.json)"
  done
done
