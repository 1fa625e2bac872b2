#!/bin/bash
# Round 6: training step with the context encoder on a side stream (default) vs in order on the caller's.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_side_enc}
mkdir -p $o
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python -u dev/probes/train_with.py FusedModel.SIDE_ENCODER=$v -- --steps 20 > $o/s$v.json 2> $o/s$v.err || { tail $o/s$v.err; exit 1; }
    echo "r$r SIDE_ENCODER=$v $(cut -c1-130 $o/s$v.json)"
  done
done
