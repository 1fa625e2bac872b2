#!/bin/bash
# Round 5: headline (no extras) twice + the training step once, on the current tree.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_quick}
mkdir -p $o
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --extras off --steps 30 --warmup 5 > $o/b4_$r.json 2> $o/b4_$r.err || { tail $o/b4_$r.err; exit 1; }
  echo "b4 r$r $(tail -1 $o/b4_$r.json | cut -c1-150)"
done
if [ -z "$NOTRAIN" ]; then
timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train.json 2> $o/train.err || { tail $o/train.err; exit 1; }
echo "train $(tail -1 $o/train.json | cut -c1-150)"
fi
