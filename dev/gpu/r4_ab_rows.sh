#!/bin/bash
# Round 4: A/B of the adaptive norm-statistics / norm-backward row blocking (training bench, same box)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_ab_rows
mkdir -p $o
for r in 1 2; do
  for v in adaptive fixed; do
    if [ $v = fixed ]; then export JR_AB_FIXED_ROWS=1; else unset JR_AB_FIXED_ROWS; fi
    timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_$v.json 2> $o/train.err || { tail $o/train.err; exit 1; }
    echo "$v r$r $(tail -1 $o/train_$v.json | cut -c1-130)"
  done
done
