#!/bin/bash
# Round 5: same-box A/B of the round-start kernels (dev/bin/_C_base.so, built from d67e02a) against the
# current tree's _C.so -- headline (no extras) and the training step, alternating.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_ab_base}
mkdir -p $o
for r in 1 2; do
  for v in base new; do
    so=""; [ $v = base ] && so=$PWD/dev/bin/_C_base.so
    JR_NATIVE_SO=$so timeout -k 10 300 python -u bench.py --extras off --steps 30 --warmup 5 > $o/b4_${v}_$r.json 2> $o/b4_${v}_$r.err || { tail $o/b4_${v}_$r.err; exit 1; }
    echo "b4 $v r$r $(tail -1 $o/b4_${v}_$r.json | cut -c100-190)"
  done
done
for r in 1 2; do
  for v in base new; do
    so=""; [ $v = base ] && so=$PWD/dev/bin/_C_base.so
    JR_NATIVE_SO=$so timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_${v}_$r.json 2> $o/train_${v}_$r.err || { tail $o/train_${v}_$r.err; exit 1; }
    echo "train $v r$r $(tail -1 $o/train_${v}_$r.json | cut -c50-130)"
  done
done
