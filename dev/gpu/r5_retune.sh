#!/bin/bash
# Round 5: re-time the persisted conv tile-config table on the current kernels (tools/autotune_db.py,
# JR_TUNE=fresh), then a same-box A/B of the new table (JR_TUNE_DB) against the packaged one.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_retune}
mkdir -p $o
JR_TUNE=fresh timeout -k 10 1500 python -u tools/autotune_db.py --out $o/gfx950.json > $o/tune.log 2>&1 || { tail -20 $o/tune.log; exit 1; }
tail -3 $o/tune.log
for r in 1 2; do
  for v in old new; do
    db=""; [ $v = new ] && db=$PWD/$o/gfx950.json
    JR_TUNE_DB=$db timeout -k 10 300 python -u bench.py --extras off --steps 30 --warmup 5 > $o/b4_${v}_$r.json 2> $o/b4_${v}_$r.err || { tail $o/b4_${v}_$r.err; exit 1; }
    echo "b4 $v r$r $(tail -1 $o/b4_${v}_$r.json | cut -c100-190)"
  done
done
for r in 1 2; do
  for v in old new; do
    db=""; [ $v = new ] && db=$PWD/$o/gfx950.json
    JR_TUNE_DB=$db timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_${v}_$r.json 2> $o/train_${v}_$r.err || { tail $o/train_${v}_$r.err; exit 1; }
    echo "train $v r$r $(tail -1 $o/train_${v}_$r.json | cut -c50-130)"
  done
done
