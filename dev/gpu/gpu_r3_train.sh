#!/bin/bash
# Vectorised pyramid-backward dC: kernel + fused-training tests, training bench x3, training kernel trace,
# and the persisted autotune table's misses (s2d stems) timed and merged.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/train
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_train_gpu.py -k "pyr_bwd or fused or train" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/train_bench.py > $o/tb_$r.json 2> $o/tb_$r.err || exit $?
  tail -1 $o/tb_$r.json | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/k -o run -- python3 tools/train_bench.py --steps 5 --warmup 2 > $o/prof.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/autotune_db.py --no-train --out gpurun_out/gfx950.json > $o/autotune.log 2>&1 || exit $?
tail -3 $o/autotune.log
