#!/bin/bash
# Native batched GEMM for the pyramid backward (no hipBLASLt): tests, training bench, training trace.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/bgemm
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "bgemm or pyr_bwd" > $o/ktests.log 2>&1 || { tail -40 $o/ktests.log; exit 1; }
tail -1 $o/ktests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_train_gpu.py > $o/ttests.log 2>&1 || { tail -40 $o/ttests.log; exit 1; }
tail -1 $o/ttests.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py > $o/tb_$r.json 2> $o/tb_$r.err || exit $?
  tail -1 $o/tb_$r.json | cut -c1-160
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/k -o run -- python3 tools/train_bench.py --steps 5 --warmup 2 > $o/prof.log 2>&1 || exit $?
