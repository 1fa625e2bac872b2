#!/bin/bash
# Round 3: fused lookup kernel check + microbenchmarks (lookup vs fused, every tile config per
# loop conv and per encoder conv, hipBLASLt yardstick).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lookup_cc1 or lookup_with_fused" > gpurun_out/r3_kernel_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/lookup_bench.py > gpurun_out/r3_lookup_bench.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/microbench.py --gemm --only "" > gpurun_out/r3_microbench_loop.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/microbench.py --gemm --encoder > gpurun_out/r3_microbench_encoder.txt 2>&1 || exit $?
