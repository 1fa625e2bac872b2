#!/bin/bash
# Round 3: fused lookup+convcorr1 kernel test, engine tests, training/loss tests,
# numerics drift at the headline config, then the bench (headline + extras).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lookup_cc1 or lookup_with_fused" > gpurun_out/r3_kernel_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  > gpurun_out/r3_engine_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_train_gpu.py \
  -k "swapped or nonfinite or native_sequence" > gpurun_out/r3_advice_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/drift.py measure --json gpurun_out/r3_drift.json > gpurun_out/r3_drift.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r3_bench.log 2>&1 || exit $?
export TMPDIR=/tmp
mkdir -p gpurun_out/r3prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3prof/b4 -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > gpurun_out/r3prof/b4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3prof/b4s -o run -- python3 bench.py --steps 5 --warmup 2 --extras off --streams off > gpurun_out/r3prof/b4s.log 2>&1 || exit $?
