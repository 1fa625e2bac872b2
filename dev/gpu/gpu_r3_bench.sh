#!/bin/bash
# Round 3: engine tests + headline bench + schedule A/B (single lane + graph pipelining at batch 4).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  "tests/test_kernels_gpu.py::test_lookup_with_fused_update_is_bitwise" > gpurun_out/r3_engine_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --extras off --streams off --pipeline graph > gpurun_out/r3_bench_b4_onelane_pipe.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --extras off --streams off --pipeline off > gpurun_out/r3_bench_b4_onelane.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --extras off > gpurun_out/r3_bench_again.log 2>&1 || exit $?
