#!/bin/bash
# Round 3: numerics drift at the headline config + a baseline bench + the new ADVICE tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/drift.py measure --json gpurun_out/r3_drift.json > gpurun_out/r3_drift.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_base.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_train_gpu.py -k "swapped or nonfinite or native_sequence" > gpurun_out/r3_advice_tests.log 2>&1 || exit $?
