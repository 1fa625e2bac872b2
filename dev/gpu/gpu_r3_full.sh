#!/bin/bash
# Round 3: full GPU test suite, the persisted autotune table (fresh timing), training-step profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1 || exit $?
JR_TUNE=fresh timeout -k 10 600 python -u tools/autotune_db.py --out gpurun_out/gfx950.json > gpurun_out/r3_autotune.log 2>&1 || exit $?
timeout -k 10 700 bash scripts/gpu_trainprof.sh > gpurun_out/r3_trainprof.log 2>&1 || exit $?
