#!/bin/bash
# Round 5: the new / tightened GPU tests (lifecycle, uint8 prep, relative engine bounds, overfit), then PMC.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5_a
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_input_prep_gpu.py tests/test_lifecycle_gpu.py tests/test_engine_gpu.py tests/test_train_gpu.py \
  > $o/tests.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $o/tests.txt | tail -80
[ $rc -eq 0 ] || { grep -B 40 -m 3 "Error\|assert" $o/tests.txt | tail -80; exit 1; }
OUT=r5_pmc bash dev/gpu/r5_pmc_loop.sh
