#!/bin/bash
# Round 4: residual-build relu fix -- GPU tests, then the GRU 4-block A/B and the stats / prologue profiles
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_fix
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_halo_gpu.py tests/test_engine_gpu.py tests/test_gru_halo_gpu.py tests/test_kernels_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
bash dev/gpu/r4_gru4.sh && bash dev/gpu/r4_stats.sh
