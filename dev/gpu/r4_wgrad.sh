#!/bin/bash
# Round 4: 256 x 256 wgrad tiles -- numerics + microbench on the training shapes
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_wgrad
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_train_gpu.py -k native_wgrad > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
PYTHONPATH=. timeout -k 10 300 python -u dev/probes/wgrad_bench.py > $o/wgrad_bench.txt 2>&1 || { tail -20 $o/wgrad_bench.txt; exit 1; }
cat $o/wgrad_bench.txt
