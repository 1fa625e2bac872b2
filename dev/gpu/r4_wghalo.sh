#!/bin/bash
# Round 4: halo weight gradient (3x3 / stride 1) -- numerics + microbench (halo vs im2col via JR_WGRAD_HALO=0)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_wghalo
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_train_gpu.py -k native_wgrad > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
PYTHONPATH=. timeout -k 10 300 python -u dev/probes/wgrad_bench.py > $o/wgrad_bench.txt 2>&1 || { tail -20 $o/wgrad_bench.txt; exit 1; }
cat $o/wgrad_bench.txt
JR_WGRAD_HALO=0 PYTHONPATH=. timeout -k 10 300 python -u dev/probes/wgrad_bench.py > $o/wgrad_bench_off.txt 2>&1 || { tail -20 $o/wgrad_bench_off.txt; exit 1; }
cat $o/wgrad_bench_off.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_train_gpu.py tests/test_autograd_gpu.py > $o/tests2.txt 2>&1 || { tail -30 $o/tests2.txt; exit 1; }
tail -1 $o/tests2.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_$r.json 2> $o/train_$r.err || { tail $o/train_$r.err; exit 1; }
  echo "train r$r $(tail -1 $o/train_$r.json | cut -c1-120)"
done
