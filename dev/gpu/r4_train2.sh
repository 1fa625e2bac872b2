#!/bin/bash
# Round 4: head weight gradients next to the BPTT chain + bf16 identity-shortcut gradient -- tests + bench
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r4_train2}
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_train_gpu.py tests/test_autograd_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train.json 2> $o/train.err || { tail $o/train.err; exit 1; }
  echo "train r$r $(tail -1 $o/train.json | cut -c1-140)"
done
