#!/bin/bash
# Round 5: channel-split ConvGRU kernel: correctness vs fp32, then per-stage times vs the fused kernels.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/r5_split
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gru_split_gpu.py \
  > $o/tests.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $o/tests.txt | tail -20
[ $rc -eq 0 ] || { grep -B 30 -m 2 "^E " $o/tests.txt | tail -60; exit 1; }
for b in 4 1; do
  timeout -k 10 300 python -u tools/gru_bench.py --arch raft_large --batch $b > $o/bench_b$b.txt 2>&1 || { tail -20 $o/bench_b$b.txt; exit 1; }
  cat $o/bench_b$b.txt
done
