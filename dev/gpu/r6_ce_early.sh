#!/bin/bash
# Round 6: context-encoder backward launched before the pyramid backward (overlapping it): tests + bench.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_ce_early}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 20 > $o/t$r.json 2> $o/t$r.err || { tail $o/t$r.err; exit 1; }
  echo "r$r $(cut -c1-130 $o/t$r.json)"
done
