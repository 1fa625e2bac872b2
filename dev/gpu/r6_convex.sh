#!/bin/bash
# Round 6: convex mask head forms (tiles 0 = current auto, 3..5 = convex_head2_kernel) -- numerics + device time.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_convex}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k convex_head_kernel --timeout 200 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for t in 0 3 4 5 0 3 4 5; do timeout -k 10 60 python -u dev/probes/convex_bench.py 4 $t 2>&1 | grep convex_head; done | tee $o/bench.txt
for t in 0 3 4 5; do timeout -k 10 60 python -u dev/probes/convex_bench.py 1 $t 2>&1 | grep convex_head; done | tee -a $o/bench.txt
