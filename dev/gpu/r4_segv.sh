#!/bin/bash
# Round 4: segfault in engine.pipelined (capture_part) -- isolate
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_segv
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_engine_gpu.py::test_graph_pipelined_matches_forward" > $o/t1.txt 2>&1; echo "isolated: rc=$? $(tail -1 $o/t1.txt)"
grep -n "engine.py\", line" $o/t1.txt | head -3
JR_PLAN_DEBUG=1 timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread "tests/test_engine_gpu.py::test_graph_pipelined_matches_forward" > $o/t2.txt 2>&1; echo "debug: rc=$?"
grep -n "\[plan\]" $o/t2.txt | tail -8
