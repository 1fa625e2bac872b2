#!/bin/bash
# Round 6: the whole GPU suite in one process WITHOUT the per-test state-release fixture
# (JR_TEST_KEEP_STATE=1, tests/conftest.py), then smoke().
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_suite_nogc}
mkdir -p $o
JR_TEST_KEEP_STATE=1 timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -2 $o/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
