#!/bin/bash
# Round 4: engine-vs-golden failure at raft_large 2 x 128x160 -- halo conv tests on every config, env bisection
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_diag
mkdir -p $o
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_conv_halo_gpu.py > $o/halo_tests.txt 2>&1; tail -15 $o/halo_tests.txt
T="tests/test_engine_gpu.py::test_engine_matches_golden"
for e in "X=1" "JR_HALO_RES=0" "JR_HALO_NORM=0" "JR_CONV_HALO=0" "JR_GRU=unfused" "JR_TUNE=fresh"; do
  env $e timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread "$T" -k "raft_large" > $o/eng_$e.txt 2>&1
  echo "$e: $(tail -1 $o/eng_$e.txt)"
  grep -E "^E .*assert [0-9]" $o/eng_$e.txt | head -3
done
