#!/bin/bash
# s2d stem + unconditional epilogue prefetch in the fused ConvGRU: tests, phases, engine/drift tests, bench,
# and a same-box A/B of the stem (JR_NO_S2D=1: the 7x7 form).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/s2d
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gru or s2d" > $o/ktests.log 2>&1 || { tail -40 $o/ktests.log; exit 1; }
tail -1 $o/ktests.log
timeout -k 10 120 python -u tools/gru_phases.py > $o/phases.txt 2>&1 || exit $?
cat $o/phases.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py > $o/etests.log 2>&1 || { tail -40 $o/etests.log; exit 1; }
tail -1 $o/etests.log
for r in 1 2; do
  for v in 0 1; do
    JR_NO_S2D=$v timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/b4_$v$r.json 2> $o/b4_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b4_$v$r.json')); print('b4 no_s2d=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit $?
