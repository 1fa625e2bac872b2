#!/bin/bash
# Fused ConvGRU: 8-wave 64 x 64 variant (JR_GRU_W8=1) vs the 16-wave default: tests, phases, headline A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/w8
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gru" > $o/ktests.log 2>&1 || { tail -40 $o/ktests.log; exit 1; }
tail -1 $o/ktests.log
timeout -k 10 120 python -u tools/gru_phases.py --w8 1 > $o/phases.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/gru_phases.py --w8 0 >> $o/phases.txt 2>&1 || exit $?
cat $o/phases.txt
JR_GRU_W8=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "fused_gru or golden or lane" > $o/etests.log 2>&1 || { tail -40 $o/etests.log; exit 1; }
tail -1 $o/etests.log
for r in 1 2; do
  for v in 0 1; do
    JR_GRU_W8=$v timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/b4_$v$r.json 2> $o/b4_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b4_$v$r.json')); print('b4 w8=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
