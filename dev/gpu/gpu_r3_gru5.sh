#!/bin/bash
# Fused ConvGRU with the epilogue operands prefetched during the last K stages: kernel tests, phase split,
# engine tests, headline.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/gru5
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gru" > $o/ktests.log 2>&1 || { tail -40 $o/ktests.log; exit 1; }
tail -1 $o/ktests.log
timeout -k 10 120 python -u tools/gru_phases.py > $o/phases.txt 2>&1 || exit $?
cat $o/phases.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py > $o/etests.log 2>&1 || { tail -40 $o/etests.log; exit 1; }
tail -1 $o/etests.log
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/b4_$r.json 2> $o/b4_$r.err || exit $?
  python -c "import json; d=json.load(open('$o/b4_$r.json')); print('b4', d['value'], d['ms_per_step'], d['step_ms_p50'])"
done
