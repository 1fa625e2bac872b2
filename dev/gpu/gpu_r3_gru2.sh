#!/bin/bash
# Fused ConvGRU + E_MASK-free mask lane (hm parity halves, flowp copy): tests, headline runs, trace.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/gru2
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py tests/test_kernels_gpu.py -k "engine or drift or gru or conv_epilogues" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/b4_$r.json 2> $o/b4_$r.err || exit $?
  python -c "import json; d=json.load(open('$o/b4_$r.json')); print('b4', d['value'], d['ms_per_step'], d['step_ms_p50'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit $?
