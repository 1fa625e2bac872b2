#!/bin/bash
# Lane-schedule fork order A/B: the lookup's successors created main-lane first (JR_FORK_ORDER=main)
# or mask-lane first (side, the round-2 order); engine tests; a kernel trace of the new order.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/fork
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in main side; do
    JR_FORK_ORDER=$v timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/bench_$v$r.json 2> $o/bench_$v$r.err || exit $?
    python -c "import json,sys; d=json.load(open('$o/bench_$v$r.json')); print('$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
JR_FORK_ORDER=main timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit $?
