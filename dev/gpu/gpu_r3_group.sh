#!/bin/bash
# Grouped corr conv + convflow2 launch (one-lane schedule): tests and batch-1 A/B (JR_CONV_GROUP=1 / 0).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/group
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_drift.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in 1 0; do
    JR_CONV_GROUP=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 group=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
    JR_CONV_GROUP=$v timeout -k 10 200 python -u bench.py --extras off --arch raft_small --batch 1 --steps 40 > $o/s1_$v$r.json 2> $o/s1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/s1_$v$r.json')); print('small b1 group=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
timeout -k 10 300 python -u bench.py --extras off --steps 30 > $o/head.json 2> $o/head.err || exit $?
cat $o/head.json
