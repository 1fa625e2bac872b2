#!/bin/bash
# Merged flow conv + deferred upsampling (one-lane schedule): tests and batch-1 A/B (JR_MERGED_UP=1 / 0).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/merged
mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in 1 0; do
    JR_MERGED_UP=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 merged=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
    JR_MERGED_UP=$v timeout -k 10 200 python -u bench.py --extras off --arch raft_small --batch 1 --steps 40 > $o/s1_$v$r.json 2> $o/s1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/s1_$v$r.json')); print('small b1 merged=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
