#!/bin/bash
# The persisted pair config of the batch-1 grouped launch: engine tests + b1 bench (default vs override 23).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/grp24
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_d$r.json 2> $o/b1_d$r.err || exit $?
  python -c "import json; d=json.load(open('$o/b1_d$r.json')); print('b1 default', d['value'], d['ms_per_step'], d['autotune']['tile_cfgs'].get('me.convcorr2'))"
  JR_CFG_OVERRIDE="me.convcorr2=23" timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_o$r.json 2> $o/b1_o$r.err || exit $?
  python -c "import json; d=json.load(open('$o/b1_o$r.json')); print('b1 cfg 23', d['value'], d['ms_per_step'])"
done
