#!/bin/bash
# convcorr1 (1x1) in the merged flow-conv grid at batch 1: tests + A/B (JR_MERGED_C1=1 / 0).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/mc1
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in 1 0; do
    JR_MERGED_C1=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 mc1=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/large -o run -- python3 bench.py --batch 1 --steps 5 --warmup 2 --extras off > $o/large.log 2>&1 || exit $?
