#!/bin/bash
# Fused ConvGRU stage: kernel tests, engine + drift tests, headline / batch-1 A/B vs the two-launch path,
# and a kernel trace of the fused headline.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/gru
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gru_stage_fused or gru_fused_fits" > $o/ktests.log 2>&1 || { tail -40 $o/ktests.log; exit 1; }
tail -1 $o/ktests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py > $o/etests.log 2>&1 || { tail -40 $o/etests.log; exit 1; }
tail -1 $o/etests.log
for r in 1 2; do
  for v in 1 0; do
    JR_GRU_FUSED=$v timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/b4_$v$r.json 2> $o/b4_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b4_$v$r.json')); print('b4 fused=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
    JR_GRU_FUSED=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 30 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 fused=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit $?
