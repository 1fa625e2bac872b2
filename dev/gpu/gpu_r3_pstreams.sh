#!/bin/bash
# Eager prologue on a side stream + loop graph (JR_PIPE_STREAMS): probe, correctness, bench A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/pstreams
mkdir -p $o
timeout -k 10 200 python -u tools/pipe_streams.py > $o/probe.txt 2>&1 || { tail -20 $o/probe.txt; exit 1; }
grep -v amdgpu.ids $o/probe.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "pipelined" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in 1 0; do
    JR_PIPE_STREAMS=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 pstreams=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
    JR_PIPE_STREAMS=$v timeout -k 10 200 python -u bench.py --extras off --arch raft_small --batch 1 --steps 40 > $o/s1_$v$r.json 2> $o/s1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/s1_$v$r.json')); print('small b1 pstreams=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
