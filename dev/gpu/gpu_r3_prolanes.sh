#!/bin/bash
# One-lane loop with the context encoder on its own prologue lane (JR_PRO_LANES=1) at batch 1: A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/prolanes2
mkdir -p $o
for r in 1 2; do
  for v in 1 0; do
    JR_PRO_LANES=$v timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('b1 prolanes=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
    JR_PRO_LANES=$v timeout -k 10 200 python -u bench.py --extras off --arch raft_small --batch 1 --steps 40 > $o/s1_$v$r.json 2> $o/s1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/s1_$v$r.json')); print('small b1 prolanes=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
JR_PRO_LANES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/large -o run -- python3 bench.py --batch 1 --steps 5 --warmup 2 --extras off > $o/large.log 2>&1 || exit $?
