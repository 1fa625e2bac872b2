#!/bin/bash
# Pipelined graph: one fork root (JR_PIPE_ROOT) and the next forward's prologue nodes interleaved over the loop's (JR_PIPE_SPREAD).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/spread2
mkdir -p $o
for r in 1 2; do
  for v in "0 0" "1 0" "1 3" "0 p"; do
    set -- $v
    if [ "$2" = p ]; then pro=first; sp=0; else pro=; sp=$2; fi
    JR_PIPE_ROOT=$1 JR_PIPE_SPREAD=$sp JR_PIPE_PROLOGUE=$pro timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$1$2$r.json 2> $o/b1_$1$2$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$1$2$r.json')); print('b1 root=$1 spread=$2', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
JR_PIPE_ROOT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/large -o run -- python3 bench.py --batch 1 --steps 5 --warmup 2 --extras off > $o/large.log 2>&1 || exit $?
