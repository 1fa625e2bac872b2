#!/bin/bash
# Round 4: with the host gate, batch-1 cross-batch pipelining auto vs off (raft_large 32 it, raft_small 32 / 12 it)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_gate_pipe_ab
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --batch 1 --steps 60 --warmup 10 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  run large_pipe_r$r && run large_off_r$r --pipeline off && run small_pipe_r$r --arch raft_small && run small_off_r$r --arch raft_small --pipeline off && run small12_pipe_r$r --arch raft_small --iters 12 && run small12_off_r$r --arch raft_small --iters 12 --pipeline off || exit 1
done
