#!/bin/bash
# Round 4: batch-1 cross-batch graph pipelining A/B (raft_large and raft_small), same box, interleaved
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_b1_pipe_ab
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --batch 1 --steps 60 --warmup 10 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  run large_auto_r$r && run large_off_r$r --pipeline off && run small_auto_r$r --arch raft_small && run small_off_r$r --arch raft_small --pipeline off || exit 1
done
