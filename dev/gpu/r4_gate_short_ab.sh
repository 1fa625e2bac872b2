#!/bin/bash
# Round 4: host gate on short forwards (raft_small 12 it) and long ones (raft_large 32 it), gate on / off, one box
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_gate_short_ab
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --batch 1 --steps 60 --warmup 10 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  for g in 1 0; do
    export JR_HOST_GATE=$g
    run small12_g${g}_r$r --arch raft_small --iters 12 && run large_g${g}_r$r && run small32_g${g}_r$r --arch raft_small || exit 1
  done
done
