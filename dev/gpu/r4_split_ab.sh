#!/bin/bash
# Round 4: batch-4 headline, independent batch parts in one graph (split) vs lanes, same box
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_split_ab
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 30 --warmup 5 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  run lanes_r$r && run split4_off_r$r --split 4 --streams off && run split2_off_r$r --split 2 --streams off && run split2_off_pipe_r$r --split 2 --streams off --pipeline graph || exit 1
done
