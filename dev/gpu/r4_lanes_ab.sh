#!/bin/bash
# Round 4: batch-4 headline schedule A/B on one box: lanes (auto) vs one lane (merged grids), split 2, graph pipeline
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_lanes_ab
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 30 --warmup 5 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120)"
}
for r in 1 2; do
  run lanes_r$r && run onelane_r$r --streams off && run onelane_pipe_r$r --streams off --pipeline graph || exit 1
done
run split2 --split 2 && run split2_off --split 2 --streams off
