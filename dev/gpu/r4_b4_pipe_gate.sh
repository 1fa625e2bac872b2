#!/bin/bash
# Round 4: with the host gate, batch-4 (lanes) cross-batch graph pipelining vs off, one box, interleaved
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_b4_pipe_gate
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 30 --warmup 5 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  run off_r$r && run pipe_r$r --pipeline graph || exit 1
done
