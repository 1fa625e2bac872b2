#!/bin/bash
# Round 4: serving-mode rows with the host gate (final-only pipelined, batch 8), README numbers
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_serving
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 30 --warmup 5 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
run final_only --final-only && run b8 --batch 8 && run final_only_b1 --final-only --batch 1
