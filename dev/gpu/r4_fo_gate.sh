#!/bin/bash
# Round 4: final-only batch-1 serving, host gate on / off, one box
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_fo_gate
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 60 --warmup 10 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  JR_HOST_GATE=1 run fo_b1_g1_r$r --final-only --batch 1 && JR_HOST_GATE=0 run fo_b1_g0_r$r --final-only --batch 1 && JR_HOST_GATE=1 run fo_b4_g1_r$r --final-only && JR_HOST_GATE=0 run fo_b4_g0_r$r --final-only || exit 1
done
