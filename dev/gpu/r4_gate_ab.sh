#!/bin/bash
# Round 4: engine host gate (launch a replay only after the previous call finished) A/B, same box, interleaved
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_gate_ab
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 60 --warmup 10 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  for g in 1 0; do
    export JR_HOST_GATE=$g
    run b1_g${g}_r$r --batch 1 && run small_g${g}_r$r --batch 1 --arch raft_small && run b4_g${g}_r$r --steps 30 || exit 1
  done
done
