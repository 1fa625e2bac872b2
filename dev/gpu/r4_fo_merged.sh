#!/bin/bash
# Round 4: final-only loop in the all-iterations one-lane order (JR_FO_MERGED) -- tests + A/B, one box
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_fo_merged
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_resolution_gpu.py -k "final_only or pipelined or golden or hires or 4k or resolution" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 40 --warmup 10 --final-only "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  JR_FO_MERGED=1 run b1_m1_r$r --batch 1 && JR_FO_MERGED=0 run b1_m0_r$r --batch 1 && JR_FO_MERGED=1 run b4_m1_r$r && JR_FO_MERGED=0 run b4_m0_r$r || exit 1
done
