#!/bin/bash
# Round 4: lane fork after convcorr1 (JR_FORK_C1=1) vs after the lookup -- correctness + batch-4 headline A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_fork_ab
mkdir -p $o
JR_FORK_C1=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "lane or streams or golden" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --steps 30 --warmup 5 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2 3; do
  run base_r$r && JR_FORK_C1=1 run fork_r$r || exit 1
done
