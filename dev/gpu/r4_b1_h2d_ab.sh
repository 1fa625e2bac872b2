#!/bin/bash
# Round 4: batch-1 streaming vs per-pair sync: which input path costs (prefetcher / sync H2D / resident inputs)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_b1_h2d_ab
mkdir -p $o
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --extras off --batch 1 --steps 60 --warmup 10 "$@" > $o/$n.json 2> $o/$n.err || { tail $o/$n.err; return 1; }
  echo "$n $(tail -1 $o/$n.json | cut -c1-120 | sed 's/.*"value"/value/')"
}
for r in 1 2; do
  run off_pf_r$r --pipeline off && run off_synch2d_r$r --pipeline off --sync-h2d && run off_noh2d_r$r --pipeline off --no-h2d && run pipe_pf_r$r && run pipe_noh2d_r$r --no-h2d || exit 1
done
