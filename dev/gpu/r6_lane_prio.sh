#!/bin/bash
# Round 6: plan lane stream priorities (temporary JR_LANE_PRIO switch): default (lane 0 greatest, others least),
# "same" (all greatest), "normal" (all 0) -- headline batch 4 and raft_large batch-1 stream.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_lane_prio}
mkdir -p $o
for r in 1 2; do
  for v in default same normal; do
    JR_LANE_PRIO=$v timeout -k 10 300 python -u bench.py --extras off --steps 20 > $o/h_$v.json 2> $o/h_$v.err || { tail $o/h_$v.err; exit 1; }
    echo "r$r prio=$v b4 $(python -c "import json;d=json.load(open('$o/h_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
