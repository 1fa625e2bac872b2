#!/bin/bash
# Round 5: what the host gate fixes (kernel traces with the gate on / off) and where the raft_small
# 12-iteration p99 steps come from (per-step device times).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_gate}
mkdir -p $o
for g in 0 1; do
  timeout -k 10 120 python3 dev/probes/gate_trace.py --gate $g --n 12 >> $o/plain.txt 2>&1 || { tail -5 $o/plain.txt; exit 1; }
done
cat $o/plain.txt
for g in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/g$g -o run -- python3 dev/probes/gate_trace.py --gate $g --n 12 > $o/g$g.log 2>&1 || { tail -5 $o/g$g.log; exit 1; }
  tail -1 $o/g$g.log
done
python3 dev/probes/trace_compare.py $(find $o/g1 -name '*kernel_trace.csv' | head -1) $(find $o/g0 -name '*kernel_trace.csv' | head -1) --top 20 > $o/compare.txt 2>&1
cat $o/compare.txt
find $o -name '*kernel_trace.csv' -delete
timeout -k 10 200 python3 -u bench.py --arch raft_small --batch 1 --iters 12 --steps 100 --warmup 15 --extras off --step-times > $o/small12.json 2> $o/small12.err || { tail -5 $o/small12.err; exit 1; }
grep step_ms $o/small12.err | head -c 2000
