#!/bin/bash
# Round 6: raft_small batch-1 kernel trace (headline-style forward, 32 iterations): breakdown,
# prologue listing and loop iteration timeline.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_small}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/t -o run -- python3 bench.py --arch raft_small --batch 1 --extras off --steps 5 --warmup 2 ${ARGS} > $o/t.log 2>&1 || { tail -5 $o/t.log; exit 1; }
f=$(find $o/t -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_breakdown.py $f --steps 5 --top 40 > $o/breakdown.txt 2>&1
python3 tools/timeline.py $f --iter 10 > $o/timeline.txt 2>&1 || true
python3 tools/timeline.py $f --prologue > $o/prologue.txt 2>&1 || true
python3 tools/prologue_timeline.py $f > $o/prologue_q.txt 2>&1 || true
rm -f $f
head -3 $o/timeline.txt; wc -l $o/prologue.txt
