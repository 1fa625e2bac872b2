#!/bin/bash
# Round 4: training step busy / idle split and the largest idle gaps (kernel trace)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_train_gaps
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 tools/train_bench.py --steps 5 --warmup 3 > $o/prof.log 2>&1 || { tail $o/prof.log; exit 1; }
db=$(ls $o/prof/*/run_results.db $o/prof/run_results.db 2>/dev/null | head -1)
PYTHONPATH=tools python dev/probes/step_gaps.py $db --top 25 > $o/gaps.txt 2>&1 || { cat $o/gaps.txt; exit 1; }
python tools/kernel_breakdown.py $db --marker "" --steps 8 --top 60 > $o/breakdown.txt 2>&1 || exit 1
rm -rf $o/prof
cat $o/gaps.txt
