#!/bin/bash
# Round 6: per-queue Gantt chart + breakdown of a steady-state training step.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_train_gantt}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -o run -- python3 tools/train_bench.py --steps 8 --warmup 3 > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_breakdown.py $f --marker seq_loss_kernel --between --steps 6 --top 70 > $o/breakdown.txt 2>&1 || { cat $o/breakdown.txt; exit 1; }
PYTHONPATH=tools python3 dev/probes/train_gantt.py $f --bucket 100 > $o/gantt.txt 2>&1 || { cat $o/gantt.txt; exit 1; }
gzip -c $f > $o/trace.csv.gz
rm -rf $o/prof
cat $o/gantt.txt
head -12 $o/breakdown.txt
