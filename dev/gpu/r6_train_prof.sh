#!/bin/bash
# Round 6: steady-state training-step kernel breakdown (whole steps between loss kernels, warm-up excluded).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_train_prof}
mkdir -p $o
timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train.json 2> $o/train.err || { tail $o/train.err; exit 1; }
cat $o/train.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -o run -- python3 tools/train_bench.py --steps 8 --warmup 3 > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_breakdown.py $f --marker seq_loss_kernel --between --steps 6 --top 70 > $o/breakdown.txt 2>&1 || { cat $o/breakdown.txt; exit 1; }
PYTHONPATH=tools python3 dev/probes/step_gaps.py $f --top 25 > $o/gaps.txt 2>&1 || { cat $o/gaps.txt; exit 1; }
rm -rf $o/prof
head -45 $o/breakdown.txt
head -8 $o/gaps.txt
