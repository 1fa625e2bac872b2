#!/bin/bash
# Round 6: idle gaps inside the batch-4 headline forward (lane schedule): kernel trace, then the
# largest gaps of one forward (dev/probes/step_gaps.py, forwards delimited by the prep kernel).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PWD/tools${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_gaps}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/t -o run -- python3 bench.py --batch 4 --extras off --steps 5 --warmup 2 > $o/t.log 2>&1 || { tail -5 $o/t.log; exit 1; }
f=$(find $o/t -name '*kernel_trace.csv' | head -1)
python3 dev/probes/step_gaps.py $f --marker prep_images --top 30 > $o/gaps.txt 2>&1 || true
python3 tools/timeline.py $f --prologue > $o/prologue.txt 2>&1 || true
rm -f $f
cat $o/gaps.txt
