#!/bin/bash
# Round 5: kernel trace of the headline forward (batch ${B:-4}) -> per-kernel breakdown + iteration timeline.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_trace}
mkdir -p $o
for b in ${BATCHES:-4 1}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/t$b -o run -- python3 bench.py --batch $b --extras off --steps 5 --warmup 2 ${ARGS} > $o/t$b.log 2>&1 || { tail -5 $o/t$b.log; exit 1; }
  f=$(find $o/t$b -name '*kernel_trace.csv' | head -1)
  python3 tools/kernel_breakdown.py $f --steps 5 --top 25 > $o/breakdown_b$b.txt 2>&1
  python3 tools/timeline.py $f > $o/timeline_b$b.txt 2>&1 || true
  head -30 $o/breakdown_b$b.txt
  head -16 $o/timeline_b$b.txt
  rm -f $f
done
