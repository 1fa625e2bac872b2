#!/bin/bash
# Round 5: training throughput after the repack fix + the headline prologue's per-queue timeline.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pro_q}
mkdir -p $o
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_$r.json 2> $o/train_$r.err || { tail $o/train_$r.err; exit 1; }
  echo "train r$r $(tail -1 $o/train_$r.json | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/k -o run -- python3 bench.py --extras off --steps 4 --warmup 2 > $o/bench.log 2>&1 || { tail -5 $o/bench.log; exit 1; }
f=$(find $o/k -name '*kernel_trace.csv' | head -1)
python3 tools/prologue_timeline.py "$f" > $o/prologue_q.txt || exit 1
tail -8 $o/prologue_q.txt
rm -rf $o/k
