#!/bin/bash
# Round 6: training step (config 5) throughput, kernel breakdown and GPU idle gaps on the current tree.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_train}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_$r.json 2> $o/train_$r.err || { tail $o/train_$r.err; exit 1; }
  echo "train r$r $(tail -1 $o/train_$r.json | cut -c1-160)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -o run -- python3 tools/train_bench.py --steps 5 --warmup 3 > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_breakdown.py $f --marker "" --steps 8 --top 60 > $o/breakdown.txt 2>&1 || exit 1
PYTHONPATH=tools python3 dev/probes/step_gaps.py $f --top 25 > $o/gaps.txt 2>&1 || { cat $o/gaps.txt; exit 1; }
rm -rf $o/prof
head -30 $o/breakdown.txt
head -20 $o/gaps.txt
