#!/bin/bash
# Round 6: convcorr1 fused into the lookup (lane schedule) -- kernel test, engine tests, headline A/B,
# and a kernel-trace timeline of the new iteration.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_c1}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fused_convcorr1 or lookup" --timeout 200 --timeout-method thread > $o/ktests.txt 2>&1 || { tail -30 $o/ktests.txt; exit 1; }
tail -1 $o/ktests.txt
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $o/etests.txt 2>&1 || { tail -30 $o/etests.txt; exit 1; }
tail -1 $o/etests.txt
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python -u dev/probes/bench_with.py LOOKUP_C1=$v -- --batch 4 --extras off --steps 20 > $o/b4_c1$v.json 2> $o/b4_c1$v.err || { tail $o/b4_c1$v.err; exit 1; }
    echo "LOOKUP_C1=$v $(python -c "import json;d=json.load(open('$o/b4_c1$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/t -o run -- python3 bench.py --batch 4 --extras off --steps 5 --warmup 2 > $o/t.log 2>&1 || { tail -5 $o/t.log; exit 1; }
f=$(find $o/t -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_breakdown.py $f --steps 5 --top 30 > $o/breakdown.txt 2>&1
python3 tools/timeline.py $f --iter 20 > $o/timeline.txt 2>&1 || true
rm -f $f
cat $o/timeline.txt
