#!/bin/bash
# Round 4: persistent convex mask head (JR_CONVEX_PERSIST=1) -- numerics + A/B at batch 4
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_convex
mkdir -p $o
JR_CONVEX_PERSIST=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "convex or upsample or golden or merged or bitwise" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for pv in 0 1 0 1; do
  JR_CONVEX_PERSIST=$pv PYTHONPATH=. timeout -k 10 100 python -u dev/probes/convex_bench.py 4 || exit 1
done
for r in 1 2; do
for pv in 1 0; do
  JR_CONVEX_PERSIST=$pv timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4.json 2> $o/b4.err || { tail $o/b4.err; exit 1; }
  echo "r$r persist=$pv b4 $(python -c "import json;d=json.load(open('$o/b4.json'));print(d['value'],d['ms_per_step'])")"
done
done
JR_CONVEX_PERSIST=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit 1
db=$(ls $o/prof/*/run_results.db $o/prof/run_results.db 2>/dev/null | head -1)
python tools/kernel_breakdown.py $db --top 20 > $o/breakdown_b4.txt 2>&1 || exit 1
rm -rf $o/prof
grep -E "convex" $o/breakdown_b4.txt
