#!/bin/bash
# Round 6: straight-line EPI_BWD epilogue -- training numerics tests, bench, steady-state breakdown.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_epibwd}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 20 > $o/train_$r.json 2> $o/train_$r.err || { tail $o/train_$r.err; exit 1; }
  cut -c1-150 $o/train_$r.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -o run -- python3 tools/train_bench.py --steps 8 --warmup 3 > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_breakdown.py $f --marker seq_loss_kernel --between --steps 6 --top 70 > $o/breakdown.txt 2>&1 || { cat $o/breakdown.txt; exit 1; }
python3 - $f <<'PY'
import csv, sys
seen = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "conv_igemm_kernel" in n and ", 5, " in n:
        seen[n[:70]] = (r["Scratch_Size"], r["VGPR_Count"], r.get("Accum_VGPR_Count"))
for k, v in seen.items(): print("scratch/vgpr/agpr", v, k)
PY
rm -rf $o/prof
head -14 $o/breakdown.txt
