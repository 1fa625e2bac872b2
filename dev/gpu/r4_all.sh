#!/bin/bash
# Round 4: validation + measurement sweep after the pyramid / encoder / training changes.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_all
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_halo_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py > $o/tests1.txt 2>&1 || { tail -40 $o/tests1.txt; exit 1; }
tail -1 $o/tests1.txt
timeout -k 10 200 python -u tools/corr_bench.py pyr --batch 4 > $o/pyr.txt 2>&1 || { tail $o/pyr.txt; exit 1; }
grep pyr $o/pyr.txt
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_$r.json 2> $o/b4_$r.err || { tail $o/b4_$r.err; exit 1; }
  echo "b4 r$r $(python -c "import json;d=json.load(open('$o/b4_$r.json'));print(d['value'],d['ms_per_step'],d['autotune'])")"
done
timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 20 > $o/b1.json 2> $o/b1.err || { tail $o/b1.err; exit 1; }
echo "b1 $(python -c "import json;d=json.load(open('$o/b1.json'));print(d['value'],d['ms_per_step'])")"
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit 1
db=$(ls $o/prof/*/run_results.db $o/prof/run_results.db 2>/dev/null | head -1)
python tools/timeline.py $db --prologue > $o/prologue_b4.txt 2>&1 || exit 1
python tools/timeline.py $db > $o/timeline_b4.txt 2>&1 || exit 1
python tools/kernel_breakdown.py $db --top 40 > $o/breakdown_b4.txt 2>&1 || exit 1
rm -rf $o/prof
head -2 $o/prologue_b4.txt
grep -E "corr_pyr" $o/breakdown_b4.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_train_gpu.py > $o/tests2.txt 2>&1 || { tail -40 $o/tests2.txt; exit 1; }
tail -1 $o/tests2.txt
for hv in 1 0; do
  JR_CONV_HALO=$hv timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_h$hv.json 2> $o/train_h$hv.err || { tail $o/train_h$hv.err; exit 1; }
  echo "train halo=$hv $(tail -1 $o/train_h$hv.json)"
done
