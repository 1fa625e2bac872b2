#!/bin/bash
# Round 4: training after the wgrad 256-tile / XCD order and the stats-final rewrite: tests, bench, profile
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_train
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_halo_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fused_train_gpu.py tests/test_train_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_$r.json 2> $o/train_$r.err || { tail $o/train_$r.err; exit 1; }
  echo "train r$r $(tail -1 $o/train_$r.json | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 tools/train_bench.py --steps 5 --warmup 3 > $o/prof.log 2>&1 || exit 1
db=$(ls $o/prof/*/run_results.db $o/prof/run_results.db 2>/dev/null | head -1)
python tools/kernel_breakdown.py $db --marker "" --steps 8 --top 50 > $o/breakdown.txt 2>&1 || exit 1
rm -rf $o/prof
head -40 $o/breakdown.txt
timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1.json 2> $o/b1.err || exit 1
echo "b1 $(python -c "import json;d=json.load(open('$o/b1.json'));print(d['value'],d['ms_per_step'])")"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_$r.json 2> $o/b4_$r.err || { tail $o/b4_$r.err; exit 1; }
  echo "b4 r$r $(python -c "import json;d=json.load(open('$o/b4_$r.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/profb4 -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/profb4.log 2>&1 || exit 1
db=$(ls $o/profb4/*/run_results.db $o/profb4/run_results.db 2>/dev/null | head -1)
python tools/timeline.py $db --prologue > $o/prologue_b4.txt 2>&1 || exit 1
python tools/kernel_breakdown.py $db --top 40 > $o/breakdown_b4.txt 2>&1 || exit 1
rm -rf $o/profb4
head -2 $o/prologue_b4.txt
for r in 1 2; do
for e in "JR_HALO_NORM=1" "JR_HALO_NORM=0" "JR_HALO_RES=0"; do
  env $e timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/ab_b1.json 2> $o/ab_b1.err || { tail $o/ab_b1.err; exit 1; }
  env $e timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/ab_b4.json 2> $o/ab_b4.err || { tail $o/ab_b4.err; exit 1; }
  echo "r$r $e b1 $(python -c "import json;d=json.load(open('$o/ab_b1.json'));print(d['value'],d['ms_per_step'])") b4 $(python -c "import json;d=json.load(open('$o/ab_b4.json'));print(d['value'],d['ms_per_step'])")"
done
done
