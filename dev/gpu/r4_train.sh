#!/bin/bash
# Round 4: halo convs in the training encoders (forward + stride-1 data gradients): tests + A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_train
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_halo_gpu.py tests/test_fused_train_gpu.py tests/test_train_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
for hv in 1 0 1; do
  JR_CONV_HALO=$hv timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_h$hv.json 2> $o/train_h$hv.err || { tail $o/train_h$hv.err; exit 1; }
  echo "halo=$hv $(tail -1 $o/train_h$hv.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 tools/train_bench.py --steps 5 --warmup 3 > $o/prof.log 2>&1 || exit 1
db=$(ls $o/prof/*/run_results.db $o/prof/run_results.db 2>/dev/null | head -1)
python tools/kernel_breakdown.py $db --marker "" --steps 8 --top 40 > $o/breakdown.txt 2>&1 || exit 1
rm -rf $o/prof
head -30 $o/breakdown.txt
