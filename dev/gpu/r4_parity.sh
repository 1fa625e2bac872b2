#!/bin/bash
# Round 4: parity-buffered mask-lane operands (no E_MASK join) -- engine tests, race check, A/B, timeline
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_parity
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_drift.py tests/test_fused_train_gpu.py -k "not wgrad" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
for pv in 1 0; do
  JR_MASK_PARITY=$pv timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4.json 2> $o/b4.err || { tail $o/b4.err; exit 1; }
  echo "r$r parity=$pv b4 $(python -c "import json;d=json.load(open('$o/b4.json'));print(d['value'],d['ms_per_step'])")"
done
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit 1
db=$(ls $o/prof/*/run_results.db $o/prof/run_results.db 2>/dev/null | head -1)
python tools/timeline.py $db --iter 10 > $o/timeline_b4.txt 2>&1 || exit 1
python tools/kernel_breakdown.py $db --top 40 > $o/breakdown_b4.txt 2>&1 || exit 1
rm -rf $o/prof
head -16 $o/timeline_b4.txt
