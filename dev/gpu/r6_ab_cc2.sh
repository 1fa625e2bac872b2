#!/bin/bash
# Round 6: same-box A/B of the cc2 batch-4 tile config (113: 6-wave whole-cout tile, 125: 12-wave
# SIMD-balanced tile), plus the new training-oracle GPU tests.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_ab_cc2}
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_fused_train_gpu.py -x -q -k "trajectory or oracle" --timeout 300 --timeout-method thread > $o/train_tests.txt 2>&1 || { tail -30 $o/train_tests.txt; exit 1; }
tail -1 $o/train_tests.txt
for r in 1 2 3; do
  for c in 125 113; do
    JR_CFG_OVERRIDE="me.convcorr2=$c" timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 > $o/b4_$c.json 2> $o/b4_$c.err || { tail $o/b4_$c.err; exit 1; }
    echo "cc2 cfg $c: $(python -c "import json;d=json.load(open('$o/b4_$c.json'));print(d['value'],d['ms_per_step'])")"
  done
done
