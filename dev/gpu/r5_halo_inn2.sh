#!/bin/bash
# Round 5: packed normalising loader -- tests, variant costs, then headline + training.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_halo_inn2}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_engine_gpu.py tests/test_fused_train_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for f in inn,stats inn,res,stats,xn; do
  timeout -k 10 180 python -u tools/conv_bench.py l1 l2 l3 --fused $f > $o/f_$f.txt 2>&1 || { tail $o/f_$f.txt; exit 1; }
  echo "== $f"; grep -E "^l|halo 10[0-6]" $o/f_$f.txt
done
OUT=$(basename $o)/q bash dev/gpu/r5_quick.sh
