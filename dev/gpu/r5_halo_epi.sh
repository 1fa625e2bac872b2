#!/bin/bash
# Round 5: cost of the fused instance-norm pieces in the halo 3x3 conv (stats partials, input norm,
# residual) on the encoder layers, per tile config.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_halo_epi}
mkdir -p $o
for f in "" stats inn inn,stats inn,res,stats inn,res,stats,xn; do
  timeout -k 10 180 python -u tools/conv_bench.py l1 l2 l3 ${f:+--fused $f} > $o/f_${f:-plain}.txt 2>&1 || { tail $o/f_${f:-plain}.txt; exit 1; }
  echo "== ${f:-plain}"; grep -v "^ *halo 1[0-9][0-9] .*[0-9]\{3\}\.[0-9] us" $o/f_${f:-plain}.txt | head -30
done
