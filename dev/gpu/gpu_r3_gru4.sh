#!/bin/bash
# Same-box A/B: mask-lane parity halves (JR_GRU_PARITY=1, no E_MASK) vs one hm copy + E_MASK before the
# last ConvGRU stage (0), x GEMM 2 on 8 / 16 waves (JR_GRU_G2=0 / 1).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/gru4
mkdir -p $o
JR_GRU_PARITY=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "fused_gru or lane" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in "0 0" "0 1" "1 0" "1 1"; do
    set -- $v
    JR_GRU_PARITY=$1 JR_GRU_G2=$2 timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/b4_$1$2$r.json 2> $o/b4_$1$2$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b4_$1$2$r.json')); print('parity=$1 g2=$2', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
