#!/bin/bash
# Tile config of the batch-1 grouped convcorr2 + convflow2 launch (JR_CFG_OVERRIDE on convcorr2).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/grpcfg
mkdir -p $o
for r in 1 2; do
  for c in 23 2 14 24 12 4; do
    JR_CFG_OVERRIDE="me.convcorr2=$c" timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$c$r.json 2> $o/b1_$c$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$c$r.json')); print('b1 cfg=$c', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
