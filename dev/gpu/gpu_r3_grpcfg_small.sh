#!/bin/bash
# Tile config of raft_small's batch-1 grouped convcorr1 + convflow2 launch (JR_CFG_OVERRIDE on convcorr1).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/grpcfg_s
mkdir -p $o
for r in 1 2; do
  for c in 15 4 24 23 2 5; do
    JR_CFG_OVERRIDE="me.convcorr1=$c" timeout -k 10 200 python -u bench.py --extras off --arch raft_small --batch 1 --steps 40 > $o/s1_$c$r.json 2> $o/s1_$c$r.err || exit $?
    python -c "import json; d=json.load(open('$o/s1_$c$r.json')); print('small b1 cfg=$c', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
