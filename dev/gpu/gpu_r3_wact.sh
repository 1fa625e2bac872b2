#!/bin/bash
# Padding wave tiles skip their MFMAs (+ channel-tile rotation over SIMDs): old / new .so A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/wact
mkdir -p $o
for r in 1 2; do
  for v in new old; do
    cp abso/_C_$v.so jax_raft_amd/_C.so
    for c in 34 22 35; do timeout -k 10 100 python -u tools/conv_one.py convcorr2 $c 200 2>/dev/null | sed "s/^/$v /" || exit $?; done
    timeout -k 10 200 python -u bench.py --extras off --steps 30 > $o/h_$v$r.json 2> $o/h_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/h_$v$r.json')); print('$v headline', d['value'], d['ms_per_step'], d['step_ms_p50'])"
    timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 > $o/b1_$v$r.json 2> $o/b1_$v$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$v$r.json')); print('$v b1', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
cp abso/_C_new.so jax_raft_amd/_C.so
