#!/bin/bash
# Input H2D modes at batch 1 / 4: overlapped prefetch (default) vs same-stream copy vs device-resident inputs.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/h2d
mkdir -p $o
for r in 1 2; do
  for m in "" "--sync-h2d" "--no-h2d"; do
    n=$(echo "x$m" | tr -d '-')
    timeout -k 10 200 python -u bench.py --extras off --batch 1 --steps 40 $m > $o/b1_$n$r.json 2> $o/b1_$n$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b1_$n$r.json')); print('b1 $m', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
  for m in "" "--sync-h2d"; do
    n=$(echo "x$m" | tr -d '-')
    timeout -k 10 200 python -u bench.py --extras off --steps 30 $m > $o/b4_$n$r.json 2> $o/b4_$n$r.err || exit $?
    python -c "import json; d=json.load(open('$o/b4_$n$r.json')); print('b4 $m', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
