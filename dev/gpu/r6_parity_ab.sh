#!/bin/bash
# Round 6: same-box A/B of the parity-buffered mask lane (no E_MASK join) at batch 4.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_parity}
mkdir -p $o
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python -u dev/probes/bench_with.py MASK_PARITY=$v -- --batch 4 --extras off --steps 20 > $o/b4_$v.json 2> $o/b4_$v.err || { tail $o/b4_$v.err; exit 1; }
    echo "MASK_PARITY=$v $(python -c "import json;d=json.load(open('$o/b4_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
