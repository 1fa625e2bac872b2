#!/bin/bash
# Round 5: A/B of engine lowering choices at the headline (dev/probes/bench_with.py), alternating runs.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_ab}
mkdir -p $o
: > $o/ab.txt
for r in 1 2; do
  for v in ${VARIANTS:-base MASK_PARITY=1}; do
    a=$v; [ "$v" = "base" ] && a=""
    timeout -k 10 300 python -u dev/probes/bench_with.py $a -- --batch ${B:-4} --extras off --steps 20 > $o/one.json 2> $o/one.err || { tail $o/one.err; exit 1; }
    echo "r$r $v $(python -c "import json;d=json.load(open('$o/one.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")" | tee -a $o/ab.txt
  done
done
