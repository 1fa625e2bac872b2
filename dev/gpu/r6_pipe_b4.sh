#!/bin/bash
# Round 6: headline batch 4 with the cross-batch graph pipeline (loop i || prologue i+1) vs the default.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_pipe_b4}
mkdir -p $o
for r in 1 2; do
  for v in auto graph; do
    timeout -k 10 300 python -u bench.py --extras off --steps 20 --pipeline $v > $o/$v.json 2> $o/$v.err || { tail $o/$v.err; exit 1; }
    echo "r$r pipeline=$v $(python -c "import json;d=json.load(open('$o/$v.json'));print(d['value'],d['ms_per_step'],d['config'].get('cross_batch_pipeline'))")"
  done
done
