#!/bin/bash
# Round 6: 1088x1920 batch 1 with the batch-1 prologue lanes (context encoder lane + one batch-2 feature-encoder chain;
# PRO_PIXELS raised) vs the default one-lane prologue at that size.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_hires_lanes}
mkdir -p $o
for r in 1 2; do
  for v in 28160 100000; do
    timeout -k 10 300 python -u dev/probes/bench_with.py PRO_PIXELS=$v -- --batch 1 --height 1088 --width 1920 --extras off --steps 20 > $o/p$v.json 2> $o/p$v.err || { tail $o/p$v.err; exit 1; }
    echo "r$r PRO_PIXELS=$v $(python -c "import json;d=json.load(open('$o/p$v.json'));print(d['value'],d['ms_per_step'],d['config'].get('cross_batch_pipeline'))")"
  done
done
