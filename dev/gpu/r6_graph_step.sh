#!/bin/bash
# Round 6: whole-step graph capture (TrainConfig.graph_step) vs the default eager step around the native plans.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_graph_step}
mkdir -p $o
for r in 1 2; do
  for v in eager graph; do
    a=""; [ $v = graph ] && a="--graph-step"
    timeout -k 10 300 python -u tools/train_bench.py --steps 20 $a > $o/$v.json 2> $o/$v.err || { tail $o/$v.err; exit 1; }
    echo "r$r $v $(python -c "import json;d=json.loads(open('$o/$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['loss'])")"
  done
done
