#!/bin/bash
# Round 6: same-box A/B of the early context-encoder backward (FusedModel.EARLY_CE).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_ce_early_ab}
mkdir -p $o
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python -u dev/probes/train_with.py FusedModel.EARLY_CE=$v -- --steps 20 > $o/e$v.json 2> $o/e$v.err || { tail $o/e$v.err; exit 1; }
    echo "r$r EARLY_CE=$v $(python -c "import json;d=json.loads(open('$o/e$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['loss'])")"
  done
done
