#!/bin/bash
# Round 6: fused training loop forward with the flow-feature / mask-head lane (FusedLoop.FWD_LANES) re-measured.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_fwd_lanes}
mkdir -p $o
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python -u dev/probes/train_with.py FusedLoop.FWD_LANES=$v -- --steps 20 > $o/f$v.json 2> $o/f$v.err || { tail $o/f$v.err; exit 1; }
    echo "r$r FWD_LANES=$v $(python -c "import json;d=json.loads(open('$o/f$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['loss'])")"
  done
done
