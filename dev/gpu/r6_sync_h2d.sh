#!/bin/bash
# Round 6: headline with the prefetched H2D (copy stream, default) vs the inputs copied on the compute stream (--sync-h2d).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_sync_h2d}
mkdir -p $o
for r in 1 2; do
  for v in prefetch sync; do
    a=""; [ $v = sync ] && a="--sync-h2d"
    timeout -k 10 300 python -u bench.py --extras off --steps 20 $a > $o/$v.json 2> $o/$v.err || { tail $o/$v.err; exit 1; }
    echo "r$r $v $(python -c "import json;d=json.load(open('$o/$v.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")"
  done
done
