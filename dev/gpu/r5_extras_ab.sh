#!/bin/bash
# Round 5: raft_small extras slower inside the full bench than standalone -- which earlier extra does it?
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_extras_ab}
mkdir -p $o
: > $o/ab.txt
for skip in "b1_sync_u8" "b1_fps,b1_sync,b1_sync_u8" "none"; do
  timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --skip-extras "$skip,fp32_b1_fps,hires_b1" > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/bench.json')); e=d['extras']
print('skip=$skip', {k: (v.get('value'), v.get('step_ms_p50') or v.get('latency_ms_p50')) for k, v in e.items() if isinstance(v, dict)})
" | tee -a $o/ab.txt
done
