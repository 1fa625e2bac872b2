#!/bin/bash
# Round 5: raft_small 12-iteration stream after the raft_large extras: leaked engines or GPU state?
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_extras_ab2}
mkdir -p $o
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --step-times --skip-extras "b1_sync_u8,small_b1_fps_32it,small_b1_sync_32it,fp32_b1_fps,hires_b1" > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
grep "^extra " $o/bench.err
python -c "
import json; d=json.load(open('$o/bench.json')); e=d['extras']
print({k: (v.get('value'), v.get('step_ms_p50') or v.get('latency_ms_p50')) for k, v in e.items() if isinstance(v, dict)})
"
