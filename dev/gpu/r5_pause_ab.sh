#!/bin/bash
# Round 5: are the raft_small extras slower after the headline because of the GPU's state (idle first)?
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pause_ab}
mkdir -p $o
: > $o/ab.txt
for p in 0 20 0 20; do
  timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --extra-pause $p --skip-extras "b1_fps,b1_sync,b1_sync_u8,small_b1_fps_32it,fp32_b1_fps,hires_b1" > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/bench.json')); e=d['extras']
print('pause=$p', {k: (v.get('value'), v.get('step_ms_p50') or v.get('latency_ms_p50')) for k, v in e.items() if isinstance(v, dict) and k.startswith('small')})
" | tee -a $o/ab.txt
done
