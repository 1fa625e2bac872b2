#!/bin/bash
# Round 6: same-box A/B of the batch-1 persistent pyramid (CORR_PERSIST_B1) on the batch-1 extras.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_b1_ab}
mkdir -p $o
SK=fp32_b1_fps,hires_b1,small_b1_sync_32it_mixed
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 600 python -u dev/probes/bench_with.py CORR_PERSIST_B1=$v -- --steps 3 --warmup 2 --extras on --skip-extras $SK > $o/b_$v.json 2> $o/b_$v.err || { tail $o/b_$v.err; exit 1; }
    python -c "
import json; d=json.load(open('$o/b_$v.json'))
ex=d.get('extras',{})
print('CORR_PERSIST_B1=$v', ' '.join(f'{k}={v[\"value\"]:.1f}' for k,v in ex.items() if isinstance(v, dict) and 'value' in v))
"
  done
done
