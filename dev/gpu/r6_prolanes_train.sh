#!/bin/bash
# Round 6: is the bench's train extra sensitive to PRO_LANES through the extras before it?
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_prolanes_train}
mkdir -p $o
ALL=b1_fps,b1_sync,b1_sync_u8,small_b1_fps_32it,small_b1_sync_32it,small_b1_fps_12it,small_b1_sync_32it_mixed,fp32_b1_fps,hires_b1
for r in 1 2; do
  for v in auto off; do
    timeout -k 10 600 python -u dev/probes/bench_with.py PRO_LANES=$v -- --steps 5 --skip-extras $ALL > $o/t_$v.json 2> $o/t_$v.err || { tail $o/t_$v.err; exit 1; }
    echo "r$r only-train PRO_LANES=$v $(python -c "import json;d=json.loads(open('$o/t_$v.json').read().strip().splitlines()[-1]);print(d['extras']['train_pairs_per_s']['value'])")"
    timeout -k 10 600 python -u dev/probes/bench_with.py PRO_LANES=$v -- --steps 5 --skip-extras small_b1_fps_32it,small_b1_sync_32it,small_b1_fps_12it,small_b1_sync_32it_mixed > $o/l_$v.json 2> $o/l_$v.err || { tail $o/l_$v.err; exit 1; }
    echo "r$r large-extras PRO_LANES=$v $(python -c "import json;d=json.loads(open('$o/l_$v.json').read().strip().splitlines()[-1]);print(d['extras']['train_pairs_per_s']['value'])")"
  done
done
