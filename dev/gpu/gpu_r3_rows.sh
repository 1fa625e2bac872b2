#!/bin/bash
# Adaptive row chunks for the instance-norm statistics / norm-backward partials: tests + old/new .so A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/rows
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_train_gpu.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2; do
  for v in new old; do
    cp abso/_C_$v.so jax_raft_amd/_C.so
    timeout -k 10 300 python -u bench.py --steps 20 > $o/h_$v$r.json 2> $o/h_$v$r.err || exit $?
    python -c "
import json; d=json.load(open('$o/h_$v$r.json')); x=d['extras']
print('$v headline', d['value'], 'b1', x['b1_fps']['value'], 'small_b1', x['small_b1_fps_32it']['value'], 'train', x['train_pairs_per_s']['value'])"
  done
done
cp abso/_C_new.so jax_raft_amd/_C.so
