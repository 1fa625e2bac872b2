#!/bin/bash
# Round 6: halo weight-gradient split count (temporary JR_WG_SLOTS: workgroup slots per conv, default 256).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_wg_slots}
mkdir -p $o
JR_WG_SLOTS=64 timeout -k 10 300 python -u -m pytest tests/test_fused_train_gpu.py tests/test_autograd_gpu.py -x -q -k "wgrad" --timeout 200 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
  for v in ${SLOTS:-256 128 64}; do
    JR_WG_SLOTS=$v timeout -k 10 300 python -u tools/train_bench.py --steps 20 > $o/s$v.json 2> $o/s$v.err || { tail $o/s$v.err; exit 1; }
    echo "r$r slots=$v $(python -c "import json;d=json.loads(open('$o/s$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['loss'])")"
  done
done
