#!/bin/bash
# Round 6: encoder weight gradients on plan lane 1 as their output gradients appear (EncoderTrain.WGRAD_LANE):
# training numerics tests + same-box A/B.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_wgrad_lane}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python -u dev/probes/train_with.py EncoderTrain.WGRAD_LANE=$v -- --steps 20 > $o/w$v.json 2> $o/w$v.err || { tail $o/w$v.err; exit 1; }
    echo "r$r WGRAD_LANE=$v $(python -c "import json;d=json.loads(open('$o/w$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['loss'])")"
  done
done
