#!/bin/bash
# Round 6: norm kernels with per-block LDS coefficients -- probe, numerics tests, train + inference benches.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_norm_check}
mkdir -p $o
timeout -k 10 120 python -u dev/probes/norm_bwd_bench.py > $o/probe.txt 2>&1 || { tail $o/probe.txt; exit 1; }
cat $o/probe.txt
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_train_gpu.py tests/test_drift.py tests/test_engine_f32.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train.json 2> $o/train.err || { tail $o/train.err; exit 1; }
cat $o/train.json
timeout -k 10 300 python -u bench.py --extras off --steps 20 > $o/b4.json 2> $o/b4.err || { tail $o/b4.err; exit 1; }
python -c "import json;d=json.load(open('$o/b4.json'));print('b4',d['value'],d['ms_per_step'])"
