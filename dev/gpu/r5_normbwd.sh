#!/bin/bash
# Round 5: norm backward with batched row loads -- fused training tests, microbench, training step.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_normbwd}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 200 python -u dev/probes/norm_bwd_bench.py > $o/nb.txt 2>&1 || { tail $o/nb.txt; exit 1; }
grep -v amdgpu $o/nb.txt | tail -20
for r in 1 2; do
timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train_$r.json 2> $o/train_$r.err || { tail $o/train_$r.err; exit 1; }
echo "train $(tail -1 $o/train_$r.json | cut -c1-150)"
done
