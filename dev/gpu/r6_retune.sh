#!/bin/bash
# Round 6: in-situ re-time of the training ConvGRU conv configs with the 256x64 tiles (44..46) as candidates.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_retune}
mkdir -p $o
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv" --timeout 100 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/base_$r.json 2> $o/base_$r.err || { tail $o/base_$r.err; exit 1; }
  cut -c1-140 $o/base_$r.json
  timeout -k 10 300 python -u dev/probes/train_retune.py --steps 15 > $o/retune_$r.txt 2> $o/retune_$r.err || { tail $o/retune_$r.err; exit 1; }
  cut -c1-140 $o/retune_$r.txt
done
