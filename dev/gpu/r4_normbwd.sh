#!/bin/bash
# Round 4: isolated instance-norm backward rate at the config-5 encoder shapes
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r4_normbwd}
mkdir -p $o
timeout -k 10 200 python -u dev/probes/norm_bwd_bench.py > $o/bench.txt 2>&1 || { tail -30 $o/bench.txt; exit 1; }
cat $o/bench.txt
