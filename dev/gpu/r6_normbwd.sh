#!/bin/bash
# Round 6: standalone encoder norm-backward timing + per-kernel trace stats.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_normbwd}
mkdir -p $o
timeout -k 10 120 python -u dev/probes/norm_bwd_bench.py > $o/bench.txt 2>&1 || { tail $o/bench.txt; exit 1; }
cat $o/bench.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 dev/probes/norm_bwd_bench.py > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 $f | head -12
