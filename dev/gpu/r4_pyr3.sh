#!/bin/bash
# Round 4: pyramid write-locality experiment (query-tile-major levels 0 / 1, JR_PYR_QT).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_pyr3
mkdir -p $o
timeout -k 10 200 python -u tools/corr_bench.py pyr --batch 4 > $o/bench.txt 2>&1 && JR_PYR_QT=1 timeout -k 10 200 python -u tools/corr_bench.py pyr --batch 4 >> $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
cat $o/bench.txt
