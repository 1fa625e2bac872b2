#!/bin/bash
# Round 4: sources of the small framework kernels in the training step
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_fills
mkdir -p $o
PYTHONPATH=. timeout -k 10 400 python -u dev/probes/train_fill_sources.py > $o/fills.txt 2>&1 || { tail -30 $o/fills.txt; exit 1; }
grep -v "^$" $o/fills.txt | head -80
