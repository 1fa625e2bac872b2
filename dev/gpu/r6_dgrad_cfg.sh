#!/bin/bash
# Round 6: the training ConvGRU data gradients (EPI_BWD) pinned to other tile configs: config 34 spills
# (scratch 44 B) with the EPI_BWD epilogue, which the plain-epilogue autotune does not see.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_dgrad_cfg}
mkdir -p $o
for c in 34 20 22 18 25 16; do
  timeout -k 10 300 python -u dev/probes/train_retune.py --set $c --steps 20 > $o/c$c.txt 2> $o/c$c.err || { tail $o/c$c.err; exit 1; }
  echo "cfg $c $(head -1 $o/c$c.txt | cut -c1-110)"
done
