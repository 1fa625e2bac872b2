#!/bin/bash
# Round 4: where does the persistent pyramid spend its time (stores off / MFMA off).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_pyr4
mkdir -p $o
: > $o/bench.txt
for d in 0 1 2 3; do
  echo "dbg=$d" >> $o/bench.txt
  JR_PYR_DBG=$d timeout -k 10 200 python -u tools/corr_bench.py pyr --batch 4 >> $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
done
cat $o/bench.txt
