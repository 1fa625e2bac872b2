#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/r5_split_phases
mkdir -p $o
for args in "--batch 4 --cfg-a 1 --cfg-b 6" "--batch 4 --cfg-a 6 --cfg-b 0" "--batch 1 --cfg-a 7 --cfg-b 3"; do
  timeout -k 10 120 python -u tools/gru_split_phases.py $args >> $o/phases.txt 2>&1 || { tail -20 $o/phases.txt; exit 1; }
done
cat $o/phases.txt
