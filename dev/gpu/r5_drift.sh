#!/bin/bash
# Round 5: drift of the engine vs the fp32 golden at the headline config (tools/drift.py measure).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_drift}
mkdir -p $o
timeout -k 10 600 python -u tools/drift.py measure --json $o/drift.json > $o/drift.txt 2>&1 || { tail -30 $o/drift.txt; exit 1; }
cat $o/drift.txt
