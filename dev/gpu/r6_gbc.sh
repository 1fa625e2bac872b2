#!/bin/bash
# Round 6: hipGraph branch concurrency probe + headline with / without loop lanes.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_gbc}
mkdir -p $o
timeout -k 10 120 python -u dev/probes/graph_branch_concurrency.py > $o/probe.txt 2>&1 || { tail $o/probe.txt; exit 1; }
cat $o/probe.txt
for v in auto off; do
  timeout -k 10 300 python -u bench.py --extras off --steps 20 --streams $v > $o/s_$v.json 2> $o/s_$v.err || { tail $o/s_$v.err; exit 1; }
  echo "streams=$v $(python -c "import json;d=json.load(open('$o/s_$v.json'));print(d['value'],d['ms_per_step'],d['config'].get('concurrent_branches'))")"
done
