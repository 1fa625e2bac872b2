#!/bin/bash
# Round 6: HIP graph-execution queue knob (DEBUG_HIP_FORCE_GRAPH_QUEUES) vs the headline and a prologue trace.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_graphq}
mkdir -p $o
for v in default 1 2 4; do
  if [ $v = default ]; then unset DEBUG_HIP_FORCE_GRAPH_QUEUES; else export DEBUG_HIP_FORCE_GRAPH_QUEUES=$v; fi
  timeout -k 10 300 python -u bench.py --extras off --steps 20 > $o/h_$v.json 2> $o/h_$v.err || { tail $o/h_$v.err; exit 1; }
  echo "graphq=$v $(python -c "import json;d=json.load(open('$o/h_$v.json'));print(d['value'],d['ms_per_step'])")"
done
unset DEBUG_HIP_FORCE_GRAPH_QUEUES
