#!/bin/bash
# Round 5: HIP runtime settings vs the graph-edge / queued-replay costs: headline (lane schedule,
# three cross-lane edges per iteration) and the gate probe (gate off), alternating settings.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_rtenv_ab}
mkdir -p $o
: > $o/ab.txt
for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "GPU_STREAMOPS_CP_WAIT=1" "AMD_DIRECT_DISPATCH=0"; do
  env $e timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 > $o/one.json 2> $o/one.err || { echo "$e bench failed" | tee -a $o/ab.txt; tail -3 $o/one.err; continue; }
  echo "$e b4 $(python -c "import json;d=json.load(open('$o/one.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")" | tee -a $o/ab.txt
  env $e timeout -k 10 120 python3 dev/probes/gate_trace.py --gate 0 --n 12 2>/dev/null | tail -1 | cut -c1-60 | sed "s/^/$e /" | tee -a $o/ab.txt
done
