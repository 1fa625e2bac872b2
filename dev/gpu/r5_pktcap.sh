#!/bin/bash
# Round 5: DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 (graph kernel packets captured at instantiation) vs the
# runtime default: gate probe (gate on / off) and the full bench with extras.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pktcap}
mkdir -p $o
: > $o/ab.txt
for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  for g in 0 1; do
    env $e timeout -k 10 120 python3 dev/probes/gate_trace.py --gate $g --n 12 2>/dev/null | tail -1 | sed "s/^/$e /" | tee -a $o/ab.txt
  done
done
for e in "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "X=0"; do
  env $e timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/bench.json')); e=d['extras']
print('$e', 'headline', d['value'], {k: (v.get('value'), v.get('step_ms_p50') or v.get('latency_ms_p50'), v.get('step_ms_p99') or v.get('latency_ms_p99')) for k, v in e.items() if isinstance(v, dict)})
" | tee -a $o/ab.txt
  cp $o/bench.json "$o/bench_${e%%=*}.json"
done
