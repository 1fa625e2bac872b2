#!/bin/bash
# Round 5: packet capture vs default, raft_small 12-iteration stream and sync 32-iteration latency, alternating.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pktcap2}
mkdir -p $o
: > $o/ab.txt
for r in 1 2 3; do
  for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
    env $e timeout -k 10 300 python -u bench.py --arch raft_small --batch 1 --iters 12 --steps 100 --warmup 15 --extras off > $o/one.json 2> $o/one.err || { tail $o/one.err; exit 1; }
    a=$(python -c "import json;d=json.load(open('$o/one.json'));print(d['value'],d['step_ms_p50'],d['step_ms_p99'])")
    b=$(env $e timeout -k 10 200 python3 -u dev/probes/sync_ab.py . --arch raft_small 2>/dev/null | tail -1 | sed 's/.*sync: //')
    echo "r$r $e small12 $a | small sync32 $b" | tee -a $o/ab.txt
  done
done
