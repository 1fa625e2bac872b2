#!/bin/bash
# Round 5: the host-gate effect under HIP kernel-argument placement settings, and the raft_small
# 12-iteration p99 steps vs Python garbage collection.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_gate2}
mkdir -p $o
: > $o/gate_env.txt
for e in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_KERNARG_OPTIMIZATION=0"; do
  for g in 0 1; do
    echo "$e" >> $o/gate_env.txt
    env $e timeout -k 10 120 python3 dev/probes/gate_trace.py --gate $g --n 12 >> $o/gate_env.txt 2>&1 || { tail -5 $o/gate_env.txt; exit 1; }
  done
done
grep -v amdgpu.ids $o/gate_env.txt
timeout -k 10 200 python3 -u dev/probes/p99_probe.py --steps 200 > $o/p99.txt 2>&1 || { tail -5 $o/p99.txt; exit 1; }
grep -v amdgpu.ids $o/p99.txt
