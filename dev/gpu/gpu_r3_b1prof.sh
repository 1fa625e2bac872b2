#!/bin/bash
# Batch-1 kernel traces (raft_large, raft_small) for the iteration timeline.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/b1prof
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/large -o run -- python3 bench.py --batch 1 --steps 5 --warmup 2 --extras off > $o/large.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/small -o run -- python3 bench.py --arch raft_small --batch 1 --steps 5 --warmup 2 --extras off > $o/small.log 2>&1 || exit $?
