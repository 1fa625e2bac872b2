#!/bin/bash
# Round 5 vs round 4 tree (worktree .r4tree, its own _C.so) on the same box: per-pair sync latency.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r5_sync_ab}
mkdir -p $o
: > $o/ab.txt
for r in 1 2; do
  for t in . .r4tree; do
    for arch in raft_small raft_large; do
      timeout -k 10 200 python3 -u dev/probes/sync_ab.py $t --arch $arch >> $o/ab.txt 2> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
    done
  done
done
cat $o/ab.txt
