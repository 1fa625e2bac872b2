#!/bin/bash
# Round 5: does creating torch's side-stream pool before the engine slow the engine's lanes?
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pipe_first_ab}
mkdir -p $o
: > $o/ab.txt
for r in 1 2; do
  for f in "" "--pipelined-first"; do
    for arch in raft_small raft_large; do
      timeout -k 10 200 python3 -u dev/probes/sync_ab.py . --arch $arch $f >> $o/ab.txt 2> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
    done
  done
done
cat $o/ab.txt
