#!/bin/bash
# Round 5: the un-pipelined batch-1 forward (the reference's per-pair protocol): prologue timeline.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pro}
mkdir -p $o
for arch in raft_small raft_large; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/t_$arch -o run -- python3 bench.py --arch $arch --batch 1 --pipeline off --extras off --steps 5 --warmup 2 > $o/t_$arch.log 2>&1 || { tail -5 $o/t_$arch.log; exit 1; }
  f=$(find $o/t_$arch -name '*kernel_trace.csv' | head -1)
  python3 tools/timeline.py $f --prologue > $o/prologue_$arch.txt 2>&1 || true
  python3 tools/timeline.py $f > $o/timeline_$arch.txt 2>&1 || true
  head -60 $o/prologue_$arch.txt
  rm -f $f
done
