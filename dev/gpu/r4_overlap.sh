#!/bin/bash
# Round 4: does the pipelined batch-1 graph overlap the next pair's prologue with the loop?
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_overlap
mkdir -p $o
for c in "raft_small:32" "raft_large:32"; do
  a=${c%%:*}; it=${c##*:}
  timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_$a -o run -- python3 bench.py --arch $a --batch 1 --iters $it --steps 6 --warmup 2 --extras off > $o/prof_$a.log 2>&1 || { tail $o/prof_$a.log; exit 1; }
  db=$(ls $o/prof_$a/*/run_results.db $o/prof_$a/run_results.db 2>/dev/null | head -1)
  python tools/overlap.py $db --list 120 > $o/overlap_$a.txt 2>&1 || { cat $o/overlap_$a.txt; exit 1; }
  rm -rf $o/prof_$a
  head -8 $o/overlap_$a.txt
done
