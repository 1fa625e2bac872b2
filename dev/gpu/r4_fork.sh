#!/bin/bash
# Round 4: pipelined / merged graphs with a fork root (JR_PIPE_FORK A/B) + overlap of one step.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_fork
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "pipelin or merge or split or part" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
for f in 1 0; do
  for c in "raft_small:1" "raft_large:1" "raft_large:4"; do
    a=${c%%:*}; b=${c##*:}
    JR_PIPE_FORK=$f timeout -k 10 200 python -u bench.py --arch $a --batch $b --extras off --steps 20 > $o/${a}_b${b}_f$f.json 2> $o/${a}_b${b}_f$f.err || { tail $o/${a}_b${b}_f$f.err; exit 1; }
    echo "fork=$f $a b$b $(python -c "import json;d=json.load(open('$o/${a}_b${b}_f$f.json'));print(d['value'],d['ms_per_step'])")"
  done
done
for a in raft_small raft_large; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_$a -o run -- python3 bench.py --arch $a --batch 1 --steps 6 --warmup 2 --extras off > $o/prof_$a.log 2>&1 || { tail $o/prof_$a.log; exit 1; }
  db=$(ls $o/prof_$a/*/run_results.db $o/prof_$a/run_results.db 2>/dev/null | head -1)
  python tools/overlap.py $db --list 200 > $o/overlap_$a.txt 2>&1 || { cat $o/overlap_$a.txt; exit 1; }
  rm -rf $o/prof_$a
  sed -n 2,6p $o/overlap_$a.txt
done
