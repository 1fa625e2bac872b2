#!/bin/bash
# Round 3 re-entry: full GPU suite, smoke, headline bench with extras, kernel stats of the headline.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r3v
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1 || { tail -30 $o/gputests.log; exit 1; }
tail -2 $o/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
tail -1 $o/smoke.log
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
cat $o/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof.log 2>&1 || exit $?
find $o/prof -name '*kernel_stats.csv'
