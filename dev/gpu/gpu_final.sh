# all GPU tests, smoke, headline bench, and a kernel trace of the pipelined batch-1 bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/final
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1 || { tail -30 $o/gputests.log; exit 1; }
tail -2 $o/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err
cut -c 1-250 $o/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_b1 -o run -- python3 bench.py --batch 1 --steps 5 --warmup 2 > $o/prof_b1.log 2>&1
ls $o/prof_b1
