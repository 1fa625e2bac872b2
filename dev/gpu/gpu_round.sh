# One GPU round: all GPU tests, smoke(), headline bench + like-for-like variants,
# a rocprofv3 kernel-stats profile of the headline bench, and the training bench.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/round
o=gpurun_out/round
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1 || { tail -30 $o/gputests.log; exit 1; }
tail -2 $o/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 200 python bench.py > $o/bench.json 2> $o/bench.err
cat $o/bench.json
: > $o/variants.log
for a in "--steps 20" "--batch 1 --steps 20" "--arch raft_small --batch 1 --steps 20" "--arch raft_small --steps 20" "--batch 8 --steps 20" "--final-only --steps 20" "--iters 12 --steps 20"; do
  echo "== $a" >> $o/variants.log
  timeout -k 10 200 python bench.py $a 2>/dev/null | grep '"value"' >> $o/variants.log
done
cut -c 1-200 $o/variants.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 > $o/prof.log 2>&1
find $o/prof -name '*kernel_stats.csv' | head -3
timeout -k 10 300 python tools/train_bench.py > $o/train.json 2> $o/train.err
cat $o/train.json
