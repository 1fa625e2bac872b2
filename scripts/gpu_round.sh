# One GPU round: kernel/engine tests, headline bench + the like-for-like
# batch-1 configs, and a rocprofv3 kernel-stats profile of the headline bench.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/round
o=gpurun_out/round
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1
tail -3 $o/gputests.log
timeout -k 10 200 python bench.py > $o/bench.json 2> $o/bench.err
cat $o/bench.json
for a in "--batch 1 --steps 20" "--arch raft_small --batch 1 --steps 20" "--arch raft_small" "--batch 8" "--final-only"; do
  echo "== $a" >> $o/variants.log
  timeout -k 10 200 python bench.py $a >> $o/variants.log 2>&1
done
cat $o/variants.log | cut -c 1-220
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 > $o/prof.log 2>&1
find $o/prof -name '*kernel_stats.csv' | head -3
