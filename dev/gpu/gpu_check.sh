# Quick GPU check: GPU tests, smoke(), headline bench, training bench.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/check
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1 || { tail -30 $o/gputests.log; exit 1; }
tail -2 $o/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 200 python bench.py --steps 20 > $o/bench.json 2> $o/bench.err
cat $o/bench.json
timeout -k 10 300 python tools/train_bench.py > $o/train.json 2> $o/train.err
cat $o/train.json
