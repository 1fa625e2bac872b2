# Graph-pipelined bench A/B (one graph = loop of batch i || prologue of batch i+1)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/copipe
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "graph_pipelined or pipelined_submit" -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { tail -40 $o/test.log; exit 1; }
tail -2 $o/test.log
: > $o/ab.log
for a in "" "--pipeline graph" "" "--pipeline graph" "--batch 1 --pipeline graph" "--batch 1" "--arch raft_small --pipeline graph" "--arch raft_small --batch 1 --pipeline graph" "--final-only --pipeline graph"; do
  echo "== $a" >> $o/ab.log
  timeout -k 10 200 python bench.py --steps 20 $a 2>>$o/ab.err | cut -c 1-330 >> $o/ab.log
done
cat $o/ab.log
