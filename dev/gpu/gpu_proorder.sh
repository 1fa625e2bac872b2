# pipelined graph: prologue nodes created first (JR_PIPE_PROLOGUE=first) vs loop first
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/proorder
mkdir -p $o
JR_PIPE_PROLOGUE=first timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "pipelined" -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { tail -30 $o/test.log; exit 1; }
tail -1 $o/test.log
: > $o/ab.log
run() { echo "== $* $BA" >> $o/ab.log; env "$@" timeout -k 10 200 python bench.py --steps 20 $BA 2>>$o/ab.err | cut -c 80-200 >> $o/ab.log; }
for BA in "--batch 1" "--arch raft_small" "--batch 1" "--pipeline graph"; do
run JR_PIPE_PROLOGUE=loop
run JR_PIPE_PROLOGUE=first
done
cat $o/ab.log
