# batch parts merged into one graph (--split N): tests + A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/merge
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "split or graph_replay" -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { tail -30 $o/test.log; exit 1; }
tail -1 $o/test.log
: > $o/ab.log
run() { echo "== $*" >> $o/ab.log; timeout -k 10 200 python bench.py --steps 20 "$@" 2>>$o/ab.err | cut -c 80-200 >> $o/ab.log; }
run
run --split 2
run --split 4
run --split 2 --no-merge-parts
run --batch 8 --split 2
run --batch 8
run --split 2
run
cat $o/ab.log
