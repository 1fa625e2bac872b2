# node copies in creation order (new) vs depth-first (old library): pipelined / split configs
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/copyorder
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "pipelined or split" -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { tail -30 $o/test.log; exit 1; }
tail -1 $o/test.log
: > $o/ab.log
run() { echo "== $* $BA" >> $o/ab.log; env "$@" timeout -k 10 200 python bench.py --steps 20 $BA 2>>$o/ab.err | cut -c 80-200 >> $o/ab.log; }
for BA in "--batch 1" "--pipeline graph" "--arch raft_small" "--split 2" "--batch 1"; do
run JR_X=new
run JR_NATIVE_SO=jax_raft_amd/_C_old.so
done
cat $o/ab.log
