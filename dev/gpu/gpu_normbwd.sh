# norm backward unroll A/B: fused training tests + train bench, old vs new library
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/normbwd
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { tail -30 $o/test.log; exit 1; }
tail -1 $o/test.log
: > $o/ab.log
for k in 1 2; do
  echo "== new" >> $o/ab.log; timeout -k 10 300 python tools/train_bench.py | cut -c 1-120 >> $o/ab.log
  echo "== old" >> $o/ab.log; JR_NATIVE_SO=jax_raft_amd/_C_old.so timeout -k 10 300 python tools/train_bench.py | cut -c 1-120 >> $o/ab.log
done
cat $o/ab.log
