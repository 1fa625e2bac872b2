# Fused training path: gradient tests + step timing (tools/train_bench.py, config 5 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/train
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_fused_train_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for i in 1 2; do
timeout -k 10 200 python3 tools/train_bench.py --steps 20 --warmup 5 > $o/tb.log 2>&1
tail -1 $o/tb.log | cut -c1-200
done
