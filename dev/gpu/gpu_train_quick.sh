set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_fused_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_train.log 2>&1; rc=$?; tail -3 gpurun_out/t_train.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_train.log | head -20; exit $rc; }
for i in 1 2; do timeout -k 10 300 python tools/train_bench.py 2>/dev/null | tail -1 | cut -c1-120 || exit 1; done
