set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_fused_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gs.log 2>&1; rc=$?; tail -2 gpurun_out/t_gs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/train_bench.py 2>/dev/null | tail -1 | cut -c1-110
