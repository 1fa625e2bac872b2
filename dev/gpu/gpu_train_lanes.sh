set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_fused_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_train.log 2>&1; rc=$?; tail -3 gpurun_out/t_train.log; [ $rc -eq 0 ] || exit $rc
for e in 1 0 1 0; do echo -n "== fwd_lanes=$e "; JR_FUSED_FWD_LANES=$e timeout -k 10 300 python tools/train_bench.py 2>/dev/null | tail -1 | cut -c1-110 || exit 1; done
