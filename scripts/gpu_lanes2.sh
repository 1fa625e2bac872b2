set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lanes.log 2>&1; rc=$?; tail -3 gpurun_out/t_lanes.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 VARIANTS=";--flow-lane side;--arch raft_small;--batch 8;--batch 2" bash scripts/gpu_variants.sh || exit 1
