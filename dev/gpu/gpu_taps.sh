set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "taps or golden or flow_lane or convex" > gpurun_out/t_taps.log 2>&1; rc=$?; tail -3 gpurun_out/t_taps.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 VARIANTS=";;--batch 1;--arch raft_small" bash scripts/gpu_variants.sh || exit 1
BATCH=4 ARCHS=raft_large TAG=taps BENCH_ARGS="--streams off" bash scripts/gpu_b1.sh > /dev/null 2>&1; grep -i "taps" gpurun_out/b4taps/raft_large_breakdown.txt
