set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv1x1 or golden or flow_lane or convex or split" > gpurun_out/t_c1.log 2>&1; rc=$?; tail -3 gpurun_out/t_c1.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 VARIANTS=";;--batch 1" bash scripts/gpu_variants.sh || exit 1
BATCH=4 ARCHS=raft_large TAG=c1 BENCH_ARGS="--streams off" bash scripts/gpu_b1.sh > /dev/null 2>&1; grep -i "conv1x1\|taps_gemm" gpurun_out/b4c1/raft_large_breakdown.txt; head -4 gpurun_out/b4c1/raft_large_timeline.txt
