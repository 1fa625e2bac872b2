set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_autograd_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "lookup or corr or golden or matches" > gpurun_out/t_lookup.log 2>&1; rc=$?; tail -3 gpurun_out/t_lookup.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=";--streams off;--batch 1" bash scripts/gpu_variants.sh || exit 1
BATCH=4 ARCHS=raft_large TAG=lk BENCH_ARGS="--streams off" bash scripts/gpu_b1.sh
