set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "corr or golden or lookup or matches or blocked" > gpurun_out/t_pyr.log 2>&1; rc=$?; tail -3 gpurun_out/t_pyr.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 VARIANTS=";--batch 1" bash scripts/gpu_variants.sh || exit 1
BATCH=4 ARCHS=raft_large TAG=pyr bash scripts/gpu_b1.sh > /dev/null 2>&1; grep -i "corr_pyramid\|corr_lookup" gpurun_out/b4pyr/raft_large_breakdown.txt
