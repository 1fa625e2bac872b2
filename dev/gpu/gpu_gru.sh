set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gru.log 2>&1; rc=$?; tail -3 gpurun_out/t_gru.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_gru.log | head; exit $rc; }
STEPS=30 VARIANTS=";;--batch 8" bash scripts/gpu_variants.sh || exit 1
BATCH=4 ARCHS=raft_large TAG=gru bash scripts/gpu_b1.sh > /dev/null 2>&1; cat gpurun_out/b4gru/raft_large_timeline.txt
