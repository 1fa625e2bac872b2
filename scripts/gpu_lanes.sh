set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "flow_lane or streams or split" > gpurun_out/t_lanes.log 2>&1; rc=$?; tail -3 gpurun_out/t_lanes.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 VARIANTS=";--flow-lane mask;;--flow-lane mask" bash scripts/gpu_variants.sh || exit 1
BATCH=4 ARCHS=raft_large TAG=mask BENCH_ARGS="--flow-lane mask" bash scripts/gpu_b1.sh
