set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "convex" > gpurun_out/t_convex.log 2>&1; rc=$?; tail -3 gpurun_out/t_convex.log; [ $rc -eq 0 ] || exit $rc
for a in "--convex fused" "--convex head" "--convex head --streams off" "--convex head --batch 1"; do echo "== $a"; timeout -k 10 200 python bench.py --steps 20 $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1; done
BATCH=4 ARCHS=raft_large TAG=head BENCH_ARGS="--convex head --streams off" bash scripts/gpu_b1.sh
