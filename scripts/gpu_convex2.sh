set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "convex" > gpurun_out/t_convex.log 2>&1; rc=$?; tail -3 gpurun_out/t_convex.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/convex_bench.py || exit 1
for a in "--convex fused" "--convex head" "--convex head --streams off"; do echo "== $a"; timeout -k 10 200 python bench.py --steps 20 $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1; done
