set -o pipefail
for q in 4 16 32 4 16 32; do echo -n "== bench GPU_MAX_HW_QUEUES=$q "; GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1; done
for q in 4 16; do echo -n "== train GPU_MAX_HW_QUEUES=$q "; GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/train_bench.py 2>/dev/null | tail -1 | cut -c60-90 || exit 1; done
