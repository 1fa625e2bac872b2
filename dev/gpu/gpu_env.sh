# bench.py under HIP runtime environment variants (one line each: env -> pairs/s, ms/step)
set -o pipefail
IFS=';' read -ra VARS <<< "${ENVS:-NONE=1}"
for e in "${VARS[@]}"; do
  echo -n "== [$e] "
  env $e timeout -k 10 ${TMO:-200} python bench.py --steps ${STEPS:-20} $BENCH_ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1
done
