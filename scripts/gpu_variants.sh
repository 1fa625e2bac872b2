# bench.py schedule variants (one line each: args -> pairs/s, ms/step)
set -o pipefail
IFS=';' read -ra VARS <<< "${VARIANTS:-;--flow-lane main;--double-buffer;--mask-head fused;--streams off}"
for a in "${VARS[@]}"; do
  echo -n "== [$a] "
  timeout -k 10 200 python bench.py --steps ${STEPS:-20} $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1
done
