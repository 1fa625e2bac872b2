#!/bin/bash
# Round 6: training side streams at high priority -- full bench with PRO_LANES auto / off.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_prio}
mkdir -p $o
summ() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras") or {}
print(round(d["value"], 1), " ".join(f"{k}={v['value']}" for k, v in ex.items() if isinstance(v, dict) and "value" in v))
PY
}
for v in off auto; do
  timeout -k 10 600 python -u dev/probes/bench_with.py PRO_LANES=$v -- > $o/p_$v.json 2> $o/p_$v.err || { tail $o/p_$v.err; exit 1; }
  echo "prio PRO_LANES=$v $(summ $o/p_$v.json)"
done
timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/tb.json 2> $o/tb.err || { tail $o/tb.err; exit 1; }
cut -c1-150 $o/tb.json
