#!/bin/bash
# Round 6: prologue lanes A/B (PRO_LANES auto vs off) on the full bench (all extras), same box.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_prolanes}
mkdir -p $o
summ() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras") or {}
print(round(d["value"], 1), " ".join(f"{k}={v['value']}" for k, v in ex.items() if isinstance(v, dict) and "value" in v))
PY
}
for r in 1 2; do
  for v in auto off; do
    timeout -k 10 600 python -u dev/probes/bench_with.py PRO_LANES=$v -- > $o/full_$v.json 2> $o/full_$v.err || { tail $o/full_$v.err; exit 1; }
    echo "r$r PRO_LANES=$v $(summ $o/full_$v.json)"
  done
done
