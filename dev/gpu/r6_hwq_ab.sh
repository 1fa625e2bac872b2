#!/bin/bash
# Round 6: HIP hardware queues per process (GPU_MAX_HW_QUEUES 4 = default vs 8) x prologue lanes, full bench.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_hwq}
mkdir -p $o
summ() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras") or {}
print(round(d["value"], 1), " ".join(f"{k}={v['value']}" for k, v in ex.items() if isinstance(v, dict) and "value" in v))
PY
}
for q in 4 8; do
  for v in auto off; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python -u dev/probes/bench_with.py PRO_LANES=$v -- > $o/q${q}_$v.json 2> $o/q${q}_$v.err || { tail $o/q${q}_$v.err; exit 1; }
    echo "hwq=$q PRO_LANES=$v $(summ $o/q${q}_$v.json)"
  done
done
