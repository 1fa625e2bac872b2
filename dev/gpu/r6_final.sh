#!/bin/bash
# Round 6 final: smoke() + the default bench (all extras) twice on the final tree.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_final}
mkdir -p $o
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
for r in 1 2; do
  timeout -k 10 700 python -u bench.py > $o/bench_$r.json 2> $o/bench_$r.err || { tail $o/bench_$r.err; exit 1; }
  python - $o/bench_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras") or {}
print(round(d["value"], 1), d["ms_per_step"], " ".join(f"{k}={v['value']}" for k, v in ex.items() if isinstance(v, dict) and "value" in v))
PY
done
