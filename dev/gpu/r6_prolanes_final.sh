#!/bin/bash
# Round 6: batch-1 prologue on one lane + training extra in a child process: engine tests + full bench x2.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_pl_final}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
summ() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras") or {}
print(round(d["value"], 1), " ".join(f"{k}={v['value']}" for k, v in ex.items() if isinstance(v, dict) and "value" in v))
PY
}
for r in 1 2; do
  timeout -k 10 700 python -u bench.py > $o/full_$r.json 2> $o/full_$r.err || { tail $o/full_$r.err; exit 1; }
  echo "r$r $(summ $o/full_$r.json)"
done
