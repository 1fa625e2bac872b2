#!/bin/bash
# Round 6: batch 1, context encoder on its own prologue lane next to the batched feature encoder (CE_LANE_B1=1)
# vs everything on one lane (default), full bench extras.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_ce_lane_b1}
mkdir -p $o
summ() { python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extras") or {}
print(round(d["value"], 1), " ".join(f"{k}={v['value']}" for k, v in ex.items() if isinstance(v, dict) and "value" in v and k != "train_pairs_per_s"))
PY
}
ALL=train_pairs_per_s
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 600 python -u dev/probes/bench_with.py CE_LANE_B1=$v -- --skip-extras fp32_b1_fps,hires_b1,small_b1_sync_32it_mixed > $o/f_$v.json 2> $o/f_$v.err || { tail $o/f_$v.err; exit 1; }
    echo "r$r CE_LANE_B1=$v $(summ $o/f_$v.json)"
  done
done
