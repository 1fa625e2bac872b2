#!/bin/bash
# Round 6: each batch-1 extra in a fresh process (bench.py --only-extra) vs inside the full bench run.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_extra_standalone}
mkdir -p $o
timeout -k 10 700 python -u bench.py > $o/full.json 2> $o/full.err || { tail $o/full.err; exit 1; }
python - $o/full.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("in-bench", round(d["value"], 1), " ".join(f"{k}={v['value']}" for k, v in d["extras"].items() if isinstance(v, dict)))
PY
for k in b1_fps b1_sync b1_sync_u8 small_b1_fps_32it small_b1_sync_32it small_b1_fps_12it; do
  timeout -k 10 300 python -u bench.py --only-extra $k > $o/$k.json 2> $o/$k.err || { tail $o/$k.err; exit 1; }
  echo "standalone $k $(python -c "import json;d=json.loads(open('$o/$k.json').read().strip().splitlines()[-1]);print(d['$k']['value'])")"
done
