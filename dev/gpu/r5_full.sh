#!/bin/bash
# Round 5: the whole GPU suite in one process, then the headline / batch-1 bench (no extras).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_full}
mkdir -p $o
timeout -k 10 1500 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -40 $o/gpu_tests.txt; exit 1; }
tail -2 $o/gpu_tests.txt
for b in 4 1; do
  timeout -k 10 300 python -u bench.py --batch $b --extras off --steps 20 > $o/b$b.json 2> $o/b$b.err || { tail $o/b$b.err; exit 1; }
  echo "b$b $(python -c "import json;d=json.load(open('$o/b$b.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['autotune']['hits'],d['autotune']['misses'])")"
done
