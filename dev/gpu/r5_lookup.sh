#!/bin/bash
# Round 5: lookup last-chunk skip -- kernel tests, engine tests, b4 / b1 bench.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_lookup}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_input_prep_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for b in 4 1; do
  timeout -k 10 300 python -u bench.py --batch $b --extras off --steps 20 > $o/b$b.json 2> $o/b$b.err || { tail $o/b$b.err; exit 1; }
  echo "b$b $(python -c "import json;d=json.load(open('$o/b$b.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")"
done
