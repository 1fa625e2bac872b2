#!/bin/bash
# Round 6: lookup queries per wave (JR_LOOKUP_QPW, temporary A/B switch): headline + batch-1 sync.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_lookup_qpw}
mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "lookup" --timeout 100 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
JR_LOOKUP_QPW=3 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "lookup" --timeout 100 --timeout-method thread >> $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
JR_LOOKUP_QPW=1 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "lookup" --timeout 100 --timeout-method thread >> $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
grep passed $o/tests.txt
for r in 1 2; do
  for v in 2 3 1; do
    JR_LOOKUP_QPW=$v timeout -k 10 300 python -u bench.py --extras off --steps 20 > $o/h_$v.json 2> $o/h_$v.err || { tail $o/h_$v.err; exit 1; }
    echo "r$r qpw=$v $(python -c "import json;d=json.load(open('$o/h_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
