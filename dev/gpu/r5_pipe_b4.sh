#!/bin/bash
# Round 5: graph pipelining at batch 4 with the lane schedule, re-measured on the round-5 kernels.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pipe_b4}
mkdir -p $o
: > $o/ab.txt
for r in 1 2; do
  for p in auto graph; do
    timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 --pipeline $p > $o/one.json 2> $o/one.err || { tail $o/one.err; exit 1; }
    echo "r$r pipeline=$p $(python -c "import json;d=json.load(open('$o/one.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")" | tee -a $o/ab.txt
  done
done
for p in auto graph; do
  timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 --pipeline $p --streams off > $o/one.json 2> $o/one.err || { tail $o/one.err; exit 1; }
  echo "one lane pipeline=$p $(python -c "import json;d=json.load(open('$o/one.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")" | tee -a $o/ab.txt
done
