#!/bin/bash
# Round 4: prologue lanes at batch 1 (JR_PRO_LANES A/B) over the full bench with extras.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_prolanes
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
summ='import json,sys;d=json.load(open(sys.argv[1]));e=d.get("extras",{});print("headline",d["value"],{k:(v.get("value") if isinstance(v,dict) else v) for k,v in e.items()})'
for pl in 1 0; do
  JR_PRO_LANES=$pl timeout -k 10 900 python -u bench.py --extras on > $o/full_pl$pl.json 2> $o/full_pl$pl.err || { tail $o/full_pl$pl.err; exit 1; }
  echo "pro_lanes=$pl $(python -c "$summ" $o/full_pl$pl.json)"
done
