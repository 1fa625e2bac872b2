#!/bin/bash
# Round 6: batch-4 headline with lanes on vs off: bench A/B + kernel-trace timelines of both.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_lanes}
mkdir -p $o
for s in on off on off; do
  timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 --streams $s > $o/b4_$s.json 2> $o/b4_$s.err || { tail $o/b4_$s.err; exit 1; }
  echo "streams=$s $(python -c "import json;d=json.load(open('$o/b4_$s.json'));print(d['value'],d['ms_per_step'])")"
done
for s in on off; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/t$s -o run -- python3 bench.py --batch 4 --extras off --steps 5 --warmup 2 --streams $s > $o/t$s.log 2>&1 || { tail -5 $o/t$s.log; exit 1; }
  f=$(find $o/t$s -name '*kernel_trace.csv' | head -1)
  python3 tools/kernel_breakdown.py $f --steps 5 --top 30 > $o/breakdown_$s.txt 2>&1
  python3 tools/timeline.py $f > $o/timeline_$s.txt 2>&1 || true
  python3 tools/timeline.py $f --iter 20 > $o/timeline20_$s.txt 2>&1 || true
  rm -f $f
done
