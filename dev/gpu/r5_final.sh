#!/bin/bash
# Round 5 rehearsal of the driver's round-end checks: the whole GPU suite in one process, smoke(), bench.py
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_final}
mkdir -p $o
timeout -k 10 1500 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -2 $o/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$o/bench.json'))
print('headline', d['value'], d['ms_per_step'])
for k,v in d.get('extras',{}).items():
    print(k, v if not isinstance(v, dict) else (v.get('value'), v.get('ms_per_step'), v.get('vs_baseline')))
"
