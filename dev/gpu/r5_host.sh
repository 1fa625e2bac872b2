#!/bin/bash
# Round 5: engine host-path change (flat staleness check) -- engine / lifecycle tests, then the full bench.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_host}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_lifecycle_gpu.py tests/test_input_prep_gpu.py tests/test_engine_f32.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$o/bench.json'))
print('headline', d['value'], d['ms_per_step'])
for k,v in d.get('extras',{}).items():
    print(k, v if not isinstance(v, dict) else (v.get('value'), v.get('ms_per_step'), v.get('step_ms_p50') or v.get('latency_ms_p50'), v.get('step_ms_p99') or v.get('latency_ms_p99')))
"
