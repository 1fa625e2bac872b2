#!/bin/bash
# Round 5: the halo-kernel stem in the engine -- engine GPU tests, the tuned table extended with the new
# (halo-keyed) stem problems (JR_TUNE=db: existing entries kept), then the headline + full bench.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_stem2}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_input_prep_gpu.py tests/test_conv_halo_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 900 python -u tools/autotune_db.py --out $o/gfx950.json > $o/tune.log 2>&1 || { tail -20 $o/tune.log; exit 1; }
tail -1 $o/tune.log
JR_TUNE_DB=$PWD/$o/gfx950.json timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$o/bench.json'))
print('headline', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"] if isinstance(v, dict) else v}' for k, v in (d.get('extras') or {}).items()))
"
