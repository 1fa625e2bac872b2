#!/bin/bash
# Round 5: same-box A/B of the full bench.py (headline + extras) -- round-start kernels (dev/bin/_C_base.so,
# built from d67e02a, via JR_NATIVE_SO) against the current tree's _C.so, alternating.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_ab_full}
mkdir -p $o
for v in base new base new; do
  so=""; [ $v = base ] && so=$PWD/dev/bin/_C_base.so
  i=$(ls $o | grep -c "^bench_$v")
  JR_NATIVE_SO=$so timeout -k 10 900 python -u bench.py > $o/bench_${v}_$i.json 2> $o/bench_${v}_$i.err || { tail $o/bench_${v}_$i.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/bench_${v}_$i.json'))
print('$v', 'headline', d['value'], ' '.join(f'{k}={v[\"value\"] if isinstance(v, dict) else v}' for k, v in d.get('extras', {}).items()))
"
done
