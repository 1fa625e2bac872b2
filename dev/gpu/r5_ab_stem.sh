#!/bin/bash
# Round 5: same-box A/B of the halo-kernel stem: base = the tree before it (dev/bin/_C_base.so + its
# tuned table dev/bin/gfx950_base.json; the stems pinned to that table's batch-4 choice, igemm cfg 15, since the
# current Python offers the halo stem configs the old library lacks), new = the current tree; headline, no extras.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_ab_stem}
mkdir -p $o
run() {  # $1 = base|new, $2 = tag, rest = bench args
  local v=$1 tag=$2; shift 2
  if [ $v = base ]; then export JR_NATIVE_SO=$PWD/dev/bin/_C_base.so JR_TUNE_DB=$PWD/dev/bin/gfx950_base.json JR_CFG_OVERRIDE=fe.stem_s2d=15,ce.stem_s2d=15; else unset JR_NATIVE_SO JR_TUNE_DB JR_CFG_OVERRIDE; fi
  timeout -k 10 900 python -u bench.py "$@" > $o/${tag}_$v.json 2> $o/${tag}_$v.err || { tail $o/${tag}_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/${tag}_$v.json'))
print('$tag $v', 'headline', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"] if isinstance(v, dict) else v}' for k, v in (d.get('extras') or {}).items()))
"
}
for r in 1 2 3; do run base b4r$r --extras off --steps 30 --warmup 5; run new b4r$r --extras off --steps 30 --warmup 5; done
