#!/bin/bash
# Round 5: the instance-norm stem's statistics in the halo stem's epilogue -- engine GPU tests, the tuned
# table extended with the new (halo-norm keyed) stem problems, then a same-box headline A/B against the
# engine before it (dev/bin/engine_base.py swapped in; same library).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_stem_stats}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_input_prep_gpu.py tests/test_lifecycle_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 900 python -u tools/autotune_db.py --out $o/gfx950.json --no-train > $o/tune.log 2>&1 || { tail -20 $o/tune.log; exit 1; }
tail -1 $o/tune.log
cp jax_raft_amd/runtime/engine.py $o/engine_new.py
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then cp dev/bin/engine_base.py jax_raft_amd/runtime/engine.py; else cp $o/engine_new.py jax_raft_amd/runtime/engine.py; fi
    JR_TUNE_DB=$PWD/$o/gfx950.json timeout -k 10 300 python -u bench.py --extras off --steps 30 --warmup 5 > $o/b4_${v}_$r.json 2> $o/b4_${v}_$r.err || { tail $o/b4_${v}_$r.err; cp $o/engine_new.py jax_raft_amd/runtime/engine.py; exit 1; }
    echo "b4 $v r$r $(python -c "import json;d=json.load(open('$o/b4_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
cp $o/engine_new.py jax_raft_amd/runtime/engine.py
