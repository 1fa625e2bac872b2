#!/bin/bash
# Round 6: gru_fused with per-tile K-stage rotation -- numerics, stage phases (new vs previous
# build), same-box batch-4 A/B.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_gru_rot}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "gru or golden" --timeout 250 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for so in new base; do
  if [ $so = base ]; then export JR_NATIVE_SO=jax_raft_amd/_C_base.so; else unset JR_NATIVE_SO; fi
  timeout -k 10 120 python -u tools/gru_phases.py --batch 4 > $o/phases_$so.txt 2>&1 || { tail -20 $o/phases_$so.txt; exit 1; }
  echo "== $so"; grep -v amdgpu.ids $o/phases_$so.txt
done
for r in 1 2 3; do
  for so in new base; do
    if [ $so = base ]; then export JR_NATIVE_SO=jax_raft_amd/_C_base.so; else unset JR_NATIVE_SO; fi
    timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 > $o/b4_$so.json 2> $o/b4_$so.err || { tail $o/b4_$so.err; exit 1; }
    echo "$so b4 $(python -c "import json;d=json.load(open('$o/b4_$so.json'));print(d['value'],d['ms_per_step'])")"
  done
done
