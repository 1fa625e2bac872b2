#!/bin/bash
# Round 6: convex head epilogue VALU diet -- numerics, isolated time, and same-box in-situ A/B
# against the previous build (JR_NATIVE_SO=jax_raft_amd/_C_base.so).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_convex_ab}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k "convex_head_kernel or golden" --timeout 250 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for so in new base; do
  if [ $so = base ]; then export JR_NATIVE_SO=jax_raft_amd/_C_base.so; else unset JR_NATIVE_SO; fi
  for b in 4 1; do timeout -k 10 60 python -u dev/probes/convex_bench.py $b 2>&1 | grep convex_head | sed "s/^/$so /"; done
done
for r in 1 2 3; do
  for so in new base; do
    if [ $so = base ]; then export JR_NATIVE_SO=jax_raft_amd/_C_base.so; else unset JR_NATIVE_SO; fi
    timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 > $o/b4_$so.json 2> $o/b4_$so.err || { tail $o/b4_$so.err; exit 1; }
    timeout -k 10 300 python -u bench.py --batch 1 --extras off --steps 40 > $o/b1_$so.json 2> $o/b1_$so.err || { tail $o/b1_$so.err; exit 1; }
    echo "$so b4 $(python -c "import json;d=json.load(open('$o/b4_$so.json'));print(d['value'],d['ms_per_step'])") b1 $(python -c "import json;d=json.load(open('$o/b1_$so.json'));print(d['value'],d['ms_per_step'])")"
  done
done
