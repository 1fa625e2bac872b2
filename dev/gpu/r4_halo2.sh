#!/bin/bash
# Round 4: halo GRU + halo conv numerics, GRU stage timing, engine numerics, bench A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_halo2
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gru_halo_gpu.py tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1
rc=$?
tail -15 $o/tests.log
[ $rc -eq 0 ] || exit $rc
for args in "--arch raft_large --batch 1" "--arch raft_large --batch 4" "--arch raft_small --batch 1" "--arch raft_small --batch 4"; do
  timeout -k 10 240 python -u tools/gru_bench.py $args >> $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
done
cat $o/bench.log
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_drift.py -x -q --timeout 200 --timeout-method thread > $o/engine.log 2>&1
rc=$?
tail -15 $o/engine.log
[ $rc -eq 0 ] || exit $rc
for g in halo unfused; do
  export JR_GRU=$g
  timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1_$g.json 2> $o/b1_$g.err || { tail $o/b1_$g.err; exit 1; }
  timeout -k 10 200 python -u bench.py --arch raft_small --batch 1 --extras off --steps 30 > $o/s1_$g.json 2> $o/s1_$g.err || { tail $o/s1_$g.err; exit 1; }
  timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_$g.json 2> $o/b4_$g.err || { tail $o/b4_$g.err; exit 1; }
  echo "$g b1 $(python -c "import json;d=json.load(open('$o/b1_$g.json'));print(d['value'],d['ms_per_step'])") small_b1 $(python -c "import json;d=json.load(open('$o/s1_$g.json'));print(d['value'],d['ms_per_step'])") b4 $(python -c "import json;d=json.load(open('$o/b4_$g.json'));print(d['value'],d['ms_per_step'], d['autotune']['tile_cfgs'])")"
done
