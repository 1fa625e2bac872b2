#!/bin/bash
# Round 4: engine numerics with the halo GRU / halo convs, bench A/B (GRU lowering, fused encoder norms).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_halo3
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_engine_gpu.py tests/test_drift.py -x -q --timeout 200 --timeout-method thread > $o/engine.log 2>&1
rc=$?
tail -15 $o/engine.log
[ $rc -eq 0 ] || exit $rc
for args in "--arch raft_large --batch 1" "--arch raft_small --batch 1"; do
  timeout -k 10 240 python -u tools/gru_bench.py $args 2>&1 | grep -v amdgpu.ids >> $o/gru_bench.log || { tail -20 $o/gru_bench.log; exit 1; }
done
grep -E "stage|halo" $o/gru_bench.log
for g in halo unfused; do
  for hn in 1 0; do
    export JR_GRU=$g JR_HALO_NORM=$hn
    timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1_${g}_$hn.json 2> $o/b1_${g}_$hn.err || { tail $o/b1_${g}_$hn.err; exit 1; }
    timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_${g}_$hn.json 2> $o/b4_${g}_$hn.err || { tail $o/b4_${g}_$hn.err; exit 1; }
    echo "$g norm=$hn b1 $(python -c "import json;d=json.load(open('$o/b1_${g}_$hn.json'));print(d['value'],d['ms_per_step'])") b4 $(python -c "import json;d=json.load(open('$o/b4_${g}_$hn.json'));print(d['value'],d['ms_per_step'])")"
  done
  timeout -k 10 200 python -u bench.py --arch raft_small --batch 1 --extras off --steps 30 > $o/s1_$g.json 2> $o/s1_$g.err || { tail $o/s1_$g.err; exit 1; }
  echo "$g small_b1 $(python -c "import json;d=json.load(open('$o/s1_$g.json'));print(d['value'],d['ms_per_step'])")"
done
python -c "import json;d=json.load(open('$o/b4_halo_1.json'));print(d['autotune'])"
