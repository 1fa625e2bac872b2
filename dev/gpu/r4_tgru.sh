#!/bin/bash
# Round 4: training forward ConvGRU stages on gru_halo (saved gates) -- tests + A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_tgru
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gru_halo_gpu.py tests/test_fused_train_gpu.py tests/test_train_gpu.py > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2; do
for e in "JR_TRAIN_GRU_HALO=1" "JR_TRAIN_GRU_HALO=0"; do
  env $e timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train.json 2> $o/train.err || { tail $o/train.err; exit 1; }
  echo "r$r $e $(tail -1 $o/train.json | cut -c1-140)"
done
done
for r in 1 2; do
for pm in graph off; do
  timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 --pipeline $pm > $o/b1_$pm.json 2> $o/b1_$pm.err || { tail $o/b1_$pm.err; exit 1; }
  timeout -k 10 200 python -u bench.py --arch raft_small --batch 1 --extras off --steps 30 --pipeline $pm > $o/s1_$pm.json 2> $o/s1_$pm.err || { tail $o/s1_$pm.err; exit 1; }
  echo "r$r pipeline=$pm b1 $(python -c "import json;d=json.load(open('$o/b1_$pm.json'));print(d['value'],d['ms_per_step'])") small_b1 $(python -c "import json;d=json.load(open('$o/s1_$pm.json'));print(d['value'],d['ms_per_step'])")"
done
done
