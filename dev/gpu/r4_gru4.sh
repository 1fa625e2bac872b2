#!/bin/bash
# Round 4: 4-block gru_halo tiles (whole 128-pixel rows at batch 4) -- tests, stage bench, A/B vs gru_fused
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_gru4
mkdir -p $o
true
tail -1 $o/tests.txt
timeout -k 10 200 python -u tools/gru_bench.py --batch 4 > $o/gru_bench_b4.txt 2>&1 || { tail $o/gru_bench_b4.txt; exit 1; }
cat $o/gru_bench_b4.txt
for r in 1 2; do
for g in halo auto; do
  JR_GRU=$g timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_${g}_$r.json 2> $o/b4_${g}_$r.err || { tail $o/b4_${g}_$r.err; exit 1; }
  echo "r$r gru=$g b4 $(python -c "import json;d=json.load(open('$o/b4_${g}_$r.json'));print(d['value'],d['ms_per_step'],d['autotune']['misses'],d.get('tile_cfgs',{}).get('gru0.halo'))")"
done
done
