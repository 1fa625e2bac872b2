#!/bin/bash
# Round 6: same-box A/B of the ConvGRU lowering at batch 4 (GRU=halo vs the default whole-row gru_fused).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_gru_ab}
mkdir -p $o
for r in 1 2 3; do
  for v in auto halo; do
    timeout -k 10 300 python -u dev/probes/bench_with.py GRU=$v -- --batch 4 --extras off --steps 20 > $o/b4_$v.json 2> $o/b4_$v.err || { tail $o/b4_$v.err; exit 1; }
    echo "r$r GRU=$v $(python -c "import json;d=json.load(open('$o/b4_$v.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")"
  done
done
