#!/bin/bash
# Round 4: A/B of the GRU lowering x halo convs at batch 4 / 1, plus kernel traces.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_ab1
mkdir -p $o
for r in 1 2; do
for cfg in "fused 0" "fused 1" "halo 1" "halo 0"; do
  set -- $cfg
  export JR_GRU=$1 JR_CONV_HALO=$2
  timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_$1_$2.json 2> $o/b4_$1_$2.err || { tail $o/b4_$1_$2.err; exit 1; }
  echo "r$r b4 gru=$1 conv_halo=$2 $(python -c "import json;d=json.load(open('$o/b4_$1_$2.json'));print(d['value'],d['ms_per_step'])")"
done
done
for cfg in "halo 1" "halo 0"; do
  set -- $cfg
  export JR_GRU=$1 JR_CONV_HALO=$2
  timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1_$1_$2.json 2> $o/b1_$1_$2.err || { tail $o/b1_$1_$2.err; exit 1; }
  echo "b1 gru=$1 conv_halo=$2 $(python -c "import json;d=json.load(open('$o/b1_$1_$2.json'));print(d['value'],d['ms_per_step'])")"
done
export JR_GRU=halo JR_CONV_HALO=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_b4 -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof_b4.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_b1 -o run -- python3 bench.py --batch 1 --steps 5 --warmup 2 --extras off > $o/prof_b1.log 2>&1 || exit 1
export JR_GRU=fused JR_CONV_HALO=0
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_b4_r3 -o run -- python3 bench.py --steps 5 --warmup 2 --extras off > $o/prof_b4_r3.log 2>&1 || exit 1
ls -R $o | head -30
