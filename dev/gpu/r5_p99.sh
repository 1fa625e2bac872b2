#!/bin/bash
# Round 5: raft_small 12-iteration stream p99: host-side stalls of the input copies, SDMA vs blit copies.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_p99}
mkdir -p $o
for e in "X=0" "HSA_ENABLE_SDMA=0"; do
  echo "== $e" >> $o/p99_env.txt
  env $e timeout -k 10 300 python3 -u dev/probes/p99_probe.py --steps 300 >> $o/p99_env.txt 2>&1 || { tail -5 $o/p99_env.txt; exit 1; }
  env $e timeout -k 10 300 python3 -u bench.py --arch raft_small --batch 1 --iters 12 --steps 200 --warmup 15 --extras off --step-times > $o/small12.json 2> $o/small12.err || { tail -5 $o/small12.err; exit 1; }
  echo "bench small12 $e: $(python3 -c "import json;d=json.load(open('$o/small12.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['step_ms_p99'])")" >> $o/p99_env.txt
  env $e timeout -k 10 300 python3 -u bench.py --batch 1 --extras off --steps 40 > $o/b1.json 2> $o/b1.err || { tail -5 $o/b1.err; exit 1; }
  echo "bench b1 $e: $(python3 -c "import json;d=json.load(open('$o/b1.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['step_ms_p99'])")" >> $o/p99_env.txt
done
grep -v amdgpu $o/p99_env.txt
