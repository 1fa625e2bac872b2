#!/bin/bash
# Round 5: engine reference probe, then the remaining new tests, evidence runs behind cited test bounds
# (resolution drift, DP gradient error), the pipelined-graph fork A/B, then the loop PMC.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/r5_b
mkdir -p $o
timeout -k 10 200 python -u dev/probes/engine_refs.py > $o/refs.txt 2>&1 || { tail -20 $o/refs.txt; exit 1; }
tail -20 $o/refs.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_input_prep_gpu.py tests/test_lifecycle_gpu.py tests/test_engine_gpu.py tests/test_train_gpu.py \
  > $o/tests.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $o/tests.txt | tail -20
[ $rc -eq 0 ] || { grep -B 60 -m 1 "^E " $o/tests.txt | tail -70; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_resolution_gpu.py \
  "tests/test_train_gpu.py::test_dp_grads_equal_full_batch" > $o/evidence.txt 2>&1 || { tail -40 $o/evidence.txt; exit 1; }
grep -E "EPE|DP vs|passed|failed" $o/evidence.txt | tail -20
for fk in 1 0; do
  JR_PIPE_FORK=$fk timeout -k 10 200 python -u bench.py --arch raft_small --batch 1 --iters 12 --extras off --steps 60 --warmup 15 \
    > $o/fork$fk.json 2> $o/fork$fk.err || { tail $o/fork$fk.err; exit 1; }
  echo "JR_PIPE_FORK=$fk $(python -c "import json;d=json.load(open('$o/fork$fk.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['step_ms_p99'])")"
done
OUT=r5_pmc bash dev/gpu/r5_pmc_loop.sh
