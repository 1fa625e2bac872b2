# A/B: GRU-B epilogue operand prefetch (JR_EPI_PREFETCH) -- microbench + headline bench + engine tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/epi
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "gru or golden or graph" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
(cd tools && JR_EPI_PREFETCH=0 timeout -k 10 120 python3 epi_cost.py) > $o/epi0.txt 2>&1
(cd tools && timeout -k 10 120 python3 epi_cost.py) > $o/epi1.txt 2>&1
echo "prefetch off"; grep gru $o/epi0.txt; echo "prefetch on"; grep gru $o/epi1.txt
for v in 1 0 1 0; do
  JR_EPI_PREFETCH=$v timeout -k 10 200 python -u bench.py --extras off --steps 20 --warmup 5 > $o/run.log 2>&1
  echo "prefetch=$v :: $(tail -1 $o/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
