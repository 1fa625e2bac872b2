#!/bin/bash
# Round 4: per-config conv microbench (halo vs implicit GEMM) + PMC passes on the halo conv
# of encoder layer 1 and the batch-4 loop convs, then the new GPU tests.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_conv
mkdir -p $o/pmc
timeout -k 10 300 python -u tools/conv_bench.py l1 l2 l3 cc2b4 cc2b1 meb4 meb1 fhb4 fh512b1 cf2b4 cf2b1 > $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
cat $o/bench.txt
for pc in l1:100 cc2b4:109 cc2b4:111 fhb4:105; do
  p=${pc%%:*}; c=${pc##*:}; i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
             "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $o/pmc/${p}_c${c}_g$i -o run -- python3 tools/conv_bench.py $p --cfg $c --run 10 > $o/pmc/${p}_c${c}_g$i.log 2>&1 || { echo "pmc $p $c g$i failed"; tail -5 $o/pmc/${p}_c${c}_g$i.log; exit 1; }
  done
done
python tools/pmc_summary.py $o/pmc > $o/pmc_summary.txt 2>&1
cat $o/pmc_summary.txt
find $o/pmc -name '*.db' -delete
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_injection_gpu.py tests/test_resolution_gpu.py tests/test_train_gpu.py tests/test_bench_contract.py > $o/tests.txt 2>&1
rc=$?
tail -40 $o/tests.txt
exit $rc
