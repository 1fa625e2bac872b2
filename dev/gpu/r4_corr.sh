#!/bin/bash
# Round 4: correlation pyramid / lookup microbench + PMC (FETCH / WRITE bytes, MFMA, L2 hits).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_corr
mkdir -p $o/pmc
timeout -k 10 200 python -u tools/corr_bench.py pyr lookup --batch 4 > $o/bench.txt 2>&1 && timeout -k 10 200 python -u tools/corr_bench.py pyr lookup --batch 1 >> $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
cat $o/bench.txt
for op in pyr:corr_pyramid lookup:corr_lookup; do
  k=${op%%:*}; f=${op##*:}; i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $o/pmc/${k}_g$i -o run -- python3 tools/corr_bench.py $k --run 5 > $o/pmc/${k}_g$i.log 2>&1 || { echo "pmc $k g$i failed"; tail -5 $o/pmc/${k}_g$i.log; exit 1; }
  done
  python tools/pmc_summary.py $o/pmc $f > $o/pmc_$k.txt 2>&1
  cat $o/pmc_$k.txt
done
find $o/pmc -name '*.db' -delete
