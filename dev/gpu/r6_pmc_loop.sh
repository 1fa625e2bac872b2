#!/bin/bash
# Round 6 (same recipe as r5_pmc_loop.sh): per-kernel PMC of the headline forward (batch 4) and the batch-1 forward: MFMA busy share,
# VALU / MFMA, LDS bank conflicts, HBM fetch / write, wait / stall shares (tools/pmc_table.py).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r6_pmc}
mkdir -p $o
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G3="FETCH_SIZE GRBM_GUI_ACTIVE"
G4="WRITE_SIZE GRBM_GUI_ACTIVE"
for b in ${BATCHES:-4 1}; do
  i=0
  for grp in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $o/b${b}_g$i -o run -- \
      python3 bench.py --batch $b --extras off --steps 2 --warmup 1 ${ARGS} > $o/b${b}_g$i.log 2>&1 \
      || { echo "pmc b$b g$i failed"; tail -5 $o/b${b}_g$i.log; exit 1; }
  done
  python3 tools/pmc_table.py $o/b${b}_g1 $o/b${b}_g2 $o/b${b}_g3 $o/b${b}_g4 --min-n 2 > $o/pmc_b$b.txt 2>&1
  head -40 $o/pmc_b$b.txt
done
find $o -name '*.db' -delete
