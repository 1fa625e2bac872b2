#!/bin/bash
# Round 6: PMC of the convex mask head forms at batch 4 (standalone, dev/probes/convex_bench.py).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_convex_pmc}
mkdir -p $o
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G3="FETCH_SIZE GRBM_GUI_ACTIVE"
G4="WRITE_SIZE GRBM_GUI_ACTIVE"
for t in 0 3; do
  i=0
  for grp in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $o/t${t}_g$i -o run -- \
      python3 dev/probes/convex_bench.py 4 $t > $o/t${t}_g$i.log 2>&1 || { echo "pmc t$t g$i failed"; tail -5 $o/t${t}_g$i.log; exit 1; }
  done
  python3 tools/pmc_table.py $o/t${t}_g1 $o/t${t}_g2 $o/t${t}_g3 $o/t${t}_g4 --min-n 2 > $o/pmc_t$t.txt 2>&1
  cat $o/pmc_t$t.txt
done
find $o -name '*.db' -delete
