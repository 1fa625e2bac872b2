#!/bin/bash
# Round 5: PMC of the halo conv on encoder layer 2 (cfg 103), plain vs the normalising variant (+ stats).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_pmc_halo}
mkdir -p $o
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G3="FETCH_SIZE GRBM_GUI_ACTIVE"
G4="WRITE_SIZE GRBM_GUI_ACTIVE"
for v in plain inn inn,stats; do
  f=""; [ $v != plain ] && f="--fused $v"
  i=0
  for grp in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $o/${v}_g$i -o run -- \
      python3 tools/conv_bench.py ${LAYER:-l2} --cfg ${CFG:-103} --run 5 $f > $o/${v}_g$i.log 2>&1 \
      || { echo "pmc $v g$i failed"; tail -5 $o/${v}_g$i.log; exit 1; }
  done
  echo "== $v"
  python3 tools/pmc_table.py $o/${v}_g1 $o/${v}_g2 $o/${v}_g3 $o/${v}_g4 --filter conv_halo > $o/pmc_$v.txt 2>&1
  cat $o/pmc_$v.txt
done
find $o -name '*.db' -delete
