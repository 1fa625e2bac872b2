#!/bin/bash
# Round 5: PMC of the channel-split ConvGRU kernels (tools/gru_bench.py, batch ${B:-4}).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/r5_split_pmc
mkdir -p $o
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G3="FETCH_SIZE GRBM_GUI_ACTIVE"
i=0
for grp in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $o/g$i -o run -- \
    python3 tools/gru_bench.py --arch raft_large --batch ${B:-4} --reps 5 > $o/g$i.log 2>&1 || { echo "pmc g$i failed"; tail -5 $o/g$i.log; exit 1; }
done
python3 tools/pmc_table.py $o/g1 $o/g2 $o/g3 --filter gru > $o/pmc.txt 2>&1
cat $o/pmc.txt
find $o -name '*.db' -delete
