# PMC passes (one counter group per rocprofv3 run) over single-conv runs.
# usage: bash scripts/gpu_pmc.sh <conv> <cfg> [<cfg> ...]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
conv=$1; shift
mkdir -p gpurun_out/pmc
for cfg in "$@"; do
  timeout -k 10 120 python3 tools/conv_one.py $conv $cfg >> gpurun_out/pmc/times.txt
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/${conv}_c${cfg}_g$i -o run -- python3 tools/conv_one.py $conv $cfg 20 > /dev/null 2>&1
  done
done
