set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/lpmc; mkdir -p gpurun_out/lpmc
i=0
for ctr in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "corr_lookup" --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/lpmc/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-graph > gpurun_out/lpmc/p$i.log 2>&1 || exit 1
done
