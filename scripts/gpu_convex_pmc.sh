set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/cpmc; mkdir -p gpurun_out/cpmc
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/cpmc/p$i -o run -- python3 tools/convex_bench.py --batch 4 > gpurun_out/cpmc/p$i.log 2>&1 || exit 1
done
