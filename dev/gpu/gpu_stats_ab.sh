# one-launch instance-norm statistics A/B + pipeline auto mode
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/stats
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "channel_stats or instance_norm or graph_pipelined or matches_golden" -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { tail -40 $o/test.log; exit 1; }
tail -2 $o/test.log
: > $o/ab.log
run() { echo "== $* $BA" >> $o/ab.log; env "$@" timeout -k 10 200 python bench.py --steps 20 $BA 2>>$o/ab.err | cut -c 1-200 >> $o/ab.log; }
for k in 1 2; do
BA="" run JR_STATS_FUSED=0
BA="" run JR_STATS_FUSED=1
done
BA="--batch 1" run JR_STATS_FUSED=1
BA="--batch 1 --pipeline off" run JR_STATS_FUSED=1
cat $o/ab.log
