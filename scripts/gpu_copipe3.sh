# Graph-pipelined bench: prologue as child node / more HW queues; one-launch stats A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/copipe
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "channel_stats or instance_norm" -x -q --timeout 120 --timeout-method thread > $o/test3.log 2>&1 || { tail -40 $o/test3.log; exit 1; }
tail -2 $o/test3.log
: > $o/ab3.log
run() { echo "== $* $BA" >> $o/ab3.log; env "$@" timeout -k 10 200 python bench.py --steps 20 $BA 2>>$o/ab.err | cut -c 1-200 >> $o/ab3.log; }
BA="" run JR_STATS_FUSED=0
BA="" run JR_STATS_FUSED=1
BA="--pipeline graph" run JR_PIPE_PROLOGUE=child
BA="--pipeline graph" run GPU_MAX_HW_QUEUES=8
BA="--pipeline graph" run GPU_MAX_HW_QUEUES=8 JR_PIPE_PROLOGUE=child
BA="" run GPU_MAX_HW_QUEUES=8
BA="--batch 1 --pipeline graph" run JR_PIPE_PROLOGUE=child
BA="" run JR_STATS_FUSED=0
BA="" run JR_STATS_FUSED=1
cat $o/ab3.log
