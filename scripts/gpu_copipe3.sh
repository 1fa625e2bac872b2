# Graph-pipelined bench: prologue as child node / more HW queues
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/copipe
mkdir -p $o
: > $o/ab3.log
run() { echo "== $*" >> $o/ab3.log; env "$@" timeout -k 10 200 python bench.py --steps 20 $BA 2>>$o/ab.err | cut -c 1-200 >> $o/ab3.log; }
BA="" run JR_X=0
BA="--pipeline graph" run JR_PIPE_PROLOGUE=child
BA="--pipeline graph" run GPU_MAX_HW_QUEUES=8
BA="--pipeline graph" run GPU_MAX_HW_QUEUES=8 JR_PIPE_PROLOGUE=child
BA="" run GPU_MAX_HW_QUEUES=8
BA="--batch 1 --pipeline graph" run JR_PIPE_PROLOGUE=child
BA="--pipeline graph" run JR_PIPE_PROLOGUE=child
BA="" run JR_X=0
cat $o/ab3.log
