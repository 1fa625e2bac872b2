# kernel trace of the headline bench (graph replay), summary + iteration timeline
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/trace
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/trace -o run -- python3 bench.py --steps 5 --warmup 2 "$@" > gpurun_out/trace/bench.log 2>&1
