set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/g -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof1/graph.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/ng -o run -- python3 bench.py --steps 5 --warmup 2 --no-graph > gpurun_out/prof1/nograph.log 2>&1
for a in "--batch 1" "--batch 2" "--batch 8" "--split 2" "--batch 1 --arch raft_small" "--arch raft_small --iters 12 --batch 1"; do
  echo "== $a" >> gpurun_out/prof1/variants.log
  timeout -k 10 200 python3 bench.py $a >> gpurun_out/prof1/variants.log 2>&1
done
