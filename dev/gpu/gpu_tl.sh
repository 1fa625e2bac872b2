# kernel traces of bench variants (one rocprofv3 run each) -> gpurun_out/tl/<i>/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for v in "$@"; do
  mkdir -p gpurun_out/tl/$i
  echo "$v" > gpurun_out/tl/$i/variant.txt
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl/$i -o run -- python3 bench.py --steps 5 --warmup 2 $v > gpurun_out/tl/$i/bench.log 2>&1
  i=$((i+1))
done
