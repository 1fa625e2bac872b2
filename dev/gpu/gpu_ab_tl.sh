# selected GPU tests ($1 = pytest -k), then per variant: bench line + kernel trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/tl; mkdir -p gpurun_out/tl
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/tl/tests.log 2>&1 || { tail -30 gpurun_out/tl/tests.log; exit 1; }
tail -2 gpurun_out/tl/tests.log
shift
i=0
for v in "$@"; do
  mkdir -p gpurun_out/tl/$i
  echo "$v" > gpurun_out/tl/$i/variant.txt
  timeout -k 10 200 python bench.py $v 2>&1 | grep '"value"' | cut -c 80-170 > gpurun_out/tl/$i/bench.txt
  echo "== $v: $(cat gpurun_out/tl/$i/bench.txt)"
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl/$i -o run -- python3 bench.py --steps 5 --warmup 2 $v > gpurun_out/tl/$i/bench.log 2>&1
  i=$((i+1))
done
