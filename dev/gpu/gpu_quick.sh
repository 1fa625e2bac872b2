# Quick GPU check: selected tests (pytest -k expression in $1), then A/B bench variants ($2..)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/q
o=gpurun_out/q
: > $o/ab.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
shift
for v in "$@"; do
  echo "== $v" >> $o/ab.log
  envs=(); args=()
  for w in $v; do if [[ $w == *=* ]]; then envs+=("$w"); else args+=("$w"); fi; done
  timeout -k 10 200 env "${envs[@]}" python bench.py "${args[@]}" 2>&1 | grep '"value"' | cut -c 80-200 >> $o/ab.log
done
cat $o/ab.log
