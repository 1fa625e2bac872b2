# corr pyramid: microbench of the launch variants (+ optional kernel tests)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/corr
o=gpurun_out/corr
if [ -n "$TESTS" ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "corr or engine" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
fi
: > $o/mb.log
for v in "$@"; do
  echo "== $v" >> $o/mb.log
  timeout -k 10 120 env $v python tools/microbench.py --only corr_pyramid 2>&1 | grep corr_pyr >> $o/mb.log
done
cat $o/mb.log
