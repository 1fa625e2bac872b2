# A/B of plan options on the headline bench (one line per variant)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
run() { echo "== $*" >> $out; timeout -k 10 200 "$@" 2>&1 | grep '"value"' | cut -c 80-200 >> $out; }
for v in "$@"; do run python bench.py $v; done
