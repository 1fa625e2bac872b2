# batch 1 / 2: lanes x graph pipelining
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/b1lanes
mkdir -p $o
: > $o/ab.log
run() { echo "== $*" >> $o/ab.log; timeout -k 10 200 python bench.py --steps 20 "$@" 2>>$o/ab.err | cut -c 1-200 >> $o/ab.log; }
run --batch 1
run --batch 1 --streams on --pipeline graph
run --batch 1 --streams on --pipeline off
run --batch 2
run --batch 2 --streams on --pipeline graph
run --batch 2 --streams on --pipeline off
run --batch 2 --pipeline off
cat $o/ab.log
