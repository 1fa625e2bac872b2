# Graph-pipelined bench A/B, lane variants at batch 4 / 2 / 8
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/copipe
mkdir -p $o
: > $o/ab2.log
for a in "" "--streams off --pipeline graph" "--streams off" "--pipeline graph" "--batch 2 --pipeline graph" "--batch 2" "--batch 8 --streams off --pipeline graph" "--batch 8" "--streams off --pipeline graph"; do
  echo "== $a" >> $o/ab2.log
  timeout -k 10 200 python bench.py --steps 20 $a 2>>$o/ab.err | cut -c 1-200 >> $o/ab2.log
done
cat $o/ab2.log
