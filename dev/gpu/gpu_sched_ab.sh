# A/B of the headline schedule: lanes (default at batch 4) vs one lane + graph pipelining.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/sched
mkdir -p $o
for v in "" "--streams off --pipeline graph" "--streams off" "--streams on --pipeline graph" "" "--streams off --pipeline graph"; do
  timeout -k 10 200 python -u bench.py --extras off --steps 20 --warmup 5 $v > $o/run.log 2>&1
  echo "$v :: $(tail -1 $o/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["cross_batch_pipeline"], d["config"]["concurrent_branches"])')"
done
