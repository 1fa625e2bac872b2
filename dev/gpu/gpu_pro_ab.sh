# A/B: prologue issue order (JR_PLAN_INTERLEAVE) + timeline of the interleaved order.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/proab
mkdir -p $o
for v in 1 0 1 0; do
  JR_PLAN_INTERLEAVE=$v timeout -k 10 200 python -u bench.py --extras off --steps 20 --warmup 5 > $o/run.log 2>&1
  echo "interleave=$v :: $(tail -1 $o/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/k -o run -- python3 bench.py --extras off --steps 4 --warmup 2 > $o/bench.log 2>&1
f=$(find $o/k -name '*kernel_trace.csv' | head -1)
python3 tools/prologue_timeline.py "$f" > $o/timeline_il.txt
tail -5 $o/timeline_il.txt
rm -f "$f"
