# Prologue timeline of the headline forward (batch 4, lanes schedule).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/pro
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/k -o run -- python3 bench.py --extras off --steps 4 --warmup 2 > $o/bench.log 2>&1
f=$(find $o/k -name '*kernel_trace.csv' | head -1)
python3 tools/prologue_timeline.py "$f" > $o/timeline.txt
tail -8 $o/timeline.txt
rm -f "$f"
