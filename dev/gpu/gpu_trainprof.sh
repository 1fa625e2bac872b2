# Training-step profile: phase timing + rocprofv3 kernel trace of tools/train_bench.py.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/trainprof
mkdir -p $o
timeout -k 10 300 python3 tools/train_phases.py > $o/phases.json 2> $o/phases.err
cat $o/phases.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/k -o run -- python3 tools/train_bench.py --steps 5 --warmup 2 > $o/bench.log 2>&1
tail -1 $o/bench.log
db=$(ls $o/k/run_results.db $o/k/*/run_results.db 2>/dev/null | head -1 || true)
if [ -z "$db" ]; then db=$(find $o/k -name '*kernel_trace.csv' | head -1); fi
python3 tools/kernel_breakdown.py "$db" --steps 5 --marker seq_loss_kernel --top 60 > $o/breakdown.txt
cat $o/breakdown.txt
(cd tools && python3 step_gaps.py "../$db") > $o/gaps.txt
cat $o/gaps.txt
