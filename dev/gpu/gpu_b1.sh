# batch-1 latency profile (the reference's own FPS config): kernel trace + one-iteration timeline
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/b${BATCH:-1}${TAG:-}
mkdir -p $o
for arch in ${ARCHS:-raft_large raft_small}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/$arch -o run -- python3 bench.py --steps 5 --warmup 2 --batch ${BATCH:-1} --arch $arch ${BENCH_ARGS:-} > $o/$arch.log 2>&1
  tail -1 $o/$arch.log | cut -c1-200
  db=$(ls $o/$arch/run_results.db $o/$arch/*/run_results.db 2>/dev/null | head -1 || true)
  if [ -z "$db" ]; then db=$(find $o/$arch -name '*kernel_trace.csv' | head -1); fi
  python3 tools/kernel_breakdown.py "$db" --steps 5 --marker corr_pyramid_kernel --top 30 > $o/${arch}_breakdown.txt
  (cd tools && python3 timeline.py "../$db" --iter 10) > $o/${arch}_timeline.txt
  cat $o/${arch}_timeline.txt
done
