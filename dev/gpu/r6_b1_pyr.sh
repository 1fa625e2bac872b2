#!/bin/bash
# Round 6: batch-1 pyramid kernel durations, tile kernel vs persistent (CORR_PERSIST_B1), both archs.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_b1_pyr}
mkdir -p $o
for arch in raft_large raft_small; do
  for v in 1 0; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t_${arch}_$v -o run -- python3 dev/probes/b1_forward.py --arch $arch CORR_PERSIST_B1=$v > $o/t_${arch}_$v.log 2>&1 || { tail -5 $o/t_${arch}_$v.log; exit 1; }
    f=$(find $o/t_${arch}_$v -name '*kernel_stats.csv' | head -1)
    echo "$arch CORR_PERSIST_B1=$v"; grep -i "corr_pyr" $f | cut -d, -f1-8 || true
    find $o/t_${arch}_$v -name '*kernel_trace.csv' -delete
  done
done
