#!/bin/bash
# Round 6: training step eager glue vs whole-step graph (TrainConfig.graph_step), same box.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_train_graph}
mkdir -p $o
for r in 1 2; do
  for g in "" "--graph-step"; do
    timeout -k 10 300 python -u tools/train_bench.py --steps 15 $g > $o/t$r$g.json 2> $o/t$r$g.err || { tail $o/t$r$g.err; exit 1; }
    echo "graph_step=${g:-off} $(tail -1 $o/t$r$g.json | cut -c1-140)"
  done
done
