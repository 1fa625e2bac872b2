#!/bin/bash
# Round 4: training step host gates A/B (JR_STEP_GATE: previous step finished; JR_PLAN_GATE: before each plan replay)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_train_gate_ab
mkdir -p $o
for r in 1 2; do
  for v in base step plan both; do
    unset JR_STEP_GATE JR_PLAN_GATE
    case $v in step) export JR_STEP_GATE=1;; plan) export JR_PLAN_GATE=1;; both) export JR_STEP_GATE=1 JR_PLAN_GATE=1;; esac
    timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/$v.json 2> $o/$v.err || { tail $o/$v.err; exit 1; }
    echo "$v r$r $(tail -1 $o/$v.json | cut -c1-120 | sed 's/.*"value"/value/')"
  done
done
