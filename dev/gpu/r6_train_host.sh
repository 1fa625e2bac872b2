#!/bin/bash
# Round 6: is the training step host-bound?  Host time per train_step vs wall, plus a cProfile.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_train_host}
mkdir -p $o
timeout -k 10 300 python -u tools/train_bench.py --steps 15 > $o/train.json 2> $o/train.err || { tail $o/train.err; exit 1; }
cat $o/train.json
timeout -k 10 300 python -u tools/train_bench.py --steps 15 --cprofile $o/cprofile.txt > $o/train_prof.json 2> $o/train_prof.err || { tail $o/train_prof.err; exit 1; }
cat $o/train_prof.json
head -60 $o/cprofile.txt
