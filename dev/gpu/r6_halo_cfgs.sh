#!/bin/bash
# Round 6: the new halo tile configs -- numerics against the golden conv, then the loop conv problems per config.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_halo}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 400 python -u tools/conv_bench.py cc2b4 meb4 fhb4 cf2b4 cc2b1 meb1 fh512b1 l3 > $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
cat $o/bench.txt
