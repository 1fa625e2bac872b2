#!/bin/bash
# Round 4: wide-channel halo conv configs (all output channels per workgroup) -- tests + microbench
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_wide
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_gpu.py > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 300 python -u tools/conv_bench.py cc2b1 meb1 fh512b1 cf2b1 cc2b4 > $o/conv_bench.txt 2>&1 || { tail -20 $o/conv_bench.txt; exit 1; }
cat $o/conv_bench.txt
