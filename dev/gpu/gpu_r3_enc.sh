#!/bin/bash
# Encoder conv study: kernel PS tests, every tile config on the encoder shapes (+ load
# ablations, hipBLASLt yardstick) and PMC passes over the layer-1 conv.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/enc
true

timeout -k 10 300 python -u tools/microbench.py --encoder --gemm --ablate 15,28,51 --json gpurun_out/enc/enc.json > gpurun_out/enc/enc.txt 2>&1 || exit $?
cat gpurun_out/enc/enc.txt
timeout -k 10 300 bash scripts/gpu_pmc.sh l1 15 28 51 > gpurun_out/enc/pmc.log 2>&1 || exit $?
mv gpurun_out/pmc gpurun_out/enc/
