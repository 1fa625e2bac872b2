#!/bin/bash
# Encoder conv study: every tile config on the encoder shapes (+ load ablations of the
# chosen layer-1 config, hipBLASLt yardstick) and PMC passes over the layer-1 conv.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/enc
timeout -k 10 300 python -u tools/microbench.py --encoder --gemm --ablate 28,25 --json gpurun_out/enc/enc.json > gpurun_out/enc/enc.txt 2>&1 || exit $?
timeout -k 10 300 bash scripts/gpu_pmc.sh l1 28 > gpurun_out/enc/pmc.log 2>&1 || exit $?
mv gpurun_out/pmc gpurun_out/enc/
