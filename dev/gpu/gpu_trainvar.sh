set -o pipefail
for cfg in "0 1" "1 1" "0 0" "1 0"; do set -- $cfg; echo -n "== lanes=$1 graph=$2 "; JR_FUSED_LANES=$1 JR_FUSED_GRAPH=$2 timeout -k 10 300 python tools/train_bench.py 2>/dev/null | tail -1 | cut -c60-110 || exit 1; done
