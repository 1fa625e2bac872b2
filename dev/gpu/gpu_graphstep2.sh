set -o pipefail
for cfg in "1 1" "1 0" "0 1" "0 0"; do set -- $cfg; echo -n "== graph_step=$1 side=$2 "; JR_GRAPH_STEP=$1 JR_FUSED_SIDE=$2 timeout -k 10 300 python tools/train_bench.py 2>/dev/null | tail -1 | cut -c60-110 || exit 1; done
