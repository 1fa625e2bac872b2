# A/B of plan options on the headline bench (one line per variant; a variant
# may start with ENV=VALUE assignments)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
for v in "$@"; do
  echo "== $v" >> $out
  envs=(); args=()
  for w in $v; do if [[ $w == *=* ]]; then envs+=("$w"); else args+=("$w"); fi; done
  timeout -k 10 200 env "${envs[@]}" python bench.py "${args[@]}" 2>&1 | grep '"value"' | cut -c 80-200 >> $out || echo "failed" >> $out
done
