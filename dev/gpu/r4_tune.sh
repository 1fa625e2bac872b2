#!/bin/bash
# Round 4: regenerate the persisted tile-config table with the halo configs as candidates,
# then bench with it (deterministic decisions) and summarise kernel traces on the box.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_tune
mkdir -p $o
JR_TUNE=fresh timeout -k 10 1000 python -u tools/autotune_db.py --out $o/gfx950.json > $o/tune.log 2>&1 || { tail -20 $o/tune.log; exit 1; }
tail -3 $o/tune.log
cp $o/gfx950.json jax_raft_amd/tuned/gfx950.json
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --extras off --steps 20 > $o/b4_$r.json 2> $o/b4_$r.err || { tail $o/b4_$r.err; exit 1; }
  echo "b4 r$r $(python -c "import json;d=json.load(open('$o/b4_$r.json'));print(d['value'],d['ms_per_step'],d['autotune']['hits'],d['autotune']['misses'])")"
done
timeout -k 10 200 python -u bench.py --batch 1 --extras off --steps 30 > $o/b1.json 2> $o/b1.err || exit 1
echo "b1 $(python -c "import json;d=json.load(open('$o/b1.json'));print(d['value'],d['ms_per_step'])")"
timeout -k 10 200 python -u bench.py --arch raft_small --batch 1 --extras off --steps 30 > $o/s1.json 2> $o/s1.err || exit 1
echo "small b1 $(python -c "import json;d=json.load(open('$o/s1.json'));print(d['value'],d['ms_per_step'])")"
for t in b4:4 b1:1; do
  n=${t%%:*}; b=${t##*:}
  timeout -k 10 200 rocprofv3 --kernel-trace -d $o/prof_$n -o run -- python3 bench.py --batch $b --steps 5 --warmup 2 --extras off > $o/prof_$n.log 2>&1 || exit 1
  db=$(ls $o/prof_$n/*/run_results.db $o/prof_$n/run_results.db 2>/dev/null | head -1)
  python tools/kernel_breakdown.py $db --top 40 > $o/breakdown_$n.txt 2>&1 || exit 1
  python tools/timeline.py $db --iter 10 > $o/timeline_$n.txt 2>&1 || exit 1
  rm -rf $o/prof_$n
done
head -25 $o/breakdown_b4.txt
head -20 $o/timeline_b1.txt
