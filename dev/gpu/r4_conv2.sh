#!/bin/bash
# Round 4: halo conv after the lane-group swizzle: tests, per-config microbench, PMC, benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_conv2
mkdir -p $o/pmc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_gpu.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 300 python -u tools/conv_bench.py ${PROBS:-l1 l2 l3 cc2b4 cc2b1 meb4 meb1 fhb4 cf2b4} > $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
cat $o/bench.txt
for pc in ${PMC:-l1:100 cc2b4:109}; do
  p=${pc%%:*}; c=${pc##*:}; i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $o/pmc/${p}_c${c}_g$i -o run -- python3 tools/conv_bench.py $p --cfg $c --run 10 > $o/pmc/${p}_c${c}_g$i.log 2>&1 || { echo "pmc $p $c g$i failed"; tail -5 $o/pmc/${p}_c${c}_g$i.log; exit 1; }
  done
done
python tools/pmc_summary.py $o/pmc > $o/pmc_summary.txt 2>&1
cat $o/pmc_summary.txt
find $o/pmc -name '*.db' -delete
for b in 4 1; do
  timeout -k 10 200 python -u bench.py --batch $b --extras off --steps 20 > $o/b$b.json 2> $o/b$b.err || { tail $o/b$b.err; exit 1; }
  echo "b$b $(python -c "import json;d=json.load(open('$o/b$b.json'));print(d['value'],d['ms_per_step'],d['autotune']['hits'],d['autotune']['misses'])")"
done
