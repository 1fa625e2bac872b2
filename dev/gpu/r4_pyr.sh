#!/bin/bash
# Round 4: persistent blocked pyramid kernel: tests, microbench A/B vs the tile kernel, PMC, bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r4_pyr
mkdir -p $o/pmc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "corr or lookup or pyr" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 200 python -u tools/corr_bench.py pyr lookup --batch 4 > $o/bench.txt 2>&1 && timeout -k 10 200 python -u tools/corr_bench.py pyr --batch 1 >> $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
JR_PYR_TILE=1 timeout -k 10 200 python -u tools/corr_bench.py pyr --batch 4 >> $o/bench.txt 2>&1 || { tail -20 $o/bench.txt; exit 1; }
cat $o/bench.txt
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $o/pmc/pyr_g$i -o run -- python3 tools/corr_bench.py pyr --run 5 > $o/pmc/pyr_g$i.log 2>&1 || { echo "pmc g$i failed"; tail -5 $o/pmc/pyr_g$i.log; exit 1; }
done
python tools/pmc_summary.py $o/pmc corr_pyr > $o/pmc_pyr.txt 2>&1
cat $o/pmc_pyr.txt
find $o/pmc -name '*.db' -delete
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py > $o/tests_engine.txt 2>&1 || { tail -30 $o/tests_engine.txt; exit 1; }
tail -2 $o/tests_engine.txt
for b in 4 1; do
  timeout -k 10 200 python -u bench.py --batch $b --extras off --steps 20 > $o/b$b.json 2> $o/b$b.err || { tail $o/b$b.err; exit 1; }
  echo "b$b $(python -c "import json;d=json.load(open('$o/b$b.json'));print(d['value'],d['ms_per_step'])")"
done
