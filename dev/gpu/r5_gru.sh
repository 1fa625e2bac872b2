#!/bin/bash
# Round 5: gru_fused with the resident tile image -- kernel + engine tests, phase split, headline bench.
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r5_gru}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -k "gru or fused or lane or drift or golden" --timeout 300 --timeout-method thread > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 120 python -u tools/gru_phases.py --batch 4 > $o/phases.txt 2>&1 || { tail -20 $o/phases.txt; exit 1; }
cat $o/phases.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --batch 4 --extras off --steps 20 > $o/b4_$r.json 2> $o/b4_$r.err || { tail $o/b4_$r.err; exit 1; }
  echo "b4 r$r $(python -c "import json;d=json.load(open('$o/b4_$r.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'])")"
done
