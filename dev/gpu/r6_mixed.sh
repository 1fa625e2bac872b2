#!/bin/bash
# Round 6: precision="mixed" (fp32 feature encoder) drift (tools/drift.py) and drift tests; the
# batch-1 persistent pyramid kernel test; the full default bench (its extras include
# small_b1_sync_32it_mixed next to small_b1_sync_32it).
set -o pipefail
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/${OUT:-r6_mixed}
mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "persistent_batch1" --timeout 150 --timeout-method thread > $o/ktests.txt 2>&1 || { tail -30 $o/ktests.txt; exit 1; }
tail -1 $o/ktests.txt
timeout -k 10 600 python -u tools/drift.py measure --arch raft_small raft_large --variants bf16 mixed mixed_corr_fp32 mixed_corr_gate_fp32 corr_fp32 --json $o/drift.json > $o/drift.txt 2>&1 || { tail -20 $o/drift.txt; exit 1; }
cat $o/drift.txt
timeout -k 10 300 python -u -m pytest tests/test_drift.py -x -q -m gpu --timeout 250 --timeout-method thread > $o/drift_tests.txt 2>&1 || { tail -30 $o/drift_tests.txt; exit 1; }
tail -1 $o/drift_tests.txt
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$o/bench.json'))
print('headline', d['value'], d['ms_per_step'])
for k,v in d.get('extras',{}).items():
    print(k, v if not isinstance(v, dict) else (v.get('value'), v.get('ms_per_step'), v.get('vs_baseline')))
"
