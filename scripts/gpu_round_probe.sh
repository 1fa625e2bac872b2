set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fused_train_gpu.py -x -q --timeout 120 --timeout-method thread -k "split or repeated or graph or pack" > gpurun_out/t.log 2>&1; echo "tests exit $?"; tail -3 gpurun_out/t.log
for a in "" "--split 2" "--split 2 --streams off"; do echo "== infer $a"; timeout -k 10 200 python bench.py --steps 20 $a 2>/dev/null | tail -1 || break; done
for b in 6 12 24; do echo "== train batch $b"; timeout -k 10 300 python tools/train_bench.py --batch $b 2>/dev/null | tail -1 || break; done
