set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/f32b
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_engine_f32.py tests/test_bench_contract.py "tests/test_engine_gpu.py::test_engine_context_parallel_single_slab" "tests/test_engine_gpu.py::test_engine_context_parallel_two_ranks" "tests/test_kernels_gpu.py::test_context_parallel_single_gpu_matches_engine" -x -v --timeout 250 --timeout-method thread -m gpu > $o/tests.log 2>&1 || { tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python -u bench.py --precision fp32 --batch 1 --steps 10 --warmup 3 > $o/bench_fp32.log 2>&1
tail -1 $o/bench_fp32.log | cut -c1-300
