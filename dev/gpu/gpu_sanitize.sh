# GPU tests with the host-sanitizer build of the runtime (build it first, on the CPU:
#   python -m jax_raft_amd._build --sanitize  -> jax_raft_amd/_C_san.so; UBSan + bounds on the
# C++ plan executor / bindings; kernels unchanged): any "runtime error" fails
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/sanitize
mkdir -p $o
export JR_NATIVE_SO=jax_raft_amd/_C_san.so UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1 || { tail -30 $o/gputests.log; exit 1; }
tail -2 $o/gputests.log
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > $o/bench.json 2> $o/bench.err
timeout -k 10 200 python bench.py --batch 1 --steps 3 --warmup 1 >> $o/bench.json 2>> $o/bench.err
timeout -k 10 300 python tools/train_bench.py --steps 3 > $o/train.json 2> $o/train.err || true
cat $o/gputests.log $o/bench.err $o/train.err > $o/all.log
n=$(grep -c "runtime error" $o/all.log || true)
echo "ubsan runtime errors: $n"
grep "runtime error" $o/all.log | sort | uniq -c | head -20 || true
[ "$n" = "0" ]
