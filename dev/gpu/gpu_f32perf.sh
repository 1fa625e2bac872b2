# fp32 conv kernel: correctness tests + raft_large fp32 forward timing (440x1024, 32 it, batch 1).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/f32p
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_engine_f32.py -x -q --timeout 200 --timeout-method thread -m gpu > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python -u - > $o/timing.log 2>&1 <<'PY'
import time, torch
from jax_raft_amd import raft_large
from jax_raft_amd.runtime.engine import RaftEngine
m = raft_large(seed=0)[0].eval().cuda()
i1 = torch.rand(1, 440, 1024, 3, device="cuda") * 2 - 1
i2 = torch.rand(1, 440, 1024, 3, device="cuda") * 2 - 1
e = RaftEngine(m, torch.device("cuda", 0), precision="fp32")
with torch.no_grad():
    for _ in range(2):
        e.forward(i1, i2, 32)
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(5):
        e.forward(i1, i2, 32)
    torch.cuda.synchronize()
print("fp32 ms/forward:", (time.time() - t) / 5 * 1e3, flush=True)
PY
cat $o/timing.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 tools/drift.py measure --arch raft_large --variants fp32 > $o/prof.log 2>&1
grep -h "fp32 " $o/prof.log | head -2
