# fp32 conv tile A/B (JR_F32_TILE) at raft_large 440x1024, 32 iterations, batch 1.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/f32t
mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_engine_f32.py -x -q --timeout 100 --timeout-method thread -m gpu -k "kernel or gru" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for t in 0 1 2 3; do
JR_F32_TILE=$t timeout -k 10 200 python -u - > $o/t$t.log 2>&1 <<'PY'
import time, torch, os
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
print("tile", os.environ["JR_F32_TILE"], "fp32 ms/forward:", (time.time() - t) / 5 * 1e3, flush=True)
PY
cat $o/t$t.log | grep tile
done
