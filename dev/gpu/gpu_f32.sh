# fp32 parity mode: kernel + engine tests, drift at the headline config, forward timing.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/f32
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_engine_f32.py -x -v --timeout 200 --timeout-method thread -m gpu > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python -u tools/drift.py measure --variants fp32 bf16 --json $o/drift.json > $o/drift.log 2>&1
cat $o/drift.log
timeout -k 10 200 python -u - > $o/timing.log 2>&1 <<'PY'
import time, torch
from jax_raft_amd import raft_large
from jax_raft_amd.runtime.engine import RaftEngine
m = raft_large(seed=0)[0].eval().cuda()
i1 = torch.rand(1, 440, 1024, 3, device="cuda") * 2 - 1
i2 = torch.rand(1, 440, 1024, 3, device="cuda") * 2 - 1
for prec in ("fp32", "bf16"):
    e = RaftEngine(m, torch.device("cuda", 0), precision=prec)
    with torch.no_grad():
        for _ in range(2):
            e.forward(i1, i2, 32)
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(5):
            e.forward(i1, i2, 32)
        torch.cuda.synchronize()
    print(prec, "ms/forward (raft_large 440x1024 32 it, batch 1):", (time.time() - t) / 5 * 1e3, flush=True)
PY
cat $o/timing.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 tools/drift.py measure --arch raft_large --variants fp32 > $o/prof.log 2>&1
ls $o/prof
