"""Worker for test_engine_gpu.py::test_engine_context_parallel_two_ranks: two
context-parallel ranks on one GPU (gloo, JR_SHARE_GPU=1), each holding the
correlation pyramid of its half of the query rows; every iteration all-gathers
the looked-up features (RaftEngine(cp_group=True)).  Saves the flows of the bf16
and the fp32 engine per rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402
from jax_raft_amd.parallel.dp import init_distributed  # noqa: E402
from jax_raft_amd.runtime.engine import RaftEngine  # noqa: E402

out = sys.argv[1]
init_distributed()
rank = torch.distributed.get_rank()
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(11)
base = torch.rand(2, 136, 264, 3, generator=g) * 2 - 1
i1 = base[:, 4:132, 4:260].contiguous().to(dev)
i2 = base[:, 2:130, 6:262].contiguous().to(dev)
model = raft_large(seed=0)[0].eval().to(dev)
res = {}
with torch.no_grad():
    for prec in ("bf16", "fp32"):
        eng = RaftEngine(model, dev, precision=prec, cp_group=True)
        res[prec] = eng.forward(i1, i2, 3).cpu()
        res[prec + "_final"] = eng.forward(i1, i2, 3, return_all_iters=False).cpu()
torch.cuda.synchronize()
torch.save(res, os.path.join(out, f"rank{rank}.pt"))
torch.distributed.barrier()
torch.distributed.destroy_process_group()
