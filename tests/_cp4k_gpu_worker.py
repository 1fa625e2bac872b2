"""Worker for test_resolution_gpu.py::test_4k_context_parallel_two_ranks: a 2160x3840
final-only forward (4 iterations) with the correlation volume split over two
context-parallel ranks sharing one GPU (gloo, JR_SHARE_GPU=1)."""
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
g = torch.Generator().manual_seed(2)
base = torch.rand(1, 2168, 3848, 3, generator=g) * 2 - 1
i1 = base[:, 4:2164, 4:3844].contiguous().to(dev)
i2 = base[:, 2:2162, 6:3846].contiguous().to(dev)
model = raft_large(seed=0)[0].eval().to(dev)
with torch.no_grad():
    eng = RaftEngine(model, dev, cp_group=True)
    flow = eng.forward(i1, i2, 4, return_all_iters=False).cpu()
torch.cuda.synchronize()
st = next(iter(eng._states.values()))
nbytes = sum(t.numel() * t.element_size() for k, t in st.bufs.items() if ".corr.l" in "." + k)
torch.save({"flow": flow, "bytes": nbytes}, os.path.join(out, f"rank{rank}.pt"))
torch.distributed.barrier()
torch.distributed.destroy_process_group()
