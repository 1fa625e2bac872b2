"""Batch-1 raft_large, 440x1024, 32 iterations: back-to-back forwards vs forward + synchronize per
pair (inputs resident), and the pipelined stream, same engine / process.  Why is the reference's
per-pair synchronous protocol (bench extra b1_sync) faster than the asynchronous stream?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from jax_raft_amd import raft_large  # noqa: E402

dev = torch.device("cuda:0")
H, W, IT, N = 440, 1024, 32, 60
B = int(os.environ.get("B", "1"))
model = raft_large(seed=0)[0].to(dev).eval()
eng = model.engine(dev)
a = (torch.rand(B, H, W, 3) * 2 - 1).to(dev)
b = (torch.rand(B, H, W, 3) * 2 - 1).to(dev)


def loop(sync: bool, pipe: bool = False, keep: bool = True):
    out = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        o = eng.pipelined(a, b, IT) if pipe else eng.forward(a, b, IT)
        if keep:
            out = o
        if sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return B * N / (time.perf_counter() - t0)


for _ in range(10):
    eng.forward(a, b, IT)
torch.cuda.synchronize()
for r in range(2):
    print(f"r{r} async {loop(False):.1f}  sync {loop(True):.1f}  async-drop {loop(False, keep=False):.1f}", flush=True)
if B >= 4:
    sys.exit(0)
for _ in range(5):
    eng.pipelined(a, b, IT)
eng.flush()
torch.cuda.synchronize()
for r in range(2):
    print(f"r{r} pipelined async {loop(False, True):.1f}  pipelined sync {loop(True, True):.1f}", flush=True)
    eng.flush()
