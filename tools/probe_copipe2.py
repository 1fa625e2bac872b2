"""Probe which capture crashes: submit() at batch 4 (loop-only capture with
lanes) and pipelined() at batch 1 (single-lane plans)."""
import sys

import torch

from jax_raft_amd import raft_large

mode, B = sys.argv[1], int(sys.argv[2])
model, _ = raft_large()
model = model.cuda()
eng = model.engine(torch.device("cuda", 0))
g = torch.Generator().manual_seed(0)
batches = [((torch.rand(B, 128, 256, 3, generator=g) * 2 - 1).cuda(), (torch.rand(B, 128, 256, 3, generator=g) * 2 - 1).cuda())
           for _ in range(3)]
refs = [eng.forward(a, b, 4) for a, b in batches]
torch.cuda.synchronize()
if mode == "submit":
    outs = [eng.submit(a, b, 4).result() for a, b in batches]
else:
    outs = [eng.pipelined(a, b, 4) for a, b in batches]
    outs = outs[1:] + [eng.flush()]
torch.cuda.synchronize()
print(mode, B, "ok", [bool(torch.equal(r, o)) for r, o in zip(refs, outs)], flush=True)
