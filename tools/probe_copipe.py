"""Probe: graph-pipelined engine steps (engine.pipelined) vs forward, one case,
with JR_PLAN_DEBUG capture tracing (GPU)."""
import sys

import torch

from jax_raft_amd import raft_large, raft_small

arch = sys.argv[1] if len(sys.argv) > 1 else "raft_large"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
model, _ = (raft_large if arch == "raft_large" else raft_small)()
model = model.cuda()
eng = model.engine(torch.device("cuda", 0))
g = torch.Generator().manual_seed(0)
batches = [((torch.rand(B, 128, 256, 3, generator=g) * 2 - 1).cuda(), (torch.rand(B, 128, 256, 3, generator=g) * 2 - 1).cuda())
           for _ in range(3)]
refs = [eng.forward(a, b, 4) for a, b in batches]
torch.cuda.synchronize()
print("forward ok", flush=True)
outs = [eng.pipelined(a, b, 4) for a, b in batches]
outs = outs[1:] + [eng.flush()]
torch.cuda.synchronize()
print("pipelined ok", [bool(torch.equal(r, o)) for r, o in zip(refs, outs)], flush=True)
