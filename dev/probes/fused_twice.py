#!/usr/bin/env python3
"""Do the persistent fused training plans give the same forward twice on the same weights?
(raft_large, converge setting; the second call replays the recorded plans)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.data import SyntheticFlow  # noqa: E402

torch.manual_seed(0)
model = raft_large()[0].cuda().train()
img1, img2, flow, valid = SyntheticFlow(size=(192, 256), seed=0, device=torch.device("cuda")).batch([0, 1])
F._LOOPS.clear()
outs = []
with torch.no_grad():
    for k in range(3):
        outs.append(model(img1, img2, train=True, num_flow_updates=6, fused=True).float().clone())
torch.cuda.synchronize()
for k in (1, 2):
    d = (outs[k] - outs[0]).abs()
    print(f"call {k + 1} vs call 1: max |diff| {d.max().item():.4e}, per iteration "
          + " ".join(f"{d[i].max().item():.2e}" for i in range(d.shape[0])), flush=True)
with torch.no_grad():
    ref = model(img1, img2, train=True, num_flow_updates=6, fused=False).float()
d = (outs[0] - ref).abs()
print(f"fused call 1 vs unfused: max {d.max().item():.4e}; fused call 3 vs unfused: {(outs[2] - ref).abs().max().item():.4e}")
