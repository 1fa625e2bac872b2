"""Which object keeps a RaftEngine alive after its last user reference (gc disabled)?"""
import gc
import weakref

import torch

from jax_raft_amd import raft_small
from jax_raft_amd.runtime.engine import RaftEngine

model = raft_small()[0].cuda()
x = torch.zeros(1, 128, 128, 3, device="cuda")
gc.disable()
eng = RaftEngine(model, torch.device("cuda", 0), autotune=False)
r = weakref.ref(eng)
print("after init refcount", len(gc.get_referrers(eng)))
eng.forward(x, x, 2)
torch.cuda.synchronize()
for o in gc.get_referrers(eng):
    if isinstance(o, dict) and "__name__" in o:
        continue
    print("REF", type(o), str(o)[:300])
    for o2 in gc.get_referrers(o):
        if isinstance(o2, dict) and "__name__" in o2:
            continue
        print("   <-", type(o2), str(o2)[:300])
del eng
print("alive:", r() is not None)
