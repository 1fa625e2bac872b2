"""Which reference cycle keeps the fused training plans (FusedModel / FusedLoop) alive after the
model is gone (gc disabled)?"""
import gc
import weakref

import torch

from jax_raft_amd import raft_large
from jax_raft_amd.train import fused as F

gc.disable()
model = raft_large(seed=0)[0].cuda().train()
g = torch.Generator().manual_seed(0)
i1 = (torch.rand(1, 128, 128, 3, generator=g) * 2 - 1).cuda()
i2 = (torch.rand(1, 128, 128, 3, generator=g) * 2 - 1).cuda()
out = model(i1, i2, train=True, num_flow_updates=2)
out.abs().mean().backward()
torch.cuda.synchronize()
objs = list(F._LOOPS[model].values())
fm = objs[0]
refs = {"fm": weakref.ref(fm), "loop": weakref.ref(fm.loop), "fe": weakref.ref(fm.fe), "ce": weakref.ref(fm.ce)}
del objs, out
model_ref = weakref.ref(model)
del model
print("model alive", model_ref() is not None)
for k, r in refs.items():
    print(k, "alive", r() is not None)
seen = set()


def show(o, depth):
    if depth > 3 or id(o) in seen:
        return
    seen.add(id(o))
    for x in gc.get_referrers(o):
        if x is globals() or type(x).__name__ in ("frame", "list_iterator"):
            continue
        if isinstance(x, dict) and "__name__" in x:
            continue
        print("  " * depth, "<-", type(x).__name__, (str(list(x.keys())[:8]) if isinstance(x, dict) else str(x)[:160]))
        show(x, depth + 1)


del fm
for k in ("loop", "fm", "fe", "ce"):
    o = refs[k]()
    if o is not None:
        print("== referrers of", k)
        show(o, 0)
        del o
