import sys, os
sys.path.insert(0, os.getcwd())
import torch
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import test_fused_train_gpu as T
from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.train import fused as F
for factory in (raft_large, raft_small):
    for enc in (True, False):
        F.FUSED_ENCODERS = enc
        F._LOOPS.clear()
        model, i1, i2, target = T._setup(factory)
        state = {k: v.clone() for k, v in model.state_dict().items()}
        mc = factory()[0]
        mc.load_state_dict({k: v.cpu() for k, v in state.items()})
        mc.train()
        iters = 3
        out_r = mc(i1, i2, train=True, num_flow_updates=iters)
        w = torch.tensor([0.8 ** (iters - k - 1) for k in range(iters)]).view(-1, 1, 1, 1, 1)
        (w * (out_r - target).abs()).mean().backward()
        g_r = {n: p.grad for n, p in mc.named_parameters() if p.grad is not None}
        _, g_u = T._run(model, i1, i2, target, iters, fused=False)
        model.load_state_dict(state)
        _, g_f = T._run(model, i1, i2, target, iters, fused=True)
        scale = max(v.norm().item() for v in g_r.values())
        ef, eu = [], []
        worst = []
        for n in g_r:
            if g_r[n].norm().item() < 1e-4 * scale:
                continue
            a, b = T._rel(g_f[n], g_r[n]), T._rel(g_u[n], g_r[n])
            ef.append(a); eu.append(b)
            worst.append((a - 1.25 * b, a, b, n))
        worst.sort(reverse=True)
        ef.sort(); eu.sort()
        print(factory.__name__, "enc" if enc else "loop", "median f/u", round(ef[len(ef)//2], 4), round(eu[len(eu)//2], 4),
              "max f/u", round(ef[-1], 4), round(eu[-1], 4))
        for x in worst[:4]:
            print("   ", [round(v, 4) for v in x[:3]], x[3])
