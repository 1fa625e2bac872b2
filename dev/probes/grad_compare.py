#!/usr/bin/env python3
"""Per-parameter gradient agreement of the GPU training paths (fused
whole-model, fused loop-only, unfused autograd) with fp32 CPU autograd of the
golden model: cosine similarity and norm ratio, one line per parameter group."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402


def grads(model, i1, i2, target, iters, **kw):
    model.zero_grad(set_to_none=True)
    out = model(i1, i2, train=True, num_flow_updates=iters, **kw)
    w = torch.tensor([0.8 ** (iters - k - 1) for k in range(iters)], device=out.device).view(-1, 1, 1, 1, 1)
    (w * (out.float() - target.to(out.device)).abs()).mean().backward()
    return {n: p.grad.detach().float().cpu().clone() for n, p in model.named_parameters() if p.grad is not None}


def cos(a, b):
    a, b = a.flatten(), b.flatten()
    return (torch.dot(a, b) / (a.norm() * b.norm() + 1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--size", type=int, nargs=2, default=[128, 160])
    a = ap.parse_args()
    factory = raft_large if a.arch == "raft_large" else raft_small
    torch.manual_seed(3)
    model, _ = factory()
    model.train()
    g = torch.Generator().manual_seed(3)
    H, W = a.size
    i1 = torch.rand(2, H, W, 3, generator=g) * 2 - 1
    i2 = torch.rand(2, H, W, 3, generator=g) * 2 - 1
    target = torch.randn(2, H, W, 2, generator=g) * 4
    state = {k: v.clone() for k, v in model.state_dict().items()}
    ref = grads(model, i1, i2, target, a.iters)
    model = model.cuda()
    res = {}
    for name, enc, kw in (("unfused", True, dict(fused=False)), ("loop", False, dict(fused=True)),
                          ("whole", True, dict(fused=True))):
        F.FUSED_ENCODERS = enc
        F._LOOPS.clear()
        model.load_state_dict(state)
        res[name] = grads(model, i1.cuda(), i2.cuda(), target, a.iters, **kw)
    scale = max(v.norm().item() for v in ref.values())
    print(f"{'parameter':60s} " + " ".join(f"{k:>16s}" for k in res))
    for n in ref:
        if ref[n].norm().item() < 1e-4 * scale:
            continue
        cells = [f"{cos(r[n], ref[n]):7.4f}/{r[n].norm().item() / ref[n].norm().item():7.3f}" for r in res.values()]
        print(f"{n[:60]:60s} " + " ".join(f"{c:>16s}" for c in cells))


if __name__ == "__main__":
    main()
