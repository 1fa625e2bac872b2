#!/usr/bin/env python3
"""Why do the fused and fp32 training trajectories of tools/train_converge.py part after the
first AdamW step?  Step-1 gradients of the converge setting (raft_large, 2 x 192x256 synthetic
batch, 6 iterations, sequence loss) on the fused native path, the unfused native path and fp32
CPU autograd of the golden model: per parameter the cosine and norm ratio against fp32, and the
share of elements whose SIGN agrees with fp32 (AdamW's first update is lr * sign(g)), worst
first; then the loss after one AdamW step taken with each path's gradients, all evaluated by the
fp32 CPU model.

    python dev/probes/converge_grads.py [--top 25]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.data import SyntheticFlow  # noqa: E402
from jax_raft_amd.train.loss import sequence_loss  # noqa: E402


def grads(state, batch, device, fused, iters):
    model = raft_large()[0]
    model.load_state_dict(state)
    model = model.to(device).train()
    F._LOOPS.clear()
    img1, img2, flow, valid = (t.to(device) for t in batch)
    preds = model(img1, img2, train=True, num_flow_updates=iters, fused=fused)
    loss, _ = sequence_loss(preds, flow, valid)
    loss.backward()
    return float(loss), {n: p.grad.detach().float().cpu().clone() for n, p in model.named_parameters()
                         if p.grad is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--iters", type=int, default=6)
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    state = {k: v.clone() for k, v in raft_large()[0].state_dict().items()}
    data = SyntheticFlow(size=(192, 256), seed=0, device=torch.device("cuda"))
    batch = [t.cpu() for t in data.batch([0, 1])]
    l_ref, g_ref = grads(state, batch, "cpu", False, a.iters)
    res = {}
    for name, fused in (("fused", True), ("unfused", False)):
        res[name] = grads(state, batch, "cuda", fused, a.iters)
    print(f"step-1 loss: fp32 cpu {l_ref:.4f}, " + ", ".join(f"{k} {v[0]:.4f}" for k, v in res.items()))
    scale = max(v.norm().item() for v in g_ref.values())
    for name, (_, g) in res.items():
        rows = []
        for n, r in g_ref.items():
            x = g[n]
            c = (torch.dot(x.flatten(), r.flatten()) / (x.norm() * r.norm() + 1e-20)).item()
            sg = ((torch.sign(x) == torch.sign(r)) | (r.abs() < 1e-12)).float().mean().item()
            rows.append((sg, c, x.norm().item() / (r.norm().item() + 1e-20), r.norm().item() / scale, n))
        rows.sort()
        print(f"\n{name}: worst sign agreement (sign-agree, cos, norm ratio, |g_ref| / max, parameter)")
        for sg, c, ratio, rel, n in rows[:a.top]:
            print(f"  {sg:6.3f} {c:8.4f} {ratio:8.3f} {rel:9.2e}  {n}")
    # one AdamW step (first step: update = lr * g / (|g| + eps)) with each gradient set, loss by fp32 cpu
    lr = 2e-4
    for name, g in [("fp32", g_ref)] + [(k, v[1]) for k, v in res.items()]:
        m = raft_large()[0]
        m.load_state_dict(state)
        m.train()
        opt = torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=1e-4)
        for n, p in m.named_parameters():
            p.grad = g[n].clone() if n in g else None
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        with torch.no_grad():
            img1, img2, flow, valid = batch
            loss, _ = sequence_loss(m(img1, img2, train=True, num_flow_updates=a.iters), flow, valid)
        print(f"loss after one AdamW step with the {name} gradients (fp32 cpu forward): {float(loss):.4f}", flush=True)


if __name__ == "__main__":
    main()
