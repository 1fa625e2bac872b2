#!/usr/bin/env python3
"""Convergence sanity check of the GPU training paths: overfit one fixed
synthetic batch for --steps steps with the fused native path and with the
unfused autograd path from the same initial weights, and (``--cpu-ref``) with fp32 CPU
autograd of the golden model (models/reference.py) as the reference trajectory; print the loss
curves (JSON).  They must descend alike (bf16 rounding differs, trajectories need not match
exactly)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.data import SyntheticFlow  # noqa: E402
from jax_raft_amd.train.loss import sequence_loss  # noqa: E402


def run(fused, state, factory, batch, steps, iters, lr, device="cuda"):
    torch.manual_seed(0)
    model, _ = factory()
    model.load_state_dict(state)
    model = model.to(device).train()
    batch = [t.to(device) for t in batch]
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=1e-4)
    F._LOOPS.clear()
    img1, img2, flow, valid = batch
    out = []
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        preds = model(img1, img2, train=True, num_flow_updates=iters, fused=fused)
        loss, _ = sequence_loss(preds, flow, valid)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        out.append(round(loss.item(), 4))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, nargs=2, default=[192, 256])
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--cpu-ref", action="store_true", help="also the fp32 CPU golden trajectory")
    a = ap.parse_args()
    factory = raft_large if a.arch == "raft_large" else raft_small
    state = {k: v.clone() for k, v in factory()[0].state_dict().items()}
    data = SyntheticFlow(size=tuple(a.size), seed=0, device=torch.device("cuda"))
    batch = data.batch(list(range(a.batch)))
    res = {"fused": run(True, state, factory, batch, a.steps, a.iters, a.lr),
           "unfused": run(False, state, factory, batch, a.steps, a.iters, a.lr)}
    if a.cpu_ref:
        torch.set_num_threads(min(16, os.cpu_count() or 8))
        res["fp32_cpu"] = run(False, state, factory, batch, a.steps, a.iters, a.lr, device="cpu")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
