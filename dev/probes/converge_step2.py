#!/usr/bin/env python3
"""The fused training trajectory of tools/train_converge.py parts from fp32 at step 2 although the
step-1 gradients agree (dev/probes/converge_grads.py).  After one fused AdamW step on the
converge setting, evaluate the SAME updated weights four ways: the fused plans that took the
step (persistent), fresh fused plans, the unfused native path, and fp32 CPU autograd.

    python dev/probes/converge_step2.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.data import SyntheticFlow  # noqa: E402
from jax_raft_amd.train.loss import sequence_loss  # noqa: E402


def loss_of(model, batch, fused, iters=6):
    img1, img2, flow, valid = (t.to(next(model.parameters()).device) for t in batch)
    with torch.no_grad():
        preds = model(img1, img2, train=True, num_flow_updates=iters, fused=fused)
        loss, _ = sequence_loss(preds, flow, valid)
    return float(loss)


def main():
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    torch.manual_seed(0)
    model = raft_large()[0].cuda().train()
    data = SyntheticFlow(size=(192, 256), seed=0, device=torch.device("cuda"))
    batch = data.batch([0, 1])
    opt = torch.optim.AdamW(model.parameters(), lr=2e-4, weight_decay=1e-4)
    F._LOOPS.clear()
    img1, img2, flow, valid = batch
    for step in range(2):
        opt.zero_grad(set_to_none=True)
        preds = model(img1, img2, train=True, num_flow_updates=6, fused=True)
        loss, _ = sequence_loss(preds, flow, valid)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        print(f"step {step + 1}: fused training loss {float(loss):.4f}", flush=True)
    res = {}
    res["fused, the plans that trained"] = loss_of(model, batch, True)
    F._LOOPS.clear()
    res["fused, fresh plans"] = loss_of(model, batch, True)
    res["unfused native"] = loss_of(model, batch, False)
    cpu = raft_large()[0]
    cpu.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    cpu.train()
    res["fp32 cpu"] = loss_of(cpu, [t.cpu() for t in batch], False)
    for k, v in res.items():
        print(f"updated weights, loss by {k}: {v:.4f}", flush=True)


if __name__ == "__main__":
    main()
