#!/usr/bin/env python3
"""Per-step gradient oracle of the fused training step along a training trajectory.

``tools/train_converge.py`` only compares loss curves.  This tool follows ONE trajectory (the
fused native path with its persistent plans, as the Trainer and ``bench.py`` run it) and at
every step k, on the exact weights of that step, also computes:

* ``fresh``  -- the fused path with freshly built plans (a second model, plans dropped first):
  any difference to the persistent plans is state the plans carry across steps (stale packed
  weights, buffers that are not rewritten, statistics);
* ``unfused`` -- the per-op native autograd path;
* ``golden`` -- fp32 autograd of the golden ops on the GPU (``ops.functional.golden_ops``),
  on the same weights.

Per step it prints the loss of each path and, per path, the worst per-parameter relative
gradient errors ``||g - g_golden|| / ||g_golden||`` (parameters whose golden gradient is below
1e-4 of the largest are skipped), and ``max|persistent - fresh|``.  Output: one JSON document.

    python tools/train_trajectory.py --steps 30 --out gpurun_out/traj.json

Reference semantics: the coordinates are detached every iteration (``jax_raft/model.py:497-498``)
and the mask head is scaled by 0.25 (``model.py:396-400``).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.ops.functional import golden_ops  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402
from jax_raft_amd.train.data import SyntheticFlow  # noqa: E402
from jax_raft_amd.train.loss import sequence_loss  # noqa: E402


def grads_of(model, batch, iters, mode):
    """(loss, {name: fp32 grad}) of one forward/backward of ``model`` in ``mode``."""
    img1, img2, flow, valid = batch
    model.zero_grad(set_to_none=True)
    if mode == "golden":
        with golden_ops():
            preds = model.forward_reference(img1, img2, True, iters)
    else:
        preds = model(img1, img2, train=True, num_flow_updates=iters, fused=(mode == "fused"))
    loss, _ = sequence_loss(preds.float(), flow, valid)
    loss.backward()
    return float(loss), {n: p.grad.detach().float().clone() for n, p in model.named_parameters()
                         if p.grad is not None}


def rel_errors(g, ref, floor):
    out = {}
    for n, r in ref.items():
        rn = r.norm().item()
        if rn < floor:
            continue
        x = g.get(n)
        out[n] = 1.0 if x is None else (x - r).norm().item() / rn
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, nargs=2, default=[192, 256])
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    factory = raft_large if a.arch == "raft_large" else raft_small
    dev = torch.device("cuda")
    torch.manual_seed(0)
    state = {k: v.clone() for k, v in factory()[0].state_dict().items()}
    data = SyntheticFlow(size=tuple(a.size), seed=0, device=dev)
    batch = [t.to(dev) for t in data.batch(list(range(a.batch)))]

    traj = factory()[0]
    traj.load_state_dict(state)
    traj = traj.to(dev).train()
    opt = torch.optim.AdamW(traj.parameters(), lr=a.lr, weight_decay=1e-4)
    scratch = factory()[0].to(dev).train()
    names = [n for n, _ in traj.named_parameters()]
    rows = []
    for k in range(a.steps):
        # every path on the weights of this step (the trajectory's BN statistics do not enter a
        # train-mode forward)
        snap = {n: t.detach().clone() for n, t in traj.state_dict().items()}
        l_f, g_f = grads_of(traj, batch, a.iters, "fused")
        res = {"step": k + 1, "loss": {"fused": l_f}}
        grads = {"fused": g_f}
        for mode in ("fresh", "unfused", "golden"):
            scratch.load_state_dict(snap)
            F._LOOPS.pop(scratch, None)
            l, g = grads_of(scratch, batch, a.iters, "fused" if mode == "fresh" else mode)
            res["loss"][mode] = l
            grads[mode] = g
        ref = grads["golden"]
        floor = 1e-4 * max(v.norm().item() for v in ref.values())
        res["grad_norm"] = {m: torch.sqrt(sum((v * v).sum() for v in g.values())).item() for m, g in grads.items()}
        for m in ("fused", "fresh", "unfused"):
            e = rel_errors(grads[m], ref, floor)
            worst = sorted(e.items(), key=lambda kv: -kv[1])[: a.top]
            res[f"rel_{m}"] = {"max": worst[0][1], "median": sorted(e.values())[len(e) // 2],
                               "worst": [[n, round(v, 5)] for n, v in worst]}
        dpf = max(((grads["fused"][n] - grads["fresh"][n]).abs().max().item(), n) for n in grads["fused"])
        res["persistent_vs_fresh"] = {"max_abs": dpf[0], "param": dpf[1],
                                      "loss_diff": l_f - res["loss"]["fresh"]}
        rows.append(res)
        print(json.dumps(res), flush=True)
        # advance the trajectory with the fused gradients (as the Trainer does)
        for n, p in traj.named_parameters():
            p.grad = g_f[n].to(p.dtype) if n in g_f else None
        torch.nn.utils.clip_grad_norm_(traj.parameters(), 1.0)
        opt.step()
    doc = {"tool": "tools/train_trajectory.py", "args": vars(a), "params": len(names), "steps": rows}
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
