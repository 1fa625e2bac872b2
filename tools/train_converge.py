#!/usr/bin/env python3
"""Convergence check of the GPU training paths: overfit one fixed synthetic batch for --steps
AdamW steps with the fused native path, the unfused autograd path and fp32 autograd of the
golden model (``--ref gpu``: golden ops on the GPU, ``--cpu-ref`` / ``--ref cpu``: on the CPU),
all from the same initial weights, and print the loss curves (JSON).

Thirty steps of AdamW on one batch are a chaotic map: two trajectories that differ only by
rounding part after ~5 steps (``tools/train_trajectory.py`` shows that the fused and unfused
gradients agree step by step on the SAME weights).  A single seed therefore says little about
a path's convergence; ``--seeds N`` repeats the comparison over N data seeds and reports, per
path, the mean of the last-10-step mean losses over the seeds."""
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


def run(path, state, factory, batch, steps, iters, lr, device="cuda"):
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
        if path == "golden":
            with golden_ops():
                preds = model.forward_reference(img1, img2, True, iters)
        else:
            preds = model(img1, img2, train=True, num_flow_updates=iters, fused=(path == "fused"))
        loss, _ = sequence_loss(preds.float(), flow, valid)
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
    ap.add_argument("--seeds", type=int, default=1)
    ap.add_argument("--ref", choices=("none", "gpu", "cpu"), default="gpu")
    ap.add_argument("--cpu-ref", action="store_true", help="same as --ref cpu")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ref = "cpu" if a.cpu_ref else a.ref
    factory = raft_large if a.arch == "raft_large" else raft_small
    state = {k: v.clone() for k, v in factory()[0].state_dict().items()}
    if ref == "cpu":
        torch.set_num_threads(min(16, os.cpu_count() or 8))
    res = {"tool": "tools/train_converge.py", "args": vars(a), "seeds": []}
    for seed in range(a.seeds):
        data = SyntheticFlow(size=tuple(a.size), seed=seed, device=torch.device("cuda"))
        batch = data.batch(list(range(a.batch)))
        r = {"seed": seed,
             "fused": run("fused", state, factory, batch, a.steps, a.iters, a.lr),
             "unfused": run("unfused", state, factory, batch, a.steps, a.iters, a.lr)}
        if ref != "none":
            r["fp32_" + ref] = run("golden", state, factory, batch, a.steps, a.iters, a.lr,
                                   device="cuda" if ref == "gpu" else "cpu")
        r["last10"] = {k: sum(v[-10:]) / len(v[-10:]) for k, v in r.items() if isinstance(v, list)}
        res["seeds"].append(r)
        print(json.dumps({"seed": seed, "last10": r["last10"]}), flush=True)
    paths = res["seeds"][0]["last10"].keys()
    res["mean_last10"] = {k: sum(s["last10"][k] for s in res["seeds"]) / len(res["seeds"]) for k in paths}
    print(json.dumps({"mean_last10": res["mean_last10"]}))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
