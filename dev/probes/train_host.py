#!/usr/bin/env python3
"""Is the training step (BASELINE config 5) host- or device-bound?  Times the host side of each
phase of Trainer._eager_step (forward + loss enqueue, backward enqueue, clip + optimizer enqueue,
the wait on the previous step in _settle) with time.perf_counter, next to the device time per
step; medians over the timed steps.

    python dev/probes/train_host.py [--steps 15]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd.train import trainer as T  # noqa: E402
from jax_raft_amd.train.loss import sequence_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=15)
    a = ap.parse_args()
    cfg = T.TrainConfig(arch="raft_large", steps=a.steps + 5, batch=6, iters=12, size=(384, 512), log_every=10 ** 9)
    tr = T.Trainer(cfg)
    batches = [tr.batch_for(i) for i in range(2)]
    for i in range(3):
        tr.train_step(batches[i % 2])
    torch.cuda.synchronize()
    ph = {k: [] for k in ("fwd", "bwd", "opt", "settle", "total")}
    orig_settle = tr._settle

    def settle(keep_last=False):
        t = time.perf_counter()
        orig_settle(keep_last)
        ph["settle"].append((time.perf_counter() - t) * 1e3)

    tr._settle = settle
    orig_loss = T.sequence_loss
    marks = {}

    def loss_hook(*args, **kw):
        marks["fwd"] = time.perf_counter()
        return orig_loss(*args, **kw)

    T.sequence_loss = loss_hook
    orig_clip = torch.nn.utils.clip_grad_norm_

    def clip_hook(*args, **kw):
        marks["bwd"] = time.perf_counter()
        return orig_clip(*args, **kw)

    torch.nn.utils.clip_grad_norm_ = clip_hook
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev[0].record()
    for i in range(a.steps):
        t0 = time.perf_counter()
        tr.train_step(batches[i % 2])
        t1 = time.perf_counter()
        ev[i + 1].record()
        ph["fwd"].append((marks["fwd"] - t0) * 1e3)
        ph["bwd"].append((marks["bwd"] - marks["fwd"]) * 1e3)
        ph["opt"].append((t1 - marks["bwd"]) * 1e3 - (ph["settle"][-1] if ph["settle"] else 0))
        ph["total"].append((t1 - t0) * 1e3)
    torch.cuda.synchronize()
    dev = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
    med = {k: round(statistics.median(v), 3) for k, v in ph.items() if v}
    print(f"host per step (median ms): {med}; device per step (median) {statistics.median(dev):.3f} ms", flush=True)
    T.sequence_loss, torch.nn.utils.clip_grad_norm_ = orig_loss, orig_clip


if __name__ == "__main__":
    main()
