#!/usr/bin/env python3
"""Which framework ops does the Trainer's whole-step graph capture (train/trainer.py:_capture, the
graph replayed by every timed training step of BASELINE config 5) record?  torch.profiler on the
CPU side of the capture: ATen fills / copies / reductions by the innermost jax_raft_amd or torch
frame, so each replayed framework kernel can be traced to its line.

    python dev/probes/train_capture_ops.py
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402

WATCH = ("fill_", "zero_", "copy_", "zeros", "clone", "to", "_to_copy", "sum", "norm", "stack", "cat", "mul", "add",
         "where", "empty", "_foreach")


def frame(ev):
    st = [s for s in (ev.stack or []) if ("jax_raft_amd" in s or "torch/" in s) and "profiler" not in s]
    own = [s for s in st if "jax_raft_amd" in s]
    return (own[0] if own else st[0] if st else "?").split("site-packages/")[-1]


def main():
    cfg = TrainConfig(steps=8, batch=6, iters=12, size=(384, 512), log_every=10 ** 9)
    tr = Trainer(cfg)
    b = tr.batch_for(0)
    for _ in range(cfg.graph_warmup):
        tr.train_step(b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        tr.train_step(b)   # the first graph step: captures, then replays
        torch.cuda.synchronize()
    agg = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if not name.startswith("aten::"):
            continue
        op = name[6:]
        if not any(op == w or op.startswith(w) for w in WATCH):
            continue
        agg[(name, frame(ev))] += 1
    for (name, fr), n in agg.most_common(60):
        print(f"{n:5d}  {name:32s} {fr}")


if __name__ == "__main__":
    main()
