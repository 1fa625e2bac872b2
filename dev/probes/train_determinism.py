#!/usr/bin/env python3
"""Is the fused training step (BASELINE config 5 shapes) bitwise deterministic?  Two fresh Trainers
from the same seed take the same K steps on the same batches; per step the loss and a checksum of
every gradient are compared, and at the first step that differs the parameters whose gradients
differ are listed (largest relative difference first).  Then the fused forward alone is run twice
on the first trainer's model.

    python dev/probes/train_determinism.py [--steps 4] [--batch 6] [--size 384 512]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402


def run(a):
    torch.manual_seed(0)
    cfg = TrainConfig(arch="raft_large", steps=a.steps + 2, batch=a.batch, iters=12, size=tuple(a.size),
                      log_every=10 ** 9)
    tr = Trainer(cfg)
    batches = [tr.batch_for(i) for i in range(2)]
    trace = []
    for i in range(a.steps):
        loss = tr.train_step(batches[i % 2])["loss"]
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().float().clone() for n, p in tr.model.named_parameters() if p.grad is not None}
        trace.append((float(loss) if loss is not None else float("nan"), grads))
    return tr, batches, trace


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--size", type=int, nargs=2, default=[384, 512])
    a = ap.parse_args()
    tr1, batches, t1 = run(a)
    _, _, t2 = run(a)
    for i, ((l1, g1), (l2, g2)) in enumerate(zip(t1, t2)):
        diff = [(float((g1[n] - g2[n]).abs().max() / (g1[n].abs().max() + 1e-30)), n) for n in g1 if not torch.equal(g1[n], g2[n])]
        print(f"step {i + 1}: loss {l1!r} vs {l2!r}; gradients differing: {len(diff)} of {len(g1)}", flush=True)
        if diff:
            for d, n in sorted(diff, reverse=True)[:15]:
                print(f"    {d:.3e}  {n}")
            break
    # the fused forward alone, twice, on the same weights and batch
    img1, img2 = batches[0][0], batches[0][1]
    m = tr1.model
    with torch.no_grad():
        o1 = [t.clone() for t in m(img1, img2, train=True, num_flow_updates=12, fused=True)]
        o2 = [t.clone() for t in m(img1, img2, train=True, num_flow_updates=12, fused=True)]
    torch.cuda.synchronize()
    same = all(torch.equal(x, y) for x, y in zip(o1, o2))
    print(f"fused forward twice: bitwise equal {same}; max |diff| {max(float((x - y).abs().max()) for x, y in zip(o1, o2)):.3e}")


if __name__ == "__main__":
    main()
