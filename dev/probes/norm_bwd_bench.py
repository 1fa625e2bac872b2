"""Isolated instance-norm backward (train.hip:jr_norm_bwd: partial + final + apply) at the
config-5 encoder shapes: time per call and effective HBM rate.  Usage: python dev/probes/norm_bwd_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from jax_raft_amd.ops import native as nat  # noqa: E402

EPS = 1e-5
dev = torch.device("cuda:0")
BF = torch.bfloat16


def one(N, HW, C, om_on, gres_on, reps=50):
    g = torch.randn(N, HW, C, device=dev).to(BF)
    y = torch.randn(N, HW, C, device=dev).to(BF)
    om = torch.randn(N, HW, C, device=dev).to(BF) if om_on else None
    st = torch.stack([y.float().mean(1), y.float().var(1)], -1).contiguous()   # [N, C, 2] mean / var
    red = torch.zeros(N, C, 2, device=dev)
    dy = torch.empty(N, HW, C, device=dev, dtype=BF)
    gres = torch.empty(N, HW, C, device=dev, dtype=BF) if gres_on else None
    p = nat.new_plan()
    p.add_norm_bwd([g, om, y, st, None, None, red, None, dy, gres], [1, 1, N, HW, C], EPS)
    p.capture(0)
    for _ in range(3):
        p.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        p.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    t = N * HW * C * 2
    nin = 2 + (1 if om_on else 0)
    byts = t * nin * 2 + t * (1 + (1 if gres_on else 0))
    print(f"N={N} HW={HW} C={C} om={int(om_on)} gres={int(gres_on)}: {us:7.1f} us  "
          f"{byts / us / 1e6:5.2f} TB/s (ideal at 5 TB/s {byts / 5e6:6.1f} us)", flush=True)
    return us


if __name__ == "__main__":
    tot = 0.0
    for N, HW, C in ((12, 49152, 64), (12, 12288, 96), (12, 3072, 128), (6, 49152, 64), (6, 12288, 96),
                     (6, 3072, 128)):
        tot += one(N, HW, C, False, False)
        one(N, HW, C, True, True)
    print(f"sum over shapes (plain): {tot:.1f} us")
