#!/usr/bin/env python3
"""Device time of the correlation pyramid build and the radius-4 pyramid lookup at the
engine's layout (bf16 levels, blocked levels 0 / 1) for raft_large at 440x1024 (55 x 128
feature map, 256 channels), as a captured graph of --reps launches; ``--run N`` launches one
of them N times (rocprofv3 --pmc passes).

  python tools/corr_bench.py pyr lookup --batch 4
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from conv_bench import graph_time  # noqa: E402


def setup(B, h=55, w=128, C=256, L=4, radius=4):
    from jax_raft_amd.ops import native as nat

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    f1 = torch.randn(B, h, w, C, device=dev, generator=g).to(torch.bfloat16)
    f2 = torch.randn(B, h, w, C, device=dev, generator=g).to(torch.bfloat16)
    M = B * h * w
    levels, hl, wl = [], h, w
    for l in range(L):
        shape = (M, -(-h // 8) * (8 >> l), -(-w // 16) * (16 >> l)) if l < 2 else (M, hl, wl)
        levels.append(torch.zeros(shape, device=dev, dtype=torch.bfloat16))
        hl //= 2
        wl //= 2
    ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
    base = torch.stack([xs, ys], -1).float().expand(B, h, w, 2)
    coords = (base + 6 * torch.rand(B, h, w, 2, device=dev, generator=g) - 3).reshape(M, 2).contiguous()
    S = 2 * radius + 1
    out = torch.empty(M, nat.round_up(L * S * S, 8), device=dev, dtype=torch.bfloat16)

    def pyr():
        nat.ops().corr([f1, f2] + levels, [B, h, w, C, L, h * w, 1], C ** -0.5)

    def lookup():
        nat.ops().lookup([coords, out] + levels, [L, B, h, w, radius, h * w, 1])

    wbytes = sum(v.numel() * 2 for v in levels)
    return dict(pyr=(pyr, f"writes {wbytes / 1e6:.0f} MB", wbytes),
                lookup=(lookup, f"out {out.numel() * 2 / 1e6:.1f} MB", None))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ops", nargs="+", choices=["pyr", "lookup"])
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--run", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    fns = setup(a.batch)
    fns["pyr"][0]()   # levels filled before any lookup
    for op in a.ops:
        fn, what, wbytes = fns[op]
        if a.run:
            for _ in range(a.run):
                fn()
            torch.cuda.synchronize()
            continue
        t = graph_time(fn, a.reps)
        extra = f", {wbytes / t / 1e6:.2f} TB/s of writes" if wbytes else ""
        print(f"{op} batch {a.batch}: {t:.1f} us ({what}{extra})")


if __name__ == "__main__":
    main()
