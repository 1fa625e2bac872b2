#!/usr/bin/env python3
"""Batch-1 loop-conv cost model: one 1x5 conv (M = 55 x 128 = 7040 pixels) timed
over its K (cin8 x 5) and tile configs -- separates the fixed cost of a launch
(ramp, epilogue, output) from the per-K-stage cost.

  python tools/conv_ksweep.py [cout] [cfg,cfg,...]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_raft_amd.ops import native as nat  # noqa: E402


def time_conv(cin, cout, cfg, kh=1, kw=5, B=1, h=55, w=128, n=50):
    torch.manual_seed(0)
    k = torch.randn(kh, kw, cin, cout) / math.sqrt(kh * kw * cin)
    spec = nat.make_spec(k, torch.randn(cout) * 0.1, (1, 1), (kh // 2, kw // 2), cin8=cin, device="cuda")
    x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
    M = B * h * w
    y = torch.empty(M, nat.round_up(cout, 8), device="cuda", dtype=torch.bfloat16)
    t, i, a = nat.conv_args(spec, x, B, h, w, y, act=nat.ACT_RELU, cfg=cfg)
    try:
        for _ in range(5):
            nat.ops().conv(t, i, a)
    except RuntimeError:
        return None
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            nat.ops().conv(t, i, a)
    g.replay()
    torch.cuda.synchronize()
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / n


def main():
    cout = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [15, 23, 24, 4, 2, 12, 14]
    nat.require()
    print(f"1x5 conv, M = 7040, cout {cout}: us per launch (graph of 50 launches)")
    print("cin8  K    " + " ".join(f"c{c:<6d}" for c in cfgs))
    for cin in (32, 64, 128, 256, 512):
        row = [time_conv(cin, cout, c) for c in cfgs]
        print(f"{cin:4d} {cin * 5:5d} " + " ".join(f"{v:7.2f}" if v else "   -   " for v in row), flush=True)
    print("3x3 convs (convcorr2-like 256 -> 192, me.conv 256 -> 126, fh1 128 -> 512)")
    for cin, co in ((256, 192), (256, 128), (128, 512), (128, 64)):
        row = [time_conv(cin, co, c, 3, 3) for c in cfgs]
        print(f"{cin:4d}->{co:3d} " + " ".join(f"{v:7.2f}" if v else "   -   " for v in row), flush=True)


if __name__ == "__main__":
    main()
