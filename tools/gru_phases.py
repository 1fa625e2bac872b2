#!/usr/bin/env python3
"""Phase timing of the fused ConvGRU stage kernel (csrc/kernels/gru_fused.hip) at the
headline geometry (raft_large, 440x1024 -> 55 x 128, batch 4): each workgroup's thread 0
stamps s_memrealtime (100 MHz) at kernel start, after GEMM 1, after epilogue 1, after
GEMM 2 and at its end; the medians over workgroups give the time split.

  python tools/gru_phases.py [--batch 4] [--g2 1]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_raft_amd.ops import native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--h", type=int, default=55)
    ap.add_argument("--w", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--g2", type=int, default=1, help="GEMM 2 on all 16 waves (1) or the 8 z waves (0)")
    a = ap.parse_args()
    nat.require()
    dev = "cuda"
    B, h, w, hd = a.batch, a.h, a.w, 128
    M = B * h * w
    torch.manual_seed(0)
    hx = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    h32 = torch.randn(M, hd, device=dev)
    bm = torch.randn(M, 384, device=dev).to(torch.bfloat16)
    names = ("GEMM 1 (z, r)", "epilogue 1 (+ sync)", "GEMM 2 (q)", "epilogue 2")
    for vertical in (0, 1):
        ks = (5, 1) if vertical else (1, 5)
        pad = (2, 0) if vertical else (0, 2)
        sa = nat.make_spec(torch.randn(*ks, 256, 256) / math.sqrt(1280), torch.zeros(256), (1, 1), pad, cin8=256, device=dev)
        sb = nat.make_spec(torch.randn(*ks, 256, 128) / math.sqrt(1280), torch.zeros(128), (1, 1), pad, cin8=256, device=dev)
        tiles = B * h if not vertical else B * (w // 2 if 2 * h <= 128 and w % 2 == 0 else w)
        dbg = torch.zeros(tiles * 6, dtype=torch.long, device=dev)
        args = ([hx, sa.w, sb.w, bm, h32, hx, None, dbg], [B, h, w, vertical, a.g2])
        for _ in range(3):
            nat.ops().gru_fused(*args)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            nat.ops().gru_fused(*args)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.reps * 1e3
        t = dbg.view(tiles, 6)[:, :5].double().cpu() * 0.01   # 100 MHz ticks -> us
        d = t[:, 1:] - t[:, :-1]
        med = d.median(dim=0).values.tolist()
        span = (t[:, 4].max() - t[:, 0].min()).item()
        start_spread = (t[:, 0].max() - t[:, 0].min()).item()
        print(f"{'5x1 columns' if vertical else '1x5 rows'}: {tiles} tiles, {us:.1f} us/launch (events), "
              f"stamp span {span:.1f} us, start spread {start_spread:.1f} us")
        for n_, v in zip(names, med):
            print(f"    {n_:22s} {v:6.2f} us (median workgroup)")


if __name__ == "__main__":
    main()
