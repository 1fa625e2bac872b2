#!/usr/bin/env python3
"""Phase timing of the channel-split ConvGRU launches (csrc/kernels/gru_split.hip): thread 0 of
every workgroup stamps s_memrealtime (100 MHz) at its start, after the first slab is staged, after
each K slab and at its end; medians over workgroups give the split, the spread of the start stamps
the dispatch skew.

  python tools/gru_split_phases.py [--batch 4] [--cfg-a 1] [--cfg-b 6]
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
    ap.add_argument("--axis", type=int, default=0)
    ap.add_argument("--cfg-a", type=int, default=1)
    ap.add_argument("--cfg-b", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    nat.require()
    dev = "cuda"
    B, h, w = a.batch, a.h, a.w
    M = B * h * w
    torch.manual_seed(0)
    hx = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    qx = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    h32 = torch.randn(M, 128, device=dev)
    bm = torch.randn(M, 384, device=dev).to(torch.bfloat16)
    zb = torch.zeros(M, 128, device=dev, dtype=torch.bfloat16)
    ks = (5, 1) if a.axis else (1, 5)
    for mode, cfg in ((0, a.cfg_a), (1, a.cfg_b)):
        nout = 256 if mode == 0 else 128
        pb, cb, kc = nat.GRU_SPLIT_CFGS[cfg]
        L, J = nat.gru_split_tile(cfg, a.axis, B, h, w)
        wt = nat.pack_gru_split(torch.randn(*ks, 256, nout, device=dev) / math.sqrt(1280), cb, kc)
        length = h if a.axis else w
        lines = B * (w if a.axis else h)
        ptiles = -(-(lines * -(-length // L)) // J)
        grid = -(-ptiles // 8) * 8 * (nout // (32 * cb))
        dbg = torch.zeros(grid * 12, dtype=torch.long, device=dev)
        t = [hx, wt, bm, zb, qx, None, None, None, dbg] if mode == 0 else [qx, wt, bm, zb, None, h32, hx, None, dbg]
        i = [B, h, w, a.axis, mode, L, J, cfg]
        for _ in range(3):
            nat.ops().gru_split(t, i)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            nat.ops().gru_split(t, i)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.reps * 1e3
        st = dbg.view(grid, 12).double().cpu() * 0.01      # 100 MHz ticks -> us
        live = st[:, 0] > 0
        st = st[live]
        nslab = 256 // kc
        cols = [0, 1] + [2 + k for k in range(min(nslab, 8))] + [10]
        t_ = st[:, cols]
        d = (t_[:, 1:] - t_[:, :-1]).median(dim=0).values.tolist()
        names = ["stage slab 0"] + [f"slab {k}" for k in range(min(nslab, 8))] + ["epilogue"]
        span = (st[:, 10].max() - st[:, 0].min()).item()
        spread = (st[:, 0].max() - st[:, 0].min()).item()
        wg = (st[:, 10] - st[:, 0]).median().item()
        print(f"mode {mode} cfg {cfg} (PB {pb}, CB {cb}, KC {kc}, L {L}, J {J}): {int(live.sum())} WGs, "
              f"{us:.1f} us/launch (events), span {span:.1f} us, start spread {spread:.1f} us, WG median {wg:.1f} us")
        print("   " + "  ".join(f"{n}: {v:.2f}" for n, v in zip(names, d)))


if __name__ == "__main__":
    main()
