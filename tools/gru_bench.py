#!/usr/bin/env python3
"""Per-launch device time of one ConvGRU stage at a RAFT loop shape: the halo-tiled fused
kernel (gru_halo.hip) for each of its tilings vs the whole-row fused kernel (gru_fused.hip,
raft_large only) and the two-launch implicit-GEMM path (EPI_GRU_A + EPI_GRU_B).  Each
variant runs as a captured graph of --reps launches (no host launch cost in the number).

  python tools/gru_bench.py --arch raft_large --batch 1 [--h 55 --w 128]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_time(fn, reps=50, rounds=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        t = s.elapsed_time(e) * 1000.0 / reps
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large", choices=["raft_large", "raft_small"])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--h", type=int, default=55)
    ap.add_argument("--w", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from jax_raft_amd.ops import native as nat

    nat.require()
    dev = torch.device("cuda", 0)
    large = a.arch == "raft_large"
    hd = 128 if large else 96
    cs = 2 * hd
    B, h, w = a.batch, a.h, a.w
    M = B * h * w
    stages = [((1, 5), 0, 0), ((5, 1), 0, 1)] if large else [((3, 3), 1, 0)]
    src = torch.randn(M, cs, device=dev).to(torch.bfloat16)
    dst = torch.randn(M, cs, device=dev).to(torch.bfloat16)
    h32 = torch.randn(M, hd, device=dev)
    bm = (torch.randn(M, 3 * hd, device=dev) * 0.3).to(torch.bfloat16)
    zb = torch.empty(M, hd, device=dev, dtype=torch.bfloat16)
    for ks, mode, axis in stages:
        kzr = torch.randn(*ks, cs, 2 * hd, device=dev) / math.sqrt(ks[0] * ks[1] * cs)
        kq = torch.randn(*ks, cs, hd, device=dev) / math.sqrt(ks[0] * ks[1] * cs)
        wa, wb = nat.pack_gru_halo(kzr, cs), nat.pack_gru_halo(kq, cs)
        print(f"{a.arch} {ks[0]}x{ks[1]} stage, B={B}, {h}x{w} map (M = {M})")
        for tile in nat.gru_halo_candidates(hd, mode, axis, B, h, w):
            t = graph_time(lambda: nat.ops().gru_halo([src, src, wa, wb, bm, h32, dst, None],
                                                      [B, h, w, mode, axis, *tile]), a.reps)
            print(f"  gru_halo tile {tile}: {nat.gru_halo_tiles(mode, axis, B, h, w, tile[0], tile[1])} WGs  "
                  f"{t:7.2f} us")
        pad = ((ks[0] - 1) // 2, (ks[1] - 1) // 2)
        sa = nat.make_spec(kzr, torch.zeros(2 * hd, device=dev), (1, 1), pad, cin8=cs, device=dev)
        sb = nat.make_spec(kq, torch.zeros(hd, device=dev), (1, 1), pad, cin8=cs, device=dev)
        best = None
        for cfg_a in nat.TUNE_CFGS:
            try:
                ta = graph_time(lambda: nat.ops().conv(*nat.conv_args(
                    sa, src, B, h, w, dst, zbuf=zb, hidden=hd, epi=nat.EPI_GRU_A, bmap=bm, cfg=cfg_a)), a.reps)
            except RuntimeError:
                continue
            best = ta if best is None else min(best, ta)
        bestb = None
        for cfg_b in nat.TUNE_CFGS:
            try:
                tb = graph_time(lambda: nat.ops().conv(*nat.conv_args(
                    sb, dst, B, h, w, src, h32=h32, zbuf=zb, hidden=hd, epi=nat.EPI_GRU_B, bmap=bm,
                    bmap_coff=2 * hd, cfg=cfg_b)), a.reps)
            except RuntimeError:
                continue
            bestb = tb if bestb is None else min(bestb, tb)
        print(f"  two-launch GEMM path (best tile configs): {best:7.2f} + {bestb:7.2f} = {best + bestb:7.2f} us")
        if large and nat.ops().gru_fused_fits(h, w, axis):
            wpa, wpb = sa.w, sb.w
            t = graph_time(lambda: nat.ops().gru_fused([src, wpa, wpb, bm, h32, src, None], [B, h, w, axis]), a.reps)
            print(f"  gru_fused (whole rows / columns): {nat.gru_fused_tiles(B, h, w, axis)} WGs  {t:7.2f} us")


if __name__ == "__main__":
    main()
