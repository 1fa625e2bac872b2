#!/usr/bin/env python3
"""Per-kernel microbenchmarks at the headline shapes (raft_large, 440x1024,
batch 4 -> fmap 55x128, M = 28160 query pixels).  Times every loop-body conv
under each tile config, the lookup, the correlation build and the upsample
with hip events; prints a table (and JSON with --json)."""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_raft_amd.ops import native as nat  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--h", type=int, default=55)
    ap.add_argument("--w", type=int, default=128)
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--gemm", action="store_true", help="also time the equivalent plain GEMM on hipBLASLt")
    ap.add_argument("--ablate", default="", help="comma list of cfgs: also time them with X / W / both loads dropped")
    ap.add_argument("--encoder", action="store_true",
                    help="time the encoder convs instead (raft_large FE half at batch 4: 4 images of 440x1024)")
    args = ap.parse_args()
    nat.require()
    dev = "cuda"
    B, h, w = args.batch, args.h, args.w
    M = B * h * w
    torch.manual_seed(0)
    res = {}

    def rnd(*s, dtype=torch.bfloat16):
        return torch.randn(*s, device=dev).to(dtype)

    # ------------------------------------------------------------- convs
    convs = [
        # name, cin, cin8/x_cs, cout, kh, kw, pad
        ("convcorr1", 324, 328, 256, 1, 1, (0, 0)),
        ("convflow1", 2, 8, 128, 7, 7, (3, 3)),
        ("convcorr2", 256, 256, 192, 3, 3, (1, 1)),
        ("convflow2", 128, 128, 64, 3, 3, (1, 1)),
        ("me.conv", 256, 256, 126, 3, 3, (1, 1)),
        # GRU convs over [h | motion | flow] (the context share is a prologue bias map)
        ("gru.a(1x5)", 256, 256, 256, 1, 5, (0, 2)),
        ("gru.b(1x5)", 256, 256, 128, 1, 5, (0, 2)),
        ("gru.a(5x1)", 256, 256, 256, 5, 1, (2, 0)),
        ("conv1x5.nobmap", 256, 256, 256, 1, 5, (0, 2)),   # gru.a without the bias-map epilogue read
        # fixed-cost probes: one / four 64-deep K stages at the loop's M and N = 256
        ("probe.k64", 64, 64, 256, 1, 1, (0, 0)),
        ("probe.k256", 256, 256, 256, 1, 1, (0, 0)),
        ("fh1+mask1", 128, 128, 512, 3, 3, (1, 1)),
        ("fh2", 256, 256, 2, 3, 3, (1, 1)),
        ("mask2", 256, 256, 576, 1, 1, (0, 0)),
    ]
    if args.encoder:   # name, cin, cs, cout, kh, kw, pad, stride, input H, W
        convs = [("stem7x7s2", 3, 8, 64, 7, 7, (3, 3), 2, 440, 1024),
                 ("l1.3x3.64", 64, 64, 64, 3, 3, (1, 1), 1, 220, 512),
                 ("l2.3x3s2.96", 64, 64, 96, 3, 3, (1, 1), 2, 220, 512),
                 ("l2.3x3.96", 96, 96, 96, 3, 3, (1, 1), 1, 110, 256),
                 ("l2.ds1x1s2", 64, 64, 96, 1, 1, (0, 0), 2, 220, 512),
                 ("l3.3x3s2.128", 96, 96, 128, 3, 3, (1, 1), 2, 110, 256),
                 ("l3.3x3.128", 128, 128, 128, 3, 3, (1, 1), 1, 55, 128),
                 ("head1x1.256", 128, 128, 256, 1, 1, (0, 0), 1, 55, 128)]
    else:
        convs = [c + (1, h, w) for c in convs]
    for name, cin, cs, cout, kh, kw, pad, st, H_, W_ in convs:
        if args.only and args.only not in name:
            continue
        k = torch.randn(kh, kw, cin, cout) / math.sqrt(kh * kw * cin)
        b = torch.randn(cout) * 0.1
        spec = nat.make_spec(k, b, (st, st), pad, cin8=cs, device=dev)
        x = rnd(B, H_, W_, cs)
        OH, OW = spec.out_hw(H_, W_)
        Mo = B * OH * OW
        y = torch.empty(Mo, nat.round_up(cout, 8), device=dev, dtype=torch.bfloat16)
        flops = 2.0 * Mo * cout * kh * kw * cin
        row = {}
        bm = torch.randn(M, 384, device=dev) if name.startswith("gru") else None
        for cfg in nat.TUNE_CFGS:
            t, i, a = nat.conv_args(spec, x, B, H_, W_, y, act=nat.ACT_RELU, cfg=cfg, bmap=bm)
            us = timeit(lambda: nat.ops().conv(t, i, a))
            row[cfg] = us
        best = min(row, key=row.get)
        for cfg in [int(c) for c in args.ablate.split(",") if c]:
            parts = []
            for ab, nm in ((1, "noX"), (2, "noW"), (3, "noXW")):
                t, i, a = nat.conv_args(spec, x, B, H_, W_, y, act=nat.ACT_RELU, cfg=cfg)
                i = list(i)
                i[20] = cfg | (ab << 8)
                parts.append(f"{nm}={timeit(lambda: nat.ops().conv(t, i, a)):6.1f}")
            print(f"{'':12s} ablate c{cfg}: full={row[cfg]:6.1f} " + " ".join(parts), flush=True)
        if args.gemm:  # same M x K x N as a library GEMM (no im2col, no epilogue): a yardstick
            K = kh * kw * cin
            a_ = rnd(Mo, K)
            b_ = rnd(K, cout)
            g_us = timeit(lambda: torch.matmul(a_, b_))
            print(f"{'':12s} hipBLASLt {Mo}x{K}x{cout}: {g_us:7.1f} us {flops / g_us / 1e6:7.1f} TF/s")
        res[name] = {"us": row, "best_cfg": best, "tflops": flops / row[best] / 1e6, "heuristic": nat.pick_cfg(Mo, cout)}
        print(f"{name:12s} " + " ".join(f"c{c}={u:7.1f}" for c, u in row.items()) +
              f"  best=c{best} {flops / row[best] / 1e6:7.1f} TF/s  heur=c{nat.pick_cfg(Mo, cout)}", flush=True)
    if args.encoder:
        if args.json:
            with open(args.json, "w") as fh:
                json.dump(res, fh, indent=1)
        return

    # ------------------------------------------------------------- correlation
    if not args.only or "corr" in args.only or "lookup" in args.only:
        C = 256
        f = rnd(2 * B, h, w, C)
        for dt in (torch.float32, torch.bfloat16):  # bf16 = the engine's default pyramid storage
            lv = []
            hl, wl = h, w
            for _ in range(4):
                lv.append(torch.empty(M, hl, wl, device=dev, dtype=dt))
                hl //= 2
                wl //= 2
            us = timeit(lambda: nat.ops().corr([f[:B], f[B:]] + lv, [B, h, w, C, 4], 1 / 16.0), iters=5)
            tag = "corr_pyramid" + ("" if dt == torch.bfloat16 else "_fp32")
            res[tag] = {"us": us, "tflops": 2.0 * B * (h * w) ** 2 * C / us / 1e6}
            print(f"{tag:12s} {us:8.1f} us  {2.0 * B * (h * w) ** 2 * C / us / 1e6:.1f} TF/s", flush=True)
        coords = (torch.stack(torch.meshgrid(torch.arange(w), torch.arange(h), indexing="xy"), -1).float()
                  .reshape(1, h * w, 2).repeat(B, 1, 1).reshape(M, 2).to(dev))
        coords += torch.randn_like(coords) * 3
        out = torch.empty(M, 328, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: nat.ops().lookup([coords, out] + lv, [4, B, h, w, 4]))
        res["lookup"] = {"us": us}
        print(f"lookup       {us:8.1f} us")
    if not args.only or "flowhead" in args.only:
        taps = torch.randn(M, 24, device=dev)
        bias = torch.zeros(2, device=dev)
        coords = torch.zeros(M, 2, device=dev)
        f32 = torch.zeros(M, 2, device=dev)
        hx = rnd(M, 400)
        f8 = rnd(M, 8)
        us = timeit(lambda: nat.ops().flow_taps([taps, bias, coords, f32, hx, hx, f8], [B, h, w, 382, 382]))
        res["flow_taps"] = {"us": us}
        print(f"flow_taps    {us:8.1f} us")
    if not args.only or "upsample" in args.only:
        mask = rnd(M, 576)
        flow = torch.randn(M, 2, device=dev)
        out = torch.empty(B, 8 * h, 8 * w, 2, device=dev)
        us = timeit(lambda: nat.ops().upsample_convex([mask, flow, out], [B, h, w, 0]))
        res["upsample_convex"] = {"us": us}
        print(f"upsample     {us:8.1f} us")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
