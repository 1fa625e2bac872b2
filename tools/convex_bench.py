#!/usr/bin/env python3
"""Microbenchmark of the inference mask head at raft_large shapes: the
dedicated convex_head kernel (per tiles-per-wave choice) vs the EPI_CONVEX conv
epilogue and the separate mask conv + upsample_convex pair."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.ops import native as nat  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 4])
    a = ap.parse_args()
    nat.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    res = {}
    for B in a.batch:
        h, w = 55, 128
        M = B * h * w
        feat = torch.randn(M, 256, generator=g).to(torch.bfloat16).to(dev)
        kern = torch.randn(1, 1, 256, 576, generator=g) * 0.06
        bias = torch.randn(576, generator=g) * 0.5
        flow = (torch.randn(M, 2, generator=g) * 3).to(dev)
        wpk, bp = nat.pack_convex_head(kern.to(dev), bias.to(dev))
        out = torch.empty(B, 8 * h, 8 * w, 2, device=dev)
        for t in (0, 1, 2):
            res[f"B{B} head tiles={t}"] = round(timeit(lambda: nat.convex_head(feat, wpk, bp, flow, B, h, w, 0.25,
                                                                               out=out, tiles=t)), 2)
        res[f"B{B} out.zero_()"] = round(timeit(lambda: out.zero_()), 2)
        mask = torch.empty(M, 576, device=dev, dtype=torch.bfloat16)
        res[f"B{B} upsample_convex only"] = round(timeit(lambda: nat.ops().upsample_convex([mask, flow, out],
                                                                                          [B, h, w, 0])), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
