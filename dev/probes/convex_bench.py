#!/usr/bin/env python3
"""Device time of the inference convex mask head (csrc/kernels/convex_head.h) at raft_large
batch 4 (55 x 128 maps), as a captured graph of 30 launches (the persistent form above 128
pixel blocks; the round-4 A/B of the two forms: profiles/r4_convex_persist_ab.txt)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd.ops import native as nat  # noqa: E402


def main():
    B, h, w = int(sys.argv[1]) if len(sys.argv) > 1 else 4, 55, 128
    tiles = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    M = B * h * w
    dev = torch.device("cuda", 0)
    feat = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    k = torch.randn(1, 1, 256, 576, device=dev) * 0.05
    wpk, bias = nat.pack_convex_head(k, torch.randn(576, device=dev) * 0.1)
    flow = torch.randn(M, 2, device=dev)
    out = torch.empty(B, 8 * h, 8 * w, 2, device=dev)

    def run():
        nat.ops().convex_head([feat, wpk, bias, flow, out], [B, h, w, 0, 0, tiles], 0.25)

    run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(30):
            run()
    best = None
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        t = s.elapsed_time(e) * 1000 / 30
        best = t if best is None else min(best, t)
    print(f"convex_head B={B} tiles={tiles}: {best:.1f} us, "
          f"checksum {out.double().abs().sum().item():.6e}")


if __name__ == "__main__":
    main()
