#!/usr/bin/env python3
"""Microbenchmark of the pointwise LDS-weight conv (conv1x1.hip) at the
convcorr1 shape (raft_large, 324 -> 256 + ReLU), batch 1 and 4;
graph-replayed like the engine."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.ops import native as nat  # noqa: E402


def main():
    nat.load()
    dev = torch.device("cuda", 0)
    res = {}
    for B in (1, 4):
        M = B * 55 * 128
        x = torch.randn(M, 328, device=dev).to(torch.bfloat16)
        w = nat.pack_conv1x1(torch.randn(1, 1, 324, 256, device=dev) * 0.05, 352)
        b = torch.randn(256, device=dev)
        y = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
        f = lambda: nat.ops().conv1x1([x, w, b, y], [M, 328, 352, 256, nat.ACT_RELU, 0])
        for _ in range(5):
            f()
        g = torch.cuda.CUDAGraph()   # graph-replayed, as in the engine (no launch overhead)
        with torch.cuda.graph(g):
            for _ in range(20):
                f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g.replay()
        torch.cuda.synchronize()
        s.record()
        for _ in range(5):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        res[f"B{B}_us"] = round(s.elapsed_time(e) * 1e3 / 100, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
