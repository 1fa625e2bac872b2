#!/usr/bin/env python3
"""Cost of the ConvGRU epilogues at the headline loop shape (raft_large, batch 4,
55x128 -> M = 28160): the same 1x5 conv (K = 5 x 256) timed with the plain
epilogue (bias only), + the context bias map, and with the GRU-A / GRU-B
epilogues (z / r*h / blend: z, fp32 h reads and writes), per tile config."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_raft_amd.ops import native as nat  # noqa: E402
from microbench import timeit  # noqa: E402


def main():
    nat.require()
    dev = "cuda"
    B, h, w, hd = 4, 55, 128, 128
    M = B * h * w
    torch.manual_seed(0)
    x = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    bm = torch.randn(M, 384, device=dev).to(torch.bfloat16)
    z = torch.rand(M, hd, device=dev).to(torch.bfloat16)
    h32 = torch.randn(M, hd, device=dev)
    for name, cout, epi in (("gru.a", 2 * hd, nat.EPI_GRU_A), ("gru.b", hd, nat.EPI_GRU_B)):
        k = torch.randn(1, 5, 256, cout) / math.sqrt(5 * 256)
        spec = nat.make_spec(k, torch.zeros(cout), (1, 1), (0, 2), cin8=256, device=dev)
        y = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
        for cfg in (21, 34, 22, 33):
            rows = []
            for tag, kw in (("plain", {}), ("bmap", dict(bmap=bm)),
                            ("epi", dict(bmap=bm, epi=epi, zbuf=z, hidden=hd,
                                         h32=h32 if epi == nat.EPI_GRU_B else None))):
                t, i, a = nat.conv_args(spec, x, B, h, w, y, cfg=cfg, **kw)
                rows.append(f"{tag}={timeit(lambda: nat.ops().conv(t, i, a), iters=50):6.1f}")
            print(f"{name} c{cfg}: " + " ".join(rows), flush=True)


if __name__ == "__main__":
    main()
