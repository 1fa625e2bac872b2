#!/usr/bin/env python3
"""Fixed (K-independent) cost of one implicit-GEMM conv launch: time a
one-stage (K = 64) 1x1 conv at the loop's M with N = 256 / 64 outputs, at a
tiny M, and with / without the X-W loads, next to a bare 16-byte memset
(the timing loop's own launch floor)."""
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
    cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "34,22,0").split(",")]
    z = torch.zeros(4, device=dev)
    print(f"launch floor (memset 16 B): {timeit(lambda: z.zero_(), iters=50):6.1f} us")
    for M, cin, cout in ((28160, 64, 256), (28160, 64, 64), (28160, 64, 512), (256, 64, 256), (2048, 64, 256),
                         (28160, 256, 256)):
        k = torch.randn(1, 1, cin, cout) / math.sqrt(cin)
        b = torch.zeros(cout)
        spec = nat.make_spec(k, b, (1, 1), (0, 0), device=dev)
        x = torch.randn(1, 1, M, cin, device=dev).to(torch.bfloat16)
        y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        row = []
        for cfg in cfgs:
            t, i, a = nat.conv_args(spec, x, 1, 1, M, y, act=nat.ACT_RELU, cfg=cfg)
            full = timeit(lambda: nat.ops().conv(t, i, a))
            i = list(i)
            i[20] = cfg | (3 << 8)
            noxw = timeit(lambda: nat.ops().conv(t, i, a))
            row.append(f"c{cfg}: {full:6.1f} (noXW {noxw:6.1f})")
        print(f"M={M:6d} K={cin:4d} N={cout:4d}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
