#!/usr/bin/env python3
"""conv_halo.hip (config 44) vs the autotuned implicit-GEMM configs on the
encoders' 3x3 convs at the headline shapes (440x1024 frames, 4 images per
encoder pass): layer1 64 -> 64 at 220x512, layer3 128 -> 128 at 55x128."""
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
    for N, H, W, cin, cout in ((4, 220, 512, 64, 64), (4, 55, 128, 128, 128), (8, 220, 512, 64, 64)):
        k = torch.randn(3, 3, cin, cout) / math.sqrt(9 * cin)
        b = torch.zeros(cout)
        spec = nat.make_spec(k, b, (1, 1), (1, 1), device=dev)
        x = torch.randn(N, H, W, cin, device=dev).to(torch.bfloat16)
        y = torch.empty(N * H * W, cout, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * N * H * W * cout * 9 * cin
        row = {}
        for cfg in tuple(nat.TUNE_CFGS) + (nat.HALO_CFG,):
            t, i, a = nat.conv_args(spec, x, N, H, W, y, act=nat.ACT_RELU, cfg=cfg)
            row[cfg] = timeit(lambda: nat.ops().conv(t, i, a), iters=10)
        best = min((c for c in row if c != nat.HALO_CFG), key=row.get)
        print(f"N={N} {H}x{W} {cin}->{cout}: halo {row[nat.HALO_CFG]:7.1f} us "
              f"({flops / row[nat.HALO_CFG] / 1e6:6.1f} TF/s)  best igemm c{best} {row[best]:7.1f} us "
              f"({flops / row[best] / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
