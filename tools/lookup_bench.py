#!/usr/bin/env python3
"""The correlation lookup at the headline shapes (raft_large, 55 x 128 feature
maps, blocked bf16 pyramid): the wide lookup kernel + the LDS-weight 1x1 conv
(MotionEncoder.convcorr1) as two kernels vs the fused lookup_cc1 kernel, with
and without the fused flow update, at batch 1 and 4 (hip events, us)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_raft_amd.models import reference as R  # noqa: E402
from jax_raft_amd.ops import native as nat  # noqa: E402
from microbench import timeit  # noqa: E402


def main():
    nat.require()
    dev = "cuda"
    h, w, C, L, r = 55, 128, 256, 4, 4
    S = 2 * r + 1
    K = L * S * S
    for B in (1, 4):
        M = B * h * w
        f = torch.randn(2 * B, h, w, C, device=dev).to(torch.bfloat16)
        nty, ntx = -(-h // 8), -(-w // 16)
        lv, hl, wl = [], h, w
        for l in range(L):
            shape = (M, nty * (8 >> l), ntx * (16 >> l)) if l < 2 else (M, hl, wl)
            lv.append(torch.zeros(shape, device=dev, dtype=torch.bfloat16))
            hl //= 2
            wl //= 2
        nat.ops().corr([f[:B], f[B:]] + lv, [B, h, w, C, L, h * w, 1], 1.0 / math.sqrt(C))
        coords = (R.make_coords_grid(B, h, w).reshape(M, 2) + torch.randn(M, 2) * 4).to(dev)
        corr = torch.zeros(M, 328, device=dev, dtype=torch.bfloat16)
        kern = torch.randn(1, 1, K, 256, device=dev) / math.sqrt(K)
        bias = torch.zeros(256, device=dev)
        w352 = nat.pack_conv1x1(kern, 352)
        y = torch.zeros(M, 256, device=dev, dtype=torch.bfloat16)
        t_lk = timeit(lambda: nat.ops().lookup([coords, corr] + lv, [L, B, h, w, r, h * w, 1]))
        t_c1 = timeit(lambda: nat.ops().conv1x1([corr, w352, bias, y], [M, 328, 352, 256, nat.ACT_RELU, 0]))
        t_f = timeit(lambda: nat.ops().lookup_cc1([coords, y] + lv + [w352, bias], [L, B, h, w, r, 1, 352, 256, 0]))
        print(f"B={B}: lookup {t_lk:6.1f} + conv1x1 {t_c1:6.1f} = {t_lk + t_c1:6.1f} us | fused lookup_cc1 {t_f:6.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
