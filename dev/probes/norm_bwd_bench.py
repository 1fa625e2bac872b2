#!/usr/bin/env python3
"""Standalone timing of the encoder normalisation backward (train.hip:jr_norm_bwd) on the
config-5 training shapes (feature encoder: 12 maps of 384x512 / 2^k), with the achieved
bandwidth of the whole op under a byte model (gout, y [, om] read twice; dy [, gres] written)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd.ops import native as nat  # noqa: E402

BF16, F32 = torch.bfloat16, torch.float32
CASES = [  # (N, HW, C, om, gres dtype or None, mode)
    (12, 192 * 256, 64, False, None, 1),
    (12, 192 * 256, 64, True, BF16, 1),
    (12, 96 * 128, 96, True, None, 1),
    (12, 96 * 128, 96, True, F32, 1),
    (12, 48 * 64, 128, True, BF16, 1),
    (6, 192 * 256, 64, True, BF16, 2),
]


def main():
    dev = torch.device("cuda")
    ops = nat.ops()
    torch.manual_seed(0)
    for N, HW, C, has_om, gdt, mode in CASES:
        sh = (N, HW, C)
        g = torch.randn(sh, device=dev).to(BF16)
        y = torch.randn(sh, device=dev).to(BF16)
        om = torch.randn(sh, device=dev).to(BF16) if has_om else None
        st = torch.stack([y.float().sum(1), (y.float() ** 2).sum(1)], -1).contiguous()
        gam = torch.rand(C, device=dev) + 0.5
        bet = torch.randn(C, device=dev) * 0.1
        red = torch.zeros(N, C, 2, device=dev)
        dy = torch.empty_like(g)
        gres = torch.empty(sh, dtype=gdt, device=dev) if gdt is not None else None
        t = [g, om, y, st, gam, bet, red, None, dy, gres]
        i = [mode, 1, N, HW, C]
        for _ in range(3):
            ops.norm_bwd(t, i, 1e-5)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 20
        for _ in range(reps):
            ops.norm_bwd(t, i, 1e-5)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        el = N * HW * C
        rd = el * 2 * (2 + (1 if has_om else 0))
        by = 2 * rd + el * 2 + (el * gres.element_size() if gres is not None else 0)
        print(f"N={N} HW={HW} C={C} om={int(has_om)} gres={gdt} mode={mode}: {us:7.1f} us  "
              f"{by / 1e6:7.1f} MB  {by / us / 1e6:5.2f} TB/s", flush=True)


ACT_CASES = [  # (N, HW, C, residual, mode): the encoders' norm -> relu [+ residual] units
    (12, 192 * 256, 64, False, 1),
    (12, 96 * 128, 96, True, 1),
    (6, 192 * 256, 64, False, 2),
    (6, 48 * 64, 128, True, 2),
    (2, 55 * 128, 128, False, 1),   # raft_small batch-1 Sintel shapes (2 frames)
    (2, 110 * 256, 32, True, 1),
]


def act_main():
    dev = torch.device("cuda")
    ops = nat.ops()
    for N, HW, C, res, mode in ACT_CASES:
        sh = (N, HW, C)
        x = torch.randn(sh, device=dev).to(BF16)
        st = torch.stack([x.float().sum(1), (x.float() ** 2).sum(1)], -1).contiguous()
        gam = torch.rand(C, device=dev) + 0.5
        bet = torch.randn(C, device=dev) * 0.1
        r = torch.randn(sh, device=dev).to(BF16) if res else None
        y = torch.empty_like(x)
        t = [x, st, gam, bet, r, st if res else None, None, None, y]
        i = [mode, mode if res else 0, N, HW, C, 3 if res else 1]
        for _ in range(3):
            ops.norm_act(t, i, 1e-5)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 20
        for _ in range(reps):
            ops.norm_act(t, i, 1e-5)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        by = N * HW * C * 2 * (3 if res else 2)
        print(f"norm_act N={N} HW={HW} C={C} res={int(res)} mode={mode}: {us:7.1f} us  {by / 1e6:7.1f} MB  "
              f"{by / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
    act_main()
