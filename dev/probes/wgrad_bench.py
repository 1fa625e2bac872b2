#!/usr/bin/env python3
"""Microbenchmark of the implicit-GEMM weight gradient (csrc/kernels/wgrad.hip)
on the training step's shapes: us per call and TF/s, vs im2col + hipBLASLt."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.ops import native as nat  # noqa: E402
from jax_raft_amd.ops.autograd import _wgrad_gemm  # noqa: E402

# name, N, H, W, cin (=cin8), cout, kh, kw, stride, pad
SHAPES = [
    ("loop gru.zr 1x5", 72, 48, 64, 256, 256, 1, 5, 1, (0, 2)),
    ("loop gru.q 1x5", 72, 48, 64, 256, 128, 1, 5, 1, (0, 2)),
    ("loop cc2 3x3", 72, 48, 64, 256, 192, 3, 3, 1, (1, 1)),
    ("loop mc 3x3", 72, 48, 64, 256, 128, 3, 3, 1, (1, 1)),
    ("loop fh1 3x3", 72, 48, 64, 128, 512, 3, 3, 1, (1, 1)),
    ("loop mask 1x1", 72, 48, 64, 256, 576, 1, 1, 1, (0, 0)),
    ("fe l1 3x3", 12, 192, 256, 64, 64, 3, 3, 1, (1, 1)),
    ("fe l2 3x3", 12, 96, 128, 96, 96, 3, 3, 1, (1, 1)),
    ("fe l3 3x3", 12, 48, 64, 128, 128, 3, 3, 1, (1, 1)),
    ("fe stem 7x7", 12, 384, 512, 8, 64, 7, 7, 2, (3, 3)),
]


def timeit(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for name, N, H, W, cin, cout, kh, kw, s, pad in SHAPES:
        OH, OW = (H + 2 * pad[0] - kh) // s + 1, (W + 2 * pad[1] - kw) // s + 1
        x = torch.randn(N, H, W, cin, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, OH, OW, cout, device="cuda").to(torch.bfloat16)
        dw = torch.empty(kh, kw, cin, cout, device="cuda")
        db = torch.empty(cout, device="cuda")
        args = ([x, dy, dw, db], [N, H, W, 0, cin, kh, kw, s, s, pad[0], pad[1], 0, OH, OW, cout, cin])
        t_nat = timeit(lambda: nat.ops().wgrad(*args))
        M = N * OH * OW
        kpad = nat.round_up(kh * kw * cin, 64)
        col = torch.empty(M, kpad, dtype=torch.bfloat16, device="cuda")

        def lib():
            nat.ops().im2col([x, col], [N, H, W, 0, cin, kh, kw, s, s, pad[0], pad[1]])
            _wgrad_gemm(dy.reshape(M, cout), col, cout)
        t_lib = timeit(lib)
        fl = 2.0 * M * kh * kw * cin * cout
        print(f"{name:18s} M={M:7d} K={kh * kw * cin:5d} N={cout:4d}  native {t_nat:8.1f} us {fl / t_nat / 1e6:6.1f} TF/s"
              f"   im2col+hipBLASLt {t_lib:8.1f} us {fl / t_lib / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
