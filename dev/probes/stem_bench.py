#!/usr/bin/env python3
"""Device time of the encoders' space-to-depth stem (4x4 / pad 2 over 16 channels, 64 outputs, output =
input size; ops/native.py:s2d_stem_kernel) at the headline shape (4 images of 440x1024 -> 220x512):
the halo kernel's stem configs against every implicit-GEMM tile config, each as a graph of 30 launches.

    python dev/probes/stem_bench.py [--n 4]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))

from conv_bench import graph_time  # noqa: E402

from jax_raft_amd.ops import native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, h, w = a.n, 220, 512
    k = torch.randn(7, 7, 3, 64, device=dev) / math.sqrt(147)
    spec = nat.make_spec(nat.s2d_stem_kernel(k), torch.zeros(64, device=dev), (1, 1), (2, 2), cin8=16, device=dev)
    x = torch.randn(N, h, w, 16, device=dev).to(torch.bfloat16)
    y = torch.empty(N * h * w, 64, device=dev, dtype=torch.bfloat16)
    flop = 2.0 * N * h * w * 64 * 16 * 16
    res = []
    for c in list(nat.HALO_STEM_CFGS) + list(nat.TUNE_CFGS):
        def launch(c=c):
            nat.ops().conv(*nat.conv_args(spec, x, N, h, w, y, act=nat.ACT_RELU, out_hw=(h, w), cfg=c))
        try:
            t = graph_time(launch)
        except RuntimeError:
            continue
        res.append((t, c))
    res.sort()
    for t, c in res[:12]:
        kind = f"halo {nat.halo_cfg(c)}" if c >= nat.HALO_CFG0 else "igemm"
        print(f"cfg {c:4d} {kind:32s} {t:7.1f} us  {flop / t / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
