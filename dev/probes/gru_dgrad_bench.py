#!/usr/bin/env python3
"""The training ConvGRU data-gradient GEMMs (config 5: 6 x 48 x 64 pixels, 1x5 taps, 256 output
channels = [h | motion | flow]) with the plain epilogue, per tile config: how much of the in-situ
EPI_BWD time (profiles/r6_train_breakdown.txt: 42-44 us per launch, config 34) is the K loop."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))

import torch  # noqa: E402

from conv_bench import graph_time  # noqa: E402
from jax_raft_amd.ops import native as nat  # noqa: E402

N, H, W = 6, 48, 64


def main():
    dev = torch.device("cuda")
    ops = nat.ops()
    for name, cin, ks, pad in (("zr-dgrad 1x5", 256, (1, 5), (0, 2)), ("q-dgrad 1x5", 128, (1, 5), (0, 2)),
                               ("zr-dgrad 5x1", 256, (5, 1), (2, 0))):
        k = torch.randn(ks[0], ks[1], cin, 256, device=dev) * 0.05
        spec = nat.make_spec(k, torch.zeros(256, device=dev), (1, 1), pad)
        x = torch.randn(N, H, W, cin, device=dev).to(torch.bfloat16)
        y = torch.empty(N * H * W, 256, device=dev, dtype=torch.bfloat16)
        flop = 2 * N * H * W * 256 * cin * ks[0] * ks[1]
        for cfg in (34, 22, 21, 20, 33, 25, 0, 18):
            t, i, a = nat.conv_args(spec, x, N, H, W, y, cfg=cfg)
            us = graph_time(lambda: ops.conv(t, i, a))
            print(f"{name} cfg {cfg:3d}: {us:6.1f} us  {flop / us / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
