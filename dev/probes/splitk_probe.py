#!/usr/bin/env python3
"""Would split-K pay off for the batch-1 loop convs (raft_large, 440x1024 ->
M = 7040)?  Times each conv (best tile config) against the same conv with half
the input channels on twice the pixels -- the work of one launch whose grid.z
holds two K halves -- plus an fp32 partial-sum read/write pass of the output size."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_raft_amd.ops import native as nat  # noqa: E402
from microbench import timeit  # noqa: E402


def best(spec, x, N, H, W, y, **kw):
    r = {}
    for cfg in nat.TUNE_CFGS:
        t, i, a = nat.conv_args(spec, x, N, H, W, y, cfg=cfg, **kw)
        r[cfg] = timeit(lambda: nat.ops().conv(t, i, a), iters=30)
    c = min(r, key=r.get)
    return r[c], c


def main():
    nat.require()
    dev = "cuda"
    h, w = 55, 128
    for name, cin, cout, kh, kw_, pad in (("gru.a 1x5", 256, 256, 1, 5, (0, 2)), ("gru.b 1x5", 256, 128, 1, 5, (0, 2)),
                                         ("convcorr2", 256, 192, 3, 3, (1, 1)), ("me.conv", 256, 126, 3, 3, (1, 1)),
                                         ("fh1+mask", 128, 512, 3, 3, (1, 1))):
        out = []
        for S in (1, 2, 4):
            c = cin // S
            k = torch.randn(kh, kw_, c, cout) / math.sqrt(kh * kw_ * cin)
            spec = nat.make_spec(k, torch.zeros(cout), (1, 1), pad, device=dev)
            x = torch.randn(S, h, w, c, device=dev).to(torch.bfloat16)
            y = torch.empty(S * h * w, nat.round_up(cout, 8), device=dev, dtype=torch.float32 if S > 1 else torch.bfloat16)
            t, cfg = best(spec, x, S, h, w, y)
            red = 0.0
            if S > 1:   # reduce pass: read S fp32 partial maps, write bf16
                part = torch.randn(S, h * w, cout, device=dev)
                red = timeit(lambda: part.sum(0).to(torch.bfloat16), iters=30)
            out.append(f"S={S}: {t:6.1f} us (c{cfg}){' + reduce %.1f' % red if S > 1 else ''}")
        print(f"{name:10s} " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
