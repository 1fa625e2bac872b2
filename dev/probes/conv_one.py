#!/usr/bin/env python3
"""Run ONE loop conv of the headline shapes under ONE tile config, N times
(for rocprofv3 --pmc passes: one kernel, many identical dispatches).

  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES ... -- python3 tools/conv_one.py gru.a 22
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_raft_amd.ops import native as nat  # noqa: E402

SHAPES = {  # name: cin, cin8, cout, kh, kw, pad, bmap
    "convcorr1": (324, 328, 256, 1, 1, (0, 0), False),
    "convcorr2": (256, 256, 192, 3, 3, (1, 1), False),
    "me.conv": (256, 256, 126, 3, 3, (1, 1), False),
    "gru.a": (256, 256, 256, 1, 5, (0, 2), True),
    "gru.b": (256, 256, 128, 1, 5, (0, 2), True),
    "fh1": (128, 128, 512, 3, 3, (1, 1), False),
    "mask2": (256, 256, 576, 1, 1, (0, 0), False),
}
# encoder convs (feature encoder half at batch 4): name -> (cin, cin8, cout, kh, kw, pad, bmap, stride, H, W)
ENC = {
    "stem": (3, 8, 64, 7, 7, (3, 3), False, 2, 440, 1024),
    "l1": (64, 64, 64, 3, 3, (1, 1), False, 1, 220, 512),
    "l2s2": (64, 64, 96, 3, 3, (1, 1), False, 2, 220, 512),
    "l2": (96, 96, 96, 3, 3, (1, 1), False, 1, 110, 256),
    "l3s2": (96, 96, 128, 3, 3, (1, 1), False, 2, 110, 256),
    "l3": (128, 128, 128, 3, 3, (1, 1), False, 1, 55, 128),
}


def main():
    name, cfg = sys.argv[1], int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    B, h, w, st = 4, 55, 128, 1
    if name in ENC:
        cin, cs, cout, kh, kw, pad, use_bm, st, h, w = ENC[name]
    else:
        cin, cs, cout, kh, kw, pad, use_bm = SHAPES[name]
    nat.require()
    torch.manual_seed(0)
    k = torch.randn(kh, kw, cin, cout) / math.sqrt(kh * kw * cin)
    spec = nat.make_spec(k, torch.randn(cout) * 0.1, (st, st), pad, cin8=cs, device="cuda")
    x = torch.randn(B, h, w, cs, device="cuda").to(torch.bfloat16)
    OH, OW = spec.out_hw(h, w)
    M = B * OH * OW
    y = torch.empty(M, nat.round_up(cout, 8), device="cuda", dtype=torch.bfloat16)
    bm = torch.randn(M, 384, device="cuda") if use_bm else None
    t, i, a = nat.conv_args(spec, x, B, h, w, y, act=nat.ACT_RELU, cfg=cfg, bmap=bm)
    for _ in range(n):
        nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        nat.ops().conv(t, i, a)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / n * 1e3
    print(f"{name} cfg {cfg}: {us:.1f} us  {2.0 * M * cout * kh * kw * cin / us / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
