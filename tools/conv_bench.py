#!/usr/bin/env python3
"""Device time of one RAFT 3x3 conv problem per tile config: the halo kernel configs
(conv_halo.hip, cfg >= 100) and the implicit-GEMM autotune set, each as a captured graph of
--reps launches.  ``--cfg C --run N`` instead launches one config N times (for rocprofv3
--pmc passes).

  python tools/conv_bench.py l1 cc2b4 meb1      # problems below
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name: (N, H, W, cin, cout)  -- encoder layers at batch 4 (4 images), loop convs at batch 4 / 1
PROBLEMS = {
    "l1": (4, 220, 512, 64, 64), "l2": (4, 110, 256, 96, 96), "l3": (4, 55, 128, 128, 128),
    "cc2b4": (4, 55, 128, 256, 192), "cc2b1": (1, 55, 128, 256, 192),
    "meb4": (4, 55, 128, 256, 126), "meb1": (1, 55, 128, 256, 126),
    "fhb4": (4, 55, 128, 128, 256), "fh512b1": (1, 55, 128, 128, 512),
    "cf2b4": (4, 55, 128, 128, 64), "cf2b1": (1, 55, 128, 128, 64),
}


def graph_time(fn, reps=30, rounds=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        t = s.elapsed_time(e) * 1000.0 / reps
        best = t if best is None else min(best, t)
    return best


def setup(name):
    from jax_raft_amd.ops import native as nat

    N, H, W, cin, cout = PROBLEMS[name]
    dev = torch.device("cuda", 0)
    x = torch.randn(N, H, W, cin, device=dev).to(torch.bfloat16)
    k = torch.randn(3, 3, cin, cout, device=dev) / math.sqrt(9 * cin)
    spec = nat.make_spec(k, torch.zeros(cout, device=dev), (1, 1), (1, 1), device=dev)
    y = torch.empty(N * H * W, nat.round_up(cout, 8), device=dev, dtype=torch.bfloat16)
    flop = 2.0 * N * H * W * cout * 9 * cin
    return nat, spec, x, y, (N, H, W), flop


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("problems", nargs="+")
    ap.add_argument("--cfg", type=int, default=None)
    ap.add_argument("--run", type=int, default=0)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--fused", default="", help="halo configs only: comma list of stats (output statistics "
                    "partials), inn (input instance norm on load), res (+ normalised residual), xn (write-back)")
    a = ap.parse_args()
    fz = set(filter(None, a.fused.split(",")))
    for name in a.problems:
        nat, spec, x, y, (N, H, W), flop = setup(name)

        cin, cout = PROBLEMS[name][3], PROBLEMS[name][4]
        dev = x.device
        kw = {}
        if fz:   # encoder-style fused norms (train/fused_encoder.py, runtime/engine.py:_encoder)
            if "stats" in fz:
                kw["stats_part"] = torch.zeros(N * (H + 8) * (W + 16) // 4 * cout * 2, device=dev)
            if "inn" in fz:
                st = torch.stack([torch.zeros(N, cin, device=dev), torch.full((N, cin), float(H * W), device=dev)], -1)
                kw.update(in_stats=st.contiguous(), in_relu=1, in_hw=H * W)
                if "res" in fz:
                    kw.update(in_res=torch.randn_like(x), in_res_stats=st.contiguous(), in_relu=3)
                if "xn" in fz:
                    kw["xn"] = torch.empty_like(x)

        def launch(cfg):
            nat.ops().conv(*nat.conv_args(spec, x, N, H, W, y, act=nat.ACT_NONE if fz else nat.ACT_RELU, cfg=cfg, **kw))

        if a.run:
            for _ in range(a.run):
                launch(a.cfg)
            torch.cuda.synchronize()
            continue
        cfgs = [a.cfg] if a.cfg is not None else list(nat.halo_cfgs_for(spec, {})) + ([] if fz else list(nat.TUNE_CFGS))
        res = []
        for c in cfgs:
            try:
                t = graph_time(lambda: launch(c), a.reps)
            except RuntimeError:
                continue
            res.append((t, c))
        res.sort()
        best_igemm = next(((t, c) for t, c in res if c < nat.HALO_CFG0), None)
        if best_igemm is None:
            print(f"{name} {PROBLEMS[name]} fused {sorted(fz)}:")
        else:
            print(f"{name} {PROBLEMS[name]}: best igemm cfg {best_igemm[1]} {best_igemm[0]:.1f} us "
                  f"({flop / best_igemm[0] / 1e6:.0f} TF/s)")
        for t, c in res:
            if c >= nat.HALO_CFG0:
                print(f"   halo {c} {nat.halo_cfg(c)}: {t:7.1f} us  {flop / t / 1e6:6.0f} TF/s")


if __name__ == "__main__":
    main()
