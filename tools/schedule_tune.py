#!/usr/bin/env python3
"""Schedule-aware tile-config search for the refinement-loop convs.

The engine's autotuner times every conv alone; inside the lane schedule the
convs run next to the mask lane's kernels, where another tile config can be
faster.  This tool times the WHOLE captured forward (raft_large, 440x1024,
32 iterations, batch 4) while one loop conv's config is swapped
(``RaftEngine(cfg_override=...)``), greedily conv by conv, and prints the
best override table as JSON (use it with ``JR_CFG_OVERRIDE`` / ``cfg_override``).

  python tools/schedule_tune.py [--batch 4] [--reps 12] [--names gru0.b,gru1.b]
"""
import argparse
import gc
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402
from jax_raft_amd.ops import native as nat  # noqa: E402
from jax_raft_amd.runtime.engine import RaftEngine  # noqa: E402

LOOP = ["me.convcorr2", "me.conv", "mask.convrelu", "me.convflow2"]   # (the ConvGRU stages are fused at batch 4)


def time_forward(model, dev, ovr, img1, img2, iters, reps):
    eng = RaftEngine(model, dev, cfg_override=ovr)
    try:
        for _ in range(3):
            eng.forward(img1, img2, iters)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(3):   # best of 3 windows
            s.record()
            for _ in range(reps):
                eng.forward(img1, img2, iters)
            e.record()
            e.synchronize()
            t = s.elapsed_time(e) / reps
            best = t if best is None else min(best, t)
        return best
    except RuntimeError as ex:   # config not valid for this conv / epilogue
        print(f"  {ovr}: {str(ex).splitlines()[0][:100]}", flush=True)
        return None
    finally:
        del eng
        gc.collect()
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--names", default=",".join(LOOP))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, _ = raft_large(seed=0)
    model = model.to(dev).eval()
    g = torch.Generator().manual_seed(0)
    img1 = (torch.rand(a.batch, 440, 1024, 3, generator=g) * 2 - 1).to(dev)
    img2 = (torch.rand(a.batch, 440, 1024, 3, generator=g) * 2 - 1).to(dev)
    ovr = {}
    base = time_forward(model, dev, ovr, img1, img2, a.iters, a.reps)
    print(f"baseline {base:.3f} ms/forward", flush=True)
    cands = [c for c in nat.TUNE_CFGS if nat.CFG_TILES[c][0] >= 64]
    for name in a.names.split(","):
        best_c, best_t = None, base
        for c in cands:
            t = time_forward(model, dev, dict(ovr, **{name: c}), img1, img2, a.iters, a.reps)
            if t is not None:
                print(f"  {name} cfg {c}: {t:.3f} ms", flush=True)
                if t < best_t * 0.995:
                    best_c, best_t = c, t
        if best_c is not None:
            ovr[name] = best_c
            base = best_t
        print(f"{name}: {'cfg %d' % best_c if best_c is not None else 'autotuned kept'} -> {base:.3f} ms", flush=True)
    print(json.dumps({"override": ovr, "ms_per_forward": round(base, 3)}), flush=True)


if __name__ == "__main__":
    main()
