#!/usr/bin/env python3
"""Regenerate the persisted conv tile-config table (jax_raft_amd/runtime/tunedb.py)
on the target GPU: build the inference plans of every benchmarked
configuration and the training plans of BASELINE config 5 with fresh timing
(``JR_TUNE=fresh``), then write the merged table.

    JR_TUNE=fresh python tools/autotune_db.py --out gpurun_out/gfx950.json
    cp gpurun_out/gfx950.json jax_raft_amd/tuned/gfx950.json
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# (arch, batch, H, W, iters, all_iters): bench.py headline + extras, Sintel eval shapes
INFER = [("raft_large", b, 440, 1024, 32, True) for b in (1, 2, 4, 8)] + [
    ("raft_large", 4, 440, 1024, 32, False), ("raft_large", 1, 440, 1024, 32, False),
    ("raft_small", 1, 440, 1024, 32, True), ("raft_small", 4, 440, 1024, 32, True),
    ("raft_small", 1, 440, 1024, 12, True)]
TRAIN = [("raft_large", 6, 384, 512, 12), ("raft_small", 6, 384, 512, 12)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--no-train", action="store_true")
    a = ap.parse_args()
    if os.environ.get("JR_TUNE") != "fresh":
        print("note: JR_TUNE is not 'fresh': entries already in the table are kept, not re-timed", flush=True)
    from jax_raft_amd import raft_large, raft_small
    from jax_raft_amd.runtime import tunedb
    from jax_raft_amd.runtime.engine import RaftEngine

    dev = torch.device("cuda", 0)
    arch = tunedb.gpu_arch(dev)
    models = {n: f(seed=0)[0].to(dev).eval() for n, f in (("raft_large", raft_large), ("raft_small", raft_small))}
    for name, B, H, W, it, all_it in INFER:
        t = time.time()
        eng = RaftEngine(models[name], dev)
        x = torch.zeros(B, H, W, 3, device=dev)
        eng.forward(x, x, it, return_all_iters=all_it)
        torch.cuda.synchronize()
        print(f"infer {name} B={B} {H}x{W} it={it} all={all_it}: {time.time() - t:.1f} s", flush=True)
        del eng
    if not a.no_train:
        from jax_raft_amd.train.loss import sequence_loss

        for name, B, H, W, it in TRAIN:
            t = time.time()
            m = (raft_large if name == "raft_large" else raft_small)(seed=0)[0].to(dev).train()
            x = torch.zeros(B, H, W, 3, device=dev)
            gt = torch.zeros(B, H, W, 2, device=dev)
            preds = m(x, x, train=True, num_flow_updates=it, autograd=True)
            loss, _ = sequence_loss(preds, gt)
            loss.backward()
            torch.cuda.synchronize()
            print(f"train {name} B={B} {H}x{W} it={it}: {time.time() - t:.1f} s", flush=True)
            del m, preds, loss
            torch.cuda.empty_cache()
    tunedb.save(arch, a.out)   # only --out: the packaged table changes by an explicit cp
    print(f"{len(tunedb._table(arch))} entries -> {a.out}; {tunedb.stats()}", flush=True)


if __name__ == "__main__":
    main()
