#!/usr/bin/env python3
"""Numerical drift of the native engine against the fp32 golden forward at the
headline configuration (440x1024, 32 refinement iterations, batch 1) -- the
reference's benchmark setting (``jax_raft/model.py:589-605``,
``scripts/validate_sintel.py:164-203``: 32 iterations on Sintel frames padded
to 440x1024, fp32 end to end).

Without the pretrained checkpoints and Sintel (no network), EPE against ground
truth is not measurable; what the bf16 kernels must show instead is how far 32
recurrent iterations drift from the fp32 golden model (models/reference.py) on
the same weights (``seed=0`` init) and the same input pair (a translated
synthetic pair, as tests/test_engine_gpu.py uses).

    python tools/drift.py golden            # CPU: write the fixtures (final flows, fp32)
    python tools/drift.py measure [--json F] # GPU: per-iteration EPE vs golden for
                                             # both archs x pyramid dtypes

The golden is recomputed on the CPU in the measuring process (about 5 s for
raft_large on 8 cores) so every iteration can be compared; its final flow is
checked against the committed fixture first.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIXDIR = os.path.join(ROOT, "tests", "fixtures")
H, W, ITERS = 440, 1024, 32


def fixture_path(arch: str) -> str:
    return os.path.join(FIXDIR, f"golden_{arch}_440x1024_32it.npz")


def inputs(B: int = 1, H_: int = H, W_: int = W, seed: int = 0):
    """A translated synthetic pair: image2 is image1 shifted by (+2, -2) px
    (tests/test_engine_gpu.py:_inputs at the headline size)."""
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(B, H_ + 8, W_ + 8, 3, generator=g) * 2 - 1
    return base[:, 4:4 + H_, 4:4 + W_].contiguous(), base[:, 2:2 + H_, 6:6 + W_].contiguous()


def model_for(arch: str):
    from jax_raft_amd import raft_large, raft_small

    return (raft_large if arch == "raft_large" else raft_small)(seed=0)[0].eval()


@torch.no_grad()
def golden(arch: str, iters: int = ITERS) -> torch.Tensor:
    """fp32 CPU golden flows (iters, 1, H, W, 2)."""
    m = model_for(arch)
    i1, i2 = inputs()
    return m(i1, i2, num_flow_updates=iters)


def epe(a: torch.Tensor, b: torch.Tensor) -> float:
    return (a.double() - b.double()).norm(dim=-1).mean().item()


def write_fixtures() -> None:
    os.makedirs(FIXDIR, exist_ok=True)
    for arch in ("raft_large", "raft_small"):
        t = time.time()
        g = golden(arch)
        mags = g.norm(dim=-1).mean(dim=(1, 2, 3)).tolist()
        np.savez_compressed(fixture_path(arch), final=g[-1, 0].numpy().astype(np.float32),
                            mean_mag=np.asarray(mags, dtype=np.float64))
        print(f"{arch}: golden in {time.time() - t:.1f} s, |flow| it1 {mags[0]:.3f} it32 {mags[-1]:.3f} "
              f"-> {fixture_path(arch)}", flush=True)


def load_fixture(arch: str):
    with np.load(fixture_path(arch), allow_pickle=False) as z:
        return torch.from_numpy(z["final"]), z["mean_mag"].tolist()


@torch.no_grad()
def measure(out_json: str | None, archs, variants) -> list:
    from jax_raft_amd.runtime.engine import RaftEngine

    dev = torch.device("cuda", 0)
    recs = []
    for arch in archs:
        t = time.time()
        g = golden(arch)
        fx, _ = load_fixture(arch)
        fix_err = (g[-1, 0] - fx).abs().max().item()
        mag = g.norm(dim=-1).mean(dim=(1, 2, 3))
        print(f"{arch}: CPU golden {time.time() - t:.1f} s, max |golden - fixture| = {fix_err:.2e}", flush=True)
        m = model_for(arch).to(dev)
        i1, i2 = inputs()
        for name, kw in variants:
            eng = RaftEngine(m, dev, **kw)
            out = eng.forward(i1.to(dev), i2.to(dev), ITERS).cpu()
            curve = [epe(out[i], g[i]) for i in range(ITERS)]
            rel = [c / max(mag[i].item(), 1e-6) for i, c in enumerate(curve)]
            rec = dict(arch=arch, variant=name, epe=curve, rel=rel, mean_mag=mag.tolist(),
                       fixture_max_abs=fix_err, final_epe_vs_fixture=epe(out[-1, 0], fx))
            recs.append(rec)
            print(f"  {name:24s} EPE it1 {curve[0]:.4f} it8 {curve[7]:.4f} it16 {curve[15]:.4f} it32 {curve[-1]:.4f} "
                  f"(rel {rel[-1]:.2e}, |flow| {mag[-1]:.2f})", flush=True)
            del eng
        del m
        torch.cuda.empty_cache()
    if out_json:
        os.makedirs(os.path.dirname(os.path.abspath(out_json)), exist_ok=True)
        with open(out_json, "w") as f:
            json.dump(recs, f)
    return recs


VARIANTS = {
    "bf16": dict(),                                  # default: bf16 pyramid, bf16 z gate / context bias map
    "corr_fp32": dict(corr_dtype=torch.float32),     # fp32 pyramid
    "corr_gate_fp32": dict(corr_dtype=torch.float32, gate_dtype=torch.float32),
    "fp32": dict(precision="fp32"),                  # fp32 engine (runtime/engine_f32.py)
    "mixed": dict(precision="mixed"),                # fp32 feature encoder, bf16 rest (RaftEngineMixed)
    "mixed_corr_fp32": dict(precision="mixed", corr_dtype=torch.float32),   # + fp32 pyramid
    "mixed_corr_gate_fp32": dict(precision="mixed", corr_dtype=torch.float32, gate_dtype=torch.float32),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["golden", "measure"])
    ap.add_argument("--json", default=None)
    ap.add_argument("--arch", nargs="*", default=["raft_large", "raft_small"])
    ap.add_argument("--variants", nargs="*", default=list(VARIANTS))
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    if a.mode == "golden":
        write_fixtures()
    else:
        measure(a.json, a.arch, [(v, VARIANTS[v]) for v in a.variants])


if __name__ == "__main__":
    main()
