#!/usr/bin/env python3
"""Optical flow over a frame sequence with graph-pipelined engine steps
(``RaftEngine.pipelined``): each call replays one hipGraph that holds the
previous pair's refinement loop and this pair's encoders + correlation
pyramid, and returns the previous pair's flow; ``flush()`` drains the last.

  python examples/video_flow.py frame_0000.png frame_0001.png ... [--arch raft_small] [--iters 12]

Without frames a synthetic drifting sequence is used.  Needs an MI355X (the
native engine); prints the pairs/s of the steady-state pipeline.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.utils.flow_io import InputPadder, normalize_image, read_image  # noqa: E402


def frames(paths, n_synth=16):
    if paths:
        for p in paths:
            yield normalize_image(read_image(p))
        return
    rng = np.random.default_rng(0)
    base = rng.integers(0, 255, (440 + 8 * n_synth, 1024 + 8 * n_synth, 3), dtype=np.uint8)
    for k in range(n_synth):
        yield normalize_image(base[3 * k:3 * k + 436, 2 * k:2 * k + 1024])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("frames", nargs="*")
    ap.add_argument("--arch", default="raft_large", choices=["raft_large", "raft_small"])
    ap.add_argument("--weights", default=None, help="Flax msgpack checkpoint (else random init)")
    ap.add_argument("--iters", type=int, default=32)
    args = ap.parse_args()
    assert torch.cuda.is_available(), "the pipelined engine runs on the GPU"
    factory = raft_large if args.arch == "raft_large" else raft_small
    model, _ = factory(weights=args.weights) if args.weights else factory()
    dev = torch.device("cuda", 0)
    model = model.to(dev).eval()
    eng = model.engine(dev)

    flows, prev, padder = [], None, None
    t0, n_pairs = None, 0
    for img in frames(args.frames):
        if padder is None:
            padder = InputPadder(img.shape, channels_last=True)
        (cur,) = padder.pad(img)
        cur = cur.to(dev)
        if prev is not None:
            out = eng.pipelined(prev, cur, args.iters, return_all_iters=False)   # the previous pair's flow
            if out is not None:
                flows.append(padder.unpad(out[-1]))
                if t0 is None:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                else:
                    n_pairs += 1
        prev = cur
    last = eng.flush()
    if last is not None:
        flows.append(padder.unpad(last[-1]))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0 if t0 is not None else 0.0
    print(f"{len(flows)} flow fields {tuple(flows[0].shape) if flows else ()}; "
          f"steady state {n_pairs / dt if dt > 0 and n_pairs else float('nan'):.1f} pairs/s")


if __name__ == "__main__":
    main()
