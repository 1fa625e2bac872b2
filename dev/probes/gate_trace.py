#!/usr/bin/env python3
"""Why does a long graph replay enqueued behind a running one run slower (the engine's host
gate, runtime/engine.py:_gate)?  Runs raft_large batch-1 32-iteration forwards back to back with
the gate on or off; run it under ``rocprofv3 --kernel-trace`` in two processes and compare the
traces with dev/probes/trace_compare.py (kernel durations vs idle gaps per forward).

    python dev/probes/gate_trace.py --gate 0|1 [--n 12] [--arch raft_large] [--iters 32]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gate", type=int, default=1)
    ap.add_argument("--n", type=int, default=12)
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    model = (raft_large if a.arch == "raft_large" else raft_small)()[0].cuda().eval()
    dev = torch.device("cuda", 0)
    eng = model.engine(dev)
    eng.host_gate = bool(a.gate)
    g = torch.Generator().manual_seed(0)
    i1 = (torch.rand(a.batch, 440, 1024, 3, generator=g) * 2 - 1).to(dev)
    i2 = (torch.rand(a.batch, 440, 1024, 3, generator=g) * 2 - 1).to(dev)
    for _ in range(3):
        eng.forward(i1, i2, a.iters)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.n + 1)]
    t0 = time.perf_counter()
    ev[0].record()
    host = []
    for k in range(a.n):
        h = time.perf_counter()
        eng.forward(i1, i2, a.iters)
        host.append((time.perf_counter() - h) * 1e3)
        ev[k + 1].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    dev_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(a.n)]
    print(f"gate={a.gate} {a.arch} b{a.batch} {a.iters} it: wall {wall / a.n:.3f} ms/fwd; device per fwd "
          + " ".join(f"{t:.2f}" for t in dev_ms) + "; host enqueue per fwd " + " ".join(f"{t:.2f}" for t in host),
          flush=True)


if __name__ == "__main__":
    main()
