#!/usr/bin/env python3
"""Where do the raft_small 12-iteration stream's p99 steps come from (bench.py extra
``small_b1_fps_12it``: p50 1.23 ms, p99 4.5 ms)?  Runs the same graph-pipelined batch-1 stream,
records every step's device time and the host time of every Python garbage collection
(gc.callbacks), and prints the slow steps next to the collections that overlapped them; then the
same stream with the collector disabled; then with the inputs copied from pinned host memory
each step (bench.py's protocol: runtime/pipeline.py:InputPrefetcher on a copy stream, or a
non-blocking copy on the compute stream).

    python dev/probes/p99_probe.py [--steps 200] [--iters 12]
"""
import argparse
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_small  # noqa: E402


def run(eng, frames, iters, steps, dev, h2d=None):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    host = [0.0] * steps
    gcs = []
    t_gc = {}

    def cb(phase, info):
        if phase == "start":
            t_gc["t"] = time.perf_counter()
        else:
            gcs.append((len([h for h in host if h > 0]), info["generation"], (time.perf_counter() - t_gc["t"]) * 1e3))

    gc.callbacks.append(cb)
    pf = None
    if h2d == "prefetch":
        from jax_raft_amd.runtime.pipeline import InputPrefetcher

        pf = InputPrefetcher([tuple(frames[0][0].shape)] * 2, dev)
        pf.put(0, list(frames[0]))
    ev[0].record()
    for k in range(steps):
        t = time.perf_counter()
        if pf is not None:
            x, y = pf.get(k)
        elif h2d == "stream":
            x, y = (v.to(dev, non_blocking=True) for v in frames[k % len(frames)])
        else:
            x, y = frames[k % len(frames)]
        eng.pipelined(x, y, iters)
        if pf is not None:
            pf.release(k)
            if k + 1 < steps:
                pf.put(k + 1, list(frames[(k + 1) % len(frames)]))
        host[k] = (time.perf_counter() - t) * 1e3
        ev[k + 1].record()
    eng.flush()
    torch.cuda.synchronize(dev)
    gc.callbacks.remove(cb)
    dev_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(steps)]
    return dev_ms, host, gcs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--iters", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = raft_small()[0].to(dev).eval()
    eng = model.engine(dev)
    g = torch.Generator().manual_seed(0)
    frames = [tuple((torch.rand(1, 440, 1024, 3, generator=g) * 2 - 1).to(dev) for _ in range(2)) for _ in range(4)]
    for _ in range(20):
        eng.pipelined(*frames[0], a.iters)
    eng.flush()
    torch.cuda.synchronize(dev)
    pinned = [tuple(v.cpu().pin_memory() for v in f) for f in frames]
    for mode in ("gc on", "gc off", "h2d prefetch", "h2d same stream"):
        if mode == "gc off":
            gc.collect()
            gc.disable()
        if mode == "h2d prefetch":
            gc.enable()
        h2d = {"h2d prefetch": "prefetch", "h2d same stream": "stream"}.get(mode)
        dev_ms, host, gcs = run(eng, pinned if h2d else frames, a.iters, a.steps, dev, h2d)
        srt = sorted(dev_ms)
        p50, p99 = srt[len(srt) // 2], srt[int(0.99 * len(srt))]
        slow = [k for k, t in enumerate(dev_ms) if t > 2 * p50]
        print(f"{mode}: p50 {p50:.3f} ms  p99 {p99:.3f} ms  mean {sum(dev_ms) / len(dev_ms):.3f} ms; "
              f"{len(slow)} steps > 2 x p50: {[(k, round(dev_ms[k], 2), round(host[k], 2)) for k in slow]}")
        print(f"   collections (step, generation, host ms): {[(s, gg, round(t, 2)) for s, gg, t in gcs]}")
        print(f"   host enqueue p50 {sorted(host)[len(host) // 2]:.3f} ms, max {max(host):.3f} ms", flush=True)
    gc.enable()


if __name__ == "__main__":
    main()
