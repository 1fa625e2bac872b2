#!/usr/bin/env python3
"""Host enqueue time vs device time per pair of the graph-pipelined batch-1 stream
(bench.py small_b1_fps_12it / b1_fps): perf_counter around each pipelined() call (the
host blocks only at its gate), and the wall time of N pairs with one final sync."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402


def prefetch_mode(eng, iters, n, variant):
    """bench.py's input path: pinned host pair -> InputPrefetcher copy stream -> pipelined()."""
    from jax_raft_amd.runtime.pipeline import InputPrefetcher

    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(2)
    img1 = (torch.rand(1, 440, 1024, 3, generator=g) * 2 - 1).pin_memory()
    img2 = (torch.rand(1, 440, 1024, 3, generator=g) * 2 - 1).pin_memory()
    if variant == "sync_copy":   # the copy on the compute stream, no overlap
        def step(i):
            eng.pipelined(img1.to(dev, non_blocking=True), img2.to(dev, non_blocking=True), iters)
        for i in range(10):
            step(i)
    else:
        depth = 3 if variant == "depth3" else 2
        pf = InputPrefetcher([(1, 440, 1024, 3), (1, 440, 1024, 3)], dev, depth=depth)
        if variant == "prio":
            pf.stream = torch.cuda.Stream(device=dev, priority=-1)

        def step(i):
            a, b = pf.get(i)
            eng.pipelined(a, b, iters)
            pf.release(i)
            pf.put(i + 1, [img1, img2])
        pf.put(0, [img1, img2])
        for i in range(10):
            step(i)
        base = 10
        step_ = step
        step = lambda i: step_(base + i)  # noqa: E731
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    dev = torch.device("cuda")
    model = raft_small(seed=0)[0].to(dev).eval()
    eng = model.engine(dev)
    for variant in ("default", "sync_copy", "depth3", "prio", "default"):
        w = prefetch_mode(eng, 12, 60, variant)
        print(f"raft_small 12 it, pinned-host inputs via {variant}: {1e3 * w:.3f} ms/pair", flush=True)
        eng.flush()
    del eng, model
    torch.cuda.empty_cache()
    for name, fac, iters in (("raft_small", raft_small, 12), ("raft_small", raft_small, 32), ("raft_large", raft_large, 32)):
        model = fac(seed=0)[0].to(dev).eval()
        eng = model.engine(dev)
        g = torch.Generator().manual_seed(1)
        pairs = [(torch.rand(1, 440, 1024, 3, generator=g).to(dev) * 2 - 1,
                  torch.rand(1, 440, 1024, 3, generator=g).to(dev) * 2 - 1) for _ in range(4)]
        for i in range(20):
            eng.pipelined(*pairs[i % 4], iters)
        torch.cuda.synchronize()
        n = 60
        host = []
        t0 = time.perf_counter()
        for i in range(n):
            h0 = time.perf_counter()
            eng.pipelined(*pairs[i % 4], iters)
            host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n
        host.sort()
        print(f"{name} {iters} it: wall {1e3 * wall:.3f} ms/pair, host p50 {1e3 * host[n // 2]:.3f} ms, "
              f"p90 {1e3 * host[int(n * 0.9)]:.3f} ms", flush=True)
        eng.flush()
        del eng, model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
