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


def main():
    dev = torch.device("cuda")
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
