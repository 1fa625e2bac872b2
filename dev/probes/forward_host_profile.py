#!/usr/bin/env python3
"""Where the host time of one RaftEngine.forward goes (cProfile over steady-
state calls; the GPU is kept busy so nothing blocks on it)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, _ = raft_large(seed=0)
    model = model.to(dev).eval()
    a = torch.rand(4, 440, 1024, 3, device=dev) * 2 - 1
    b = torch.rand(4, 440, 1024, 3, device=dev) * 2 - 1
    eng = model.engine(dev)
    for _ in range(3):
        eng.forward(a, b, 32)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(4):
        out = eng.forward(a, b, 32)
        del out
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main()
