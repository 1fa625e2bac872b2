#!/usr/bin/env python3
"""N synchronous batch-1 forwards of raft_large / raft_small at 440x1024 (the reference's
per-pair protocol without the timing): a short program to run under rocprofv3 for kernel
durations of the non-pipelined (RaftEngine.forward) plans.

    python dev/probes/b1_forward.py [--arch raft_large] [--n 5] [ATTR=VALUE ...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.runtime.engine import RaftEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("attrs", nargs="*")
    a = ap.parse_args()
    for item in a.attrs:
        k, v = item.split("=")
        old = getattr(RaftEngine, k)
        setattr(RaftEngine, k, (v not in ("0", "false", "False")) if isinstance(old, bool) else type(old)(v))
    m = (raft_large if a.arch == "raft_large" else raft_small)(seed=0)[0].cuda().eval()
    g = torch.Generator().manual_seed(0)
    i1 = (torch.rand(1, 440, 1024, 3, generator=g) * 2 - 1).cuda()
    i2 = (torch.rand(1, 440, 1024, 3, generator=g) * 2 - 1).cuda()
    for _ in range(a.n):
        m(i1, i2, num_flow_updates=a.iters)
        torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
