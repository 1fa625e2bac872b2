#!/usr/bin/env python3
"""Host-side time of RaftEngine.forward vs the pipelined submit() (per call,
and per graph replay inside submit): shows whether a graph launch blocks the
host (which serialises the prologue graph of batch i+1 behind the loop graph
of batch i)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, _ = raft_large(seed=0)
    model = model.to(dev).eval()
    B, H, W = 4, 440, 1024
    a = torch.rand(B, H, W, 3, device=dev) * 2 - 1
    b = torch.rand(B, H, W, 3, device=dev) * 2 - 1
    eng = model.engine(dev)
    for _ in range(3):
        eng.forward(a, b, 32)
    torch.cuda.synchronize()
    hs = []
    t0 = time.perf_counter()
    for _ in range(6):
        h0 = time.perf_counter()
        eng.forward(a, b, 32)
        hs.append(1e3 * (time.perf_counter() - h0))
    torch.cuda.synchronize()
    print("forward host ms/call", [round(x, 2) for x in hs], "device ms/step", round(1e3 * (time.perf_counter() - t0) / 6, 2))
    for _ in range(3):
        eng.submit(a, b, 32)
    torch.cuda.synchronize()
    # instrument the two graph replays
    import types
    plan_cls_calls = []
    hs = []
    t0 = time.perf_counter()
    for _ in range(6):
        h0 = time.perf_counter()
        eng.submit(a, b, 32)
        hs.append(1e3 * (time.perf_counter() - h0))
    torch.cuda.synchronize()
    print("submit host ms/call", [round(x, 2) for x in hs], "device ms/step", round(1e3 * (time.perf_counter() - t0) / 6, 2))
    st = [v for k, v in eng._states.items() if "slot" in k]
    plan = st[0].plan
    for part in (0, 1):
        torch.cuda.synchronize()
        hs = []
        for _ in range(4):
            h0 = time.perf_counter()
            plan.replay_part(part)
            hs.append(1e3 * (time.perf_counter() - h0))
        torch.cuda.synchronize()
        print(f"replay_part({part}) host ms/call", [round(x, 2) for x in hs])


if __name__ == "__main__":
    main()
