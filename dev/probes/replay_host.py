#!/usr/bin/env python3
"""Host-side duration of a hipGraph replay (raft_large forward, batch 4):
single-lane vs multi-lane plan graphs.  A host time close to the device time
means the launch blocks until the graph has (nearly) finished."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd import raft_large  # noqa: E402


def main():
    model, _ = raft_large(seed=0)
    model = model.cuda().eval()
    x1 = torch.rand(4, 440, 1024, 3, device="cuda") * 2 - 1
    x2 = torch.rand(4, 440, 1024, 3, device="cuda") * 2 - 1
    for streams in (False, True):
        kw = dict(num_flow_updates=32, streams=streams, copy_output=False)
        for _ in range(3):
            model(x1, x2, **kw)
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for _ in range(10):
            h0 = time.perf_counter()
            model(x1, x2, **kw)
            host.append(1e3 * (time.perf_counter() - h0))
        torch.cuda.synchronize()
        dev = 1e3 * (time.perf_counter() - t0) / 10
        print({"streams": streams, "host_ms_per_call": [round(h, 2) for h in host], "device_ms_per_call": round(dev, 2)})


if __name__ == "__main__":
    main()
