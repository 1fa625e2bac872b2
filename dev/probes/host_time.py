#!/usr/bin/env python3
"""Host-side cost of one training step: wall time of train_step() calls
(enqueue only; they block only at host syncs) vs the device time per step.
A host time close to the device time means the launch queue runs dry."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402


def main():
    tr = Trainer(TrainConfig(batch=6, iters=12, steps=40, log_every=10 ** 9))
    b = [tr.batch_for(0), tr.batch_for(1)]
    for i in range(4):
        tr.train_step(b[i % 2])
    torch.cuda.synchronize()
    n = 10
    host = []
    t0 = time.perf_counter()
    for i in range(n):
        h0 = time.perf_counter()
        tr.train_step(b[i % 2])
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    dev = (time.perf_counter() - t0) / n
    # pure host cost: the same steps with the GPU far behind is not separable; report the
    # per-call enqueue times and the device step time
    print({"host_ms_per_call": [round(1e3 * h, 2) for h in host], "device_ms_per_step": round(1e3 * dev, 2)})
    import torch.profiler as P
    with P.profile(activities=[P.ProfilerActivity.CPU]) as prof:
        for i in range(3):
            tr.train_step(b[i % 2])
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
