#!/usr/bin/env python3
"""Which Python lines launch the small framework kernels (fills / copies / elementwise) of one
fused training step (BASELINE config 5)?  torch.profiler with stacks, aggregated by kernel name
and the innermost jax_raft_amd / torch frame."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402


def main():
    cfg = TrainConfig(steps=8, batch=6, iters=12, size=(384, 512), log_every=10 ** 9)
    tr = Trainer(cfg)
    b = tr.batch_for(0)
    for _ in range(3):
        tr.train_step(b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True,
                 experimental_config=torch._C._profiler._ExperimentalConfig(verbose=True)) as prof:
        tr.train_step(b)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=40,
                                                       max_src_column_width=90))
    agg = collections.Counter()
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.stack:
            continue
        name = ev.name
        if not any(k in name for k in ("fill", "copy", "zero", "empty", "clone", "to", "cat", "mul", "add", "norm", "sum", "where")):
            continue
        frame = next((f for f in ev.stack if "jax_raft_amd" in f or "trainer" in f), ev.stack[0])
        agg[(name, frame)] += 1
    for (name, frame), n in agg.most_common(40):
        print(f"{n:4d}  {name:40s}  {frame}")


if __name__ == "__main__":
    main()
