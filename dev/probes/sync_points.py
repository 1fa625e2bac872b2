#!/usr/bin/env python3
"""Host-device synchronisation points of a training step: runs Trainer steps
with torch.cuda.set_sync_debug_mode("warn") and prints the Python stack of
every synchronising call (each one drains the launch queue: the GPU idles
while the host enqueues what follows)."""
import collections
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402


def main():
    tr = Trainer(TrainConfig(batch=6, iters=12, steps=40, log_every=10 ** 9))
    for i in range(4):
        tr.train_step(tr.batch_for(i))
    torch.cuda.synchronize()
    seen = collections.Counter()
    stacks = {}

    def show(message, category, filename, lineno, file=None, line=None):
        st = "".join(traceback.format_stack()[-9:-1])
        key = str(message)[:80] + " @ " + st.strip().splitlines()[-2] if st else str(message)
        seen[key] += 1
        stacks[key] = st

    warnings.showwarning = show
    torch.cuda.set_sync_debug_mode("warn")
    for i in range(2):
        tr.train_step(tr.batch_for(4 + i))
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    for k, n in seen.most_common():
        print(f"== {n}x {k}\n{stacks[k]}")
    print(f"{sum(seen.values())} synchronising calls in 2 steps")


if __name__ == "__main__":
    with warnings.catch_warnings():
        warnings.simplefilter("always")
        main()
