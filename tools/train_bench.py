#!/usr/bin/env python3
"""Training throughput (BASELINE config 5): raft_large on synthetic
FlyingChairs-shaped 384x512 pairs, 12 refinement iterations, sequence loss,
AdamW + one-cycle, grad clip 1.0, RCCL gradient all-reduce when launched
with torchrun.  Prints one JSON line (rank 0): pairs/s over the whole job."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_raft_amd.parallel import dp  # noqa: E402
from jax_raft_amd.train.trainer import TrainConfig, Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--size", type=int, nargs=2, default=[384, 512])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graph-step", action="store_true", help="replay the whole step as one captured graph")
    ap.add_argument("--fresh-batches", action="store_true",
                    help="synthesise every step's batch inside the timed loop (bench.py's train extra)")
    ap.add_argument("--settle-lag", type=int, default=None, help="Trainer.SETTLE_LAG override (A/B)")
    ap.add_argument("--cprofile", default="", help="write the host-side cProfile of the timed steps (top 40) here")
    a = ap.parse_args()
    cfg = TrainConfig(arch=a.arch, steps=a.steps + a.warmup, batch=a.batch, iters=a.iters, size=tuple(a.size),
                      log_every=10 ** 9, graph_step=a.graph_step)
    if a.settle_lag is not None:
        Trainer.SETTLE_LAG = a.settle_lag
    tr = Trainer(cfg)
    batches = [tr.batch_for(i) for i in range(2)]
    for i in range(a.warmup):
        tr.train_step(batches[i % 2])
    torch.cuda.synchronize()
    if dp.is_dist():
        torch.distributed.barrier()
    prof = None
    if a.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    host = 0.0
    t0 = time.perf_counter()
    for i in range(a.steps):
        h0 = time.perf_counter()
        m = tr.train_step(tr.batch_for(a.warmup + i) if a.fresh_batches else batches[i % 2])
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    if prof is not None:
        import io
        import pstats
        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(40)
        with open(a.cprofile, "w") as f:
            f.write(buf.getvalue())
    dt = torch.tensor([time.perf_counter() - t0], device=tr.device, dtype=torch.float64)
    if dp.is_dist():
        torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    el = dt.item()
    if tr.rank == 0:
        print(json.dumps({"metric": "training image-pairs/sec (config 5)", "value": round(tr.world * a.batch * a.steps / el, 3),
                          "unit": "image-pairs/s", "n_gpus": tr.world, "ms_per_step": round(1000 * el / a.steps, 2),
                          # host time inside train_step (includes its one wait on the previous step's flag)
                          "host_ms_per_step": round(1000 * host / a.steps, 2),
                          "loss": float(m["loss"]), "config": {"model": a.arch, "per_gpu_batch": a.batch,
                          "image_size": list(a.size), "num_flow_updates": a.iters, "parallelism": f"dp{tr.world}",
                          "dtype": "bf16 (fp32 master weights)"}}), flush=True)
    if dp.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
