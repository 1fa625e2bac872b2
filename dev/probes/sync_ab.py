#!/usr/bin/env python3
"""The bench's per-pair synchronous protocol (bench.py:run_sync_latency) for one arch, run
against the framework tree given on the command line (e.g. an older round's worktree with its
own _C.so), so two trees can be compared on the same box:

    python dev/probes/sync_ab.py <tree root> [--arch raft_small] [--iters 32] [--steps 60]
"""
import argparse
import os
import sys
import types


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--arch", default="raft_small")
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--pool-first", action="store_true",
                    help="create a torch side stream (torch's per-device stream pool) before the engine")
    ap.add_argument("--pipelined-first", action="store_true",
                    help="run (and drop) a graph-pipelined stream of the same model before the sync protocol")
    a = ap.parse_args()
    root = os.path.abspath(a.root)
    sys.path.insert(0, root)
    import torch

    import bench
    import jax_raft_amd
    from jax_raft_amd import raft_large, raft_small

    assert os.path.dirname(os.path.dirname(os.path.abspath(jax_raft_amd.__file__))) == root, jax_raft_amd.__file__
    ctx = bench.Ctx(types.SimpleNamespace(dist_backend="nccl", step_times=False))
    if a.pool_first:
        side = torch.cuda.Stream(device=ctx.dev)
        with torch.cuda.stream(side):
            torch.zeros(1, device=ctx.dev)
    model = (raft_small if a.arch == "raft_small" else raft_large)(seed=0)[0].to(ctx.dev).eval()
    kw = dict(use_graph=True, streams="auto", split=1, gate_dtype=torch.bfloat16, corr_dtype=torch.bfloat16,
              copy_output=True, precision="bf16")
    if a.pipelined_first:
        m2 = (raft_small if a.arch == "raft_small" else raft_large)(seed=0)[0].to(ctx.dev).eval()
        bench.run_inference(ctx, m2, B=1, H=440, W=1024, iters=a.iters, steps=30, warmup=10, final_only=False,
                            gather=False, seed=99, engine_kw=kw, guarded=True)
        del m2
        torch.cuda.empty_cache()
    r = bench.run_sync_latency(ctx, model, H=440, W=1024, iters=a.iters, steps=a.steps, warmup=15, seed=99,
                               engine_kw=kw)
    print(f"{root}{' (pool first)' if a.pool_first else ''}{' (pipelined first)' if a.pipelined_first else ''}: {a.arch} {a.iters} it sync: {r['value']} FPS, p50 {r['latency_ms_p50']} ms, "
          f"p99 {r['latency_ms_p99']} ms", flush=True)


if __name__ == "__main__":
    main()
