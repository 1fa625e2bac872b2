#!/usr/bin/env python3
"""Headline benchmark: raft_large inference throughput (image pairs / s) on
Sintel-shaped 440x1024 frames (436 padded to /8, like scripts/validate_sintel.py
of the reference), 32 refinement iterations, all 32 upsampled predictions
produced (the reference's output), bf16 compute on the native HIP kernels with
the whole forward replayed as one hipGraph.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched by torch.distributed.run, one rank per GPU (RCCL).  Weak scaling:
each rank processes ``--batch`` pairs per step (default 4, so 8 GPUs = the
BASELINE config's batch of 32).  Each timed step includes the host->device
copy of its input pair (the reference times H2D + forward as well,
validate_sintel.py:185-186); the copy of step i+1 is overlapped with step i
on a copy stream (runtime/pipeline.py), as a serving loop would.  With
``--pipeline auto`` (default) the configs whose plan runs on one lane (batch
< 4, raft_small, final-only) replay graph-pipelined steps (engine.pipelined):
one hipGraph per step holding batch i's refinement loop and batch i+1's
encoders + correlation pyramid, so every timed step does exactly one forward's
work (K loops + K prologues; the pipeline is filled before the warmup and the
last prologue's batch is drained after the timer).  The headline config
(raft_large, batch 4) runs the lane schedule without it.  Timing: W untimed warmup steps, then exactly K
steps bracketed by barrier + synchronize; the MAX over ranks is reported.
Weights are random-init (no network for checkpoints), data is synthetic, so
EPE is not measurable here and is reported as null.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_FPS = 11.8  # README.md:9 of the reference (RTX 3090 Ti, raft_large, 32 iters, batch 1)
METRIC = "image-pairs/sec + Sintel-clean EPE, raft_large 32 iters at 1/2/4/8 MI355X"


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _relaunch(n: int) -> int:
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    print("bench.py: --gpus {} without a launcher, running: {}".format(n, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4, help="image pairs per GPU per step")
    ap.add_argument("--arch", default="raft_large", choices=["raft_large", "raft_small"])
    ap.add_argument("--height", type=int, default=440)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="inputs already resident on the GPU")
    ap.add_argument("--sync-h2d", action="store_true", help="copy each step's inputs synchronously (no prefetch overlap)")
    ap.add_argument("--streams", default="auto", choices=["auto", "on", "off"],
                    help="concurrent model branches on plan lanes: auto = at batch >= 4 per GPU with all iterations upsampled (measured break-even)")
    ap.add_argument("--no-streams", action="store_true", help="same as --streams off")
    ap.add_argument("--flow-head", default="taps", choices=["taps", "conv", "fused"],
                    help="flow head output conv: 1x1 GEMM + tap sum (default), 3x3 conv, or the halo-tiled kernel")
    ap.add_argument("--final-only", action="store_true",
                    help="serving mode: upsample/return only the final flow (not the reference's output)")
    ap.add_argument("--gate-dtype", default="bf16", choices=["bf16", "fp32"],
                    help="storage of the GRU z gate / folded context bias map (the hidden state is fp32 either way)")
    ap.add_argument("--flow-lane", default="mask", choices=["side", "main", "mask"])
    ap.add_argument("--no-copy-output", action="store_true",
                    help="return the engine's static output buffer instead of a fresh copy (measurement knob)")
    ap.add_argument("--convex", default="head", choices=["fused", "separate", "head"],
                    help="mask predictor 1x1 conv + convex upsampling: conv epilogue / two kernels / dedicated kernel")
    ap.add_argument("--mask-head", default="split", choices=["split", "fused"],
                    help="mask predictor 3x3 conv on the mask lane (split) or batched with the flow head's (fused)")
    ap.add_argument("--double-buffer", action="store_true", help="parity double-buffering of the flow head outputs")
    ap.add_argument("--no-taps-epi", action="store_true",
                    help="FlowHead conv1 stores its features and a separate GEMM forms conv2's taps")
    ap.add_argument("--no-fuse-update", action="store_true",
                    help="separate flow-update kernel after the flow head instead of inside the next lookup")
    ap.add_argument("--no-fe-split", action="store_true",
                    help="one feature-encoder pass over both images instead of one per image on two lanes")
    ap.add_argument("--fork-after", default="lookup", choices=["lookup", "cc1"],
                    help="main-lane kernel after which the mask lane forks each iteration")
    ap.add_argument("--no-direct-flow", action="store_true", help="flow branch 7x7 conv on the implicit GEMM instead of the direct VALU kernel")
    ap.add_argument("--no-merge-parts", action="store_true",
                    help="with --split: one graph per part on its own stream instead of all parts in one graph")
    ap.add_argument("--split", type=int, default=1, help="independent batch parts (one hipGraph each) run concurrently per GPU")
    ap.add_argument("--pipeline", default="auto", choices=["auto", "off", "graph", "streams"],
                    help="cross-batch software pipelining: 'auto' = 'graph' where the engine runs one lane (batch < 4, "
                         "raft_small, final-only; measured faster there) else off; 'graph' = each step replays ONE hipGraph holding batch i's "
                         "refinement loop and batch i+1's encoders + correlation pyramid as parallel branches "
                         "(engine.pipelined); 'streams' = the two phases as separate graphs on two streams "
                         "(engine.submit, measured to serialise)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL on ROCm) for real runs; gloo only to rehearse >1 rank on fewer GPUs")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` without a launcher: start torch.distributed.run as a
        # child (nothing has touched the GPU yet) and exit with its return code,
        # rather than silently benchmarking one GPU.
        sys.exit(_relaunch(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} != WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    ndev = torch.cuda.device_count()
    dev_index = local_rank % ndev if args.dist_backend == "gloo" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    pg = None
    if world > 1:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        pg = dist

    from jax_raft_amd import raft_large, raft_small

    model, _ = (raft_large if args.arch == "raft_large" else raft_small)(seed=0)
    model = model.to(dev).eval()
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator().manual_seed(1234 + rank)
    img1 = (torch.rand(B, H, W, 3, generator=g) * 2 - 1)
    img2 = (torch.rand(B, H, W, 3, generator=g) * 2 - 1)
    if args.no_h2d:
        img1, img2 = img1.to(dev), img2.to(dev)
    else:
        img1, img2 = img1.pin_memory(), img2.pin_memory()
    from jax_raft_amd.runtime.pipeline import InputPrefetcher

    # Every step copies its input pair host -> device (the reference times H2D
    # too); the copy of step i+1 runs on a copy stream while step i computes
    # (InputPrefetcher), so only the first copy of a run is exposed.
    pf = None if (args.no_h2d or args.sync_h2d) else InputPrefetcher([(B, H, W, 3), (B, H, W, 3)], dev)

    streams = False if args.no_streams else {"auto": "auto", "on": True, "off": False}[args.streams]
    engine_kw = dict(use_graph=not args.no_graph, streams=streams, split=args.split,
                     flow_head=args.flow_head, double_buffer=args.double_buffer, direct_flow=not args.no_direct_flow,
                     gate_dtype=torch.bfloat16 if args.gate_dtype == "bf16" else torch.float32,
                     flow_lane=args.flow_lane, mask_head=args.mask_head,
                     convex=args.convex, copy_output=not args.no_copy_output, taps_epi=not args.no_taps_epi,
                     fuse_update=not args.no_fuse_update, fe_split=not args.no_fe_split,
                     fork_after=args.fork_after, merge_parts=not args.no_merge_parts)
    mode = args.pipeline
    if mode == "auto":
        lanes = model.engine(dev, **engine_kw).uses_lanes(B, not args.final_only)
        mode = "off" if (lanes or args.split > 1) else "graph"
    pipelined = mode == "streams" and not args.no_graph
    copipe = mode == "graph" and not args.no_graph
    eng = model.engine(dev, **engine_kw) if (pipelined or copipe) else None
    if copipe:
        # fill the pipeline: the first batch's prologue (its loop runs in the first warmup / timed step)
        eng.pipelined(img1.to(dev), img2.to(dev), args.iters, return_all_iters=not args.final_only)

    def forward(a, b):
        """One step; returns (flows, stream the step's work ends on).  Pipelined
        'graph' mode: the flows of the previous step's inputs (one loop + one
        prologue of work per step)."""
        if copipe:
            return (eng.pipelined(a, b, args.iters, return_all_iters=not args.final_only),
                    torch.cuda.current_stream(dev))
        if pipelined:
            # batch i's encoders + correlation pyramid overlap batch i-1's refinement loop
            h = eng.submit(a, b, args.iters, return_all_iters=not args.final_only)
            return h.out, eng.loop_stream
        return (model(a, b, num_flow_updates=args.iters, return_all_iters=not args.final_only, **engine_kw),
                torch.cuda.current_stream(dev))

    def run(n, events=None):
        if pf is None:
            for i in range(n):
                out, s = forward(img1.to(dev, non_blocking=True), img2.to(dev, non_blocking=True))
                if events is not None:
                    events[i + 1].record(s)
            return out
        pf.put(0, [img1, img2])
        for i in range(n):
            a, b = pf.get(i)
            out, s = forward(a, b)
            if events is not None:
                events[i + 1].record(s)
            pf.release(i)
            if i + 1 < n:
                pf.put(i + 1, [img1, img2])
        return out

    def barrier():
        if pg is not None:
            pg.barrier()
        torch.cuda.synchronize(dev)

    out = run(args.warmup)
    torch.cuda.synchronize(dev)
    if out is None:   # pipelined with --warmup 0: nothing finished yet
        out = torch.zeros((1 if args.final_only else args.iters, B, H, W, 2))
    assert out.shape == (1 if args.final_only else args.iters, B, H, W, 2) and bool(torch.isfinite(out[-1]).all())

    # per-step device timestamps (hipEvents on the compute stream) for the
    # step-time distribution; the headline uses the host clock around all K steps
    events = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    barrier()
    t0 = time.perf_counter()
    events[0].record()
    out = run(args.steps, events)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    barrier()
    if copipe:
        eng.flush()   # the last prologue's batch (untimed)
        torch.cuda.synchronize(dev)
    step_seq = [events[i].elapsed_time(events[i + 1]) for i in range(args.steps)]
    if os.environ.get("JR_BENCH_STEPS"):   # per-step device times in order (diagnostics)
        print("step_ms", [round(t, 3) for t in step_seq], file=sys.stderr)
    step_ms = sorted(step_seq)
    pct = lambda q: round(step_ms[min(len(step_ms) - 1, int(q * len(step_ms)))], 3)
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    if pg is not None:
        pg.all_reduce(dt, op=pg.ReduceOp.MAX)
    elapsed = dt.item()
    ms_per_step = 1000.0 * elapsed / args.steps
    pairs_per_s = world * B * args.steps / elapsed
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(pairs_per_s, 3),
            "unit": "image-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "step_ms_p50": pct(0.5),
            "step_ms_p99": pct(0.99),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(pairs_per_s / BASELINE_FPS, 3) if args.arch == "raft_large" and args.iters == 32 and not args.final_only else None,
            "dtype": "bf16",
            "data": "synthetic (random Sintel-shaped 440x1024 frames, random-init weights; EPE not measurable)",
            "epe_sintel_clean": None,
            "config": {
                "model": args.arch,
                "global_batch": world * B,
                "per_gpu_batch": B,
                "image_size": [H, W],
                "seq_len": None,
                "num_flow_updates": args.iters,
                "outputs": "final iteration only (serving mode)" if args.final_only else "all iterations upsampled (reference semantics)",
                "hipgraph": not args.no_graph,
                "concurrent_branches": (streams if streams != "auto" else ("auto (on: batch >= 4 with a mask predictor)" if not args.final_only else "auto (off in final-only mode)")),
                "flow_head": args.flow_head,
                "gate_dtype": args.gate_dtype,
                "flow_lane": args.flow_lane,
                "mask_head": args.mask_head,
                "convex": args.convex,
                "direct_flow_conv": not args.no_direct_flow,
                "taps_epilogue": not args.no_taps_epi,
                "update_in_lookup": not args.no_fuse_update,
                "feature_encoder_split": not args.no_fe_split,
                "fork_after": args.fork_after,
                "batch_parts": args.split,
                "cross_batch_pipeline": mode if not args.no_graph else "off",
                "h2d_in_timed_region": not args.no_h2d,
                "h2d_overlapped": not (args.no_h2d or args.sync_h2d),
                "parallelism": f"dp{world}",
            },
        }
        print(json.dumps(rec), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
