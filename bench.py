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
validate_sintel.py:185-186), overlapped with the previous step on a copy
stream (runtime/pipeline.py), and -- for N>1 -- the RCCL gather of every
rank's final flows to rank 0 (the DP batched-inference result
gather), issued asynchronously so it overlaps the next step's compute.  W
untimed warmup steps, then exactly K steps bracketed by barrier + synchronize;
the MAX over ranks is reported.

After the headline, the secondary BASELINE configurations are measured the same
way and added to the SAME JSON line (``extras``; a failure in an extra's untimed
set-up gives ``null`` on every rank without losing the headline): raft_large batch
1 as a pipelined stream (``b1_fps``) and with the reference's synchronous per-pair
protocol (``b1_sync``: H2D + forward + sync, 1 / mean latency,
validate_sintel.py:185-188), raft_small batch 1 at 32 iterations (stream and
sync) and at 12 iterations (config 2), the fp32 engine at batch 1, 1088x1920
frames (``hires_b1``), and training (config 5: raft_large, 384x512, 12
iterations, batch 6 per GPU, sequence loss + AdamW through the Trainer, RCCL
gradient all-reduce for N>1, synthetic data generated inside each timed step).

Weights are random-init (no network for checkpoints), data is synthetic, so
EPE is not measurable here and is reported as null; the numerical drift of the
bf16 engine against the fp32 golden model at this configuration is in
profiles/r5_drift.md (tools/drift.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_FPS = 11.8         # README.md:9 of the reference (RTX 3090 Ti, raft_large, 32 iters, batch 1)
BASELINE_SMALL_FPS = 36.6   # README.md:11 (raft_small, 32 iters, batch 1)
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


class Ctx:
    """Process / device / process-group context of one benchmark run."""

    def __init__(self, args):
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        ndev = torch.cuda.device_count()
        self.gloo = args.dist_backend == "gloo"
        self.step_times = bool(getattr(args, "step_times", False))
        idx = local_rank % ndev if self.gloo else local_rank
        torch.cuda.set_device(idx)
        self.dev = torch.device("cuda", idx)
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist

            if self.gloo:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=self.dev)
            self.pg = dist

    def barrier(self):
        if self.pg is not None:
            self.pg.barrier()
        torch.cuda.synchronize(self.dev)

    def _coll_dev(self):
        return "cpu" if self.gloo else self.dev

    def max_all(self, v: float) -> float:
        if self.pg is None:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self._coll_dev())
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return t.item()

    def all_values(self, v: float):
        if self.pg is None:
            return [v]
        t = torch.tensor([v], dtype=torch.float64, device=self._coll_dev())
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.pg.all_gather(out, t)
        return [x.item() for x in out]

    def world_check(self) -> int:
        """All-reduce of ones over the job's process group: must equal N."""
        if self.pg is None:
            return 1
        t = torch.ones(1, device=self._coll_dev())
        self.pg.all_reduce(t)
        return int(round(t.item()))


class FlowGather:
    """Gather every rank's final flows (B, H, W, 2) fp32 to rank 0.  With RCCL the
    collective is asynchronous (its own stream, ordered after the producing
    step by the process group) and overlaps the next step's compute; at most
    ``depth`` are in flight.  With gloo (the CPU-side rehearsal) it is a
    synchronous gather of host copies."""

    def __init__(self, ctx: Ctx, shape, depth: int = 2):
        self.ctx, self.depth = ctx, depth
        dev = "cpu" if ctx.gloo else ctx.dev
        self.recv = ([[torch.empty(shape, dtype=torch.float32, device=dev) for _ in range(ctx.world)]
                      for _ in range(depth)] if ctx.rank == 0 else None)
        self.inflight = []
        self.n = 0

    def __call__(self, flows: torch.Tensor) -> None:
        dist = self.ctx.pg
        if len(self.inflight) >= self.depth:
            self.inflight.pop(0).wait()
        slot = self.n % self.depth
        self.n += 1
        glist = self.recv[slot] if self.recv is not None else None
        if self.ctx.gloo:
            dist.gather(flows.cpu(), gather_list=glist, dst=0)
            return
        self.inflight.append(dist.gather(flows, gather_list=glist, dst=0, async_op=True))

    def drain(self) -> None:
        while self.inflight:
            self.inflight.pop(0).wait()


class ExtraFailed(RuntimeError):
    """An extra failed on some rank (every rank raises it together, so the ranks' collectives
    stay paired and every rank reports the extra as null)."""


def agree(ctx: Ctx, ok: bool, what: str) -> None:
    """All ranks learn whether every rank got here without an error (MIN of a flag): a
    failure on one rank must not leave the others waiting in a collective the failed rank
    never enters (bench.py extras on N > 1)."""
    if ctx.pg is None:
        if not ok:
            raise ExtraFailed(what)
        return
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=ctx._coll_dev())
    ctx.pg.all_reduce(t, op=ctx.pg.ReduceOp.MIN)
    if t.item() < 0.5:
        raise ExtraFailed(what)


def run_inference(ctx: Ctx, model, *, B: int, H: int, W: int, iters: int, steps: int, warmup: int,
                  final_only: bool, gather: bool, seed: int, engine_kw: dict, pipeline: str = "auto",
                  h2d: bool = True, sync_h2d: bool = False, guarded: bool = False) -> dict:
    """Time ``steps`` inference steps of ``B`` pairs per rank; returns the run record.
    ``guarded``: the untimed part (engine, plan build, warmup: no collectives) may fail on
    one rank; the ranks then agree on the failure before any collective (:func:`agree`)."""
    from jax_raft_amd.runtime.pipeline import InputPrefetcher

    dev = ctx.dev
    g = torch.Generator().manual_seed(seed + ctx.rank)
    img1 = torch.rand(B, H, W, 3, generator=g) * 2 - 1
    img2 = torch.rand(B, H, W, 3, generator=g) * 2 - 1
    if h2d:
        img1, img2 = img1.pin_memory(), img2.pin_memory()
    else:
        img1, img2 = img1.to(dev), img2.to(dev)
    pf = InputPrefetcher([(B, H, W, 3), (B, H, W, 3)], dev) if (h2d and not sync_h2d) else None
    all_iters = not final_only
    eng, mode, copipe, gat = None, pipeline, False, None

    def forward(a, b):
        if copipe:
            return eng.pipelined(a, b, iters, return_all_iters=all_iters)
        return eng.forward(a, b, iters, return_all_iters=all_iters)

    def run(n, events=None):
        out = None
        if pf is not None:
            pf.put(0, [img1, img2])
        for i in range(n):
            if pf is not None:
                a, b = pf.get(i)
            else:
                a, b = img1.to(dev, non_blocking=True), img2.to(dev, non_blocking=True)
            out = forward(a, b)
            if gat is not None and out is not None:
                gat(out[-1])
            if events is not None:
                events[i + 1].record()
            if pf is not None:
                pf.release(i)
                if i + 1 < n:
                    pf.put(i + 1, [img1, img2])
        return out

    err, out = None, None
    try:
        eng = model.engine(dev, **engine_kw)
        if mode == "auto":
            mode = "off" if (eng.uses_lanes(B, not final_only) or engine_kw.get("split", 1) > 1
                             or getattr(eng, "fe_external", False)) else "graph"
        copipe = mode == "graph" and engine_kw.get("use_graph", True)
        if copipe:   # fill the pipeline: the first batch's prologue (its loop runs in the first step)
            eng.pipelined(img1.to(dev), img2.to(dev), iters, return_all_iters=all_iters)
        out = run(warmup)              # gat is None: no collective in the warmup (see `guarded`)
        torch.cuda.synchronize(dev)
        if out is not None:
            assert out.shape == ((iters if all_iters else 1), B, H, W, 2) and bool(torch.isfinite(out[-1]).all())
    except Exception as e:  # noqa: BLE001
        if not guarded:
            raise
        err = e
    if guarded:
        agree(ctx, err is None, f"{type(err).__name__}: {err}" if err is not None else "")
    gat = FlowGather(ctx, (B, H, W, 2)) if (gather and ctx.world > 1) else None
    if gat is not None:   # one untimed gather: the collective's first-use setup stays out of the timing
        gat(out[-1] if out is not None else torch.zeros(B, H, W, 2, device=dev))
        gat.drain()
    events = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ctx.barrier()
    t0 = time.perf_counter()
    events[0].record()
    run(steps, events)
    if gat is not None:
        gat.drain()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    ctx.barrier()
    if copipe:
        eng.flush()   # the last prologue's batch (untimed)
        torch.cuda.synchronize(dev)
    step_ms = [events[i].elapsed_time(events[i + 1]) for i in range(steps)]
    if ctx.step_times:   # per-step device times in order (diagnostics)
        print("step_ms " + " ".join(f"{t:.2f}" for t in step_ms), file=sys.stderr, flush=True)
    step_ms.sort()
    pct = lambda q: round(step_ms[min(len(step_ms) - 1, int(q * len(step_ms)))], 3)
    el = t1 - t0
    per_rank = [round(1000.0 * e / steps, 3) for e in ctx.all_values(el)]
    elapsed = ctx.max_all(el)
    rec = dict(value=round(ctx.world * B * steps / elapsed, 3), ms_per_step=round(1000.0 * elapsed / steps, 3),
               steps=steps, warmup=warmup, step_ms_p50=pct(0.5), step_ms_p99=pct(0.99), per_rank_ms_per_step=per_rank,
               cross_batch_pipeline=mode if engine_kw.get("use_graph", True) else "off",
               concurrent_branches=bool(eng.uses_lanes(B, all_iters)))
    if gat is not None:
        rec["gather"] = "final flows of every rank -> rank 0, async (overlapped with the next step)"
        rec["gather_ms"] = round(_gather_ms(ctx, gat, out[-1] if out is not None else None, (B, H, W, 2)), 3)
    rec["tile_cfgs"] = dict(sorted(eng.chosen_cfgs.items()))
    return rec


def run_sync_latency(ctx: Ctx, model, *, H: int, W: int, iters: int, steps: int, warmup: int, seed: int,
                     engine_kw: dict, raw: bool = False) -> dict:
    """The reference's own FPS protocol (validate_sintel.py:185-188,201-203), batch 1, one pair
    at a time: host->device copy of the pair (from pageable host memory, like numpy inputs),
    the forward with all ``iters`` upsampled predictions, then a synchronisation on the
    result -- no overlap of consecutive pairs at all.  FPS = 1 / mean latency (x ranks for
    N > 1, each rank timing its own pairs).  ``raw``: the pair is raw uint8 H x W frames (any
    size: Sintel's 436 x 1024), normalised and replicate-padded to /8 on the device by the
    engine's prep kernel, the flows cropped back (validate_sintel.py:177-191 on the device)."""
    dev = ctx.dev
    g = torch.Generator().manual_seed(seed + ctx.rank)
    if raw:
        pairs = [(torch.randint(0, 256, (1, H, W, 3), generator=g, dtype=torch.uint8),
                  torch.randint(0, 256, (1, H, W, 3), generator=g, dtype=torch.uint8)) for _ in range(4)]
        h2d = lambda x: x   # noqa: E731 -- the engine copies host frames straight into its plan input
    else:
        pairs = [(torch.rand(1, H, W, 3, generator=g) * 2 - 1, torch.rand(1, H, W, 3, generator=g) * 2 - 1)
                 for _ in range(4)]
        h2d = lambda x: x.to(dev)   # noqa: E731
    err, lat = None, []
    try:
        eng = model.engine(dev, **dict(engine_kw, split=1))
        for i in range(warmup):
            a, b = pairs[i % 4]
            eng.forward(h2d(a), h2d(b), iters)[-1]
        torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001
        err = e
    agree(ctx, err is None, f"{type(err).__name__}: {err}" if err is not None else "")
    ctx.barrier()
    for i in range(steps):
        a, b = pairs[i % 4]
        t0 = time.perf_counter()
        flow = eng.forward(h2d(a), h2d(b), iters)[-1]
        torch.cuda.synchronize(dev)
        lat.append(time.perf_counter() - t0)
        assert flow.shape == (1, H, W, 2)
    ctx.barrier()
    mean = sum(lat) / len(lat)
    mean_max = ctx.max_all(mean)
    lat.sort()
    proto = ("per pair: raw uint8 frames H2D (pageable) + on-device normalise / replicate pad to /8 + forward "
             "(all iterations upsampled) + crop + sync; no cross-pair overlap (validate_sintel.py:177-191)" if raw else
             "per pair: H2D (pageable) + forward (all iterations upsampled) + sync; no cross-pair overlap "
             "(validate_sintel.py:185-188)")
    return dict(value=round(ctx.world / mean_max, 3), latency_ms_mean=round(1000 * mean_max, 3),
                latency_ms_p50=round(1000 * lat[len(lat) // 2], 3),
                latency_ms_p99=round(1000 * lat[min(len(lat) - 1, int(0.99 * len(lat)))], 3),
                steps=steps, warmup=warmup, protocol=proto)


def _gather_ms(ctx: Ctx, gat: FlowGather, flows, shape) -> float:
    """Stand-alone time of one final-flow gather (barrier-bracketed, mean of 3)."""
    flows = flows if flows is not None else torch.zeros(shape, device=ctx.dev)
    ts = []
    for _ in range(3):
        ctx.barrier()
        t0 = time.perf_counter()
        gat(flows)
        gat.drain()
        torch.cuda.synchronize(ctx.dev)
        ts.append(time.perf_counter() - t0)
    return 1000.0 * ctx.max_all(sum(ts) / len(ts))


def run_training_child(*, arch: str, B: int, size, iters: int, steps: int, warmup: int) -> dict:
    """Single GPU: the training extra in a fresh child process (tools/train_bench.py; the parent
    has finished its GPU work and waits).  In-process, after the inference extras, the step's
    side streams share hardware queues with whatever streams the process created before
    (GPU_MAX_HW_QUEUES = 4), and the same step measured 174-376 pairs/s depending on which
    extras ran first (profiles/r6_hwq_ab.txt); a training job starts in a fresh process."""
    import subprocess

    cmd = [sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "train_bench.py"),
           "--arch", arch, "--batch", str(B), "--iters", str(iters), "--size", str(size[0]), str(size[1]),
           "--steps", str(steps), "--warmup", str(warmup), "--fresh-batches"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"train_bench.py exited {r.returncode}: {r.stderr[-2000:]}")
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return dict(value=d["value"], ms_per_step=d["ms_per_step"], steps=steps, warmup=warmup, loss=round(d["loss"], 4),
                per_rank_ms_per_step=[d["ms_per_step"]], process="fresh child (tools/train_bench.py)",
                config=dict(model=arch, per_gpu_batch=B, global_batch=B, image_size=list(size), num_flow_updates=iters,
                            optimizer="AdamW + one-cycle, clip 1.0", loss="sequence loss gamma 0.8",
                            grad_allreduce=None, data="synthetic, generated on the GPU inside each timed step"))


def run_training(ctx: Ctx, *, arch: str, B: int, size, iters: int, steps: int, warmup: int) -> dict:
    """BASELINE config 5 through the Trainer (fused native step, AdamW, RCCL
    gradient all-reduce for N>1); each step synthesises its batch on the GPU."""
    from jax_raft_amd.train.trainer import TrainConfig, Trainer

    cfg = TrainConfig(arch=arch, steps=steps + warmup, batch=B, iters=iters, size=tuple(size), log_every=10 ** 9)
    tr = Trainer(cfg, device=ctx.dev)
    for i in range(warmup):
        tr.train_step(tr.batch_for(i))
    tr.flush()
    ctx.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        m = tr.train_step(tr.batch_for(warmup + i))
    tr.flush()
    torch.cuda.synchronize(ctx.dev)
    el = time.perf_counter() - t0
    ctx.barrier()
    elapsed = ctx.max_all(el)
    return dict(value=round(ctx.world * B * steps / elapsed, 3), ms_per_step=round(1000.0 * elapsed / steps, 3),
                steps=steps, warmup=warmup, loss=round(float(m["loss"]), 4),
                per_rank_ms_per_step=[round(1000.0 * e / steps, 3) for e in ctx.all_values(el)],
                config=dict(model=arch, per_gpu_batch=B, global_batch=ctx.world * B, image_size=list(size),
                            num_flow_updates=iters, optimizer="AdamW + one-cycle, clip 1.0",
                            loss="sequence loss gamma 0.8", grad_allreduce="RCCL" if ctx.world > 1 else None,
                            data="synthetic, generated on the GPU inside each timed step"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4, help="image pairs per GPU per step")
    ap.add_argument("--arch", default="raft_large", choices=["raft_large", "raft_small"])
    ap.add_argument("--height", type=int, default=440)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="inputs already resident on the GPU")
    ap.add_argument("--sync-h2d", action="store_true", help="copy each step's inputs synchronously (no prefetch overlap)")
    ap.add_argument("--streams", default="auto", choices=["auto", "on", "off"],
                    help="concurrent model branches on plan lanes: auto = at batch >= 4 per GPU with all "
                         "iterations upsampled (measured break-even)")
    ap.add_argument("--final-only", action="store_true",
                    help="serving mode: upsample/return only the final flow (not the reference's output)")
    ap.add_argument("--gate-dtype", default="bf16", choices=["bf16", "fp32"],
                    help="storage of the GRU z gate / folded context bias map (the hidden state is fp32 either way)")
    ap.add_argument("--corr-dtype", default="bf16", choices=["bf16", "fp32"], help="correlation pyramid storage")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "mixed"],
                    help="engine compute precision: bf16 MFMA operands (default), the fp32 parity mode, or "
                         "mixed (fp32 feature encoder, bf16 rest: runtime/engine_f32.py:RaftEngineMixed)")
    ap.add_argument("--no-copy-output", action="store_true",
                    help="return the engine's static output buffer instead of a fresh tensor (measurement knob)")
    ap.add_argument("--split", type=int, default=1, help="independent batch parts captured into one hipGraph")
    ap.add_argument("--pipeline", default="auto", choices=["auto", "off", "graph"],
                    help="cross-batch software pipelining: 'auto' = 'graph' where the engine runs one lane (batch < 4, "
                         "raft_small, final-only; measured faster there) else off; 'graph' = each step replays ONE "
                         "hipGraph holding batch i's refinement loop and batch i+1's encoders + correlation pyramid")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the RCCL gather of the final flows")
    ap.add_argument("--extras", default="auto", choices=["auto", "on", "off"],
                    help="secondary configs after the headline (auto: on for the default headline config)")
    ap.add_argument("--extra-steps", type=int, default=20)
    ap.add_argument("--step-times", action="store_true", help="print every timed step's device time (stderr)")
    ap.add_argument("--skip-extras", default="", help="comma list of extras to leave out (diagnostics)")
    ap.add_argument("--only-extra", default="", help="run just this extra in this process (no headline; prints "
                                                     "its record as one JSON line) -- diagnostics / child runs")
    ap.add_argument("--extra-pause", type=float, default=0.0, help="seconds of idle before each extra (diagnostics)")
    ap.add_argument("--train-batch", type=int, default=6, help="extras: training batch per GPU (config 5: 6)")
    ap.add_argument("--train-size", type=int, nargs=2, default=[384, 512], help="extras: training image size")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL on ROCm) for real runs; gloo only to rehearse >1 rank on fewer GPUs")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` without a launcher: start torch.distributed.run as a
        # child (nothing has touched the GPU yet) and exit with its return code,
        # rather than silently benchmarking one GPU.
        sys.exit(_relaunch(args.gpus))

    ctx = Ctx(args)
    if args.gpus != ctx.world and ctx.world > 1:
        print(f"warning: --gpus {args.gpus} != WORLD_SIZE {ctx.world}; using WORLD_SIZE", file=sys.stderr)
    from jax_raft_amd import raft_large, raft_small
    from jax_raft_amd.runtime import tunedb

    factory = raft_large if args.arch == "raft_large" else raft_small
    model = factory(seed=0)[0].to(ctx.dev).eval()
    streams = {"auto": "auto", "on": True, "off": False}[args.streams]
    engine_kw = dict(use_graph=not args.no_graph, streams=streams, split=args.split,
                     gate_dtype=torch.bfloat16 if args.gate_dtype == "bf16" else torch.float32,
                     corr_dtype=torch.bfloat16 if args.corr_dtype == "bf16" else torch.float32,
                     copy_output=not args.no_copy_output, precision=args.precision)
    B, H, W = args.batch, args.height, args.width
    if args.only_extra:
        head, rccl_world = None, ctx.world
    else:
        head = run_inference(ctx, model, B=B, H=H, W=W, iters=args.iters, steps=args.steps, warmup=args.warmup,
                             final_only=args.final_only, gather=not args.no_gather, seed=1234, engine_kw=engine_kw,
                             pipeline=args.pipeline, h2d=not args.no_h2d, sync_h2d=args.sync_h2d)
        rccl_world = ctx.world_check()
    del model
    torch.cuda.empty_cache()

    default_cfg = (args.arch == "raft_large" and (B, H, W, args.iters) == (4, 440, 1024, 32) and not args.final_only
                   and not args.no_graph and args.precision == "bf16")
    extras = {}
    if args.extras == "on" or (args.extras == "auto" and default_cfg) or args.only_extra:
        t_ex = time.perf_counter()
        ks, kw_ = args.extra_steps, max(3, args.warmup)
        # *_b1_fps: batch-1 stream throughput (graph-pipelined: pair i's loop overlaps pair i+1's
        # encoders); *_b1_sync: the reference's per-pair synchronous latency protocol (no overlap);
        # fp32_b1_fps: the reference's own precision -- fp32 end to end (runtime/engine_f32.py);
        # hires_b1: 1088x1920 frames (a 136x240 feature map), batch 1, 32 iterations
        plan = [("b1_fps", "raft_large", 32, BASELINE_FPS, "bf16", "stream", (H, W)),
                ("b1_sync", "raft_large", 32, BASELINE_FPS, "bf16", "sync", (H, W)),
                # raw 436 x 1024 uint8 Sintel-size frames, prepared on the device
                ("b1_sync_u8", "raft_large", 32, BASELINE_FPS, "bf16", "sync_u8", (H - 4, W)),
                ("small_b1_fps_32it", "raft_small", 32, BASELINE_SMALL_FPS, "bf16", "stream", (H, W)),
                ("small_b1_sync_32it", "raft_small", 32, BASELINE_SMALL_FPS, "bf16", "sync", (H, W)),
                ("small_b1_fps_12it", "raft_small", 12, None, "bf16", "stream", (H, W)),
                # precision="mixed": fp32 feature encoder (raft_small's bf16 drift, profiles/r6_drift_mixed.md)
                ("small_b1_sync_32it_mixed", "raft_small", 32, BASELINE_SMALL_FPS, "mixed", "sync", (H, W)),
                ("fp32_b1_fps", "raft_large", 32, BASELINE_FPS, "fp32", "stream", (H, W)),
                ("hires_b1", "raft_large", 32, None, "bf16", "stream", (1088, 1920))]
        skip = set(filter(None, args.skip_extras.split(",")))
        for key, arch, it, base, prec, proto, (eh, ew) in plan:
            if key in skip or (args.only_extra and key != args.only_extra):
                continue
            if args.extra_pause:   # diagnostics: idle the GPU before each extra
                time.sleep(args.extra_pause)
            if args.step_times:   # diagnostics: what earlier extras left alive
                import gc

                from jax_raft_amd.runtime.engine import RaftEngine
                live = sum(isinstance(o, RaftEngine) for o in gc.get_objects())
                print(f"extra {key}: {live} live engines, {torch.cuda.memory_allocated(ctx.dev) / 2**20:.0f} MiB "
                      f"allocated", file=sys.stderr, flush=True)
            # the short forwards (raft_small: 1.2-2.3 ms) get more steps, so that one host-side
            # hiccup in a ~25 ms timed region does not decide the number
            mul = 3 if arch == "raft_small" else 1
            try:
                m = (raft_large if arch == "raft_large" else raft_small)(seed=0)[0].to(ctx.dev).eval()
                if proto in ("sync", "sync_u8"):
                    r = run_sync_latency(ctx, m, H=eh, W=ew, iters=it, steps=ks * mul, warmup=kw_ * mul,
                                         seed=99, engine_kw=dict(engine_kw, precision=prec), raw=proto == "sync_u8")
                else:
                    r = run_inference(ctx, m, B=1, H=eh, W=ew, iters=it, steps=ks * mul, warmup=kw_ * mul,
                                      final_only=False, gather=not args.no_gather, seed=99,
                                      engine_kw=dict(engine_kw, split=1, precision=prec), guarded=True)
                    r.pop("tile_cfgs", None)
                r["config"] = dict(model=arch, per_gpu_batch=1, num_flow_updates=it, image_size=[eh, ew], dtype=prec)
                r["vs_baseline"] = round(r["value"] / ctx.world / base, 3) if base else None
                extras[key] = r
                del m
            except ExtraFailed as e:   # failed on some rank; every rank lands here together
                extras[key] = None
                print(f"bench.py: extra {key} failed on a rank: {e}", file=sys.stderr)
            except Exception as e:  # noqa: BLE001 -- single-rank: a failed extra must not lose the headline
                if ctx.world > 1:
                    raise   # a failure inside a timed (collective) phase cannot be isolated per rank
                extras[key] = None
                print(f"bench.py: extra {key} failed: {type(e).__name__}: {e}", file=sys.stderr)
            torch.cuda.empty_cache()
        if args.only_extra:
            if ctx.rank == 0:
                print(json.dumps({args.only_extra: extras.get(args.only_extra)}), flush=True)
            return
        try:
            if ctx.world == 1:
                extras["train_pairs_per_s"] = run_training_child(arch="raft_large", B=args.train_batch,
                                                                 size=tuple(args.train_size), iters=12,
                                                                 steps=max(10, ks), warmup=3)
            else:
                extras["train_pairs_per_s"] = run_training(ctx, arch="raft_large", B=args.train_batch,
                                                           size=tuple(args.train_size), iters=12,
                                                           steps=max(2, ks // 2), warmup=3)
        except Exception as e:  # noqa: BLE001
            if ctx.world > 1:
                raise   # the DP step's gradient all-reduce cannot be left mid-way on one rank
            extras["train_pairs_per_s"] = None
            print(f"bench.py: extra train_pairs_per_s failed: {type(e).__name__}: {e}", file=sys.stderr)
        extras["extras_wall_s"] = round(time.perf_counter() - t_ex, 1)

    if ctx.rank == 0:
        rec = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "image-pairs/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "step_ms_p50": head["step_ms_p50"],
            "step_ms_p99": head["step_ms_p99"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(head["value"] / BASELINE_FPS, 3)
                            if args.arch == "raft_large" and args.iters == 32 and not args.final_only else None),
            "vs_baseline_note": "batch-4-per-GPU throughput / the reference's batch-1 FPS; "
                                "extras.b1_fps.vs_baseline is the like-for-like batch-1 ratio",
            "dtype": args.precision,
            "data": "synthetic (random Sintel-shaped 440x1024 frames, random-init weights; EPE not measurable)",
            "epe_sintel_clean": None,
            "rccl_world": rccl_world,
            "per_rank_ms_per_step": head["per_rank_ms_per_step"],
            "gather_ms": head.get("gather_ms"),
            "config": {
                "model": args.arch,
                "global_batch": ctx.world * B,
                "per_gpu_batch": B,
                "image_size": [H, W],
                "seq_len": None,
                "num_flow_updates": args.iters,
                "outputs": ("final iteration only (serving mode)" if args.final_only
                            else "all iterations upsampled (reference semantics)"),
                "hipgraph": not args.no_graph,
                "concurrent_branches": head["concurrent_branches"],
                "cross_batch_pipeline": head["cross_batch_pipeline"],
                "gate_dtype": args.gate_dtype,
                "corr_dtype": args.corr_dtype,
                "batch_parts": args.split,
                "h2d_in_timed_region": not args.no_h2d,
                "h2d_overlapped": not (args.no_h2d or args.sync_h2d),
                "result_gather": head.get("gather"),
                "parallelism": f"dp{ctx.world}",
            },
            "autotune": {"source": "jax_raft_amd/tuned/<arch>.json + in-process timing of misses",
                         **tunedb.stats(), "tile_cfgs": head["tile_cfgs"]},
            "extras": extras or None,
        }
        print(json.dumps(rec), flush=True)
    if ctx.pg is not None:
        ctx.pg.destroy_process_group()


if __name__ == "__main__":
    main()
