"""Data-parallel RAFT training (BASELINE config 5: raft_large, FlyingChairs-
shaped 384x512 pairs, sequence loss over 12 iterations, RCCL gradient
all-reduce).  The reference has no training code; this
follows the original RAFT recipe: AdamW + one-cycle LR (linear anneal, 5%
warm-up), gradient clipping at 1.0, gamma = 0.8, max_flow = 400.

Run (one process per GPU)::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m jax_raft_amd.train.trainer \\
        --arch raft_large --steps 1000 --batch 6 --iters 12

Checkpoints: ``<dir>/step_<n>.msgpack`` (Flax-format weights, loadable with
``raft_large(weights=...)``) + ``step_<n>.opt.pt`` (optimizer / scheduler
state, tensors only) + ``latest.json``; ``--resume`` continues from latest.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, Optional

import torch

from .. import raft_large, raft_small
from ..parallel import dp
from ..utils import checkpoint as ckpt
from .data import SyntheticFlow
from .loss import sequence_loss


@dataclass
class TrainConfig:
    arch: str = "raft_large"
    steps: int = 100
    batch: int = 6                 # per GPU
    iters: int = 12
    size: tuple = (384, 512)
    lr: float = 4e-4
    weight_decay: float = 1e-4
    eps: float = 1e-8
    clip: float = 1.0
    gamma: float = 0.8
    max_flow: float = 400.0
    seed: int = 0
    log_every: int = 10
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0
    resume: bool = False
    freeze_bn: bool = False
    sync_bn: bool = False          # synchronised BatchNorm statistics across DP ranks
    bucket_mb: float = 32.0
    skip_nonfinite: bool = True    # drop a step whose (all-reduced) gradient is NaN/Inf
    max_skipped: int = 10          # ... but abort after this many consecutive drops
    fault_nan_step: int = -1       # fault injection: poison the loss of this step (tests)
    # GPU, one rank: replay the whole step (fwd + bwd + clip + AdamW) as one captured graph.
    # Bitwise equal to the eager step, but measured slower on MI355X / ROCm 7 (config 5:
    # 259-265 vs 288 pairs/s: the native plans' own hipGraphs + eager PyTorch glue beat
    # one ~2000-node graph), so off by default.
    graph_step: bool = False
    graph_warmup: int = 3          # eager steps before the capture (plan build, autotune, allocator warm-up)


def _adamw(params, cfg: TrainConfig, device, capturable: bool = False):
    """AdamW; on the GPU the single-kernel (fused) implementation when this
    PyTorch build provides it -- one launch for all ~230 parameter tensors.
    ``capturable``: graph-replayable (device-side step counters, the learning
    rate a device tensor that the LR schedule updates in place)."""
    params = list(params)
    kw = dict(lr=cfg.lr, weight_decay=cfg.weight_decay, eps=cfg.eps)
    if device is not None and torch.device(device).type == "cuda":
        if capturable:
            try:
                return torch.optim.AdamW(params, fused=True, capturable=True,
                                         **dict(kw, lr=torch.tensor(cfg.lr, device=device)))
            except (RuntimeError, TypeError, ValueError):
                pass
        try:
            return torch.optim.AdamW(params, fused=True, **kw)
        except (RuntimeError, TypeError, ValueError):
            pass
    return torch.optim.AdamW(params, **kw)


class Trainer:
    # steps the host may run ahead of the GPU's non-finite flags (each step waits for the flag of
    # the step SETTLE_LAG before it, so the launch queue holds about that many steps)
    SETTLE_LAG = 1

    def __init__(self, cfg: TrainConfig, device: Optional[torch.device] = None):
        self.cfg = cfg
        self.rank, self.world, dev = dp.init_distributed()
        self.device = device or dev
        torch.manual_seed(cfg.seed)
        factory = raft_large if cfg.arch == "raft_large" else raft_small
        self.model, _ = factory(seed=cfg.seed)
        self.model = self.model.to(self.device).train()
        dp.broadcast_module(self.model)
        if cfg.sync_bn and self.world > 1:
            dp.convert_sync_batchnorm(self.model)
        self.flat_comm = dp.FlatGradComm() if self.world > 1 else None
        self.sync = dp.GradAllReducer(self.model, bucket_mb=cfg.bucket_mb, flat_comm=self.flat_comm)
        self._graph_ok = cfg.graph_step and self.device.type == "cuda" and self.world == 1
        self.opt = _adamw(self.model.parameters(), cfg, self.device, capturable=self._graph_ok)
        self._graph = None         # captured whole-step graph (see _graph_step)
        self.sched = torch.optim.lr_scheduler.OneCycleLR(
            self.opt, cfg.lr, total_steps=cfg.steps + 100, pct_start=0.05, cycle_momentum=False,
            anneal_strategy="linear")
        self.data = SyntheticFlow(size=tuple(cfg.size), seed=cfg.seed, device=self.device)
        self.step = 0
        self.skipped = 0           # total dropped steps
        self._skip_run = 0         # consecutive dropped steps
        self._pending = []         # (step, pinned non-finite flag, event): GPU steps not yet settled
        if cfg.resume and cfg.ckpt_dir and os.path.exists(os.path.join(cfg.ckpt_dir, "latest.json")):
            self.load(cfg.ckpt_dir)

    # ------------------------------------------------------------------ step
    def train_step(self, batch) -> Dict[str, float]:
        cfg = self.cfg
        if (self._graph_ok and self.step >= cfg.graph_warmup and cfg.fault_nan_step < 0
                and self.opt.defaults.get("capturable") and self._async_skip()):
            return self._graph_step(batch)
        return self._eager_step(batch)

    def _graph_step(self, batch) -> Dict[str, float]:
        """The whole step as one replayed graph: the native plans enqueue
        eagerly into the capture (fused.py), the loss, backward, clipping,
        the non-finite guard and fused AdamW (device-side step, tensor LR) are
        captured with them, so the launch queue never runs dry on Python or
        launch overhead between the pieces.  Captured once, after the eager
        warm-up steps; the batch is copied into static inputs each step."""
        if self._graph is None:
            self._capture(batch)
        for dst, src in zip(self._static_in, batch):
            dst.copy_(src)
        self._graph.replay()
        if self.cfg.skip_nonfinite:
            flag = torch.empty((), dtype=torch.float32, pin_memory=True)
            flag.copy_(self._static_bad, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._settle(keep_last=True)
            self._pending.append((self.step + 1, flag, ev))
        self.sched.step()
        self.step += 1
        return {k: v.clone() for k, v in self._static_out.items()}

    def _capture(self, batch) -> None:
        cfg = self.cfg
        self._static_in = [t.clone() for t in batch]
        torch.cuda.synchronize(self.device)
        self.opt.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            img1, img2, flow, valid = self._static_in
            preds = self.model(img1, img2, train=not cfg.freeze_bn, num_flow_updates=cfg.iters, autograd=True)
            loss, metrics = sequence_loss(preds, flow, valid, cfg.gamma, cfg.max_flow)
            with self._comm():
                loss.backward()
            gnorm = torch.nn.utils.clip_grad_norm_(self.model.parameters(), cfg.clip)
            bad = (~torch.isfinite(gnorm)).float()
            if cfg.skip_nonfinite:
                self.opt.found_inf = bad
            self.opt.step()
            self.opt.found_inf = None
        self._graph = g
        self._static_bad = bad
        self._static_out = {"loss": loss.detach(), "grad_norm": gnorm.detach(),
                            **{k: v.detach() for k, v in metrics.items()}}

    def _eager_step(self, batch) -> Dict[str, float]:
        img1, img2, flow, valid = batch
        cfg = self.cfg
        self.opt.zero_grad(set_to_none=True)
        train_bn = not cfg.freeze_bn
        preds = self.model(img1, img2, train=train_bn, num_flow_updates=cfg.iters, autograd=True)
        loss, metrics = sequence_loss(preds, flow, valid, cfg.gamma, cfg.max_flow)
        if self.step + 1 == cfg.fault_nan_step:
            loss = loss * float("nan")
        with self._comm():
            loss.backward()
        self.sync.finish()
        gnorm = torch.nn.utils.clip_grad_norm_(self.model.parameters(), cfg.clip)
        # Failure detection: the gradient is all-reduced, so every rank sees the
        # same norm and takes the same decision (no extra collective needed).
        if cfg.skip_nonfinite and self._async_skip():
            # GPU, fused AdamW: the optimizer kernel itself drops the update when
            # the norm is non-finite (found_inf), so no host sync stalls the
            # launch queue here; the host-side bookkeeping (skip counters, the
            # consecutive-skip abort) reads the flag one step later, when the
            # GPU is already busy with the next step (see _settle).
            bad = (~torch.isfinite(gnorm)).float()
            self.opt.found_inf = bad
            self.opt.step()
            self.opt.found_inf = None
            flag = torch.empty((), dtype=torch.float32, pin_memory=True)
            flag.copy_(bad, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._settle(keep_last=True)
            self._pending.append((self.step + 1, flag, ev))
        elif cfg.skip_nonfinite and not bool(torch.isfinite(gnorm)):
            self.opt.zero_grad(set_to_none=True)
            self._record_skip(self.step + 1, True)
        else:
            if cfg.skip_nonfinite:
                self._record_skip(self.step + 1, False)
            self.opt.step()
        self.sched.step()
        self.step += 1
        out = {"loss": loss.detach(), "grad_norm": gnorm.detach(), **{k: v.detach() for k, v in metrics.items()}}
        return out

    def _comm(self):
        """The fused native backward's flat-arena all-reduce, registered for
        this model only while its step's backward runs (train/fused.py:grad_comm)."""
        from . import fused

        return fused.grad_comm(self.model, self.flat_comm if self.device.type == "cuda" else None)

    def _async_skip(self) -> bool:
        return self.device.type == "cuda" and bool(getattr(self.opt, "defaults", {}).get("fused"))

    def _record_skip(self, step: int, bad: bool) -> None:
        if bad:
            self.skipped += 1
            self._skip_run += 1
            if self._skip_run > self.cfg.max_skipped:
                raise FloatingPointError(f"{self._skip_run} consecutive non-finite gradients at step {step}")
        else:
            self._skip_run = 0

    def _settle(self, keep_last: bool = False) -> None:
        """Fold the non-finite flags of finished steps into the skip counters
        (``keep_last``: leave the newest ``SETTLE_LAG`` pending steps, which may still run)."""
        while len(self._pending) > (self.SETTLE_LAG if keep_last else 0):
            step, flag, ev = self._pending.pop(0)
            ev.synchronize()
            self._record_skip(step, bool(flag.item()))

    def flush(self) -> None:
        """Settle every pending failure-detection flag (waits for the GPU)."""
        self._settle()

    def batch_for(self, step: int):
        cfg = self.cfg
        base = (step * self.world + self.rank) * cfg.batch
        return self.data.batch(list(range(base, base + cfg.batch)))

    def fit(self, log=print, stop_at: Optional[int] = None) -> Dict[str, float]:
        """Train to ``cfg.steps`` (or stop early after step ``stop_at``)."""
        cfg = self.cfg
        end = cfg.steps if stop_at is None else min(stop_at, cfg.steps)
        t0 = time.perf_counter()
        last = {}
        while self.step < end:
            batch = self.batch_for(self.step)
            m = self.train_step(batch)
            if self.step % cfg.log_every == 0 or self.step == cfg.steps:
                self.flush()
                vals = dp.all_reduce_scalars({k: float(v) for k, v in m.items()}, self.device)
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                dt = time.perf_counter() - t0
                vals.update(step=self.step, skipped=self.skipped, lr=float(self.sched.get_last_lr()[0]), elapsed_s=dt,
                            pairs_per_s=self.step * cfg.batch * self.world / dt)
                last = vals
                if self.rank == 0:
                    log(json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in vals.items()}))
            if cfg.ckpt_dir and cfg.ckpt_every and self.step % cfg.ckpt_every == 0:
                self.save(cfg.ckpt_dir)
        if cfg.ckpt_dir:
            self.save(cfg.ckpt_dir)
        return last

    # ------------------------------------------------------------ checkpoint
    def save(self, d: str) -> None:
        self.flush()
        if self.rank != 0:
            if dp.is_dist():
                torch.distributed.barrier()
            return
        os.makedirs(d, exist_ok=True)
        name = f"step_{self.step}"
        ckpt.save_msgpack(self.model, os.path.join(d, name + ".msgpack"))
        torch.save({"opt": self.opt.state_dict(), "sched": self.sched.state_dict(), "step": self.step,
                    "skipped": self.skipped},
                   os.path.join(d, name + ".opt.pt"))
        with open(os.path.join(d, "latest.json"), "w") as f:
            json.dump({"step": self.step, "weights": name + ".msgpack", "opt": name + ".opt.pt",
                       "config": {k: (list(v) if isinstance(v, tuple) else v) for k, v in asdict(self.cfg).items()}}, f)
        if dp.is_dist():
            torch.distributed.barrier()

    def load(self, d: str) -> None:
        with open(os.path.join(d, "latest.json")) as f:
            meta = json.load(f)
        ckpt.load_variables_into(self.model, ckpt.load_msgpack(os.path.join(d, meta["weights"])), strict=True)
        st = torch.load(os.path.join(d, meta["opt"]), map_location=self.device, weights_only=True)
        self.opt.load_state_dict(st["opt"])
        self.sched.load_state_dict(st["sched"])
        self.step = int(st["step"])
        self.skipped = int(st.get("skipped", 0))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    for f_ in TrainConfig.__dataclass_fields__.values():
        if f_.name == "size":
            ap.add_argument("--size", type=int, nargs=2, default=list(f_.default))
        elif f_.type in ("bool", bool):
            ap.add_argument(f"--{f_.name.replace('_', '-')}", action=argparse.BooleanOptionalAction,
                            default=f_.default)
        else:
            typ = {"int": int, "float": float, "str": str}.get(str(f_.type).replace("Optional[str]", "str"), str)
            ap.add_argument(f"--{f_.name.replace('_', '-')}", type=typ if f_.default is not None else str,
                            default=f_.default)
    a = ap.parse_args(argv)
    cfg = TrainConfig(**{k: (tuple(v) if k == "size" else v) for k, v in vars(a).items()})
    tr = Trainer(cfg)
    tr.fit()
    if dp.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
