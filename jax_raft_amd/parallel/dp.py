"""Data parallelism over RCCL (``torch.distributed`` backend ``"nccl"`` on ROCm
is RCCL; ``"gloo"`` is used for CPU processes and tests).

The reference is single-device (zero collective call
sites).  Here, one process per GPU:

* :func:`init_distributed` -- env-driven (torchrun: RANK/WORLD_SIZE/LOCAL_RANK,
  MASTER_ADDR/PORT), binds the local GPU, fail-fast timeouts;
* :func:`broadcast_module` -- params + BN batch_stats from rank 0 (21 MB for
  raft_large);
* :class:`GradAllReducer` -- bucketed gradient all-reduce launched from
  post-accumulate-grad hooks while backward is still running (overlap), one
  flat fp32 buffer per bucket.  Buckets default to 32 MB: raft_large's whole
  gradient (5.26 M params = 21 MB) is a single ring all-reduce over xGMI
  (~0.25 ms on 8 GPUs), small enough that more buckets only add launch latency;
  the bucket size is a knob for larger models;
* :func:`shard` / :func:`gather` -- batched-inference sharding helpers;
* :func:`all_reduce_scalars` -- metric reduction.
"""
from __future__ import annotations

import datetime
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import knobs


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> Tuple[int, int, torch.device]:
    """Initialise the default process group from torchrun-style env vars.

    Returns ``(rank, world_size, device)``.  Single-process runs (no
    WORLD_SIZE) return ``(0, 1, device)`` without creating a group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or knobs.get("JR_DIST_BACKEND")
    # JR_SHARE_GPU=1: ranks share the visible GPUs round-robin over gloo (a
    # rehearsal of >1 rank on a 1-GPU box; RCCL refuses two ranks per GPU)
    share = knobs.flag("JR_SHARE_GPU") and torch.cuda.is_available()
    use_gpu = torch.cuda.is_available() and (backend != "gloo" or share)
    if share:
        backend = "gloo"
        local = local % torch.cuda.device_count()
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if world > 1 and not is_dist():
        backend = backend or ("nccl" if use_gpu else "gloo")
        # fail fast: a rank that dies or hangs in a collective tears the job
        # down after ``timeout_s`` instead of blocking every other rank forever
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank(), world_size(), device


def convert_sync_batchnorm(module: torch.nn.Module, group=True) -> int:
    """Switch every BatchNorm of ``module`` (raft_large's context encoder: 15
    layers, 1,440 channels) to synchronised statistics over ``group`` (``True``
    = the default process group); returns the number of layers converted.

    Cost: one all-reduce of 2C+1 floats per BN layer per forward (11.5 KB in
    total for raft_large), latency- not bandwidth-bound on xGMI.  The default
    policy stays per-replica BN (like the original RAFT recipe, which freezes BN
    after the first stage); SyncBN is the choice for small per-GPU batches."""
    from ..models.layers import BatchNorm

    n = 0
    for m in module.modules():
        if isinstance(m, BatchNorm):
            m.sync_group = group
            n += 1
    return n


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Broadcast parameters and buffers (BN running stats) from ``src``."""
    if not is_dist():
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)
            t.add_(0)  # bump the version counter (.data writes do not): invalidates cached weight packs


class FlatGradComm:
    """Asynchronous averaging of flat gradient buffers for the fused native
    training step (:class:`jax_raft_amd.train.fused.FusedModel`), whose
    gradients live in three flat fp32 arenas (refinement loop, feature
    encoder, context encoder).  :meth:`start` launches an all-reduce of one
    buffer on the communicator right when the backward has produced it -- the
    loop's (~13 MB for raft_large) overlaps the encoders' backward -- with no
    per-bucket concatenation; :meth:`finish` waits and divides by the world
    size.  The parameters are then marked as reduced so the hook-based
    :class:`GradAllReducer` skips them."""

    def __init__(self, group=None):
        self.group = group
        self.world = world_size()
        self._works: List[Tuple[object, torch.Tensor]] = []
        self.reduced_ids: set = set()

    def start(self, flat: torch.Tensor) -> None:
        if self.world > 1:
            self._works.append((dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True), flat))

    def finish(self, params=()) -> None:
        for work, flat in self._works:
            work.wait()
            flat.div_(self.world)
        self._works = []
        self.reduced_ids = {id(p) for p in params}


class GradAllReducer:
    """Bucketed, backward-overlapped gradient averaging.

    Usage::

        sync = GradAllReducer(model)
        loss.backward()
        sync.finish()            # waits for the in-flight buckets, writes averaged grads
    """

    def __init__(self, module: torch.nn.Module, bucket_mb: float = 32.0, group=None,
                 flat_comm: Optional[FlatGradComm] = None):
        self.group = group
        self.flat_comm = flat_comm
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.world = world_size()
        cap = int(bucket_mb * 1024 * 1024 / 4)
        # buckets in reverse registration order ~ the order gradients become ready
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel()
            if size >= cap:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        self._pending = [0] * len(self.buckets)
        self._works: Dict[int, Tuple[object, torch.Tensor]] = {}
        self._hooks = []
        if self.world > 1:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset()

    def _reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._works = {}

    def _prereduced(self, p) -> bool:
        return self.flat_comm is not None and id(p) in self.flat_comm.reduced_ids

    def _on_grad(self, p: torch.nn.Parameter):
        if self._prereduced(p):
            return  # averaged by the fused step's flat-buffer all-reduce
        b = self._bucket_of[id(p)]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def _launch(self, b: int):
        ps = [p for p in self.buckets[b] if not self._prereduced(p)]
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]
        flat = torch.cat([g.reshape(-1).float() for g in grads])
        work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._works[b] = (work, flat)

    def finish(self):
        """Complete every bucket (also those with unused parameters) and write
        the averaged gradients back."""
        if self.world == 1:
            return
        for b in range(len(self.buckets)):
            if b not in self._works and not all(self._prereduced(p) for p in self.buckets[b]):
                self._launch(b)
        for b, (work, flat) in self._works.items():
            work.wait()
            flat.div_(self.world)
            off = 0
            for p in [p for p in self.buckets[b] if not self._prereduced(p)]:
                n = p.numel()
                g = flat[off:off + n].view_as(p).to(p.dtype)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n
        if self.flat_comm is not None:
            self.flat_comm.reduced_ids = set()
        self._reset()

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def all_reduce_scalars(values: Dict[str, float], device, average: bool = True) -> Dict[str, float]:
    if not is_dist():
        return dict(values)
    keys = sorted(values)
    t = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    if average:
        t /= world_size()
    return {k: v for k, v in zip(keys, t.tolist())}


def shard(x: torch.Tensor, r: Optional[int] = None, w: Optional[int] = None) -> torch.Tensor:
    """Contiguous batch shard of rank ``r`` (equal shards; batch % world == 0)."""
    r = rank() if r is None else r
    w = world_size() if w is None else w
    assert x.shape[0] % w == 0, f"batch {x.shape[0]} not divisible by world size {w}"
    n = x.shape[0] // w
    return x[r * n:(r + 1) * n]


def gather(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """All-gather equal shards along ``dim`` (batched-inference results)."""
    if not is_dist():
        return x
    parts = [torch.empty_like(x) for _ in range(world_size())]
    dist.all_gather(parts, x.contiguous())
    return torch.cat(parts, dim=dim)
