"""Context parallelism of the all-pairs correlation volume ("corr-volume CP").

The reference materialises the full (h*w) x (h*w) volume on one device
(``CorrBlock._compute_corr_volume``, ``jax_raft/model.py:472-481``; pyramid
``:418-446``): O(P^2) memory, P = H*W/64.  One MI355X (288 GB HBM3E) holds the
bf16 pyramid up to about 4K-5K frames; an 8K pair needs ~714 GB.  This module
shards the volume over the ranks of a process group:

* every rank runs the O(P) encoders on the full frames (replicated; they are
  a small share of the memory at these sizes);
* rank ``r`` owns a contiguous slab of QUERY rows ``[r0, r1)`` of ``fmap1`` and
  builds only that slab's pyramid against all of ``fmap2``
  (:func:`~jax_raft_amd.ops.functional.build_pyramid_queries`: on the GPU the
  MFMA corr kernel with ``nq`` = slab pixels): memory ``P * P_r`` per rank;
* a query's lookup window only touches that query's own correlation maps, so
  every rank looks up its own queries with NO communication (the lookup kernel
  with ``nq`` queries against full-size maps);
* per iteration the (B, h_r, w, L*(2r+1)^2) features (bf16 on the GPU:
  4.6 MB per pair at 440x1024, ~0.3 GB at 8K) are all-gathered along rows
  (RCCL over xGMI: one all-gather per iteration, every link busy), and the
  update block runs replicated on the gathered features.  Identical inputs and
  deterministic kernels keep the recurrent state identical on every rank, so
  no further synchronisation is needed.

On the GPU the wrapper runs the native engine in context-parallel mode
(``RaftEngine(cp_group=...)``, runtime/engine.py): each rank's plan holds its
slab's pyramid (the MFMA corr kernel with ``nq`` = slab pixels, row-major
levels), segment 1 of every iteration runs the slab lookups, the engine
all-gathers the features into the full map, and segment 3 runs the rest of the
iteration -- all kernels launched from C++ (``Plan.run_segment``).  On the CPU
(and as the executable specification) the module path below does the same with
PyTorch ops.

Inference only (``torch.no_grad``): training resolutions (368x496 crops) never
need the volume sharded, and a CP backward would need the encoder gradients
all-reduced over the query slabs.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..models import reference as R
from ..ops import functional as F


def row_slabs(h: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous near-equal partition of ``h`` query rows over ``world`` ranks
    (sizes differ by at most one; the first ``h % world`` slabs get the extra row)."""
    assert 1 <= world <= h, f"context parallelism needs at least one feature row per rank ({h} rows, {world} ranks)"
    base, extra = divmod(h, world)
    out, r0 = [], 0
    for r in range(world):
        n = base + (1 if r < extra else 0)
        out.append((r0, r0 + n))
        r0 += n
    return out


def pyramid_bytes(B: int, H: int, W: int, num_levels: int = 4, dtype_bytes: int = 2,
                  query_rows: Optional[int] = None) -> int:
    """Bytes of the correlation pyramid of B pairs at image size H x W (bf16 by
    default) when this rank holds ``query_rows`` of the H/8 feature rows (all by default)."""
    h, w = H // 8, W // 8
    q = (h if query_rows is None else query_rows) * w
    total, hl, wl = 0, h, w
    for _ in range(num_levels):
        total += hl * wl
        hl, wl = hl // 2, wl // 2
    return B * q * total * dtype_bytes


def gather_rows(x: torch.Tensor, slabs: Sequence[Tuple[int, int]], group=None) -> torch.Tensor:
    """All-gather row slabs ``x`` (B, h_r, w, C) of every rank into (B, h, w, C).
    Slabs may differ in height by one: each is zero-padded to the tallest and
    trimmed after the collective (one all-gather, equal message sizes)."""
    world = len(slabs)
    if world == 1:
        return x
    hmax = max(r1 - r0 for r0, r1 in slabs)
    B, hr, w, C = x.shape
    if hr < hmax:
        pad = x.new_zeros(B, hmax, w, C)
        pad[:, :hr] = x
    else:
        pad = x.contiguous()
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:, : r1 - r0] for p, (r0, r1) in zip(parts, slabs)], dim=1)


class ContextParallelRAFT:
    """Inference wrapper running ``model`` with its correlation volume sharded by
    query rows over ``group`` (default: the default process group; a single
    process without a group is the degenerate one-slab case).

    ``cp(image1, image2, num_flow_updates)`` returns the same (N, B, H, W, 2)
    flows as ``model.apply`` on every rank."""

    def __init__(self, model, group=None, **engine_kw):
        self.model = model
        self.group = group
        self.engine_kw = engine_kw   # native engine options on the GPU (e.g. precision="fp32")
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1

    def slabs(self, h: int) -> List[Tuple[int, int]]:
        return row_slabs(h, self.world)

    @torch.no_grad()
    def __call__(self, image1: torch.Tensor, image2: torch.Tensor, num_flow_updates: int = 12,
                 return_all_iters: bool = True) -> torch.Tensor:
        m = self.model
        B, H, W, _ = image1.shape
        assert tuple(image2.shape) == tuple(image1.shape), "input images should have the same shape"
        assert H % 8 == 0 and W % 8 == 0, "input image H and W should be divisible by 8"
        if image1.is_cuda:
            eng = m.engine(image1.device, cp_group=True if self.group is None else self.group, **self.engine_kw)
            return eng.forward(image1, image2, num_flow_updates, return_all_iters=return_all_iters)
        fmaps = m.feature_encoder(torch.cat([image1, image2], dim=0), False)
        fmap1, fmap2 = torch.chunk(fmaps, 2, dim=0)
        h, w = fmap1.shape[1], fmap1.shape[2]
        cb = m.corr_block
        min_sz = 2 * (2 ** (cb.num_levels - 1))
        assert h >= min_sz and w >= min_sz, (
            f"Feature maps are too small to be down-sampled by the correlation pyramid: need >= {min_sz}, got {(h, w)}")
        slabs = self.slabs(h)
        r0, r1 = slabs[self.rank]
        pyr = F.build_pyramid_queries(fmap1[:, r0:r1].contiguous(), fmap2.contiguous(), cb.num_levels)
        del fmaps, fmap1, fmap2
        ctx = m.context_encoder(image1, False)
        hs = m.update_block.hidden_state_size
        hidden = torch.tanh(ctx[..., :hs])
        context = torch.relu(ctx[..., hs:])
        coords0 = R.make_coords_grid(B, h, w, device=image1.device)
        coords1 = coords0.clone()
        preds = []
        for it in range(num_flow_updates):
            local = F.index_pyramid(pyr, coords1[:, r0:r1].contiguous(), cb.radius)
            corr = gather_rows(local, slabs, self.group)
            hidden, delta = m.update_block(hidden, context, corr, coords1 - coords0, False)
            coords1 = coords1 + delta
            if not return_all_iters and it + 1 < num_flow_updates:
                continue
            up_mask = None if m.mask_predictor is None else m.mask_predictor(hidden, False)
            preds.append(R.upsample_flow(coords1 - coords0, up_mask))
        return torch.stack(preds, dim=0)
