"""Golden pure-PyTorch RAFT primitives (exact reference semantics, NHWC, fp32).

This module is the numerical oracle for every HIP kernel in ``csrc/`` and the
whole CPU execution path (BASELINE config 1).  Each function reproduces the
behaviour of one primitive of the reference JAX/Flax model; the reference
line ranges are cited per function.  Implementations deliberately use plain
PyTorch indexing / ``F.conv2d`` so they can be cross-checked against
independent PyTorch primitives (``F.grid_sample``, ``F.avg_pool2d``,
``F.unfold``, ``F.interpolate``) in ``tests/test_reference.py``.

All tensors are channels-last (NHWC), like the reference.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

__all__ = [
    "grid_sample",
    "make_coords_grid",
    "resize_with_aligned_corners",
    "upsample_flow",
    "conv2d_nhwc",
    "instance_norm_nhwc",
    "batch_norm_nhwc",
    "corr_volume",
    "build_pyramid",
    "index_pyramid",
    "neighborhood_offsets",
]


def grid_sample(img: torch.Tensor, grid: torch.Tensor) -> torch.Tensor:
    """Bilinear sampling at *pixel* coordinates with zero padding.

    Reference: ``jax_raft/model.py:24-34`` (``map_coordinates(order=1,
    mode='constant')`` vmapped over batch and channel).  ``grid[..., 0]`` is
    x (column) and ``grid[..., 1]`` is y (row).  Each of the 4 taps that falls
    outside the image contributes 0; in-bounds taps keep their weight (no
    renormalisation).

    img: (N, H, W, C); grid: (N, h, w, 2) -> (N, h, w, C)
    """
    assert img.shape[-3] > 1
    assert grid.ndim == 4 and grid.shape[-1] == 2
    n, H, W, C = img.shape
    x = grid[..., 0]
    y = grid[..., 1]
    x0 = torch.floor(x)
    y0 = torch.floor(y)
    wx1 = x - x0
    wy1 = y - y0
    wx0 = 1.0 - wx1
    wy0 = 1.0 - wy1
    x0i = x0.long()
    y0i = y0.long()
    flat = img.reshape(n, H * W, C)
    out = torch.zeros(grid.shape[:-1] + (C,), dtype=img.dtype, device=img.device)
    bidx = torch.arange(n, device=img.device).view(n, 1, 1)
    for dy, wy in ((0, wy0), (1, wy1)):
        for dx, wx in ((0, wx0), (1, wx1)):
            xi = x0i + dx
            yi = y0i + dy
            valid = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
            lin = (yi.clamp(0, H - 1) * W + xi.clamp(0, W - 1))
            vals = flat[bidx.expand_as(lin), lin]  # (n, h, w, C)
            wgt = (wx * wy * valid.to(img.dtype)).unsqueeze(-1)
            out = out + wgt * vals
    return out


def make_coords_grid(batch_size: int, h: int, w: int, device=None) -> torch.Tensor:
    """``coords[b, y, x] = (x, y)`` float32.  Reference ``model.py:37-40``."""
    ys, xs = torch.meshgrid(
        torch.arange(h, device=device, dtype=torch.float32),
        torch.arange(w, device=device, dtype=torch.float32),
        indexing="ij",
    )
    coords = torch.stack([xs, ys], dim=-1)
    return coords.unsqueeze(0).repeat(batch_size, 1, 1, 1)


def _linear_resize_axis(x: torch.Tensor, axis: int, out_size: int) -> torch.Tensor:
    in_size = x.shape[axis]
    if in_size == out_size:
        return x
    # x_in = x_out * (in - 1) / (out - 1)   (align_corners=True)
    pos = torch.arange(out_size, dtype=torch.float64, device=x.device) * (
        (in_size - 1.0) / (out_size - 1.0)
    )
    i0 = torch.floor(pos).long().clamp(0, in_size - 1)
    i1 = (i0 + 1).clamp(max=in_size - 1)
    w1 = (pos - i0.double()).to(x.dtype)
    w0 = 1.0 - w1
    shape = [1] * x.ndim
    shape[axis] = out_size
    a = x.index_select(axis, i0)
    b = x.index_select(axis, i1)
    return a * w0.view(shape) + b * w1.view(shape)


def resize_with_aligned_corners(
    image: torch.Tensor, shape: Tuple[int, ...], method: str = "bilinear", antialias: bool = True
) -> torch.Tensor:
    """Bilinear resize emulating ``align_corners=True``.

    Reference ``model.py:43-66`` (``jax.image.scale_and_translate`` with
    ``scale=(out-1)/(in-1)``, ``translation=0.5-scale/2``).  Only the dims whose
    size changes are resized.  Only upsampling is exercised by RAFT; with
    ``antialias`` the triangle kernel is identical to plain linear
    interpolation for upsampling, so the flag does not change the result.
    """
    assert method == "bilinear", "currently only bilinear interpolation is supported"
    assert len(shape) == image.ndim
    out = image
    for axis in range(image.ndim):
        if image.shape[axis] != shape[axis]:
            out = _linear_resize_axis(out, axis, shape[axis])
    return out


def upsample_flow(flow: torch.Tensor, up_mask: Optional[torch.Tensor] = None, factor: int = 8) -> torch.Tensor:
    """x8 flow upsampling (bilinear when ``up_mask is None``, else convex).

    Reference ``model.py:69-98``.  Convex mode: mask channel index is
    ``k*64 + a*8 + b`` (k = 3x3 neighbour, row-major; a = sub-row; b = sub-col),
    softmax over k, weighted sum of the zero-padded 3x3 neighbourhood of
    ``factor*flow``, then pixel shuffle to (B, 8h, 8w, C).
    """
    B, h, w, C = flow.shape
    nh, nw = h * factor, w * factor
    if up_mask is None:
        up = resize_with_aligned_corners(flow, (B, nh, nw, C), method="bilinear", antialias=False)
        return factor * up
    assert up_mask.shape == (B, h, w, 9 * factor * factor)
    flow = flow.float()
    m = up_mask.float().reshape(B, h, w, 9, factor, factor)
    m = torch.softmax(m, dim=3)
    fp = F.pad((factor * flow).permute(0, 3, 1, 2), (1, 1, 1, 1))  # (B, C, h+2, w+2)
    neigh = []
    for ky in range(3):
        for kx in range(3):
            neigh.append(fp[:, :, ky:ky + h, kx:kx + w])
    neigh = torch.stack(neigh, dim=2)  # (B, C, 9, h, w)
    neigh = neigh.permute(0, 3, 4, 1, 2)  # (B, h, w, C, 9)
    # out[n,y,x,c,a,b] = sum_k m[n,y,x,k,a,b] * neigh[n,y,x,c,k]
    # as broadcast multiply + reduction: the einsum lowers to B*h*w tiny
    # (C x 9) @ (9 x 64) batched GEMMs, which the GPU library runs ~5x slower
    # than this memory-bound form (training profile, profiles/r1_train_kernel_breakdown_v1.txt)
    mm = m.reshape(B, h, w, 1, 9, factor * factor)
    up = (neigh.unsqueeze(-1) * mm).sum(dim=4)  # (B, h, w, C, 64)
    up = up.reshape(B, h, w, C, factor, factor).permute(0, 1, 4, 2, 5, 3).reshape(B, nh, nw, C)
    return up


def conv2d_nhwc(
    x: torch.Tensor,
    kernel: torch.Tensor,
    bias: Optional[torch.Tensor],
    stride: Tuple[int, int] = (1, 1),
    padding: Tuple[int, int] = (0, 0),
) -> torch.Tensor:
    """NHWC conv with an HWIO kernel (Flax layout), symmetric explicit padding.

    Reference: ``flax.linen.Conv`` as used by ``model.py:101-159`` (padding
    ``(k-1)//2`` per dim from ``model.py:137-141``) and the plain convs at
    ``model.py:304-310,347-349,394``.
    """
    w = kernel.permute(3, 2, 0, 1)  # HWIO -> OIHW
    y = F.conv2d(x.permute(0, 3, 1, 2), w, bias, stride=stride, padding=padding)
    return y.permute(0, 2, 3, 1)


def conv2d_nhwc_gemm(
    x: torch.Tensor,
    kernel: torch.Tensor,
    bias: Optional[torch.Tensor],
    stride: Tuple[int, int] = (1, 1),
    padding: Tuple[int, int] = (0, 0),
) -> torch.Tensor:
    """:func:`conv2d_nhwc` as explicit im2col + one fp32 GEMM (the same sum, no
    convolution library): the golden conv of GPU-side references (ops/functional.py
    ``golden_ops``), which must not depend on a conv library's algorithm search."""
    N, H, W, C = x.shape
    kh, kw, _, co = kernel.shape
    cols = F.unfold(x.permute(0, 3, 1, 2), (kh, kw), padding=padding, stride=stride)   # (N, C*kh*kw, L)
    OH = (H + 2 * padding[0] - kh) // stride[0] + 1
    OW = (W + 2 * padding[1] - kw) // stride[1] + 1
    w = kernel.permute(2, 0, 1, 3).reshape(C * kh * kw, co)          # unfold order: (c, i, j)
    y = torch.matmul(cols.transpose(1, 2), w)                        # (N, L, co)
    if bias is not None:
        y = y + bias
    return y.reshape(N, OH, OW, co)


def instance_norm_nhwc(x: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """Flax ``nn.InstanceNorm(epsilon=1e-5, use_bias=False, use_scale=False)``
    (``model.py:706-707``): per (n, c) over H, W, biased variance.  Statistics
    in fp32 whatever the input dtype."""
    if torch.is_grad_enabled() and x.requires_grad:
        return _InstanceNormNHWC.apply(x, eps)
    xf = x.to(torch.promote_types(x.dtype, torch.float32))
    var, mean = torch.var_mean(xf, dim=(1, 2), unbiased=False, keepdim=True)
    return ((xf - mean) * torch.rsqrt(var + eps)).to(x.dtype)


class _InstanceNormNHWC(torch.autograd.Function):
    """Instance norm with a closed-form backward: saves only the input and the
    per-(n, c) statistics (no fp32 copies of the activation), and computes
    dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) in one expression chain
    instead of autograd's trace through the mean / square / rsqrt graph."""

    @staticmethod
    def forward(ctx, x, eps: float):
        xf = x.to(torch.promote_types(x.dtype, torch.float32))
        var, mean = torch.var_mean(xf, dim=(1, 2), unbiased=False, keepdim=True)
        rstd = torch.rsqrt(var + eps)
        ctx.save_for_backward(x, mean, rstd)
        return ((xf - mean) * rstd).to(x.dtype)

    @staticmethod
    def backward(ctx, gy):
        x, mean, rstd = ctx.saved_tensors
        ft = torch.promote_types(x.dtype, torch.float32)
        g = gy.to(ft)
        xhat = (x.to(ft) - mean) * rstd
        gm = g.mean(dim=(1, 2), keepdim=True)
        gxm = (g * xhat).mean(dim=(1, 2), keepdim=True)
        return (rstd * (g - gm - xhat * gxm)).to(x.dtype), None


def batch_norm_nhwc(
    x: torch.Tensor,
    scale: torch.Tensor,
    bias: torch.Tensor,
    mean: torch.Tensor,
    var: torch.Tensor,
    train: bool,
    eps: float = 1e-5,
    momentum: float = 0.99,
    sync_group=None,
):
    """Flax ``nn.BatchNorm`` (defaults: momentum 0.99, eps 1e-5) as used by the
    raft_large context encoder (``model.py:147,157,711``).

    Returns ``(y, new_mean, new_var)``; in eval mode the running statistics are
    used and returned unchanged.  ``sync_group`` (a torch.distributed group, or
    ``True`` for the default group) makes it a synchronised BatchNorm over the
    data-parallel ranks (Flax ``axis_name=`` semantics): the batch statistics
    come from one differentiable all-reduce of (sum x, sum x^2, count) per
    layer, so every rank normalises with -- and back-propagates through -- the
    global-batch mean/variance.
    """
    dt = x.dtype
    x = x.float()
    if train:
        if sync_group is not None and torch.distributed.is_available() and torch.distributed.is_initialized():
            from torch.distributed.nn.functional import all_reduce as _ar

            n = torch.full((1,), float(x.numel() // x.shape[-1]), device=x.device)
            packed = torch.cat([x.sum(dim=(0, 1, 2)), (x * x).sum(dim=(0, 1, 2)), n])
            packed = _ar(packed) if sync_group is True else _ar(packed, group=sync_group)
            C = x.shape[-1]
            tot = packed[2 * C]
            bmean = packed[:C] / tot
            bvar = packed[C:2 * C] / tot - bmean * bmean
        else:
            bmean = x.mean(dim=(0, 1, 2))
            bvar = (x * x).mean(dim=(0, 1, 2)) - bmean * bmean
        bvar = bvar.clamp_min(0.0)
        new_mean = momentum * mean + (1.0 - momentum) * bmean.detach()
        new_var = momentum * var + (1.0 - momentum) * bvar.detach()
        m, v = bmean, bvar
    else:
        new_mean, new_var = mean, var
        m, v = mean, var
    y = (x - m) * torch.rsqrt(v + eps) * scale + bias
    return y.to(dt), new_mean, new_var


def corr_volume(fmap1: torch.Tensor, fmap2: torch.Tensor) -> torch.Tensor:
    """All-pairs correlation ``fmap1 @ fmap2^T / sqrt(C)`` -> (B, h, w, h, w).

    Reference ``CorrBlock._compute_corr_volume``, ``model.py:472-481``.
    """
    B, h, w, C = fmap1.shape
    f1 = fmap1.reshape(B, h * w, C)
    f2 = fmap2.reshape(B, h * w, C)
    corr = torch.matmul(f1, f2.transpose(1, 2))
    return corr.reshape(B, h, w, h, w) / math.sqrt(C)


def build_pyramid(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int) -> List[torch.Tensor]:
    """Correlation pyramid: level 0 is the (B*h*w, h, w) volume, each further
    level a 2x2/stride-2 VALID (floor) average pool.  Reference
    ``CorrBlock.build_pyramid``, ``model.py:418-446``.  Levels are returned as
    (B*h*w, h_l, w_l) (channel dim of size 1 squeezed)."""
    assert fmap1.shape == fmap2.shape, "Input feature maps should have the same shapes"
    min_fmap_size = 2 * (2 ** (num_levels - 1))
    assert not any(s < min_fmap_size for s in fmap1.shape[-3:-1]), (
        "Feature maps are too small to be down-sampled by the correlation pyramid. "
        f"H and W of feature maps should be at least {min_fmap_size}; got: {tuple(fmap1.shape[-3:-1])}. "
        f"Input image dimensions should be at least 8 * {min_fmap_size} = {8 * min_fmap_size}."
    )
    return build_pyramid_queries(fmap1, fmap2, num_levels)


def build_pyramid_queries(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int) -> List[torch.Tensor]:
    """:func:`build_pyramid` for a subset of query pixels: ``fmap1`` (B, hq, wq, C)
    holds the queries (e.g. a slab of query rows, context parallelism), ``fmap2``
    (B, h, w, C) every target pixel.  Levels are (B*hq*wq, h_l, w_l); each query's
    maps are exactly its rows of the full pyramid (pooling acts on target dims only)."""
    B, hq, wq, C = fmap1.shape
    _, h, w, _ = fmap2.shape
    f1 = fmap1.reshape(B, hq * wq, C)
    f2 = fmap2.reshape(B, h * w, C)
    vol = (torch.matmul(f1, f2.transpose(1, 2)) / math.sqrt(C)).reshape(B * hq * wq, h, w)
    pyr = [vol]
    for _ in range(num_levels - 1):
        hh, ww = vol.shape[-2] // 2, vol.shape[-1] // 2
        vol = vol[:, : 2 * hh, : 2 * ww].reshape(vol.shape[0], hh, 2, ww, 2).mean(dim=(2, 4))
        pyr.append(vol)
    return pyr


def neighborhood_offsets(radius: int, device=None) -> torch.Tensor:
    """``delta[i, j] = (i - r, j - r)`` -- x gets the slow index.  ``model.py:451-455``."""
    d = torch.linspace(-radius, radius, 2 * radius + 1, device=device)
    di, dj = torch.meshgrid(d, d, indexing="ij")
    return torch.stack([di, dj], dim=-1)  # (2r+1, 2r+1, 2)


def index_pyramid(pyramid: Sequence[torch.Tensor], coords: torch.Tensor, radius: int) -> torch.Tensor:
    """Radius-r bilinear lookup of every pyramid level around ``coords / 2^l``.

    Reference ``CorrBlock.index_pyramid``, ``model.py:448-470``.  Output
    channel = ``l*(2r+1)^2 + i*(2r+1) + j`` with x-offset ``i-r`` and y-offset
    ``j-r``.  coords: (B, h, w, 2) -> (B, h, w, L*(2r+1)^2)
    """
    B, h, w, _ = coords.shape
    side = 2 * radius + 1
    delta = neighborhood_offsets(radius, coords.device).reshape(1, side, side, 2)
    c = coords.reshape(B * h * w, 1, 1, 2)
    out = []
    for vol in pyramid:
        sc = c + delta
        s = grid_sample(vol.unsqueeze(-1), sc).reshape(B, h, w, side * side)
        out.append(s)
        c = c / 2
    return torch.cat(out, dim=-1)
