"""Autograd Functions over the native gfx950 kernels (the GPU training path).

=====================  ==========================================  ==========================================
op                     forward                                     backward
=====================  ==========================================  ==========================================
conv2d (NHWC, HWIO)    implicit-GEMM MFMA kernel                   dX: same kernel, flipped/transposed weights,
                                                                   input-dilation mode for strided convs;
                                                                   dW: native im2col + library GEMM; db: sum
corr pyramid           MFMA GEMM with fused 2x2 pooling (fp32)     pooling adjoint + library GEMMs
pyramid lookup         radius-r bilinear gather kernel             native scatter kernel (no atomics)
=====================  ==========================================  ==========================================

Everything else in the RAFT graph (norms, gates, concat, upsampling, loss)
is PyTorch glue on the framework layer.  ``coords`` never receive a gradient
(``stop_gradient`` at ``jax_raft/model.py:498``).
"""
from __future__ import annotations

import math
import weakref
from typing import List, Sequence, Tuple

import torch

from . import native as nat

BF16 = torch.bfloat16


def _pad_channels(x: torch.Tensor, c8: int) -> torch.Tensor:
    """bf16 contiguous NHWC with the channel dim zero-padded to ``c8``."""
    C = x.shape[-1]
    if C == c8 and x.dtype == BF16 and x.is_contiguous():
        return x
    out = torch.zeros(x.shape[:-1] + (c8,), dtype=BF16, device=x.device)
    out[..., :C] = x
    return out


def _log2_stride(s: int) -> int:
    if s not in (1, 2, 4, 8):
        raise NotImplementedError(f"native conv backward supports strides 1/2/4/8, got {s}")
    return int(math.log2(s))


_SPEC_CACHE: dict = {}
_SPEC_CACHE_MAX = 512


def _cached_spec(kernel: torch.Tensor, bias, stride, padding, cin8: int, transposed: bool):
    """Packed-weight ConvSpec, reused while the parameter is unchanged.

    The update block's weights are shared by every refinement iteration, so a
    12-iteration training step would otherwise re-pack each of them 12x in the
    forward and 12x (flipped) in the backward.  The key is the parameter's
    identity (weakref-checked) and its in-place ``_version`` counter, which
    every optimizer step bumps, so a stale pack is never reused."""
    key = (id(kernel), kernel._version, None if bias is None else (id(bias), bias._version),
           tuple(stride), tuple(padding), cin8, transposed, kernel.device)
    hit = _SPEC_CACHE.get(key)
    if hit is not None and hit[0]() is kernel and (bias is None or hit[1]() is bias):
        return hit[2]
    kh, kw, cin, cout = kernel.shape
    if transposed:
        # dX = conv(dilate_s(dY), flip(W)^T), padding k-1-p
        wt = torch.flip(kernel.detach().float(), dims=(0, 1)).permute(0, 1, 3, 2).contiguous()
        spec = nat.make_spec(wt, torch.zeros(cin, device=kernel.device), (1, 1),
                             (kh - 1 - padding[0], kw - 1 - padding[1]), cin8=cin8, device=kernel.device)
    else:
        spec = nat.make_spec(kernel.detach(), bias.detach(), tuple(stride), tuple(padding), cin8=cin8,
                             device=kernel.device)
    if len(_SPEC_CACHE) >= _SPEC_CACHE_MAX:
        _SPEC_CACHE.clear()
    _SPEC_CACHE[key] = (weakref.ref(kernel), None if bias is None else weakref.ref(bias), spec)
    return spec


_WGRAD_TILES_PER_CU = 2   # split-K target of the weight-gradient GEMMs: ~2 tiles per CU


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b (bf16 operands) with the product kept in fp32 (no bf16 rounding of dW)."""
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError):
        return torch.mm(a.float(), b.float())


def _wgrad_gemm(gy2: torch.Tensor, col: torch.Tensor, cout: int) -> torch.Tensor:
    """dW = im2col(X)^T @ dY as (kpad, cout) fp32, i.e. already the HWIO
    kernel layout (no transpose copy).  A long-K GEMM (K = batch pixels) with
    a small output, i.e. only a handful of output tiles for 256 CUs (the
    encoder's 576 x 64 weight grads ran as 9 library tiles, ~550 us each):
    split K into S batches so there are ~2 tiles per CU, bf16 MFMA with fp32
    partials, then reduce the partials in fp32."""
    M, cout8 = gy2.shape
    kpad = col.shape[1]
    tiles = -(-cout // 64) * -(-kpad // 64)
    S = 1
    while S < 64 and tiles * S * 2 <= _WGRAD_TILES_PER_CU * nat.NUM_CUS and M % (2 * S) == 0 and M // (2 * S) >= 1024:
        S *= 2
    if S == 1 or not gy2.is_cuda:
        return _mm_f32(col.t(), gy2[:, :cout])
    a = col.reshape(S, M // S, kpad).transpose(1, 2)
    b = gy2.reshape(S, M // S, cout8)[:, :, :cout]
    try:
        part = torch.bmm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError):
        part = torch.bmm(a, b).float()
    return part.sum(0)


class Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, bias, stride: Tuple[int, int], padding: Tuple[int, int]):
        kh, kw, cin, cout = kernel.shape
        N, H, W, C = x.shape
        assert C == cin, f"conv input has {C} channels, kernel expects {cin}"
        cin8 = nat.round_up(cin, 8)
        xb = _pad_channels(x, cin8)
        spec = _cached_spec(kernel, bias, stride, padding, cin8, transposed=False)
        y = nat.conv2d(spec, xb, out_dtype=BF16)
        ctx.save_for_backward(xb, kernel)
        ctx.meta = (N, H, W, cin, cout, tuple(stride), tuple(padding))
        ctx.bias_requires_grad = bias.requires_grad
        return y.contiguous() if not y.is_contiguous() else y

    @staticmethod
    def backward(ctx, gy):
        xb, kernel = ctx.saved_tensors
        N, H, W, cin, cout, (sh, sw), (ph, pw) = ctx.meta
        kh, kw = kernel.shape[:2]
        OH, OW = gy.shape[1], gy.shape[2]
        cout8 = nat.round_up(cout, 8)
        gyb = _pad_channels(gy, cout8)
        gx = gk = gb = None
        if ctx.needs_input_grad[0]:
            # dX = conv(dilate_s(dY), flip(W)^T), padding k-1-p, output size forced to (H, W)
            spec = _cached_spec(kernel, None, (1, 1), (ph, pw), cout8, transposed=True)
            gxp = torch.empty(N, H, W, nat.round_up(cin, 8), dtype=BF16, device=gy.device)
            t, i, a = nat.conv_args(spec, gyb, N, OH, OW, gxp)
            i = i + [H, W, _log2_stride(sh), _log2_stride(sw)]
            nat.ops().conv(t, i, a)
            gx = gxp[..., :cin]
        if ctx.needs_input_grad[1]:
            cin8 = xb.shape[-1]
            kpad = nat.round_up(kh * kw * cin8, 64)
            M = N * OH * OW
            col = torch.empty(M, kpad, dtype=BF16, device=gy.device)
            nat.ops().im2col([xb, col], [N, H, W, 0, cin8, kh, kw, sh, sw, ph, pw])
            gw = _wgrad_gemm(gyb.reshape(M, cout8), col, cout)  # (kpad, cout) fp32
            gk = gw[: kh * kw * cin8].reshape(kh, kw, cin8, cout)
            if cin8 != cin:
                gk = gk[:, :, :cin].contiguous()
        if ctx.bias_requires_grad:
            gb = gy.sum(dim=(0, 1, 2), dtype=torch.float32)
        return gx, gk, gb, None, None


def conv2d_nhwc(x, kernel, bias, stride=(1, 1), padding=(0, 0)):
    return Conv2dNHWC.apply(x, kernel, bias, tuple(stride), tuple(padding))


class CorrPyramid(torch.autograd.Function):
    """fmap1 (B, hq, wq, C) query pixels, fmap2 (B, h, w, C) -> L fp32 levels
    (B*hq*wq, h_l, w_l).  The queries are normally the whole map (hq, wq = h, w);
    context parallelism (:mod:`jax_raft_amd.parallel.cp`) passes a slab of rows."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, num_levels: int):
        B, hq, wq, C = fmap1.shape
        _, h, w, _ = fmap2.shape
        nq = hq * wq
        f1 = fmap1.to(BF16).contiguous()
        f2 = fmap2.to(BF16).contiguous()
        M = B * nq
        levels = []
        hl, wl = h, w
        for _ in range(num_levels):
            levels.append(torch.empty(M, hl, wl, device=fmap1.device, dtype=torch.float32))
            hl //= 2
            wl //= 2
        if C % 64 == 0:
            nat.ops().corr([f1, f2] + levels + [None] * (4 - num_levels), [B, h, w, C, num_levels, nq],
                           1.0 / math.sqrt(C))
        else:  # channel count the MFMA kernel does not tile: library GEMM + pooling
            vol = torch.matmul(f1.float().reshape(B, nq, C), f2.float().reshape(B, h * w, C).transpose(1, 2))
            vol = (vol / math.sqrt(C)).reshape(M, h, w)
            levels[0].copy_(vol)
            for l in range(1, num_levels):
                p = levels[l - 1]
                hh, ww = p.shape[1] // 2, p.shape[2] // 2
                levels[l].copy_(p[:, : 2 * hh, : 2 * ww].reshape(M, hh, 2, ww, 2).mean(dim=(2, 4)))
        ctx.save_for_backward(f1, f2)
        ctx.shape = (B, hq, wq, h, w, C, num_levels)
        # lookups of these levels accumulate their gradient into one shared buffer
        # (see _LookupGradAcc) and hand it over here instead of through autograd
        ctx.acc = _LookupGradAcc()
        levels[0]._jr_lookup_acc = ctx.acc
        ctx.set_materialize_grads(False)
        return tuple(levels)

    @staticmethod
    def backward(ctx, *glevels):
        f1, f2 = ctx.saved_tensors
        shared = ctx.acc.take()
        if shared is not None:
            glevels = tuple(s if g is None else s + g for s, g in zip(shared, glevels))
        g1, g2 = pyramid_backward(f1, f2, ctx.shape, glevels)
        return g1, g2, None


def pyramid_backward(f1, f2, shape, glevels):
    """Gradients of the correlation pyramid w.r.t. the query / target feature
    maps: the 2x2 average-pooling adjoints summed into the full-resolution
    volume gradient dC, then the two GEMMs of ``C = f1 f2^T / sqrt(C)``."""
    B, hq, wq, h, w, C, L = shape
    nq = hq * wq
    dC = torch.zeros(B * nq, h, w, device=f1.device, dtype=torch.float32)
    for l, g in enumerate(glevels):
        if g is None:
            continue
        s = 2 ** l
        hl, wl = g.shape[1], g.shape[2]
        up = g.float().repeat_interleave(s, dim=1).repeat_interleave(s, dim=2) / float(s * s)
        dC[:, : hl * s, : wl * s] += up
    dC = dC.reshape(B, nq, h * w) / math.sqrt(C)
    g1 = torch.matmul(dC, f2.float().reshape(B, h * w, C)).reshape(B, hq, wq, C)
    g2 = torch.matmul(dC.transpose(1, 2), f1.float().reshape(B, nq, C)).reshape(B, h, w, C)
    return g1, g2


def build_pyramid(fmap1, fmap2, num_levels: int) -> List[torch.Tensor]:
    return list(CorrPyramid.apply(fmap1, fmap2, num_levels))


class _LookupGradAcc:
    """One fp32 gradient accumulator per pyramid, shared by all of its lookups.

    Every refinement iteration looks up the same pyramid, so per-call level
    gradients would cost a full zero-filled fp32 pyramid per iteration plus
    an autograd add of it (hundreds of MB each at training resolution).  The
    backward kernel accumulates (read-modify-write) instead: every lookup's
    backward adds into this one buffer and returns no level gradient; the
    pyramid's own backward (:class:`CorrPyramid`) takes the sum.

    The buffer is tagged with the autograd graph task (one ``backward`` /
    ``autograd.grad`` call) that filled it, so a sum left behind by a pass in
    which the pyramid's backward did not run (gradients requested w.r.t. the
    levels themselves, or a pass that never reached the pyramid) is discarded
    instead of leaking into a later pass."""

    def __init__(self):
        self.bufs = None
        self.task = None

    def buffers(self, shapes, device) -> List[torch.Tensor]:
        task = torch._C._current_graph_task_id()
        if self.bufs is None or self.task != task:
            self.bufs = [torch.zeros(s, device=device, dtype=torch.float32) for s in shapes]
            self.task = task
        return self.bufs

    def take(self):
        bufs = self.bufs if self.task == torch._C._current_graph_task_id() else None
        self.bufs, self.task = None, None
        return bufs


def _lookup_acc(levels):
    """The shared accumulator of a pyramid built by :class:`CorrPyramid` (None
    for levels from elsewhere, whose lookups return their own gradients)."""
    return getattr(levels[0], "_jr_lookup_acc", None)


class PyramidLookup(torch.autograd.Function):
    """levels (fp32), coords (B, h, w, 2) -> (B, h, w, L*(2r+1)^2) bf16."""

    @staticmethod
    def forward(ctx, coords, radius: int, *levels):
        # queries: coords (B, hq, wq); level-0 maps: (h, w) (hq, wq = h, w unless a row slab)
        B, hq, wq, _ = coords.shape
        h, w = levels[0].shape[1], levels[0].shape[2]
        nq = hq * wq
        L = len(levels)
        S = 2 * radius + 1
        ocs = nat.round_up(L * S * S, 8)
        c = coords.detach().float().reshape(B * nq, 2).contiguous()
        out = torch.empty(B * nq, ocs, dtype=BF16, device=coords.device)
        lv = [l.contiguous() for l in levels]
        nat.ops().lookup([c, out] + lv + [None] * (4 - L), [L, B, h, w, radius, nq])
        ctx.save_for_backward(c)
        ctx.meta = (B, h, w, nq, radius, L, [tuple(l.shape) for l in levels])
        ctx.acc = _lookup_acc(levels)
        return out.reshape(B, hq, wq, ocs)[..., : L * S * S]

    @staticmethod
    def backward(ctx, g):
        (c,) = ctx.saved_tensors
        B, h, w, nq, radius, L, shapes = ctx.meta
        g = g.reshape(B * nq, -1)
        g = g.contiguous() if g.dtype in (BF16, torch.float32) else g.float().contiguous()
        acc = ctx.acc
        if acc is None:
            dls = [torch.zeros(s, device=g.device, dtype=torch.float32) for s in shapes]
            nat.ops().lookup_bwd([c, g] + dls + [None] * (4 - L), [L, B, h, w, radius, nq])
            return (None, None) + tuple(dls)
        nat.ops().lookup_bwd([c, g] + acc.buffers(shapes, g.device) + [None] * (4 - L), [L, B, h, w, radius, nq])
        return (None, None) + (None,) * L


def index_pyramid(pyramid: Sequence[torch.Tensor], coords, radius: int):
    return PyramidLookup.apply(coords, radius, *pyramid)


def raft_forward_autograd(model, image1, image2, train: bool, num_flow_updates: int, fused=None):
    """GPU forward with autograd.  Default: the correlation pyramid + refinement
    loop as one fused native node (:mod:`jax_raft_amd.train.fused`; encoders on
    the Functions above).  ``fused=False`` (or ``train.fused.FUSED_TRAIN = False``): the module
    graph of :meth:`RAFT.forward_reference` with its conv / correlation / lookup
    nodes dispatched to the native Functions above (see
    :mod:`jax_raft_amd.ops.functional`)."""
    from ..train import fused as F

    if fused is None:
        fused = F.enabled()
    if fused and F.supported(model):
        return F.forward_train(model, image1, image2, train, num_flow_updates)
    return model.forward_reference(image1, image2, train, num_flow_updates)
