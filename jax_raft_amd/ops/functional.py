"""Device-dispatching functional ops used by the model modules.

One implementation per device: CPU tensors run the golden PyTorch ops of
:mod:`jax_raft_amd.models.reference`; GPU tensors run the native gfx950 kernels
through the autograd Functions of :mod:`jax_raft_amd.ops.autograd`.  There is
no silent fallback: if the native library is missing, GPU calls raise.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager
from typing import List, Sequence

import torch

from ..models import reference as R

_mode = threading.local()


@contextmanager
def golden_ops():
    """Run the module forwards on the golden PyTorch ops on ANY device (a plain fp32
    reference on the GPU, e.g. for engine-vs-golden tests at sizes the CPU cannot afford)."""
    prev = getattr(_mode, "golden", False)
    _mode.golden = True
    try:
        yield
    finally:
        _mode.golden = prev


def _native(x: torch.Tensor) -> bool:
    return x.is_cuda and not getattr(_mode, "golden", False)


def conv2d_nhwc(x: torch.Tensor, kernel: torch.Tensor, bias, stride=(1, 1), padding=(0, 0)) -> torch.Tensor:
    if _native(x):
        from .autograd import conv2d_nhwc as native_conv

        return native_conv(x, kernel, bias, stride, padding)
    if x.is_cuda:   # golden_ops on the GPU: im2col + GEMM (no convolution-library search)
        return R.conv2d_nhwc_gemm(x, kernel, bias, stride, padding)
    return R.conv2d_nhwc(x, kernel, bias, stride, padding)


def build_pyramid(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int) -> List[torch.Tensor]:
    if _native(fmap1):
        from .autograd import build_pyramid as native_pyr

        B, h, w, _ = fmap1.shape
        min_fmap_size = 2 * (2 ** (num_levels - 1))
        assert h >= min_fmap_size and w >= min_fmap_size, (
            "Feature maps are too small to be down-sampled by the correlation pyramid. "
            f"H and W of feature maps should be at least {min_fmap_size}; got: {(h, w)}.")
        return native_pyr(fmap1, fmap2, num_levels)
    return R.build_pyramid(fmap1, fmap2, num_levels)


def build_pyramid_queries(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int) -> List[torch.Tensor]:
    """Pyramid of a subset of query pixels ``fmap1`` (B, hq, wq, C) against all of
    ``fmap2`` (B, h, w, C): levels (B*hq*wq, h_l, w_l) (context parallelism)."""
    if _native(fmap1):
        from .autograd import build_pyramid as native_pyr

        return native_pyr(fmap1, fmap2, num_levels)
    return R.build_pyramid_queries(fmap1, fmap2, num_levels)


def index_pyramid(pyramid: Sequence[torch.Tensor], coords: torch.Tensor, radius: int) -> torch.Tensor:
    if _native(coords):
        from .autograd import index_pyramid as native_lookup

        return native_lookup(pyramid, coords, radius)
    return R.index_pyramid(pyramid, coords, radius)
