"""Synthetic FlyingChairs-shaped training data (no datasets reachable offline).

Each sample is a random smooth texture (image2) and a random smooth flow field
(affine motion + low-frequency deformation); image1 is image2 warped by the
flow so brightness constancy holds exactly: ``image1(x) = image2(x + f(x))``
(bilinear, border clamp).  Ground truth is therefore exact and the sequence
loss is a meaningful training signal.  Deterministic per (seed, index) for a
given device type; generated directly on the target device (a GPU batch is a
few small kernels, cheap enough to synthesise inside a timed training step).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F


def _smooth_noise(g: torch.Generator, B: int, C: int, H: int, W: int, scales=(4, 16, 64)) -> torch.Tensor:
    """Sum of bicubically upsampled Gaussian noise octaves, on ``g``'s device."""
    dev = g.device
    out = torch.zeros(B, C, H, W, device=dev)
    for s in scales:
        n = torch.randn(B, C, max(2, H // s), max(2, W // s), generator=g, device=dev)
        out += F.interpolate(n, size=(H, W), mode="bicubic", align_corners=False) * (s / max(scales))
    return out


class SyntheticFlow:
    """``ds[i] -> (image1, image2, flow, valid)``; images NHWC-ready (H, W, 3) in [-1, 1]."""

    def __init__(self, size: Tuple[int, int] = (384, 512), length: int = 22232, max_motion: float = 20.0,
                 seed: int = 0, device="cpu"):
        self.H, self.W = size
        self.length = length
        self.max_motion = max_motion
        self.seed = seed
        self.device = torch.device(device)

    def __len__(self):
        return self.length

    def batch(self, indices) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        """(image1, image2, flow, valid) for a list of indices: NHWC tensors."""
        B = len(indices)
        dev = self.device
        g = torch.Generator(device=dev).manual_seed(self.seed * 1000003 + int(indices[0]) * 7919 + B)
        H, W = self.H, self.W
        tex = torch.tanh(_smooth_noise(g, B, 3, H, W) * 1.5)
        # flow: affine + smooth deformation
        ys, xs = torch.meshgrid(torch.linspace(-1, 1, H, device=dev), torch.linspace(-1, 1, W, device=dev),
                                indexing="ij")
        A = torch.rand(B, 2, 3, generator=g, device=dev) * 2 - 1
        A[:, :, 2] *= self.max_motion
        A[:, :, :2] *= 0.1 * self.max_motion
        fx = A[:, 0, 0, None, None] * xs + A[:, 0, 1, None, None] * ys + A[:, 0, 2, None, None]
        fy = A[:, 1, 0, None, None] * xs + A[:, 1, 1, None, None] * ys + A[:, 1, 2, None, None]
        d = _smooth_noise(g, B, 2, H, W, scales=(32, 64)) * (0.25 * self.max_motion)
        flow = torch.stack([fx + d[:, 0], fy + d[:, 1]], dim=-1)  # (B, H, W, 2)
        # image1(x) = image2(x + flow(x)): sample image2 at x + flow
        base_x = torch.arange(W, device=dev).float().view(1, 1, W)
        base_y = torch.arange(H, device=dev).float().view(1, H, 1)
        sx = (base_x + flow[..., 0]) / (W - 1) * 2 - 1
        sy = (base_y + flow[..., 1]) / (H - 1) * 2 - 1
        img1 = F.grid_sample(tex, torch.stack([sx, sy], -1), mode="bilinear", padding_mode="border",
                             align_corners=True)
        inside = (sx.abs() <= 1) & (sy.abs() <= 1)
        img1 = img1.permute(0, 2, 3, 1).contiguous()
        img2 = tex.permute(0, 2, 3, 1).contiguous()
        return img1, img2, flow, inside.float()
