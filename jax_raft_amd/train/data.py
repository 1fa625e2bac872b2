"""Synthetic FlyingChairs-shaped training data (no datasets reachable offline).

Each sample is a random smooth texture (image2) and a random smooth flow field
(affine motion + low-frequency deformation); image1 is image2 warped by the
flow so brightness constancy holds exactly: ``image1(x) = image2(x + f(x))``
(bilinear, border clamp).  Ground truth is therefore exact and the sequence
loss is a meaningful training signal.  Deterministic per (seed, index);
generated directly on the target device.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F


def _smooth_noise(g: torch.Generator, B: int, C: int, H: int, W: int, scales=(4, 16, 64), device="cpu") -> torch.Tensor:
    out = torch.zeros(B, C, H, W)
    for s in scales:
        n = torch.randn(B, C, max(2, H // s), max(2, W // s), generator=g)
        out += F.interpolate(n, size=(H, W), mode="bicubic", align_corners=False) * (s / max(scales))
    return out.to(device)


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
        g = torch.Generator().manual_seed(self.seed * 1000003 + int(indices[0]) * 7919 + B)
        H, W = self.H, self.W
        tex = _smooth_noise(g, B, 3, H, W, device=self.device)
        tex = torch.tanh(tex * 1.5)
        # flow: affine + smooth deformation
        ys, xs = torch.meshgrid(torch.linspace(-1, 1, H), torch.linspace(-1, 1, W), indexing="ij")
        A = (torch.rand(B, 2, 3, generator=g) * 2 - 1)
        A[:, :, 2] *= self.max_motion
        A[:, :, :2] *= 0.1 * self.max_motion
        fx = A[:, 0, 0, None, None] * xs + A[:, 0, 1, None, None] * ys + A[:, 0, 2, None, None]
        fy = A[:, 1, 0, None, None] * xs + A[:, 1, 1, None, None] * ys + A[:, 1, 2, None, None]
        d = _smooth_noise(g, B, 2, H, W, scales=(32, 64), device="cpu") * (0.25 * self.max_motion)
        flow = torch.stack([fx + d[:, 0], fy + d[:, 1]], dim=-1).to(self.device)  # (B, H, W, 2)
        # image1(x) = image2(x + flow(x)): sample image2 at x + flow
        base_x = torch.arange(W, device=self.device).float().view(1, 1, W)
        base_y = torch.arange(H, device=self.device).float().view(1, H, 1)
        sx = (base_x + flow[..., 0]) / (W - 1) * 2 - 1
        sy = (base_y + flow[..., 1]) / (H - 1) * 2 - 1
        img1 = F.grid_sample(tex, torch.stack([sx, sy], -1), mode="bilinear", padding_mode="border",
                             align_corners=True)
        inside = (sx.abs() <= 1) & (sy.abs() <= 1)
        img1 = img1.permute(0, 2, 3, 1).contiguous()
        img2 = tex.permute(0, 2, 3, 1).contiguous()
        return img1, img2, flow, inside.float()
