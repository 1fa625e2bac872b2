"""Optical-flow I/O and input padding.

* ``.flo`` (Middlebury) read/write -- reference ``scripts/validate_sintel.py:42-61``
  (``readFlow``; magic 202021.25, little-endian int32 w, h, float32 (u, v)).
* :class:`InputPadder` -- replicate padding to a multiple of 8, 'sintel' mode
  centred, else bottom-only (``validate_sintel.py:23-40``).  Works on NCHW or
  NHWC tensors (``channels_last=True``).
* image loading to NHWC float in [-1, 1] (``examples/demo.py:7-10``,
  ``validate_sintel.py:177-178``).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

FLO_MAGIC = 202021.25


def read_flo(path: str) -> Optional[np.ndarray]:
    """Read a Middlebury ``.flo`` file -> (H, W, 2) float32, or None on a bad magic."""
    with open(path, "rb") as f:
        magic = np.fromfile(f, np.float32, count=1)
        if magic.size == 0 or magic[0] != np.float32(FLO_MAGIC):
            return None
        w = int(np.fromfile(f, np.int32, count=1)[0])
        h = int(np.fromfile(f, np.int32, count=1)[0])
        data = np.fromfile(f, np.float32, count=2 * w * h)
    return data.reshape(h, w, 2)


def write_flo(path: str, flow: np.ndarray) -> None:
    flow = np.asarray(flow, dtype=np.float32)
    assert flow.ndim == 3 and flow.shape[2] == 2
    h, w = flow.shape[:2]
    with open(path, "wb") as f:
        np.array([FLO_MAGIC], np.float32).tofile(f)
        np.array([w, h], np.int32).tofile(f)
        flow.tofile(f)


def read_image(path: str) -> np.ndarray:
    """RGB uint8 (H, W, 3); grayscale is replicated (``validate_sintel.py:113-119``)."""
    from PIL import Image

    img = np.array(Image.open(path))
    if img.ndim == 2:
        img = np.tile(img[..., None], (1, 1, 3))
    return img[..., :3].astype(np.uint8)


def normalize_image(img_uint8: np.ndarray) -> torch.Tensor:
    """uint8 (H, W, 3) -> float32 NHWC (1, H, W, 3) in [-1, 1]."""
    return torch.from_numpy(img_uint8.astype(np.float32) / 255.0 * 2.0 - 1.0)[None]


class InputPadder:
    """Pads images so H and W are divisible by 8 (replicate mode)."""

    def __init__(self, dims: Sequence[int], mode: str = "sintel", channels_last: bool = False):
        self.channels_last = channels_last
        if channels_last:
            self.ht, self.wd = dims[-3], dims[-2]
        else:
            self.ht, self.wd = dims[-2], dims[-1]
        pad_ht = (((self.ht // 8) + 1) * 8 - self.ht) % 8
        pad_wd = (((self.wd // 8) + 1) * 8 - self.wd) % 8
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    def pad(self, *inputs: torch.Tensor) -> List[torch.Tensor]:
        out = []
        for x in inputs:
            if self.channels_last:
                x = F.pad(x.permute(0, 3, 1, 2), self._pad, mode="replicate").permute(0, 2, 3, 1).contiguous()
            else:
                x = F.pad(x, self._pad, mode="replicate")
            out.append(x)
        return out

    def unpad(self, x: torch.Tensor) -> torch.Tensor:
        if self.channels_last:
            ht, wd = x.shape[-3], x.shape[-2]
            c = [self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]]
            return x[..., c[0]:c[1], c[2]:c[3], :]
        ht, wd = x.shape[-2:]
        c = [self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]]
        return x[..., c[0]:c[1], c[2]:c[3]]


def flow_to_color(flow: np.ndarray, max_flow: Optional[float] = None) -> np.ndarray:
    """Middlebury-style colour coding of a (H, W, 2) flow field -> uint8 RGB."""
    u, v = flow[..., 0], flow[..., 1]
    rad = np.sqrt(u * u + v * v)
    maxr = max_flow if max_flow is not None else max(float(rad.max()), 1e-6)
    ang = np.arctan2(-v, -u) / np.pi  # [-1, 1]
    hue = (ang + 1.0) / 2.0
    sat = np.clip(rad / maxr, 0, 1)
    hsv = np.stack([hue, sat, np.ones_like(sat)], -1)
    i = np.floor(hsv[..., 0] * 6).astype(int) % 6
    f = hsv[..., 0] * 6 - np.floor(hsv[..., 0] * 6)
    p, q, t = 1 - sat, 1 - sat * f, 1 - sat * (1 - f)
    rgb = np.select([i[..., None] == k for k in range(6)],
                    [np.stack(c, -1) for c in ((np.ones_like(t), t, p), (q, np.ones_like(t), p), (p, np.ones_like(t), t),
                                               (p, q, np.ones_like(t)), (t, p, np.ones_like(t)), (np.ones_like(t), p, q))])
    return (rgb * 255).astype(np.uint8)
