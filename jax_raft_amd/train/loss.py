"""RAFT sequence loss (original RAFT training recipe; absent from the reference,
which only returns every iteration's prediction for this purpose,
``jax_raft/model.py:510,605``).

``loss = sum_i gamma^(N-i-1) * mean(valid * |f_gt - f_i|_1)`` with
``valid = valid_in & (|f_gt| < max_flow)``; metrics on the final prediction.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch


def sequence_loss(flow_preds: torch.Tensor, flow_gt: torch.Tensor, valid: Optional[torch.Tensor] = None,
                  gamma: float = 0.8, max_flow: float = 400.0) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """flow_preds (N, B, H, W, 2); flow_gt (B, H, W, 2); valid (B, H, W) or None."""
    n = flow_preds.shape[0]
    gt = flow_gt.float()
    mag = gt.norm(dim=-1)
    v = mag < max_flow
    if valid is not None:
        v = v & (valid >= 0.5)
    vf = v.unsqueeze(-1).float()
    loss = flow_preds.new_zeros((), dtype=torch.float32)
    for i in range(n):
        w = gamma ** (n - i - 1)
        loss = loss + w * (vf * (flow_preds[i].float() - gt).abs()).mean()
    epe = (flow_preds[-1].float() - gt).norm(dim=-1)[v]
    metrics = {
        "epe": epe.mean() if epe.numel() else loss.new_zeros(()),
        "1px": (epe < 1).float().mean() if epe.numel() else loss.new_zeros(()),
        "3px": (epe < 3).float().mean() if epe.numel() else loss.new_zeros(()),
        "5px": (epe < 5).float().mean() if epe.numel() else loss.new_zeros(()),
    }
    return loss, metrics
