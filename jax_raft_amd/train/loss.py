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
    """flow_preds (N, B, H, W, 2); flow_gt (B, H, W, 2); valid (B, H, W) or None.

    GPU tensors run the native one-pass kernel (csrc/kernels/train.hip:
    loss + metrics in one read of the predictions, gradient in one more pass,
    no host synchronisation); CPU tensors the PyTorch expression below."""
    if flow_preds.is_cuda and flow_preds.shape[0] <= 32:
        return _native_sequence_loss(flow_preds, flow_gt, valid, gamma, max_flow)
    return sequence_loss_reference(flow_preds, flow_gt, valid, gamma, max_flow)


def sequence_loss_reference(flow_preds, flow_gt, valid=None, gamma: float = 0.8, max_flow: float = 400.0):
    """PyTorch sequence loss (the CPU path and the GPU kernel's test oracle)."""
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


class _SeqLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, preds, gt, valid, gamma: float, max_flow: float):
        from ..ops import native as nat

        ops = nat.ops()
        n = preds.shape[0]
        P = gt.numel() // 2
        part = torch.empty(ops.seq_loss_blocks(P), 37, device=preds.device, dtype=torch.float32)
        ops.seq_loss([preds, gt, valid, part], [P, n], max_flow)
        s = part.sum(0)
        w = gamma ** torch.arange(n - 1, -1, -1, device=preds.device, dtype=torch.float64)
        w = (w / (2.0 * P)).float()
        loss = (w * s[:n]).sum()
        cnt = s[36]
        inv = torch.where(cnt > 0, 1.0 / cnt.clamp_min(1.0), torch.zeros_like(cnt))
        mets = torch.stack([s[32] * inv, s[33] * inv, s[34] * inv, s[35] * inv])
        ctx.save_for_backward(preds, gt, valid, w)
        ctx.max_flow = max_flow
        ctx.mark_non_differentiable(mets)
        return loss, mets

    @staticmethod
    def backward(ctx, gl, _gm):
        from ..ops import native as nat

        preds, gt, valid, w = ctx.saved_tensors
        grad = torch.empty_like(preds)
        n = preds.shape[0]
        nat.ops().seq_loss_bwd([preds, gt, valid, (w * gl).contiguous(), grad], [gt.numel() // 2, n], ctx.max_flow)
        return grad, None, None, None, None


def _native_sequence_loss(flow_preds, flow_gt, valid, gamma, max_flow):
    preds = flow_preds.float().contiguous()
    gt = flow_gt.float().contiguous()
    v = None if valid is None else valid.float().reshape(-1).contiguous()
    loss, m = _SeqLoss.apply(preds, gt, v, float(gamma), float(max_flow))
    return loss, {"epe": m[0], "1px": m[1], "3px": m[2], "5px": m[3]}
