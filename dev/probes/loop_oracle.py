#!/usr/bin/env python3
"""Per-parameter gradient error of the fused refinement-loop node (train/fused.py:FusedRefine)
against fp32 autograd of the golden ops on the GPU, on bf16-rounded operands (weights, feature
maps, context): the loop alone, T iterations, so the error is the loop kernels' own and not the
encoders' bf16 cancellation noise.

    python dev/probes/loop_oracle.py --iters 1 2 4
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from jax_raft_amd import raft_large, raft_small  # noqa: E402
from jax_raft_amd.models import reference as R  # noqa: E402
from jax_raft_amd.ops.functional import golden_ops  # noqa: E402
from jax_raft_amd.train import fused as F  # noqa: E402


def _ste_bf16(x):
    """bf16-rounded forward value, identity gradient (what a bf16-stored activation does)."""
    return x + (x.bfloat16().float() - x).detach()


def golden_loop(model, f1, f2, ctx, T, round_corr=False):
    """models/raft.py:forward_reference after the encoders; ``round_corr``: the pyramid levels
    and the looked-up correlation features rounded to bf16 in the forward, as the native paths
    store them."""
    B, h, w, _ = f1.shape
    pyr = model.corr_block.build_pyramid(f1, f2)
    if round_corr:
        pyr = [_ste_bf16(p) for p in pyr]
    hs = model.update_block.hidden_state_size
    hidden, context = torch.tanh(ctx[..., :hs]), torch.relu(ctx[..., hs:])
    c0 = R.make_coords_grid(B, h, w, device=f1.device)
    c1 = c0.clone()
    preds = []
    for _ in range(T):
        c1 = c1.detach()
        corr = model.corr_block.index_pyramid(pyr, c1)
        if round_corr:
            corr = _ste_bf16(corr)
        hidden, delta = model.update_block(hidden, context, corr, c1 - c0, True)
        c1 = c1 + delta
        m = None if model.mask_predictor is None else model.mask_predictor(hidden, True)
        preds.append(R.upsample_flow(c1 - c0, m))
    return torch.stack(preds, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="raft_large")
    ap.add_argument("--iters", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--size", type=int, nargs=2, default=[192, 256])
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    factory = raft_large if a.arch == "raft_large" else raft_small
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = factory()[0].to(dev).train()
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(p.bfloat16().float())
    B, (H, W) = a.batch, a.size
    h, w = H // 8, W // 8
    g = torch.Generator(device=dev).manual_seed(1)
    C = model.feature_encoder.out_channels
    f1 = torch.randn(B, h, w, C, generator=g, device=dev).bfloat16().float()
    f2 = (0.7 * f1 + 0.7 * torch.randn(B, h, w, C, generator=g, device=dev)).bfloat16().float()
    ctx = torch.randn(B, h, w, model.context_encoder.out_channels, generator=g, device=dev).bfloat16().float()
    target = torch.randn(B, H, W, 2, generator=g, device=dev) * 4
    for T in a.iters:
        wts = torch.tensor([0.8 ** (T - k - 1) for k in range(T)], device=dev).view(-1, 1, 1, 1, 1)
        res = {}
        for path in ("fused", "unfused", "golden", "golden_bf16corr"):
            model.zero_grad(set_to_none=True)
            x1, x2, xc = (t.clone().requires_grad_(True) for t in (f1, f2, ctx))
            if path == "fused":
                F._LOOPS.clear()
                loop = F.get_loop(model, B, H, W, T, dev)
                out = F.FusedRefine.apply(loop, x1, x2, xc, *loop.params)
            elif path == "unfused":   # the per-op native autograd path (ops/autograd.py)
                out = golden_loop(model, x1, x2, xc, T)
            else:
                with golden_ops():
                    out = golden_loop(model, x1, x2, xc, T, round_corr=path != "golden")
            (wts * (out.float() - target).abs()).mean().backward()
            gr = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
            gr.update({"d_fmap1": x1.grad, "d_fmap2": x2.grad, "d_ctx": xc.grad})
            res[path] = (out.detach(), gr)
        og, gg = res["golden"]
        (of, gf), (ou, gu), (_, gs) = res["fused"], res["unfused"], res["golden_bf16corr"]
        scale = max(v.norm().item() for v in gg.values())
        rows = []
        for n, r in gg.items():
            if r.norm().item() < 1e-4 * scale:
                continue
            rn = r.norm().item()
            rows.append(((gf[n] - r).norm().item() / rn, (gu[n] - r).norm().item() / rn,
                         (gf[n] - gu[n]).norm().item() / rn, (gs[n] - r).norm().item() / rn,
                         (gf[n] - gs[n]).norm().item() / rn, n))
        rows.sort(reverse=True)
        ef = sorted(e[0] for e in rows)
        eu = sorted(e[1] for e in rows)
        print(f"T={T}: output rel fused {(of - og).norm().item() / og.norm().item():.2e} unfused "
              f"{(ou - og).norm().item() / og.norm().item():.2e}; gradient rel error vs golden: fused median "
              f"{ef[len(ef) // 2]:.2e} max {ef[-1]:.2e}, unfused median {eu[len(eu) // 2]:.2e} max {eu[-1]:.2e} "
              f"over {len(ef)} tensors")
        print("   fused-vs-golden unfused-vs-golden fused-vs-unfused golden(bf16 corr)-vs-golden "
              "fused-vs-golden(bf16 corr)  tensor")
        for e in rows[: a.top]:
            print("   " + " ".join(f"{v:.3e}" for v in e[:5]) + f"  {e[5]}")


if __name__ == "__main__":
    main()
