"""Native autograd Functions (GPU training path) against fp32 PyTorch autograd
of the golden ops on CPU."""
import math

import pytest
import torch

from jax_raft_amd import raft_small, raft_large
from jax_raft_amd.models import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / (b.float().norm() + 1e-8)).item()


CASES = [
    # N, H, W, cin, cout, kh, kw, stride, pad
    (2, 12, 16, 64, 64, 3, 3, 1, (1, 1)),
    (2, 12, 16, 64, 96, 3, 3, 2, (1, 1)),
    (2, 13, 17, 32, 64, 1, 1, 2, (0, 0)),
    (1, 24, 32, 3, 64, 7, 7, 2, (3, 3)),
    (2, 9, 11, 384, 128, 1, 5, 1, (0, 2)),
    (2, 9, 11, 384, 128, 5, 1, 1, (2, 0)),
    (1, 10, 12, 256, 2, 3, 3, 1, (1, 1)),
    (1, 10, 12, 2, 128, 7, 7, 1, (3, 3)),
    (1, 10, 12, 324, 256, 1, 1, 1, (0, 0)),
    (2, 11, 9, 242, 96, 3, 3, 1, (1, 1)),
]


@pytest.mark.parametrize("case", CASES)
def test_conv_backward(case):
    from jax_raft_amd.ops.autograd import conv2d_nhwc

    N, H, W, cin, cout, kh, kw, s, pad = case
    torch.manual_seed(0)
    x = torch.randn(N, H, W, cin).to(torch.bfloat16).float()
    k = (torch.randn(kh, kw, cin, cout) / math.sqrt(kh * kw * cin)).to(torch.bfloat16).float()
    b = torch.randn(cout) * 0.1
    xr, kr, br = (t.clone().requires_grad_(True) for t in (x, k, b))
    yr = R.conv2d_nhwc(xr, kr, br, (s, s), pad)
    gy = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(gy)
    xg, kg, bg = (t.cuda().requires_grad_(True) for t in (x, k, b))
    y = conv2d_nhwc(xg, kg, bg, (s, s), pad)
    assert y.shape == yr.shape
    y.backward(gy.cuda().to(y.dtype))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-2
    assert _rel(xg.grad, xr.grad) < 2e-2, "dX"
    assert _rel(kg.grad, kr.grad) < 2e-2, "dW"
    assert _rel(bg.grad, br.grad) < 1e-2, "db"


def test_corr_pyramid_backward():
    from jax_raft_amd.ops.autograd import build_pyramid

    torch.manual_seed(1)
    B, h, w, C = 2, 17, 19, 64
    f1 = torch.randn(B, h, w, C).to(torch.bfloat16).float()
    f2 = torch.randn(B, h, w, C).to(torch.bfloat16).float()
    gs = None
    a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    ref = R.build_pyramid(a1, a2, 4)
    gs = [torch.randn_like(l) for l in ref]
    sum((l * g).sum() for l, g in zip(ref, gs)).backward()
    b1, b2 = f1.cuda().requires_grad_(True), f2.cuda().requires_grad_(True)
    out = build_pyramid(b1, b2, 4)
    for o, r in zip(out, ref):
        assert _rel(o, r) < 1e-3
    sum((l * g.cuda()).sum() for l, g in zip(out, gs)).backward()
    torch.cuda.synchronize()
    assert _rel(b1.grad, a1.grad) < 1e-3
    assert _rel(b2.grad, a2.grad) < 1e-3


@pytest.mark.parametrize("radius", [4, 3])
def test_lookup_backward(radius):
    from jax_raft_amd.ops.autograd import index_pyramid

    torch.manual_seed(2)
    B, h, w = 2, 16, 20
    M = B * h * w
    pyr = []
    hl, wl = h, w
    for _ in range(4):
        pyr.append(torch.randn(M, hl, wl))
        hl //= 2
        wl //= 2
    coords = R.make_coords_grid(B, h, w) + torch.randn(B, h, w, 2) * 3
    coords[0, 0, 0] = torch.tensor([-6.3, 2.5])
    pr = [p.clone().requires_grad_(True) for p in pyr]
    ref = R.index_pyramid(pr, coords, radius)
    g = torch.randn_like(ref).to(torch.bfloat16).float()
    ref.backward(g)
    pg = [p.cuda().requires_grad_(True) for p in pyr]
    out = index_pyramid(pg, coords.cuda(), radius)
    assert _rel(out, ref) < 1e-2
    out.backward(g.cuda())
    torch.cuda.synchronize()
    for a, b in zip(pg, pr):
        assert _rel(a.grad, b.grad) < 1e-5


def _pyr_case(seed, B=2, h=16, w=20, C=64, n=3):
    torch.manual_seed(seed)
    f1 = torch.randn(B, h, w, C).to(torch.bfloat16).float()
    f2 = torch.randn(B, h, w, C).to(torch.bfloat16).float()
    cs = [R.make_coords_grid(B, h, w) + torch.randn(B, h, w, 2) * 3 for _ in range(n)]
    return f1, f2, cs


def _pyr_losses(build, index, f1, f2, cs, radius=4):
    pyr = build(f1, f2, 4)
    return [(k + 1) * index(pyr, c, radius).float().sum() for k, c in enumerate(cs)], pyr


def test_lookup_backward_shared_accumulator():
    """Several lookups of one pyramid (the refinement loop's pattern) sum their
    level gradients in one shared buffer that the pyramid's backward takes; a
    retain_graph second pass repeats exactly."""
    from jax_raft_amd.ops.autograd import build_pyramid, index_pyramid

    f1, f2, cs = _pyr_case(5)
    a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    ref, _ = _pyr_losses(R.build_pyramid, R.index_pyramid, a1, a2, cs)
    sum(ref).backward()
    b1, b2 = f1.cuda().requires_grad_(True), f2.cuda().requires_grad_(True)
    out, _ = _pyr_losses(build_pyramid, index_pyramid, b1, b2, [c.cuda() for c in cs])
    sum(out).backward(retain_graph=True)
    torch.cuda.synchronize()
    assert _rel(b1.grad, a1.grad) < 1e-2 and _rel(b2.grad, a2.grad) < 1e-2
    first = (b1.grad.clone(), b2.grad.clone())
    sum(out).backward()
    torch.cuda.synchronize()
    assert _rel(b1.grad, 2 * first[0]) < 1e-6 and _rel(b2.grad, 2 * first[1]) < 1e-6


def test_lookup_backward_partial_passes():
    """Partial backward passes: a retain_graph loss over a subset of
    the lookups, then a pass whose gradients stop at the levels (the pyramid's
    backward never runs), then the full loss: each pass sees exactly its own
    lookups' gradients."""
    from jax_raft_amd.ops.autograd import build_pyramid, index_pyramid

    f1, f2, cs = _pyr_case(9)
    a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    ref, _ = _pyr_losses(R.build_pyramid, R.index_pyramid, a1, a2, cs)
    g_sub = torch.autograd.grad(ref[0] + ref[1], (a1, a2), retain_graph=True)
    g_all = torch.autograd.grad(sum(ref), (a1, a2))
    b1, b2 = f1.cuda().requires_grad_(True), f2.cuda().requires_grad_(True)
    out, pyr = _pyr_losses(build_pyramid, index_pyramid, b1, b2, [c.cuda() for c in cs])
    h_sub = torch.autograd.grad(out[0] + out[1], (b1, b2), retain_graph=True)
    for x, y in zip(h_sub, g_sub):
        assert _rel(x, y) < 1e-2
    # gradients w.r.t. the levels themselves: lookups run, the pyramid's backward does not
    torch.autograd.grad(out[2], pyr[0], retain_graph=True, allow_unused=True)
    h_all = torch.autograd.grad(sum(out), (b1, b2))
    torch.cuda.synchronize()
    for x, y in zip(h_all, g_all):
        assert _rel(x, y) < 1e-2


def test_conv_spec_cache_tracks_inplace_updates():
    from jax_raft_amd.ops.autograd import conv2d_nhwc

    torch.manual_seed(6)
    x = torch.randn(1, 12, 12, 16, device="cuda")
    k = torch.randn(3, 3, 16, 32, device="cuda", requires_grad=True)
    b = torch.randn(32, device="cuda", requires_grad=True)
    y0 = conv2d_nhwc(x, k, b, (1, 1), (1, 1)).float()
    y0b = conv2d_nhwc(x, k, b, (1, 1), (1, 1)).float()
    assert torch.equal(y0, y0b)
    with torch.no_grad():
        k.mul_(2.0)
        b.mul_(2.0)
    y1 = conv2d_nhwc(x, k, b, (1, 1), (1, 1)).float()
    assert _rel(y1, 2 * y0) < 1e-2


@pytest.mark.parametrize("factory", [raft_small, raft_large])
def test_model_gradients_match_cpu(factory):
    torch.manual_seed(3)
    model, _ = factory()
    model.train()
    g = torch.Generator().manual_seed(0)
    i1 = torch.rand(2, 128, 128, 3, generator=g) * 2 - 1
    i2 = torch.rand(2, 128, 128, 3, generator=g) * 2 - 1
    target = torch.randn(2, 128, 128, 2, generator=g)
    out = model(i1, i2, train=True, num_flow_updates=2)
    (out - target).abs().mean().backward()
    ref = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad()
    # restore BN running stats (train step mutated them) so both runs see the same state
    model = model.cuda()
    outg = model(i1.cuda(), i2.cuda(), train=True, num_flow_updates=2)
    assert outg.shape == out.shape
    (outg.float() - target.cuda()).abs().mean().backward()
    torch.cuda.synchronize()
    cos = []
    scale = max(v.norm().item() for v in ref.values())
    for n, p in model.named_parameters():
        # biases feeding an InstanceNorm have an exactly-zero true gradient (IN removes
        # per-channel shifts): their fp32 values are rounding noise, so skip tiny grads
        if n in ref and ref[n].norm().item() > 1e-4 * scale:
            a, b = p.grad.float().cpu().flatten(), ref[n].flatten()
            cos.append((torch.dot(a, b) / (a.norm() * b.norm() + 1e-12)).item())
    cos = torch.tensor(cos)
    assert cos.median() > 0.97, cos
    assert cos.min() > 0.7, cos


@pytest.mark.parametrize("M,cout,kpad", [(65536, 64, 576), (18432, 128, 1152), (3000, 32, 64)])
def test_wgrad_split_k(M, cout, kpad):
    from jax_raft_amd.ops.autograd import _wgrad_gemm

    torch.manual_seed(7)
    gy = torch.randn(M, cout, device="cuda").to(torch.bfloat16)
    col = torch.randn(M, kpad, device="cuda").to(torch.bfloat16)
    got = _wgrad_gemm(gy, col, cout)
    ref = col.float().t() @ gy.float()
    assert got.dtype == torch.float32 and got.shape == (kpad, cout)
    assert _rel(got, ref) < 1e-2
