"""The golden CPU ops against independent PyTorch primitives."""
import math

import pytest
import torch
import torch.nn.functional as F

from jax_raft_amd.models import reference as R


def test_make_coords_grid():
    c = R.make_coords_grid(2, 3, 4)
    assert c.shape == (2, 3, 4, 2)
    assert c[1, 2, 3, 0] == 3 and c[1, 2, 3, 1] == 2  # (x, y)


@pytest.mark.parametrize("H,W", [(5, 7), (2, 2), (16, 9)])
def test_grid_sample_matches_torch(H, W):
    torch.manual_seed(0)
    n, C = 3, 4
    img = torch.randn(n, H, W, C)
    grid = torch.rand(n, 6, 5, 2) * torch.tensor([W + 4.0, H + 4.0]) - 2.0
    grid[0, 0, 0] = torch.tensor([W - 1.0, H - 1.0])  # exact corner
    grid[0, 0, 1] = torch.tensor([-1.0, 0.5])  # fully outside on x
    ours = R.grid_sample(img, grid)
    gx = 2 * grid[..., 0] / (W - 1) - 1
    gy = 2 * grid[..., 1] / (H - 1) - 1
    theirs = F.grid_sample(img.permute(0, 3, 1, 2), torch.stack([gx, gy], -1), mode="bilinear",
                           padding_mode="zeros", align_corners=True).permute(0, 2, 3, 1)
    assert torch.allclose(ours, theirs, atol=1e-5)


def test_build_pyramid_matches_avgpool_and_matmul():
    torch.manual_seed(1)
    B, h, w, C = 2, 17, 23, 8
    f1, f2 = torch.randn(B, h, w, C), torch.randn(B, h, w, C)
    pyr = R.build_pyramid(f1, f2, 4)
    vol = torch.einsum("bijc,bklc->bijkl", f1, f2) / math.sqrt(C)
    assert torch.allclose(pyr[0], vol.reshape(B * h * w, h, w), atol=1e-5)
    x = pyr[0].unsqueeze(1)
    for l in range(1, 4):
        x = F.avg_pool2d(x, 2, 2)
        assert torch.allclose(pyr[l], x.squeeze(1), atol=1e-5)
    assert pyr[3].shape[-2:] == (2, 2)


def test_pyramid_min_size_assert():
    f = torch.randn(1, 15, 20, 8)
    with pytest.raises(AssertionError):
        R.build_pyramid(f, f, 4)


def test_index_pyramid_channel_order():
    """channel l*S^2 + i*S + j samples x-offset i-r, y-offset j-r (model.py:451-468)."""
    B, h, w, r = 1, 16, 16, 2
    S = 2 * r + 1
    # level map value = 100*y + x (of the TARGET pixel), identical for every query
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")
    vol = (100 * ys + xs).expand(B * h * w, h, w).contiguous()
    coords = torch.full((B, h, w, 2), 7.0)
    coords[..., 1] = 6.0  # x = 7, y = 6
    out = R.index_pyramid([vol], coords, r)
    for i in range(S):
        for j in range(S):
            assert out[0, 0, 0, i * S + j].item() == pytest.approx(100 * (6 + j - r) + (7 + i - r))


def test_upsample_convex_matches_unfold():
    torch.manual_seed(2)
    B, h, w = 2, 5, 6
    flow = torch.randn(B, h, w, 2)
    mask = torch.randn(B, h, w, 576)
    ours = R.upsample_flow(flow, mask)
    # torchvision-style NCHW implementation
    fl = flow.permute(0, 3, 1, 2)
    m = mask.permute(0, 3, 1, 2).view(B, 1, 9, 8, 8, h, w)
    m = torch.softmax(m, dim=2)
    up = F.unfold(8 * fl, kernel_size=3, padding=1).view(B, 2, 9, 1, 1, h, w)
    up = torch.sum(m * up, dim=2).permute(0, 1, 4, 2, 5, 3).reshape(B, 2, 8 * h, 8 * w)
    assert torch.allclose(ours, up.permute(0, 2, 3, 1), atol=1e-5)


def test_upsample_bilinear_matches_interpolate():
    torch.manual_seed(3)
    flow = torch.randn(2, 5, 7, 2)
    ours = R.upsample_flow(flow, None)
    theirs = 8 * F.interpolate(flow.permute(0, 3, 1, 2), size=(40, 56), mode="bilinear", align_corners=True)
    assert torch.allclose(ours, theirs.permute(0, 2, 3, 1), atol=1e-5)


def test_instance_norm_matches_torch():
    torch.manual_seed(4)
    x = torch.randn(3, 9, 11, 5) * 3 + 1
    ours = R.instance_norm_nhwc(x)
    theirs = F.instance_norm(x.permute(0, 3, 1, 2), eps=1e-5).permute(0, 2, 3, 1)
    assert torch.allclose(ours, theirs, atol=1e-4)


def test_batch_norm_train_and_eval():
    torch.manual_seed(5)
    x = torch.randn(4, 6, 7, 3)
    sc, bi = torch.rand(3) + 0.5, torch.randn(3)
    mean, var = torch.zeros(3), torch.ones(3)
    y, nm, nv = R.batch_norm_nhwc(x, sc, bi, mean, var, train=True)
    bm = x.mean((0, 1, 2))
    bv = x.var((0, 1, 2), unbiased=False)
    assert torch.allclose(nm, 0.01 * bm, atol=1e-6) and torch.allclose(nv, 0.99 + 0.01 * bv, atol=1e-6)
    assert torch.allclose(y, (x - bm) / torch.sqrt(bv + 1e-5) * sc + bi, atol=1e-4)
    y2, m2, v2 = R.batch_norm_nhwc(x, sc, bi, nm, nv, train=False)
    assert m2 is nm and torch.allclose(y2, (x - nm) / torch.sqrt(nv + 1e-5) * sc + bi, atol=1e-5)


def test_conv2d_nhwc_matches_conv2d():
    torch.manual_seed(6)
    x = torch.randn(2, 9, 10, 4)
    k = torch.randn(1, 5, 4, 6)
    b = torch.randn(6)
    ours = R.conv2d_nhwc(x, k, b, (1, 1), (0, 2))
    theirs = F.conv2d(x.permute(0, 3, 1, 2), k.permute(3, 2, 0, 1), b, padding=(0, 2)).permute(0, 2, 3, 1)
    assert torch.allclose(ours, theirs, atol=1e-5)


def test_instance_norm_closed_form_backward():
    """The instance norm's custom backward matches finite differences (float64)
    and autograd through the plain E[x^2]-E[x]^2 formula."""
    import torch

    from jax_raft_amd.models import reference as R

    torch.manual_seed(0)
    x = torch.randn(2, 5, 6, 3, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda t: R.instance_norm_nhwc(t), (x,))
    x2 = torch.randn(2, 9, 7, 4, requires_grad=True)
    g = torch.randn(2, 9, 7, 4)
    (R.instance_norm_nhwc(x2) * g).sum().backward()
    ga = x2.grad.clone()
    x2.grad = None
    m = x2.mean(dim=(1, 2), keepdim=True)
    v = (x2 * x2).mean(dim=(1, 2), keepdim=True) - m * m
    ((x2 - m) * torch.rsqrt(v + 1e-5) * g).sum().backward()
    assert (ga - x2.grad).abs().max() < 1e-5


def test_conv_gemm_equals_conv():
    """The GEMM-form golden conv (GPU-side references) is the same operator."""
    torch.manual_seed(0)
    for (kh, kw), s, p in (((3, 3), (1, 1), (1, 1)), ((7, 7), (2, 2), (3, 3)), ((1, 5), (1, 1), (0, 2)),
                           ((1, 1), (2, 2), (0, 0))):
        x = torch.randn(2, 11, 14, 6)
        k = torch.randn(kh, kw, 6, 5)
        b = torch.randn(5)
        a = R.conv2d_nhwc(x, k, b, s, p)
        g = R.conv2d_nhwc_gemm(x, k, b, s, p)
        assert a.shape == g.shape and torch.allclose(a, g, atol=1e-4, rtol=1e-4)
