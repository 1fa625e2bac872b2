"""Numerics of every HIP kernel against the fp32 PyTorch golden ops
(:mod:`jax_raft_amd.models.reference`).  Inputs are rounded to bf16 first so
the comparison isolates kernel arithmetic (fp32 accumulate) from the input
quantisation."""
import math

import pytest
import torch

from jax_raft_amd.models import reference as R
from jax_raft_amd.ops.native import CFG_TILES

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _nat():
    from jax_raft_amd.ops import native

    native.require()
    return native


def _bf(x):
    return x.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


CONV_CASES = [
    # N, H, W, cin, cout, kh, kw, stride, pad
    (2, 17, 23, 64, 64, 3, 3, 1, 1),
    (2, 20, 24, 64, 96, 3, 3, 2, 1),
    (2, 20, 24, 64, 96, 1, 1, 2, 0),
    (1, 40, 48, 3, 64, 7, 7, 2, 3),
    (2, 13, 16, 384, 256, 1, 5, 1, (0, 2)),
    (2, 13, 16, 384, 128, 5, 1, 1, (2, 0)),
    (1, 12, 18, 324, 256, 1, 1, 1, 0),
    (1, 12, 18, 2, 128, 7, 7, 1, 3),
    (1, 12, 18, 256, 126, 3, 3, 1, 1),
    (1, 12, 18, 256, 2, 3, 3, 1, 1),
    (1, 12, 18, 242, 96, 3, 3, 1, 1),
    (2, 9, 11, 24, 24, 3, 3, 2, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("cfg", [None] + sorted(CFG_TILES))
def test_conv_matches_reference(case, cfg):
    nat = _nat()
    N, H, W, cin, cout, kh, kw, s, p = case
    pad = p if isinstance(p, tuple) else (p, p)
    torch.manual_seed(0)
    x = torch.randn(N, H, W, cin)
    k = torch.randn(kh, kw, cin, cout) / math.sqrt(kh * kw * cin)
    b = torch.randn(cout) * 0.1
    ref = R.conv2d_nhwc(_bf(x), _bf(k), b, (s, s), pad)
    spec = nat.make_spec(k, b, (s, s), pad, device=DEV)
    cin8 = spec.cin8
    xg = torch.zeros(N, H, W, cin8, dtype=torch.bfloat16, device=DEV)
    xg[..., :cin] = x.to(DEV, torch.bfloat16)
    y = nat.conv2d(spec, xg, out_dtype=torch.float32, cfg=cfg)
    torch.cuda.synchronize()
    assert y.shape == ref.shape
    err = _rel(y.cpu(), ref)
    assert err < 2e-3, err


@pytest.mark.parametrize("case", [CONV_CASES[0], CONV_CASES[4], CONV_CASES[6], CONV_CASES[8]])
@pytest.mark.parametrize("cfg", [2, 12, 24])
def test_conv_lowering_variants_are_bitwise(case, cfg):
    """The conv's lowering variants (cfg bit 10: XCD-aware tile order, conv_igemm.h:tile_of_block;
    bit 11: the generic im2col loader instead of FAST) change only where / how tiles load, so the
    outputs are bitwise those of the default lowering (binding.cpp:build_conv)."""
    nat = _nat()
    N, H, W, cin, cout, kh, kw, s, p = case
    pad = p if isinstance(p, tuple) else (p, p)
    torch.manual_seed(1)
    k = torch.randn(kh, kw, cin, cout) / math.sqrt(kh * kw * cin)
    spec = nat.make_spec(k, torch.randn(cout) * 0.1, (s, s), pad, device=DEV)
    xg = torch.zeros(N, H, W, spec.cin8, dtype=torch.bfloat16, device=DEV)
    xg[..., :cin] = torch.randn(N, H, W, cin).to(DEV, torch.bfloat16)
    OH, OW = spec.out_hw(H, W)
    outs = []
    for bits in (0, 1 << 10, 1 << 11, 3 << 10):
        y = torch.full((N, OH, OW, nat.round_up(cout, 8)), 7.0, device=DEV)
        t, i, al = nat.conv_args(spec, xg, N, H, W, y, cfg=cfg)
        i[20] = cfg | bits   # (the op's cfg int; tools/microbench.py --ablate patches it the same way)
        nat.ops().conv(t, i, al)
        outs.append(y)
    torch.cuda.synchronize()
    for bits, y in zip((1 << 10, 1 << 11, 3 << 10), outs[1:]):
        assert torch.equal(y, outs[0]), (cfg, bits)


@pytest.mark.parametrize("cfg", [0, 4, 6, 7, 9, 10, 11, 12, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 33, 34,
                                 35, 36, 37, 38, 39, 40, 41, 42, 43])
def test_conv_epilogues(cfg):
    """relu / residual (pre and post) / alpha / bf16 output / channel offsets."""
    nat = _nat()
    torch.manual_seed(1)
    N, H, W, cin, cout = 2, 10, 12, 32, 48
    x = torch.randn(N, H, W, cin)
    k = torch.randn(3, 3, cin, cout) / math.sqrt(9 * cin)
    b = torch.randn(cout) * 0.1
    res = torch.randn(N, H, W, cout)
    base = R.conv2d_nhwc(_bf(x), _bf(k), b, (1, 1), (1, 1))
    spec = nat.make_spec(k, b, (1, 1), (1, 1), device=DEV)
    xg = x.to(DEV, torch.bfloat16).contiguous()
    rg = res.to(DEV, torch.bfloat16).contiguous()
    y = nat.conv2d(spec, xg, act=nat.ACT_RELU, out_dtype=torch.float32, res=rg, res_post=0, cfg=cfg)
    assert _rel(y.cpu(), torch.relu(base + _bf(res))) < 3e-3
    y = nat.conv2d(spec, xg, act=nat.ACT_RELU, out_dtype=torch.float32, res=rg, res_post=1, cfg=cfg)
    assert _rel(y.cpu(), torch.relu(torch.relu(base) + _bf(res))) < 3e-3
    y = nat.conv2d(spec, xg, act=nat.ACT_NONE, out_dtype=torch.float32, alpha=0.25, cfg=cfg)
    assert _rel(y.cpu(), 0.25 * base) < 3e-3
    # write into a channel slice of a wider buffer, plus a second copy
    big = torch.full((N * H * W, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    big2 = torch.zeros((N * H * W, 64), dtype=torch.bfloat16, device=DEV)
    t, i, a = nat.conv_args(spec, xg, N, H, W, big, y_coff=8, act=nat.ACT_TANH, y2=big2, y2_coff=16, cfg=cfg)
    nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    exp = torch.tanh(base).reshape(-1, cout)
    assert _rel(big[:, 8:56].float().cpu(), exp) < 1e-2
    assert (big[:, :8] == 7).all() and (big[:, 56:] == 7).all()
    assert _rel(big2[:, 16:64].float().cpu(), exp) < 1e-2


def _gru_ref(h, x, kz, bz, kr, br, kq, bq, pad):
    hx = torch.cat([h, x], -1)
    z = torch.sigmoid(R.conv2d_nhwc(_bf(hx), _bf(kz), bz, (1, 1), pad))
    r = torch.sigmoid(R.conv2d_nhwc(_bf(hx), _bf(kr), br, (1, 1), pad))
    q = torch.tanh(R.conv2d_nhwc(_bf(torch.cat([r * h, x], -1)), _bf(kq), bq, (1, 1), pad))
    return (1 - z) * h + z * q


@pytest.mark.parametrize("cfg", [None, 0, 6, 8, 9, 10, 11, 12, 13, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 33, 34,
                                 35, 36, 37, 38, 39, 40, 41, 42, 43])
@pytest.mark.parametrize("hidden,xin,ks,pad", [(128, 256, (1, 5), (0, 2)), (128, 256, (5, 1), (2, 0)),
                                               (96, 146, (3, 3), (1, 1))])
def test_gru_fused_epilogues(hidden, xin, ks, pad, cfg):
    nat = _nat()
    torch.manual_seed(2)
    B, h, w = 2, 11, 13
    M = B * h * w
    cin = hidden + xin
    cs = nat.round_up(cin, 8)
    hs = torch.tanh(torch.randn(B, h, w, hidden))
    xs = torch.randn(B, h, w, xin)
    ks_ = [torch.randn(*ks, cin, hidden) / math.sqrt(ks[0] * ks[1] * cin) for _ in range(3)]
    bs_ = [torch.randn(hidden) * 0.1 for _ in range(3)]
    ref = _gru_ref(hs, xs, ks_[0], bs_[0], ks_[1], bs_[1], ks_[2], bs_[2], pad)
    hx = torch.zeros(M, cs, dtype=torch.bfloat16, device=DEV)
    hx[:, :hidden] = hs.reshape(M, hidden).to(DEV, torch.bfloat16)
    hx[:, hidden:cin] = xs.reshape(M, xin).to(DEV, torch.bfloat16)
    qx = hx.clone()
    h32 = hs.reshape(M, hidden).to(DEV).contiguous()
    zb = torch.empty(M, hidden, device=DEV)
    sa = nat.make_spec(torch.cat([ks_[0], ks_[1]], 3), torch.cat([bs_[0], bs_[1]]), (1, 1), pad, cin8=cs, device=DEV)
    sb = nat.make_spec(ks_[2], bs_[2], (1, 1), pad, cin8=cs, device=DEV)
    nat.ops().conv(*nat.conv_args(sa, hx, B, h, w, qx, h32=h32, zbuf=zb, hidden=hidden, epi=nat.EPI_GRU_A, cfg=cfg))
    nat.ops().conv(*nat.conv_args(sb, qx, B, h, w, hx, h32=h32, zbuf=zb, hidden=hidden, epi=nat.EPI_GRU_B, cfg=cfg))
    torch.cuda.synchronize()
    out = h32.cpu().reshape(B, h, w, hidden)
    # r*h is quantised to bf16 before the q conv in the kernel; reference uses fp32 r*h -> bf16 as well
    assert (out - ref).abs().max().item() < 2e-2
    assert (hx[:, :hidden].float().cpu() - ref.reshape(M, hidden)).abs().max().item() < 2.5e-2


@pytest.mark.parametrize("g2", [0, 1])
@pytest.mark.parametrize("map_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,h,w,vertical", [(2, 7, 13, 0), (2, 7, 13, 1), (2, 9, 12, 1), (1, 55, 128, 0),
                                            (1, 55, 128, 1), (3, 5, 3, 1), (1, 64, 20, 1), (1, 4, 128, 0)])
def test_gru_stage_fused_kernel(B, h, w, vertical, map_dtype, g2):
    """gru_fused.hip (one launch per ConvGRU stage, r*h and z kept in the CU) vs the fp32
    ConvGRU of the reference with the context share as a per-pixel bias map (model.py:301-312):
    row tiles (1x5) and 1- / 2-column tiles (5x1), incl. the headline's 55 x 128 grid."""
    nat = _nat()
    torch.manual_seed(5)
    hd, M = 128, B * h * w
    ks = (5, 1) if vertical else (1, 5)
    pad = (2, 0) if vertical else (0, 2)
    hs = torch.tanh(torch.randn(B, h, w, hd))
    xs = torch.randn(B, h, w, hd)
    kz, kr, kq = [torch.randn(*ks, 2 * hd, hd) / math.sqrt(5 * 2 * hd) for _ in range(3)]
    bm = torch.randn(B, h, w, 384) * 0.5
    if map_dtype == torch.bfloat16:
        bm = _bf(bm)
    zero = torch.zeros(hd)
    hxr = torch.cat([hs, xs], -1)
    z = torch.sigmoid(R.conv2d_nhwc(_bf(hxr), _bf(kz), zero, (1, 1), pad) + bm[..., :hd])
    r = torch.sigmoid(R.conv2d_nhwc(_bf(hxr), _bf(kr), zero, (1, 1), pad) + bm[..., hd:2 * hd])
    q = torch.tanh(R.conv2d_nhwc(_bf(torch.cat([_bf(r * _bf(hs)), xs], -1)), _bf(kq), zero, (1, 1), pad)
                   + bm[..., 2 * hd:])
    ref = ((1 - z) * hs + z * q).reshape(M, hd)
    hx = torch.cat([hs, xs], -1).reshape(M, 2 * hd).to(DEV, torch.bfloat16).contiguous()
    h32 = hs.reshape(M, hd).to(DEV).contiguous()
    sa = nat.make_spec(torch.cat([kz, kr], 3), torch.zeros(2 * hd), (1, 1), pad, cin8=256, device=DEV)
    sb = nat.make_spec(kq, zero, (1, 1), pad, cin8=256, device=DEV)
    assert nat.ops().gru_fused_fits(h, w, vertical)
    hm = torch.full((M, hd), 7.0, dtype=torch.bfloat16, device=DEV)
    bmg = bm.reshape(M, 384).to(DEV, map_dtype).contiguous()
    # g2: GEMM 2 on the 8 z waves (0) or all 16 waves (1, the engine's choice)
    nat.ops().gru_fused([hx, sa.w, sb.w, bmg, h32, hx, hm], [B, h, w, vertical, g2])
    torch.cuda.synchronize()
    assert (h32.cpu() - ref).abs().max().item() < 2e-2
    assert (hx[:, :hd].float().cpu() - ref).abs().max().item() < 2.5e-2
    assert torch.equal(hm, hx[:, :hd])
    assert torch.equal(hx[:, hd:].float().cpu(), _bf(xs.reshape(M, hd)))   # x untouched


def test_gru_fused_fits():
    nat = _nat()
    assert nat.ops().gru_fused_fits(55, 128, 0) and nat.ops().gru_fused_fits(55, 128, 1)
    assert not nat.ops().gru_fused_fits(55, 129, 0)      # a row wider than a tile
    assert not nat.ops().gru_fused_fits(130, 64, 1)      # a column taller than a tile


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("h,w,C,L", [(16, 16, 64, 4), (23, 37, 128, 4), (55, 128, 256, 4), (17, 20, 64, 2),
                                     (13, 48, 64, 3)])
def test_corr_pyramid(h, w, C, L, dtype):
    """All-pairs volume + pooled levels vs the fp32 reference; bf16 levels of
    /16-wide maps take the LDS-staged wide-store epilogue (odd heights: partial
    tiles and floor-pooled rows), the rest the per-lane stores."""
    nat = _nat()
    torch.manual_seed(4)
    B = 2
    f1 = torch.randn(B, h, w, C)
    f2 = torch.randn(B, h, w, C)
    ref = R.build_pyramid(_bf(f1), _bf(f2), L)
    M = B * h * w
    lv = []
    hl, wl = h, w
    for _ in range(L):
        lv.append(torch.full((M, hl, wl), float("nan"), device=DEV, dtype=dtype))
        hl //= 2
        wl //= 2
    g1 = f1.to(DEV, torch.bfloat16).contiguous()
    g2 = f2.to(DEV, torch.bfloat16).contiguous()
    nat.ops().corr([g1, g2] + lv + [None] * (4 - L), [B, h, w, C, L], 1.0 / math.sqrt(C))
    torch.cuda.synchronize()
    tol = 1e-3 if dtype == torch.float32 else 8e-3
    for l in range(L):
        got = lv[l].float().cpu()
        assert not torch.isnan(got).any(), f"level {l} has unwritten cells"
        assert (got - ref[l]).abs().max().item() < tol * max(1.0, ref[l].abs().max().item()), l


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("h,w", [(17, 19), (17, 64)])
@pytest.mark.parametrize("radius,L", [(4, 4), (3, 4), (2, 2), (5, 2)])
def test_corr_lookup(radius, L, h, w, dtype):
    """Radius-r pyramid lookup vs the fp32 reference (model.py:448-470): odd
    widths take the per-lane column kernel, /64 widths (every level a whole
    number of 16-byte chunks) the wide-load kernel (radius <= 4)."""
    nat = _nat()
    torch.manual_seed(5)
    B = 2
    M = B * h * w
    pyr = []
    hl, wl = h, w
    for _ in range(L):
        pyr.append(torch.randn(M, hl, wl).to(dtype).float())
        hl //= 2
        wl //= 2
    # coords: in range, fractional, and far outside (zero padding)
    coords = R.make_coords_grid(B, h, w) + torch.randn(B, h, w, 2) * 4
    coords[0, 0, 0] = torch.tensor([-30.5, 3.25])
    coords[1, 2, 3] = torch.tensor([h + 40.0, w + 7.5])
    ref = R.index_pyramid(pyr, coords, radius)
    S = 2 * radius + 1
    ocs = nat.round_up(L * S * S, 8)
    out = torch.full((M, ocs), 5.0, dtype=torch.bfloat16, device=DEV)
    nat.ops().lookup([coords.reshape(M, 2).to(DEV).contiguous(), out] + [p.to(DEV, dtype) for p in pyr]
                     + [None] * (4 - L), [L, B, h, w, radius])
    torch.cuda.synchronize()
    got = out.float().cpu()
    assert (got[:, L * S * S:] == 0).all()
    err = (got[:, : L * S * S] - ref.reshape(M, -1)).abs().max().item()
    assert err < 3e-2 * ref.abs().max().item(), err


def test_upsample_convex_and_bilinear():
    nat = _nat()
    torch.manual_seed(6)
    B, h, w = 2, 7, 9
    M = B * h * w
    flow = torch.randn(B, h, w, 2) * 3
    mask = torch.randn(B, h, w, 576)
    ref = R.upsample_flow(flow, _bf(mask))
    out = torch.zeros(2, B, 8 * h, 8 * w, 2, device=DEV)
    nat.ops().upsample_convex([mask.reshape(M, 576).to(DEV, torch.bfloat16).contiguous(),
                               flow.reshape(M, 2).to(DEV).contiguous(), out], [B, h, w, B * 64 * h * w * 2])
    torch.cuda.synchronize()
    # eager ops run as iteration 0 of a plan: the per-iteration stride only applies inside plans
    assert (out[0].cpu() - ref).abs().max().item() < 1e-3 * ref.abs().max().item() + 1e-4
    assert (out[1] == 0).all()
    refb = R.upsample_flow(flow, None)
    outb = torch.zeros(1, B, 8 * h, 8 * w, 2, device=DEV)
    nat.ops().upsample_bilinear([flow.reshape(M, 2).to(DEV).contiguous(), outb], [B, h, w, 0])
    torch.cuda.synchronize()
    assert (outb[0].cpu() - refb).abs().max().item() < 1e-4 * refb.abs().max().item() + 1e-5


@pytest.mark.parametrize("C", [64, 96, 128, 24])
def test_instance_norm_stats_apply(C):
    nat = _nat()
    torch.manual_seed(7)
    N, H, W = 3, 37, 29
    x = _bf(torch.randn(N, H, W, C) * 2 + 0.5)
    r = _bf(torch.randn(N, H, W, C))
    xg = x.to(DEV, torch.bfloat16).contiguous()
    rg = r.to(DEV, torch.bfloat16).contiguous()
    st = torch.empty(N, C, 2, device=DEV)
    sr = torch.empty(N, C, 2, device=DEV)
    nat.ops().stats([xg, st], [N, H * W, C])
    nat.ops().stats([rg, sr], [N, H * W, C])
    y = torch.empty_like(xg)
    # relu(relu(IN(x)) + IN(r))
    nat.ops().norm_act([xg, st, None, None, rg, sr, None, None, y], [1, 1, N, H * W, C, 3], 1e-5)
    torch.cuda.synchronize()
    ref = torch.relu(torch.relu(R.instance_norm_nhwc(x)) + R.instance_norm_nhwc(r))
    assert (y.float().cpu() - ref).abs().max().item() < 3e-2
    y2 = torch.empty_like(xg)
    nat.ops().norm_act([xg, st, None, None, rg, None, None, None, y2], [1, 0, N, H * W, C, 2], 1e-5)
    torch.cuda.synchronize()
    ref2 = torch.relu(R.instance_norm_nhwc(x) + r)
    assert (y2.float().cpu() - ref2).abs().max().item() < 3e-2
    # BatchNorm statistics (mode 2: over batch and map) with an affine, relu only
    gam = torch.rand(C) + 0.5
    bet = torch.randn(C) * 0.1
    y3 = torch.empty_like(xg)
    nat.ops().norm_act([xg, st, gam.to(DEV), bet.to(DEV), None, None, None, None, y3], [2, 0, N, H * W, C, 1], 1e-5)
    torch.cuda.synchronize()
    xb = x.to(torch.bfloat16).float()
    m, v = xb.mean((0, 1, 2)), xb.var((0, 1, 2), unbiased=False)
    ref3 = torch.relu((xb - m) * torch.rsqrt(v + 1e-5) * gam + bet)
    assert (y3.float().cpu() - ref3).abs().max().item() < 3e-2


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 12, 13, 14, 15, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 33, 34,
                                 35, 36, 37, 38, 39, 40, 41, 42, 43])
def test_conv_bias_map(cfg):
    """Per-pixel fp32 bias map (the folded context share of the GRU gates):
    conv(x) + bias + bmap[:, coff:coff+cout] before the activation."""
    nat = _nat()
    torch.manual_seed(7)
    N, H, W, cin, cout = 2, 9, 21, 64, 96
    x = torch.randn(N, H, W, cin)
    k = torch.randn(1, 5, cin, cout) * 0.05
    b = torch.randn(cout) * 0.1
    bm = torch.randn(N * H * W, 136)
    base = R.conv2d_nhwc(_bf(x), _bf(k), b, (1, 1), (0, 2)).reshape(-1, cout)
    spec = nat.make_spec(k, b, (1, 1), (0, 2), device=DEV)
    xg = x.to(DEV, torch.bfloat16).contiguous()
    y = torch.zeros(N * H * W, cout, dtype=torch.float32, device=DEV)
    t, i, a = nat.conv_args(spec, xg, N, H, W, y, act=nat.ACT_SIGMOID, cfg=cfg, bmap=bm.to(DEV), bmap_coff=40)
    nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    assert _rel(y.cpu(), torch.sigmoid(base + bm[:, 40:40 + cout])) < 3e-3
    # bf16 bias map
    t, i, a = nat.conv_args(spec, xg, N, H, W, y, act=nat.ACT_SIGMOID, cfg=cfg, bmap=bm.to(DEV, torch.bfloat16),
                            bmap_coff=40)
    nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    assert _rel(y.cpu(), torch.sigmoid(base + _bf(bm[:, 40:40 + cout]))) < 3e-3


@pytest.mark.parametrize("cfg", [None, 4, 5, 24])
def test_flow_taps(cfg):
    """FlowHead.conv2 as a 1x1 conv to 9 x 2 per-tap partials (tap-major
    output channels) + flow_taps (shifted-partial sum, coords update, flow copies)."""
    nat = _nat()
    torch.manual_seed(8)
    B, h, w, cin = 2, 9, 70, 256
    M = B * h * w
    fm = torch.randn(B, h, w, cin) * 0.5
    k = torch.randn(3, 3, cin, 2) / math.sqrt(9 * cin)
    b = torch.randn(2) * 0.1
    coords = torch.randn(M, 2) * 5
    delta = R.conv2d_nhwc(_bf(fm), _bf(k), b, (1, 1), (1, 1)).reshape(M, 2)
    new = coords + delta
    grid = torch.stack(torch.meshgrid(torch.arange(w).float(), torch.arange(h).float(), indexing="xy"), -1)
    flow_ref = new - grid[None].expand(B, h, w, 2).reshape(M, 2)
    k18 = k.reshape(9, cin, 2).permute(1, 0, 2).reshape(1, 1, cin, 18)
    spec = nat.make_spec(k18, torch.zeros(18), device=DEV)
    taps = torch.zeros(M, 24, device=DEV)
    fmg = fm.to(DEV, torch.bfloat16).contiguous()
    nat.ops().conv(*nat.conv_args(spec, fmg, B, h, w, taps, cfg=cfg))
    cg = coords.to(DEV).contiguous()
    f32 = torch.zeros(M, 2, device=DEV)
    hx = torch.zeros(M, 24, device=DEV, dtype=torch.bfloat16)
    qx = torch.zeros(M, 24, device=DEV, dtype=torch.bfloat16)
    f8 = torch.zeros(M, 8, device=DEV, dtype=torch.bfloat16)
    nat.ops().flow_taps([taps, b.to(DEV), cg, f32, hx, qx, f8], [B, h, w, 16, 8])
    torch.cuda.synchronize()
    tol = 1e-3 * flow_ref.abs().max().item() + 1e-3
    assert (cg.cpu() - new).abs().max().item() < tol
    assert (f32.cpu() - flow_ref).abs().max().item() < tol
    assert torch.equal(hx[:, 16:18], qx[:, 8:10]) and torch.equal(hx[:, 16:18], f8[:, :2])
    assert (hx[:, :16] == 0).all() and (hx[:, 18:] == 0).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_corr_query_slab_and_lookup(dtype):
    """Context-parallel query slabs (parallel/cp.py): the corr kernel on rows
    [r0, r1) of fmap1 (nq = slab pixels) reproduces those rows of the full
    pyramid, and the lookup of the slab's coords against slab-sized level
    buffers reproduces those rows of the full lookup."""
    nat = _nat()
    torch.manual_seed(9)
    B, h, w, C, L, radius = 2, 23, 37, 128, 4, 4
    r0, r1 = 7, 16
    nq = (r1 - r0) * w
    f1 = torch.randn(B, h, w, C).to(DEV, torch.bfloat16)
    f2 = torch.randn(B, h, w, C).to(DEV, torch.bfloat16)

    def levels(M):
        out, hl, wl = [], h, w
        for _ in range(L):
            out.append(torch.full((M, hl, wl), float("nan"), device=DEV, dtype=dtype))
            hl //= 2
            wl //= 2
        return out

    full = levels(B * h * w)
    nat.ops().corr([f1, f2] + full, [B, h, w, C, L], 1.0 / math.sqrt(C))
    part = levels(B * nq)
    nat.ops().corr([f1[:, r0:r1].contiguous(), f2] + part, [B, h, w, C, L, nq], 1.0 / math.sqrt(C))
    torch.cuda.synchronize()
    for a, b in zip(full, part):
        rows = a.reshape(B, h, w, *a.shape[1:])[:, r0:r1].reshape(B * nq, *a.shape[1:])
        assert not torch.isnan(b).any()
        assert torch.equal(b, rows)
    S = 2 * radius + 1
    ocs = nat.round_up(L * S * S, 8)
    coords = (R.make_coords_grid(B, h, w) + torch.randn(B, h, w, 2) * 3).to(DEV)
    out_full = torch.empty(B * h * w, ocs, dtype=torch.bfloat16, device=DEV)
    nat.ops().lookup([coords.reshape(-1, 2).contiguous(), out_full] + full, [L, B, h, w, radius])
    cs = coords[:, r0:r1].reshape(-1, 2).contiguous()
    out_part = torch.empty(B * nq, ocs, dtype=torch.bfloat16, device=DEV)
    nat.ops().lookup([cs, out_part] + part, [L, B, h, w, radius, nq])
    torch.cuda.synchronize()
    ref = out_full.reshape(B, h, w, ocs)[:, r0:r1].reshape(B * nq, ocs)
    assert torch.equal(out_part, ref)
    if dtype == torch.float32:  # backward of the slab lookup == rows of the full backward
        g = torch.randn(B * h * w, ocs, device=DEV)
        dfull = [torch.zeros_like(l) for l in full]
        nat.ops().lookup_bwd([coords.reshape(-1, 2).contiguous(), g] + dfull, [L, B, h, w, radius])
        dpart = [torch.zeros_like(l) for l in part]
        gp = g.reshape(B, h, w, ocs)[:, r0:r1].reshape(B * nq, ocs).contiguous()
        nat.ops().lookup_bwd([cs, gp] + dpart, [L, B, h, w, radius, nq])
        torch.cuda.synchronize()
        for a, b in zip(dfull, dpart):
            assert torch.equal(b, a.reshape(B, h, w, *a.shape[1:])[:, r0:r1].reshape(B * nq, *a.shape[1:]))


def test_context_parallel_single_gpu_matches_engine():
    """ContextParallelRAFT (one slab: the native slab kernels + module path)
    against the golden fp32 forward on the same weights."""
    from jax_raft_amd import raft_small
    from jax_raft_amd.parallel.cp import ContextParallelRAFT

    model, variables = raft_small(seed=0)
    g = torch.Generator().manual_seed(4)
    i1 = torch.rand(1, 128, 160, 3, generator=g) * 2 - 1
    i2 = torch.rand(1, 128, 160, 3, generator=g) * 2 - 1
    ref = model.apply(variables, i1, i2, num_flow_updates=3)
    out = ContextParallelRAFT(model.cuda())(i1.cuda(), i2.cuda(), num_flow_updates=3).cpu()
    epe = (out[-1] - ref[-1]).norm(dim=-1).mean().item()
    assert epe < 0.05 * ref[-1].norm(dim=-1).mean().item() + 0.05, epe


@pytest.mark.parametrize("kh,cout,xcs,ycs,ycoff", [(7, 128, 8, 128, 0), (7, 128, 2, 128, 0), (7, 64, 8, 96, 32),
                                                   (7, 64, 2, 64, 0), (3, 32, 2, 32, 0)])
def test_conv_direct(kh, cout, xcs, ycs, ycoff):
    """Direct VALU conv (conv_direct.hip: the flow branch's 7x7 on 2 channels) vs fp32 conv."""
    nat = _nat()
    torch.manual_seed(12)
    N, H, W = 2, 19, 27
    x = torch.randn(N, H, W, 2) * 3
    k = torch.randn(kh, kh, 2, cout) * 0.2
    b = torch.randn(cout)
    p = kh // 2
    ref = torch.relu(R.conv2d_nhwc(_bf(x), k, b, (1, 1), (p, p)))
    xb = torch.zeros(N, H, W, xcs, dtype=torch.bfloat16)
    xb[..., :2] = x.to(torch.bfloat16)
    y = torch.full((N * H * W, ycs), 7.0, dtype=torch.bfloat16, device=DEV)
    nat.ops().conv_direct([xb.to(DEV), nat.pack_direct_weight(k).to(DEV), b.to(DEV), y],
                          [N, H, W, 2, kh, kh, p, p, cout, 1, ycoff])
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert (got[:, :ycoff] == 7.0).all() and (got[:, ycoff + cout:] == 7.0).all()
    assert _rel(got[:, ycoff:ycoff + cout], ref.reshape(-1, cout)) < 1e-2


@pytest.mark.parametrize("h,w,L,radius,C", [(55, 128, 4, 4, 64), (13, 48, 3, 3, 64), (16, 32, 2, 4, 64),
                                             (55, 128, 4, 4, 256), (13, 48, 3, 3, 128), (21, 32, 4, 4, 256),
                                             (8, 16, 1, 2, 128)])
def test_corr_blocked_layout_pyramid_and_lookup(h, w, L, radius, C):
    """Blocked level layout (levels 0 / 1 stored as the pyramid kernel's 8x16
    tiles): the pyramid written blocked equals the row-major reference once
    un-blocked, and the lookup on it (wide and per-lane kernels) matches the
    reference lookup of the row-major pyramid.  C = 128 / 256: the persistent
    kernel of corr_pyr.hip (partial query tiles at 13 x 48, 21 x 32); C = 64: the
    tile kernel of corr.hip."""
    nat = _nat()
    torch.manual_seed(9)
    B = 2
    f1 = torch.randn(B, h, w, C)
    f2 = torch.randn(B, h, w, C)
    ref = R.build_pyramid(_bf(f1), _bf(f2), L)
    M = B * h * w
    nty, ntx = -(-h // 8), -(-w // 16)
    lv = []
    hl, wl = h, w
    for l in range(L):
        shape = (M, nty * (8 >> l), ntx * (16 >> l)) if l < 2 else (M, hl, wl)
        lv.append(torch.full(shape, float("nan"), device=DEV, dtype=torch.bfloat16))
        hl //= 2
        wl //= 2
    g1 = f1.to(DEV, torch.bfloat16).contiguous()
    g2 = f2.to(DEV, torch.bfloat16).contiguous()
    nat.ops().corr([g1, g2] + lv + [None] * (4 - L), [B, h, w, C, L, h * w, 1], 1.0 / math.sqrt(C))
    torch.cuda.synchronize()
    hl, wl = h, w
    for l in range(L):
        got = lv[l].float().cpu()
        if l < 2:
            bh, bw = 8 >> l, 16 >> l
            got = got.reshape(M, nty, ntx, bh, bw).permute(0, 1, 3, 2, 4).reshape(M, nty * bh, ntx * bw)[:, :hl, :wl]
        assert not torch.isnan(got).any(), f"level {l} has unwritten cells"
        assert (got - ref[l]).abs().max().item() < 8e-3 * max(1.0, ref[l].abs().max().item()), l
        hl //= 2
        wl //= 2
    coords = R.make_coords_grid(B, h, w) + torch.randn(B, h, w, 2) * 5
    coords[0, 0, 0] = torch.tensor([-30.5, 3.25])
    coords[1, 2, 3] = torch.tensor([w + 9.0, h - 0.5])
    want = R.index_pyramid([r.to(torch.bfloat16).float() for r in ref], coords, radius)
    S = 2 * radius + 1
    ocs = nat.round_up(L * S * S, 8)
    out = torch.full((M, ocs), 5.0, dtype=torch.bfloat16, device=DEV)
    nat.ops().lookup([coords.reshape(M, 2).to(DEV).contiguous(), out] + lv + [None] * (4 - L),
                     [L, B, h, w, radius, h * w, 1])
    torch.cuda.synchronize()
    got = out.float().cpu()
    assert (got[:, L * S * S:] == 0).all()
    err = (got[:, : L * S * S] - want.reshape(M, -1)).abs().max().item()
    assert err < 3e-2 * want.abs().max().item(), err


@pytest.mark.parametrize("blocked,w", [(1, 64), (0, 20)])
def test_lookup_with_fused_update_is_bitwise(blocked, w):
    """The flow update fused into the lookup (corr.hip: lookup_coords; the engine
    runs iteration i's update inside iteration i+1's lookup) = the separate
    flow_taps kernel followed by the plain lookup, bitwise: coordinates, flow
    copies and sampled features (wide blocked-level kernel and per-lane kernel)."""
    nat = _nat()
    torch.manual_seed(19)
    B, h, C, L, radius = 2, 16, 64, 4, 4
    M = B * h * w
    g1 = torch.randn(B, h, w, C).to(DEV, torch.bfloat16)
    g2 = torch.randn(B, h, w, C).to(DEV, torch.bfloat16)
    nty, ntx = -(-h // 8), -(-w // 16)
    lv, hl, wl = [], h, w
    for l in range(L):
        shape = (M, nty * (8 >> l), ntx * (16 >> l)) if (blocked and l < 2) else (M, hl, wl)
        lv.append(torch.zeros(shape, device=DEV, dtype=torch.bfloat16))
        hl //= 2
        wl //= 2
    nat.ops().corr([g1, g2] + lv, [B, h, w, C, L, h * w, blocked], 1.0 / math.sqrt(C))
    taps = (torch.randn(M, 24) * 2).to(DEV)
    bias = torch.randn(2).to(DEV)
    coords0 = (R.make_coords_grid(B, h, w).reshape(M, 2) + torch.randn(M, 2) * 3).to(DEV)
    S = 2 * radius + 1
    ocs = nat.round_up(L * S * S, 8)
    res = []
    for fused in (False, True):
        coords = coords0.clone()
        f32 = torch.zeros(M, 2, device=DEV)
        hx = torch.zeros(M, 24, device=DEV, dtype=torch.bfloat16)
        qx = torch.zeros(M, 24, device=DEV, dtype=torch.bfloat16)
        f8 = torch.zeros(M, 2, device=DEV, dtype=torch.bfloat16)
        out = torch.zeros(M, ocs, device=DEV, dtype=torch.bfloat16)
        if fused:
            nat.ops().lookup([coords, out] + lv + [taps, bias, f32, hx, qx, f8], [L, B, h, w, radius, h * w, blocked, 16, 8])
        else:
            nat.ops().flow_taps([taps, bias, coords, f32, hx, qx, f8], [B, h, w, 16, 8])
            nat.ops().lookup([coords, out] + lv, [L, B, h, w, radius, h * w, blocked])
        torch.cuda.synchronize()
        res.append((coords, f32, hx, qx, f8, out))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("K,cs,coff,M", [(256, 256, 0, 1000), (256, 512, 0, 28160), (128, 136, 8, 777)])
def test_taps_gemm_matches_fp32(K, cs, coff, M):
    """flowhead.hip taps GEMM (the flow head's 3x3 output conv as 9 x 2 per-pixel
    taps) vs an fp32 matmul with the engine's tap order (tap * 2 + channel)."""
    nat = _nat()
    g = torch.Generator().manual_seed(K + M)
    fm = torch.randn(M, cs, generator=g).to(torch.bfloat16)
    kern = torch.randn(3, 3, K, 2, generator=g) * 0.05
    wpk = nat.pack_taps(kern)
    got = nat.taps_gemm(fm.to(DEV), wpk.to(DEV), K, coff).cpu()
    w = kern.reshape(9, K, 2).permute(1, 0, 2).reshape(K, 18)
    ref = fm[:, coff:coff + K].float() @ w.to(torch.bfloat16).float()
    assert (got[:, 18:] == 0).all()
    assert (got[:, :18] - ref).abs().max().item() < 1e-3 * ref.abs().max().item() + 1e-4


@pytest.mark.parametrize("K,cs,kpad,N,M", [(324, 328, 352, 256, 28160), (324, 328, 352, 256, 1001), (256, 256, 256, 128, 777),
                                           (120, 128, 128, 64, 64)])
def test_conv1x1_lds_matches_fp32(K, cs, kpad, N, M):
    """conv1x1.hip (weights per 64-channel group in LDS, all k-steps of a
    wave's pixels loaded up front, packed row permutation) vs fp32 matmul +
    bias + ReLU; channels past K in the input rows are zero-weighted."""
    nat = _nat()
    g = torch.Generator().manual_seed(K + M)
    x = torch.randn(M, cs, generator=g)
    x[:, K:] = 0
    x = x.to(torch.bfloat16)
    kern = torch.randn(1, 1, K, N, generator=g) * 0.05
    bias = torch.randn(N, generator=g) * 0.1
    wpk = nat.pack_conv1x1(kern, kpad)
    y = nat.conv1x1(x.to(DEV), wpk.to(DEV), bias.to(DEV), cs, kpad, N, act=nat.ACT_RELU).float().cpu()
    ref = torch.relu(x[:, :K].float() @ kern.reshape(K, N).to(torch.bfloat16).float() + bias)
    assert (y - ref).abs().max().item() < 1e-2 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("cfg", [34, 22, 35, 38])
def test_conv_taps_epilogue(cfg):
    """EPI_TAPS: FlowHead conv1 (3x3, 128 -> 256, relu) whose epilogue multiplies
    its features by the 18 taps of conv2 (MFMA) -> fp32 taps [M][24]; against
    fp32 torch of relu(conv1) . Wt (features rounded to bf16 as the kernel feeds them)."""
    nat = _nat()
    torch.manual_seed(11)
    N, H, W, cin = 2, 11, 37, 128
    M = N * H * W
    x = torch.randn(N, H, W, cin)
    k1 = torch.randn(3, 3, cin, 256) / math.sqrt(9 * cin)
    b1 = torch.randn(256) * 0.1
    k2 = torch.randn(3, 3, 256, 2) * 0.05
    fm = torch.relu(R.conv2d_nhwc(_bf(x), _bf(k1), b1, (1, 1), (1, 1))).reshape(M, 256)
    wt = k2.reshape(9, 256, 2).permute(1, 0, 2).reshape(256, 18)
    ref = _bf(fm) @ _bf(wt)
    spec = nat.make_spec(k1, b1, (1, 1), (1, 1), device=DEV)
    xg = x.to(DEV, torch.bfloat16).contiguous()
    taps = torch.full((M, 24), 7.0, device=DEV)
    t, i, a = nat.conv_args(spec, xg, N, H, W, taps, act=nat.ACT_RELU, epi=nat.EPI_TAPS, cfg=cfg,
                            tapw=nat.pack_taps_epi(k2.to(DEV)))
    nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    out = taps.cpu()
    assert _rel(out[:, :18], ref) < 5e-3
    assert (out[:, 18:] == 7.0).all()


@pytest.mark.parametrize("B,H,W", [(1, 16, 24), (2, 40, 56)])
def test_s2d_stem_matches_7x7_stride2(B, H, W):
    """Space-to-depth prep (elementwise.hip:prep_images_s2d_kernel) + the 4x4 / stride-1 form of
    the 7x7 / stride-2 stem (ops/native.py:s2d_stem_kernel, top / left pad 2, output H/2 x W/2)
    vs the fp32 7x7 conv of the reference (model.py:238-240)."""
    nat = _nat()
    torch.manual_seed(6)
    i1, i2 = torch.rand(B, H, W, 3) * 2 - 1, torch.rand(B, H, W, 3) * 2 - 1
    k = torch.randn(7, 7, 3, 64) / math.sqrt(147)
    b = torch.randn(64) * 0.1
    x0 = torch.zeros(2 * B, H // 2, W // 2, 16, dtype=torch.bfloat16, device=DEV)
    nat.ops().prep([i1.to(DEV), i2.to(DEV), x0], [B, H, W, 1])
    spec = nat.make_spec(nat.s2d_stem_kernel(k), b, (1, 1), (2, 2), cin8=16, device=DEV)
    y = torch.empty(2 * B, H // 2, W // 2, 64, dtype=torch.float32, device=DEV)
    nat.ops().conv(*nat.conv_args(spec, x0, 2 * B, H // 2, W // 2, y, out_hw=(H // 2, W // 2)))
    torch.cuda.synchronize()
    ref = R.conv2d_nhwc(_bf(torch.cat([i1, i2])), _bf(k), b, (2, 2), (3, 3))
    assert y.shape == ref.shape
    assert _rel(y.cpu(), ref) < 3e-3


@pytest.mark.parametrize("B,h,w,L", [(2, 12, 16, 4), (1, 9, 12, 3), (2, 16, 24, 4), (1, 9, 16, 4), (1, 13, 40, 2)])
def test_pyr_bwd_dc(B, h, w, L):
    """Correlation-pyramid backward, first half (train.hip: pyr_bwd_dc, pyr_bwd_dc8v for w % 8 == 0):
    dC = s (g0 + sum_l nearest-upsampled g_l / 4^l) over the floor-pooled region, bf16."""
    nat = _nat()
    torch.manual_seed(7)
    M = B * h * w
    gs, hl, wl = [], h, w
    for _ in range(L):
        gs.append(torch.randn(M, hl, wl))
        hl //= 2
        wl //= 2
    ref = gs[0].clone()
    for l in range(1, L):
        g = gs[l]
        up = g.repeat_interleave(2 ** l, 1).repeat_interleave(2 ** l, 2) / 4 ** l
        ref[:, :up.shape[1], :up.shape[2]] += up
    ref *= 0.0625
    dc = torch.empty(B, h * w, h * w, dtype=torch.bfloat16, device=DEV)
    nat.ops().pyr_bwd_dc([dc] + [g.to(DEV) for g in gs] + [None] * (4 - L), [L, M, h, w], 0.0625)
    torch.cuda.synchronize()
    assert _rel(dc.float().cpu().reshape(M, h, w), ref) < 8e-3


@pytest.mark.parametrize("a_kmajor", [0, 1])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("batch,M,N,K", [(2, 128, 256, 192), (3, 384, 128, 512), (1, 256, 256, 3072)])
def test_bgemm(batch, M, N, K, a_kmajor, out_dtype):
    """bgemm.hip (the pyramid backward's dfmap1 = dC . fmap2 / dfmap2 = dC^T . fmap1): batched
    bf16 GEMM with A row-major or k-major vs fp32 matmul of the same bf16 operands."""
    nat = _nat()
    torch.manual_seed(8)
    a = torch.randn(batch, M, K)
    b = torch.randn(batch, K, N)
    ref = torch.bmm(_bf(a), _bf(b)) * 0.5
    ag = (a.transpose(1, 2) if a_kmajor else a).contiguous().to(DEV, torch.bfloat16)
    c = torch.full((batch, M, N), float("nan"), dtype=out_dtype, device=DEV)
    nat.ops().bgemm([ag, b.to(DEV, torch.bfloat16), c], [M, N, K, a_kmajor], 0.5)
    torch.cuda.synchronize()
    assert not torch.isnan(c.float()).any()
    assert _rel(c.float().cpu(), ref) < (3e-3 if out_dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("C", [128, 256])
def test_corr_blocked_persistent_batch1(C):
    """Blocked layout 2 (runtime/engine.py CORR_PERSIST_B1): the persistent pyramid kernel of
    corr_pyr.hip at batch 1 (the tile kernel of corr.hip served batch 1 before) -- every level
    equals the row-major reference pyramid once un-blocked, and equals the tile kernel's output
    (layout 1) within bf16 rounding."""
    nat = _nat()
    torch.manual_seed(31 + C)
    B, h, w, L = 1, 55, 128, 4
    f1 = torch.randn(B, h, w, C)
    f2 = torch.randn(B, h, w, C)
    ref = R.build_pyramid(_bf(f1), _bf(f2), L)
    M = B * h * w
    nty, ntx = -(-h // 8), -(-w // 16)
    outs = []
    for mode in (1, 2):
        lv, hl, wl = [], h, w
        for l in range(L):
            shape = (M, nty * (8 >> l), ntx * (16 >> l)) if l < 2 else (M, hl, wl)
            lv.append(torch.full(shape, float("nan"), device=DEV, dtype=torch.bfloat16))
            hl //= 2
            wl //= 2
        nat.ops().corr([f1.to(DEV, torch.bfloat16), f2.to(DEV, torch.bfloat16)] + lv,
                       [B, h, w, C, L, h * w, mode], 1.0 / math.sqrt(C))
        torch.cuda.synchronize()
        outs.append(lv)
    hl, wl = h, w
    for l in range(L):
        for lv in outs:
            got = lv[l].float().cpu()
            if l < 2:
                bh, bw = 8 >> l, 16 >> l
                got = got.reshape(M, nty, ntx, bh, bw).permute(0, 1, 3, 2, 4).reshape(M, nty * bh, ntx * bw)[:, :hl, :wl]
            assert not torch.isnan(got).any(), f"level {l} has unwritten cells"
            assert (got - ref[l]).abs().max().item() < 8e-3 * max(1.0, ref[l].abs().max().item()), l
        hl //= 2
        wl //= 2
