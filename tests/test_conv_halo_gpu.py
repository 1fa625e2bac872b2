"""conv_halo.hip (the halo 3x3 / stride-1 conv: LDS input footprint, tap-shifted B
fragments, streamed weights) against the fp32 golden conv (reference.conv2d_nhwc) with
bf16-rounded operands, for every tile config: map sizes that are not multiples of the tile,
a partial last channel block (126 = the motion encoder's conv), channel slices of wider
buffers, the residual epilogue (pre / post), the output copy and the statistics partials."""
import math

import pytest
import torch

from jax_raft_amd.models import reference as R
from jax_raft_amd.ops.native import HALO_3X3 as _HALO

_IDS = sorted(_HALO)   # every 3x3 config id

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(x):
    return x.to(torch.bfloat16).float()


def _nat():
    from jax_raft_amd.ops import native

    native.require()
    return native


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("cfg", _IDS)
def test_conv_halo_matches_reference(cfg):
    nat = _nat()
    cin = nat.halo_cfg(cfg)[0]
    torch.manual_seed(cfg)
    for (N, H, W, cout) in ((1, 19, 37, 64 if cin != 256 else 192), (2, 9, 20, 126)):
        x = torch.randn(N, H, W, cin)
        k = torch.randn(3, 3, cin, cout) / math.sqrt(9 * cin)
        b = torch.randn(cout) * 0.1
        ref = R.conv2d_nhwc(_bf(x), _bf(k), b, (1, 1), (1, 1))
        spec = nat.make_spec(k, b, (1, 1), (1, 1), device=DEV)
        assert spec.wh is not None and cfg in nat.halo_cfgs_for(spec, {})
        # input as a channel slice of a wider buffer (offset 8)
        xg = torch.zeros(N, H, W, cin + 16, dtype=torch.bfloat16, device=DEV)
        xg[..., 8:8 + cin] = x.to(DEV, torch.bfloat16)
        y = torch.full((N * H * W, nat.round_up(cout, 8) + 16), 5.0, dtype=torch.bfloat16, device=DEV)
        t, i, a = nat.conv_args(spec, xg, N, H, W, y, x_coff=8, y_coff=0, cfg=cfg)
        nat.ops().conv(t, i, a)
        torch.cuda.synchronize()
        got = y[:, :cout].float().cpu().reshape(N, H, W, cout)
        assert _rel(got, ref) < 1e-2, (cfg, N, H, W, cout)
        assert (y[:, cout:] == 5.0).all()
        # relu + residual (pre / post) + copy
        res = torch.randn(N, H, W, cout)
        rg = torch.zeros(N * H * W, nat.round_up(cout, 8) + 8, dtype=torch.bfloat16, device=DEV)
        rg[:, :cout] = res.reshape(-1, cout).to(DEV, torch.bfloat16)
        for post in (0, 1):
            y2 = torch.zeros(N * H * W, nat.round_up(cout, 8), dtype=torch.bfloat16, device=DEV)
            t, i, a = nat.conv_args(spec, xg, N, H, W, y, x_coff=8, act=nat.ACT_RELU, res=rg, res_post=post,
                                    y2=y2, cfg=cfg)
            nat.ops().conv(t, i, a)
            torch.cuda.synchronize()
            want = torch.relu(torch.relu(ref) + _bf(res)) if post else torch.relu(ref + _bf(res))
            assert _rel(y[:, :cout].float().cpu().reshape(N, H, W, cout), want) < 1e-2, (cfg, post)
            assert torch.equal(y2[:, :cout], y[:, :cout])


@pytest.mark.parametrize("cfg", _IDS)
def test_conv_halo_stats_partials(cfg):
    """Per-channel (sum, sumsq) of the stored outputs, per tile, reduced by the stats final
    kernel: equals the statistics of the output tensor (what channel_stats computes)."""
    nat = _nat()
    cin, wco, wpx, tn, tr, tc = nat.halo_cfg(cfg)
    torch.manual_seed(3)
    N, H, W, cout = 2, 21, 35, 96 if cin == 96 else 64
    x = torch.randn(N, H, W, cin).to(DEV, torch.bfloat16)
    k = torch.randn(3, 3, cin, cout) / math.sqrt(9 * cin)
    spec = nat.make_spec(k, torch.randn(cout) * 0.1, (1, 1), (1, 1), device=DEV)
    y = torch.empty(N * H * W, cout, dtype=torch.bfloat16, device=DEV)
    nb = -(-H // tr) * -(-W // tc) * wpx
    part = torch.full((N, nb, cout, 2), float("nan"), device=DEV)
    stats = torch.empty(N, cout, 2, device=DEV)
    t, i, a = nat.conv_args(spec, x, N, H, W, y, cfg=cfg)
    nat.ops().conv(t + [part], i, a)
    nat.ops().stats_final([part, stats], [N, nb, cout])
    torch.cuda.synchronize()
    yf = y.float().reshape(N, H * W, cout)
    want = torch.stack([yf.sum(1), (yf * yf).sum(1)], -1)
    assert torch.allclose(stats, want, rtol=1e-4, atol=1e-2), (stats - want).abs().max()


@pytest.mark.parametrize("cfg", _IDS)
def test_conv_halo_input_instance_norm(cfg):
    """The producer's instance norm + relu applied while the footprint is loaded equals
    norm_act (jr_norm_act mode 1, relu) followed by the conv; padding stays zero."""
    nat = _nat()
    cin = nat.halo_cfg(cfg)[0]
    torch.manual_seed(4)
    N, H, W, cout = 2, 13, 30, 64
    x = (torch.randn(N, H, W, cin) * 2 + 0.5).to(DEV, torch.bfloat16)
    stats = torch.empty(N, cin, 2, device=DEV)
    xf = x.float().reshape(N, H * W, cin)
    stats.copy_(torch.stack([xf.sum(1), (xf * xf).sum(1)], -1))
    k = torch.randn(3, 3, cin, cout) / math.sqrt(9 * cin)
    b = torch.randn(cout) * 0.1
    spec = nat.make_spec(k, b, (1, 1), (1, 1), device=DEV)
    mean = xf.mean(1, keepdim=True)
    var = (xf * xf).mean(1, keepdim=True) - mean * mean
    xn = torch.relu((xf - mean) * torch.rsqrt(var.clamp_min(0) + 1e-5)).reshape(N, H, W, cin)
    ref = R.conv2d_nhwc(_bf(xn.cpu()), _bf(k), b, (1, 1), (1, 1))
    y = torch.empty(N * H * W, cout, dtype=torch.bfloat16, device=DEV)
    t, i, a = nat.conv_args(spec, x, N, H, W, y, cfg=cfg, in_stats=stats, in_relu=1, in_hw=H * W)
    nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    assert _rel(y.float().cpu().reshape(N, H, W, cout), ref) < 1.5e-2


@pytest.mark.parametrize("cfg,res_norm", [(i, rn) for i in _IDS for rn in (False, True)])
def test_conv_halo_builds_residual_block_output(cfg, res_norm):
    """A residual block's output relu(relu(IN(x)) + r) (model.py:171-180; r the identity input
    or an instance-normalised downsample output) built while the footprint is loaded
    (in_relu = 3) equals norm_act + the conv, and the tile-own pixels of it are written out
    (xn) exactly once."""
    nat = _nat()
    cin = nat.halo_cfg(cfg)[0]
    torch.manual_seed(5 + cfg)
    N, H, W, cout = 2, 13, 30, 64
    x = (torch.randn(N, H, W, cin) * 2 + 0.5).to(DEV, torch.bfloat16)
    r = (torch.randn(N, H, W, cin) * 1.5 - 0.2).to(DEV, torch.bfloat16)

    def st(t):
        f = t.float().reshape(N, H * W, cin)
        return torch.stack([f.sum(1), (f * f).sum(1)], -1).contiguous()

    def inorm(t):
        f = t.float().reshape(N, H * W, cin)
        m = f.mean(1, keepdim=True)
        v = (f * f).mean(1, keepdim=True) - m * m
        return ((f - m) * torch.rsqrt(v.clamp_min(0) + 1e-5)).reshape(N, H, W, cin)

    built = torch.relu(torch.relu(inorm(x)) + (inorm(r) if res_norm else r.float()))
    k = torch.randn(3, 3, cin, cout) / math.sqrt(9 * cin)
    b = torch.randn(cout) * 0.1
    spec = nat.make_spec(k, b, (1, 1), (1, 1), device=DEV)
    ref = R.conv2d_nhwc(_bf(built.cpu()), _bf(k), b, (1, 1), (1, 1))
    y = torch.empty(N * H * W, cout, dtype=torch.bfloat16, device=DEV)
    xn = torch.full((N, H, W, cin), float("nan"), dtype=torch.bfloat16, device=DEV)
    t, i, a = nat.conv_args(spec, x, N, H, W, y, cfg=cfg, in_stats=st(x), in_relu=3, in_hw=H * W, in_res=r,
                            in_res_stats=st(r) if res_norm else None, xn=xn)
    nat.ops().conv(t, i, a)
    torch.cuda.synchronize()
    assert _rel(y.float().cpu().reshape(N, H, W, cout), ref) < 1.5e-2
    assert not torch.isnan(xn.float()).any()
    assert _rel(xn.float(), built) < 1e-2


@pytest.mark.parametrize("cin,cout", [(64, 64), (96, 96), (128, 192), (256, 126)])
def test_training_repack_of_halo_weights(cin, cout):
    """The training step's one-launch weight repack (train.hip:pack_pieces_kernel, modes 4 / 5)
    writes the halo conv's weight stream of a conv and of its data gradient exactly as
    ops/native.py:pack_halo_conv does from the (flipped, transposed) kernel."""
    from jax_raft_amd.ops import native as nat
    from jax_raft_amd.train.fused import Packer, _flip_t

    torch.manual_seed(cin + cout)
    k = torch.randn(3, 3, cin, cout, device=DEV)
    b = torch.zeros(cout, device=DEV)
    sp = nat.make_spec(k, b, (1, 1), (1, 1), device=DEV)
    kt = _flip_t(k)
    tp = nat.make_spec(kt, torch.zeros(cin, device=DEV), (1, 1), (1, 1), cin8=nat.round_up(cout, 8), device=DEV)
    assert sp.wh is not None
    want_f = sp.wh.clone()
    want_t = tp.wh.clone() if tp.wh is not None else None
    sp.wh.zero_()
    if tp.wh is not None:
        tp.wh.zero_()
    k2 = k.clone().contiguous()
    pk = Packer()
    pk.piece(k2, sp, 4, (0, cout), (0, cin))
    if tp.wh is not None:
        pk.piece(k2, tp, 5, (0, cin), (0, cout))
    pk.record(None)
    torch.cuda.synchronize()
    assert torch.equal(sp.wh, want_f)
    if want_t is not None:
        assert torch.equal(tp.wh, want_t)


@pytest.mark.parametrize("cfg", sorted(__import__("jax_raft_amd.ops.native", fromlist=["x"]).HALO_STEM_CFGS))
def test_conv_halo_stem_matches_reference(cfg):
    """The encoders' 7x7 / stride-2 / pad-3 stem as the halo kernel's 4x4 configs over the 2x2
    space-to-depth input (ops/native.py:s2d_stem_kernel; pads 2 / 1, output = input size)
    against the fp32 golden 7x7 conv, with relu, on maps that are not tile multiples."""
    nat = _nat()
    torch.manual_seed(cfg)
    for (N, H, W) in ((1, 38, 74), (2, 22, 36)):
        x = torch.randn(N, H, W, 3)
        k = torch.randn(7, 7, 3, 64) / math.sqrt(147)
        b = torch.randn(64) * 0.1
        ref = torch.relu(R.conv2d_nhwc(_bf(x), _bf(k), b, (2, 2), (3, 3)))
        h, w = H // 2, W // 2
        xs = torch.zeros(N, h, w, 16)
        for sy in range(2):
            for sx in range(2):
                c0 = (sy * 2 + sx) * 3
                xs[..., c0:c0 + 3] = x[:, sy::2, sx::2]
        spec = nat.make_spec(nat.s2d_stem_kernel(k), b, (1, 1), (2, 2), cin8=16, device=DEV)
        assert spec.halo_ks == 4 and cfg in nat.halo_cfgs_for(spec, {"out_hw": (h, w)})
        xg = xs.to(DEV, torch.bfloat16)
        for c in (cfg, None):   # the halo stem and the implicit GEMM it replaces
            y = torch.full((N * h * w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
            t, i, a = nat.conv_args(spec, xg, N, h, w, y, act=nat.ACT_RELU, out_hw=(h, w), cfg=c)
            nat.ops().conv(t, i, a)
            torch.cuda.synchronize()
            assert _rel(y.float().cpu().reshape(N, h, w, 64), ref) < 1e-2, (cfg, c, N, H, W)
