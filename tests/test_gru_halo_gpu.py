"""gru_halo.hip -- the halo-tiled fused ConvGRU stage -- against the fp32 ConvGRU of the
reference (jax_raft/model.py:293-312) with the loop-invariant context share as a per-pixel
bias map, for raft_large's 1x5 / 5x1 stages (hidden 128) and raft_small's 3x3 GRU (hidden
96, x = 80 motion + 2 flow channels padded to 96), at map sizes whose rows / columns are
not multiples of a tile (widths 37 / 129 / 240, heights 55 / 136) and every tiling the
engine may pick.  Operands are bf16-rounded as the kernel sees them."""
import math

import pytest
import torch

from jax_raft_amd.models import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(x):
    return x.to(torch.bfloat16).float()


def _nat():
    from jax_raft_amd.ops import native

    native.require()
    return native


def _case(hd, xreal, ks, B, h, w, seed):
    torch.manual_seed(seed)
    cs = 2 * hd
    cin = hd + xreal
    hs = torch.tanh(torch.randn(B, h, w, hd))
    xs = torch.randn(B, h, w, xreal)
    kz, kr, kq = [torch.randn(*ks, cin, hd) / math.sqrt(ks[0] * ks[1] * cin) for _ in range(3)]
    bm = _bf(torch.randn(B, h, w, 3 * hd) * 0.5)
    pad = ((ks[0] - 1) // 2, (ks[1] - 1) // 2)
    zero = torch.zeros(hd)
    hxr = torch.cat([hs, xs], -1)
    z = torch.sigmoid(R.conv2d_nhwc(_bf(hxr), _bf(kz), zero, (1, 1), pad) + bm[..., :hd])
    r = torch.sigmoid(R.conv2d_nhwc(_bf(hxr), _bf(kr), zero, (1, 1), pad) + bm[..., hd:2 * hd])
    q = torch.tanh(R.conv2d_nhwc(_bf(torch.cat([_bf(r * _bf(hs)), xs], -1)), _bf(kq), zero, (1, 1), pad)
                   + bm[..., 2 * hd:])
    M = B * h * w
    ref = ((1 - z) * hs + z * q).reshape(M, hd)
    src = torch.zeros(M, cs, dtype=torch.bfloat16)
    src[:, :hd] = hs.reshape(M, hd).to(torch.bfloat16)
    src[:, hd:cin] = xs.reshape(M, xreal).to(torch.bfloat16)
    return dict(ref=ref, src=src, hs=hs, kzr=torch.cat([kz, kr], 3), kq=kq, bm=bm.reshape(M, 3 * hd), cs=cs)


def _run(nat, c, hd, mode, axis, B, h, w, tile, two_src=False):
    TR, TC, nb1, nb2 = tile
    M = B * h * w
    src = c["src"].to(DEV)
    xsrc = src
    if two_src:   # h from one buffer, x from another (raft_large's second stage reads h' from qx)
        xsrc = src.clone()
        src = src.clone()
        src[:, hd:] = 0
        xsrc[:, :hd] = 0
    wa = nat.pack_gru_halo(c["kzr"].to(DEV), c["cs"])
    wb = nat.pack_gru_halo(c["kq"].to(DEV), c["cs"])
    h32 = c["hs"].reshape(M, hd).to(DEV).contiguous()
    y = torch.full((M, c["cs"]), 3.0, dtype=torch.bfloat16, device=DEV)
    y2 = torch.full((M, hd), 7.0, dtype=torch.bfloat16, device=DEV)
    bmg = c["bm"].to(DEV, torch.bfloat16).contiguous()
    nat.ops().gru_halo([src, xsrc, wa, wb, bmg, h32, y, y2], [B, h, w, mode, axis, TR, TC, nb1, nb2])
    torch.cuda.synchronize()
    return h32.cpu(), y.cpu(), y2.cpu()


LARGE = [(1, 55, 128), (1, 55, 37), (2, 136, 129), (1, 136, 240), (1, 17, 16)]


@pytest.mark.parametrize("axis", [0, 1])
@pytest.mark.parametrize("B,h,w", LARGE)
def test_gru_halo_large(B, h, w, axis):
    nat = _nat()
    hd, ks = 128, ((5, 1) if axis else (1, 5))
    c = _case(hd, 128, ks, B, h, w, seed=11 + axis)
    cands = nat.gru_halo_candidates(hd, 0, axis, B, h, w)
    assert cands
    for tile in cands:
        assert nat.ops().gru_halo_geom_ok(hd, 0, *tile)
        h32, y, y2 = _run(nat, c, hd, 0, axis, B, h, w, tile)
        err = (h32 - c["ref"]).abs().max().item()
        assert err < 2e-2, (tile, err)
        assert (y[:, :hd].float() - c["ref"]).abs().max().item() < 2.5e-2, tile
        assert (y[:, hd:] == 3.0).all(), tile           # only h' channels written
        assert torch.equal(y2, y[:, :hd]), tile


@pytest.mark.parametrize("B,h,w", [(1, 55, 128), (2, 55, 37), (1, 136, 240), (1, 16, 16)])
def test_gru_halo_small(B, h, w):
    nat = _nat()
    hd = 96
    c = _case(hd, 82, (3, 3), B, h, w, seed=21)
    for tile in nat.gru_halo_candidates(hd, 1, 0, B, h, w):
        assert nat.ops().gru_halo_geom_ok(hd, 1, *tile)
        h32, y, _ = _run(nat, c, hd, 1, 0, B, h, w, tile)
        err = (h32 - c["ref"]).abs().max().item()
        assert err < 2e-2, (tile, err)
        assert (y[:, :hd].float() - c["ref"]).abs().max().item() < 2.5e-2, tile


def test_gru_halo_two_sources():
    """h read from one buffer and x from another (raft_large's second stage)."""
    nat = _nat()
    B, h, w = 1, 23, 41
    c = _case(128, 128, (5, 1), B, h, w, seed=5)
    h32, _, _ = _run(nat, c, 128, 0, 1, B, h, w, (1, 28, 1, 1), two_src=True)
    assert (h32 - c["ref"]).abs().max().item() < 2e-2


def test_gru_halo_rejects_in_place():
    nat = _nat()
    M = 4 * 20
    src = torch.zeros(M, 256, dtype=torch.bfloat16, device=DEV)
    wa = torch.zeros(256 * 5 * 256, dtype=torch.bfloat16, device=DEV)
    wb = torch.zeros(128 * 5 * 256, dtype=torch.bfloat16, device=DEV)
    bm = torch.zeros(M, 384, dtype=torch.bfloat16, device=DEV)
    h32 = torch.zeros(M, 128, device=DEV)
    with pytest.raises(RuntimeError, match="alias"):
        nat.ops().gru_halo([src, src, wa, wb, bm, h32, src], [1, 4, 20, 0, 0, 1, 20, 1, 1])
    assert not nat.ops().gru_halo_geom_ok(128, 0, 1, 29, 1, 1)    # 33 region pixels > one block
    assert not nat.ops().gru_halo_geom_ok(96, 1, 6, 6, 2, 1)      # 36 output pixels > one block
