"""gru_split.hip -- the channel-split ConvGRU stage (launch A: z, r*h; launch B: q + blend) --
against the fp32 ConvGRU of the reference (jax_raft/model.py:293-312) with the loop-invariant
context share as a per-pixel bias map, for raft_large's 1x5 / 5x1 stages (hidden 128, x = 128
channels), at map sizes whose lines are not multiples of a tile and every config the engine may
pick.  Operands are bf16-rounded as the kernels see them (z and r*h also pass through bf16)."""
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


def _case(ks, B, h, w, seed):
    hd = 128
    torch.manual_seed(seed)
    hs = torch.tanh(torch.randn(B, h, w, hd))
    xs = torch.randn(B, h, w, hd)
    kz, kr, kq = [torch.randn(*ks, 2 * hd, hd) / math.sqrt(5 * 2 * hd) for _ in range(3)]
    bm = _bf(torch.randn(B, h, w, 3 * hd) * 0.5)
    pad = ((ks[0] - 1) // 2, (ks[1] - 1) // 2)
    zero = torch.zeros(hd)
    hxr = _bf(torch.cat([hs, xs], -1))
    z = _bf(torch.sigmoid(R.conv2d_nhwc(hxr, _bf(kz), zero, (1, 1), pad) + bm[..., :hd]))
    r = torch.sigmoid(R.conv2d_nhwc(hxr, _bf(kr), zero, (1, 1), pad) + bm[..., hd:2 * hd])
    q = torch.tanh(R.conv2d_nhwc(_bf(torch.cat([_bf(r * _bf(hs)), xs], -1)), _bf(kq), zero, (1, 1), pad)
                   + bm[..., 2 * hd:])
    M = B * h * w
    ref = ((1 - z) * hs + z * q).reshape(M, hd)
    return dict(ref=ref, hs=hs, xs=xs, kzr=torch.cat([kz, kr], 3), kq=kq, bm=bm.reshape(M, 3 * hd))


def _run(nat, c, axis, B, h, w, ca, cb, hm=True):
    M = B * h * w
    hd = 128
    hx = torch.zeros(M, 256, dtype=torch.bfloat16)
    hx[:, :hd] = c["hs"].reshape(M, hd).to(torch.bfloat16)
    hx[:, hd:] = c["xs"].reshape(M, hd).to(torch.bfloat16)
    hx = hx.to(DEV)
    qx = torch.full((M, 256), 5.0, dtype=torch.bfloat16, device=DEV)
    qx[:, hd:] = hx[:, hd:]                       # the engine keeps [motion | flow] in both buffers
    bm = c["bm"].to(DEV, torch.bfloat16).contiguous()
    zb = torch.zeros(M, hd, dtype=torch.bfloat16, device=DEV)
    h32 = c["hs"].reshape(M, hd).to(DEV).contiguous()
    y2 = torch.full((M, hd), 7.0, dtype=torch.bfloat16, device=DEV) if hm else None
    (cfa, La, Ja), (cfb, Lb, Jb) = ca, cb
    pa, pb = nat.GRU_SPLIT_CFGS[cfa], nat.GRU_SPLIT_CFGS[cfb]
    wa = nat.pack_gru_split(c["kzr"].to(DEV), pa[1], pa[2])
    wb = nat.pack_gru_split(c["kq"].to(DEV), pb[1], pb[2])
    nat.ops().gru_split([hx, wa, bm, zb, qx, None, None, None], [B, h, w, axis, 0, La, Ja, cfa])
    nat.ops().gru_split([qx, wb, bm, zb, None, h32, hx, y2], [B, h, w, axis, 1, Lb, Jb, cfb])
    torch.cuda.synchronize()
    return h32.cpu(), hx.cpu(), qx.cpu(), None if y2 is None else y2.cpu()


SIZES = [(1, 55, 128), (4, 55, 128), (1, 55, 37), (2, 136, 129), (1, 136, 240), (1, 17, 16)]


@pytest.mark.parametrize("axis", [0, 1])
@pytest.mark.parametrize("B,h,w", SIZES)
def test_gru_split_matches_fp32(B, h, w, axis):
    nat = _nat()
    ks = (5, 1) if axis else (1, 5)
    c = _case(ks, B, h, w, seed=31 + axis + h)
    ca_all = nat.gru_split_candidates(0, axis, B, h, w)
    cb_all = nat.gru_split_candidates(1, axis, B, h, w)
    assert ca_all and cb_all
    n = max(len(ca_all), len(cb_all))
    for k in range(n):   # every candidate of both launches at least once
        ca, cb = ca_all[k % len(ca_all)], cb_all[k % len(cb_all)]
        h32, hx, qx, y2 = _run(nat, c, axis, B, h, w, ca, cb)
        err = (h32 - c["ref"]).abs().max().item()
        assert err < 2e-2, (ca, cb, err)
        assert (hx[:, :128].float() - c["ref"]).abs().max().item() < 2.5e-2, (ca, cb)
        assert torch.equal(hx[:, 128:], c["xs"].reshape(-1, 128).to(torch.bfloat16)), (ca, cb)   # x untouched
        assert torch.equal(y2, hx[:, :128]), (ca, cb)


def test_gru_split_rejects_bad_tiles():
    nat = _nat()
    B, h, w = 1, 55, 128
    M = B * h * w
    src = torch.zeros(M, 256, dtype=torch.bfloat16, device=DEV)
    wa = torch.zeros(256 * 5 * 256, dtype=torch.bfloat16, device=DEV)
    bm = torch.zeros(M, 384, dtype=torch.bfloat16, device=DEV)
    zb = torch.zeros(M, 128, dtype=torch.bfloat16, device=DEV)
    rh = torch.zeros(M, 256, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError):   # 2 runs of 128 do not fit 4 pixel blocks
        nat.ops().gru_split([src, wa, bm, zb, rh, None, None, None], [B, h, w, 0, 0, 128, 2, 2])
    with pytest.raises(RuntimeError):   # rh aliasing the source
        nat.ops().gru_split([src, wa, bm, zb, src, None, None, None], [B, h, w, 0, 0, 128, 1, 2])
