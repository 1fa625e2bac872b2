"""Device-side input preparation of raw frames: uint8 NHWC frames of any size are
normalised to [-1, 1], replicate-padded to /8 (InputPadder 'sintel') and laid out for the encoders
by one kernel (elementwise.hip:prep_u8_kernel), the flows cropped back to the frame size.

Oracle: the reference's host protocol (scripts/validate_sintel.py:177-191 -- x / 255 * 2 - 1,
InputPadder.pad, NHWC, unpad) as implemented by utils/flow_io.py, followed by the float path."""
import numpy as np
import pytest
import torch

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.ops import native as nat
from jax_raft_amd.runtime.engine import RaftEngine, sintel_pad, u8_table
from jax_raft_amd.utils.flow_io import InputPadder, normalize_image

pytestmark = pytest.mark.gpu


def _frames(B, H0, W0, seed):
    g = np.random.default_rng(seed)
    return (g.integers(0, 256, (B, H0, W0, 3), dtype=np.uint8), g.integers(0, 256, (B, H0, W0, 3), dtype=np.uint8))


def _host(a, b):
    """The reference protocol on the host: normalise, pad (replicate, 'sintel'), NHWC float."""
    i1 = torch.cat([normalize_image(x) for x in a])
    i2 = torch.cat([normalize_image(x) for x in b])
    p = InputPadder(i1.shape, channels_last=True)
    i1, i2 = p.pad(i1, i2)
    return i1, i2, p


@pytest.mark.parametrize("s2d", [1, 0])
@pytest.mark.parametrize("B,H0,W0", [(1, 436, 1024), (2, 130, 141), (1, 128, 128), (3, 121, 255)])
def test_prep_u8_kernel_bitwise(B, H0, W0, s2d):
    """The u8 kernel's output equals, bit for bit, the float prep kernel's output on the host-
    normalised + padded frames, over the whole padded image (the replicated border included)."""
    a, b = _frames(B, H0, W0, seed=H0 + W0)
    f1, f2, p = _host(a, b)
    H, W = f1.shape[1:3]
    pt, pb, pl, pr = sintel_pad(H0, W0)
    assert (pl, pr, pt, pb) == tuple(p._pad)
    C = 16 if s2d else 8
    shape = (2 * B, H // 2, W // 2, C) if s2d else (2 * B, H, W, C)
    ref = torch.zeros(shape, dtype=torch.bfloat16, device="cuda")
    got = torch.full(shape, 7.0, dtype=torch.bfloat16, device="cuda")
    nat.ops().prep([f1.cuda(), f2.cuda(), ref], [B, H, W] + ([1] if s2d else []))
    nat.ops().prep([torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), got, u8_table("cuda")],
                   [B, H, W, s2d, H0, W0, pt, pl])
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


def test_u8_table_is_the_reference_expression():
    x = torch.arange(256, dtype=torch.float32)
    assert torch.equal(u8_table("cpu"), x / 255.0 * 2.0 - 1.0)
    assert torch.equal(u8_table("cpu"), normalize_image(np.arange(256, dtype=np.uint8).reshape(1, 256, 1).repeat(3, 2))[0, 0, :, 0])


@pytest.mark.parametrize("factory", [raft_small, raft_large])
@pytest.mark.parametrize("final_only", [False, True])
def test_engine_u8_frames_equal_host_protocol(factory, final_only):
    """forward(uint8 frames) == crop(forward(host-normalised, padded frames)), bitwise: after the
    prep kernel the two plans run the same kernels on the same bits."""
    model, _ = factory()
    model = model.cuda()
    a, b = _frames(2, 130, 141, seed=5)
    f1, f2, p = _host(a, b)
    eng = model.engine(torch.device("cuda", 0))
    ref = eng.forward(f1.cuda(), f2.cuda(), 3, return_all_iters=not final_only)
    got = eng.forward(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), 3, return_all_iters=not final_only)
    torch.cuda.synchronize()
    pl, pr, pt, pb = p._pad
    assert got.shape == (3 if not final_only else 1, 2, 130, 141, 2)
    assert torch.equal(got, ref[:, :, pt:ref.shape[2] - pb, pl:ref.shape[3] - pr])
    # the model-level API takes raw frames too (host numpy arrays: H2D of 1/4 the bytes)
    got2 = model(a, b, num_flow_updates=3, return_all_iters=not final_only)
    torch.cuda.synchronize()
    assert got2.is_cuda and torch.equal(got2, got)


def test_engine_u8_pipelined_and_fp32():
    """pipelined() takes raw frames (the result of each batch cropped like forward()), and the
    fp32 engine prepares them with framework ops (same values: its output equals its float path)."""
    model, _ = raft_small()
    model = model.cuda()
    eng = model.engine(torch.device("cuda", 0))
    frames = [tuple(torch.from_numpy(x).cuda() for x in _frames(1, 130, 141, seed=10 + k)) for k in range(3)]
    refs = [eng.forward(x, y, 3) for x, y in frames]
    outs = [eng.pipelined(x, y, 3) for x, y in frames]
    outs = outs[1:] + [eng.flush()]
    torch.cuda.synchronize()
    for r, o in zip(refs, outs):
        assert torch.equal(r, o)
    e32 = RaftEngine(model, torch.device("cuda", 0), precision="fp32")
    x, y = (torch.from_numpy(v).cuda() for v in _frames(1, 125, 250, seed=9))   # fp32 engine: h * w % 4 == 0
    f1, f2, p = _host(x.cpu().numpy(), y.cpu().numpy())
    a = e32.forward(x, y, 2)
    b = e32.forward(f1.cuda(), f2.cuda(), 2)
    pl, pr, pt, pb = p._pad
    torch.cuda.synchronize()
    assert torch.equal(a, b[:, :, pt:b.shape[2] - pb, pl:b.shape[3] - pr])
