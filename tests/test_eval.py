"""Sintel validation pipeline on a synthetic mini-Sintel tree (no real data offline;
EPE parity with the reference's published numbers is unpinned)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from jax_raft_amd import raft_small
from jax_raft_amd.eval.sintel import MpiSintel, validate_sintel
from jax_raft_amd.utils.flow_io import InputPadder, flow_to_color, read_flo, write_flo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make_sintel(root, scenes=2, frames=3, H=124, W=132, seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    for dst in ("clean", "final"):
        for s in range(scenes):
            d = os.path.join(root, "training", dst, f"scene{s}")
            os.makedirs(d, exist_ok=True)
            for f in range(frames):
                Image.fromarray(rng.integers(0, 255, (H, W, 3), dtype=np.uint8)).save(os.path.join(d, f"frame_{f:04d}.png"))
    for s in range(scenes):
        d = os.path.join(root, "training", "flow", f"scene{s}")
        os.makedirs(d, exist_ok=True)
        for f in range(frames - 1):
            write_flo(os.path.join(d, f"frame_{f:04d}.flo"), rng.normal(size=(H, W, 2)).astype(np.float32))


def test_flo_roundtrip_and_bad_magic(tmp_path):
    x = np.random.default_rng(1).normal(size=(7, 9, 2)).astype(np.float32)
    p = str(tmp_path / "a.flo")
    write_flo(p, x)
    assert np.array_equal(read_flo(p), x)
    with open(p, "r+b") as f:
        f.write(b"\x00\x00\x00\x00")
    assert read_flo(p) is None


@pytest.mark.parametrize("H,W", [(436, 1024), (124, 132), (128, 128)])
def test_input_padder(H, W):
    x = torch.randn(1, 3, H, W)
    p = InputPadder(x.shape)
    (y,) = p.pad(x)
    assert y.shape[-2] % 8 == 0 and y.shape[-1] % 8 == 0
    assert torch.equal(p.unpad(y), x)
    if (H, W) == (436, 1024):
        assert y.shape[-2:] == (440, 1024)
        assert p._pad == [0, 0, 2, 2]
    xl = x.permute(0, 2, 3, 1).contiguous()
    pl = InputPadder(xl.shape, channels_last=True)
    (yl,) = pl.pad(xl)
    assert torch.equal(yl, y.permute(0, 2, 3, 1))
    assert torch.equal(pl.unpad(yl), xl)


def test_mpi_sintel_and_validate_cpu(tmp_path):
    _make_sintel(str(tmp_path))
    ds = MpiSintel(str(tmp_path), "training", "clean")
    assert len(ds) == 4
    a, b, flow = ds[0]
    assert a.shape == (124, 132, 3) and flow.shape == (124, 132, 2)
    model, _ = raft_small()
    res = validate_sintel(model, str(tmp_path), iters=2, device=torch.device("cpu"), verbose=False)
    assert set(res) == {"clean", "final"}
    for r in res.values():
        assert r["pairs"] == 4 and np.isfinite(r["epe"]) and 0 <= r["1px"] <= r["3px"] <= r["5px"] <= 1


def test_validate_batched_equals_per_pair(tmp_path):
    """batch_size > 1 (a partial last batch included) gives the per-pair metrics."""
    _make_sintel(str(tmp_path), scenes=2, frames=3)
    model, _ = raft_small()
    kw = dict(iters=2, device=torch.device("cpu"), verbose=False, dstypes=("clean",))
    r1 = validate_sintel(model, str(tmp_path), batch_size=1, **kw)["clean"]
    r3 = validate_sintel(model, str(tmp_path), batch_size=3, **kw)["clean"]
    assert r3["batch_size"] == 3 and r3["pairs"] == r1["pairs"] == 4
    for k in ("epe", "1px", "3px", "5px"):
        assert abs(r1[k] - r3[k]) < 1e-5 * max(1.0, abs(r1[k])), k


def test_flow_to_color():
    img = flow_to_color(np.random.default_rng(2).normal(size=(5, 6, 2)))
    assert img.shape == (5, 6, 3) and img.dtype == np.uint8


def test_demo_and_convert_cli(tmp_path):
    out = tmp_path / "f.png"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "demo.py"), "--iters", "1", "--out", str(out)],
                       capture_output=True, text=True, env={**os.environ, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, r.stderr
    assert out.exists()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "convert_checkpoint.py")], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stdout


def test_validate_u8_prep_equals_host_prep(tmp_path):
    """device_prep: the model receives raw uint8 frames (normalise + 'sintel' replicate padding
    inside the model, unpadded flows back; the GPU default) -- the same metrics as the
    reference's host-side protocol (validate_sintel.py:177-191)."""
    _make_sintel(str(tmp_path), scenes=1, frames=3)
    model, _ = raft_small()
    kw = dict(iters=2, device=torch.device("cpu"), verbose=False, dstypes=("clean",))
    rh = validate_sintel(model, str(tmp_path), device_prep=False, **kw)["clean"]
    ru = validate_sintel(model, str(tmp_path), device_prep=True, **kw)["clean"]
    for k in ("epe", "1px", "3px", "5px"):
        assert abs(rh[k] - ru[k]) < 1e-5 * max(1.0, abs(rh[k])), k
