"""Long-context analogue (resolution): the engine beyond the Sintel size.

* 376x1248 (KITTI-shaped) and 1088x1920 (a 136x240 feature map): the bf16 and fp32
  engines against the fp32 golden forward of the same weights, computed on the GPU
  (ops/functional.py ``golden_ops``: plain PyTorch fp32 ops, GEMM convs), 4 iterations;
  reference ``jax_raft/model.py:431-436,472-481,557-560``.
* 2160x3840 (4K): a final-only forward on one GPU (a 44.6 GB bf16 pyramid: the 64-bit
  pyramid indexing of csrc/kernels/corr.hip), finite and shaped right.
* 2160x3840 over 2 context-parallel ranks sharing the GPU: each rank holds the pyramid
  of its half of the query rows (recorded bytes), the result equals the single-GPU one.
"""
import os
import subprocess
import sys

import pytest
import torch

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.ops.functional import golden_ops

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bf16 engine vs fp32 golden, max over iterations of EPE / mean |golden flow| (measured on
# MI355X: profiles/r5_resolution.txt, max 0.026 / 0.020); fp32 engine vs golden: EPE / (1 + mean |flow|)
REL_EPE_BF16 = {"raft_small": 0.065, "raft_large": 0.026}
REL_EPE_FP32 = 1e-4


def _inputs(H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(1, H + 8, W + 8, 3, generator=g) * 2 - 1
    return base[:, 4:4 + H, 4:4 + W].contiguous().cuda(), base[:, 2:2 + H, 6:6 + W].contiguous().cuda()


def _golden(model, i1, i2, iters):
    with torch.no_grad(), golden_ops():
        return model.forward_reference(i1, i2, False, iters)


def _epes(out, ref):
    return [(out[i] - ref[i]).norm(dim=-1).mean().item() for i in range(ref.shape[0])]


@pytest.mark.parametrize("factory", [raft_large, raft_small])
@pytest.mark.parametrize("H,W", [(376, 1248), (1088, 1920)])
def test_hires_bf16_engine_matches_golden(factory, H, W):
    model = factory(seed=0)[0].eval().cuda()
    i1, i2 = _inputs(H, W)
    ref = _golden(model, i1, i2, 4)
    out = model(i1, i2, num_flow_updates=4)
    torch.cuda.synchronize()
    assert out.shape == ref.shape == (4, 1, H, W, 2) and torch.isfinite(out).all()
    mag = ref.norm(dim=-1).mean().item()
    e = _epes(out, ref)
    print(f"{factory.__name__} {H}x{W} bf16: EPE/|flow| per iteration {[round(x / mag, 5) for x in e]}")
    assert max(e) < REL_EPE_BF16[factory.__name__] * mag, (e, mag)


@pytest.mark.parametrize("H,W", [(376, 1248), (1088, 1920)])
def test_hires_fp32_engine_matches_golden(H, W):
    from jax_raft_amd.runtime.engine import RaftEngine

    model = raft_large(seed=0)[0].eval().cuda()
    i1, i2 = _inputs(H, W, seed=1)
    ref = _golden(model, i1, i2, 4)
    with torch.no_grad():
        out = RaftEngine(model, torch.device("cuda", 0), precision="fp32").forward(i1, i2, 4)
    torch.cuda.synchronize()
    mag = ref.norm(dim=-1).mean().item()
    e = _epes(out, ref)
    print(f"raft_large {H}x{W} fp32: EPE per iteration {e}, |flow| {mag:.4f}")
    assert max(e) < REL_EPE_FP32 * (1 + mag), (e, mag)


def _pyramid_bytes(eng):
    st = next(iter(eng._states.values()))
    return sum(t.numel() * t.element_size() for k, t in st.bufs.items() if ".corr.l" in "." + k)


@pytest.fixture(scope="module")
def single_4k():
    """One 2160x3840 final-only forward on one GPU (the engine is released afterwards)."""
    model = raft_large(seed=0)[0].eval().cuda()
    i1, i2 = _inputs(2160, 3840, seed=2)
    eng = model.engine(torch.device("cuda", 0))
    with torch.no_grad():
        out = eng.forward(i1, i2, 4, return_all_iters=False)
    torch.cuda.synchronize()
    res = {"flow": out.cpu(), "bytes": _pyramid_bytes(eng)}
    del eng, model, out
    torch.cuda.empty_cache()
    return res


def test_4k_final_only_single_gpu(single_4k):
    out, nbytes = single_4k["flow"], single_4k["bytes"]
    assert out.shape == (1, 1, 2160, 3840, 2) and torch.isfinite(out).all()
    # 270 x 480 queries x (1 + 1/4 + 1/16 + 1/64) of a 270 x 480 map, bf16
    assert nbytes > 44e9, nbytes
    print(f"4K single GPU: pyramid {nbytes / 1e9:.2f} GB")


def test_4k_context_parallel_two_ranks(tmp_path, single_4k):
    """2 CP ranks on one GPU (gloo, JR_SHARE_GPU=1): pyramid bytes per rank ~ half of the
    single-GPU pyramid; flows equal across ranks and to the single-GPU forward."""
    env = dict(os.environ, JR_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29641",
           os.path.join(ROOT, "tests", "_cp4k_gpu_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    a = torch.load(tmp_path / "rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert torch.equal(a["flow"], b["flow"]) and torch.isfinite(a["flow"]).all()
    print(f"4K CP: pyramid bytes per rank {a['bytes'] / 1e9:.2f} / {b['bytes'] / 1e9:.2f} GB")
    full = single_4k
    assert 0.45 * full["bytes"] < a["bytes"] < 0.56 * full["bytes"], (a["bytes"], full["bytes"])
    ref = full["flow"]
    mag = ref.norm(dim=-1).mean().item()
    e = (a["flow"] - ref).norm(dim=-1).mean().item()
    assert e < 0.02 * mag + 1e-3, (e, mag)
