"""Numerical drift at the headline configuration (440x1024, 32 iterations,
batch 1; tools/drift.py, profiles/r5_drift.md): the committed fp32 golden
fixtures are reproducible on the CPU, and the bf16 native engine's final flow
stays within a bound derived from the measured drift curve."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import drift  # noqa: E402

# measured on MI355X (profiles/r5_drift.md, round-5 tree; round 3: 1.69e-2 / 4.20e-2):
# final-iteration EPE / mean |golden flow| = 1.70e-2 (raft_large) and 4.22e-2 (raft_small) with
# the default bf16 engine; the bound leaves 1.5x headroom for tile-config (a re-tuned table picks
# other configs, whose summation orders differ) and device differences
REL_BOUND = {"raft_large": 1.5 * 1.70e-2, "raft_small": 1.5 * 4.22e-2}
# precision="mixed" (fp32 feature encoder): measured 1.55e-2 (raft_large) / 2.51e-2 (raft_small,
# from 4.21e-2 in bf16), profiles/r6_drift_mixed.md; 1.5x headroom as above
REL_BOUND_MIXED = {"raft_large": 1.5 * 1.55e-2, "raft_small": 1.5 * 2.51e-2}
# fp32 engine (precision="fp32"): measured 5.5e-6 / 9.4e-6 (fp32 summation order only)
REL_BOUND_FP32 = 3e-5


@pytest.mark.slow
def test_golden_fixture_reproduces_on_cpu():
    """The fp32 CPU golden forward (models/reference.py) reproduces the committed
    fixture (fixtures were written by ``tools/drift.py golden`` on this image;
    another CPU's summation order moved the 32-iteration flow by <= 0.03 px)."""
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    g = drift.golden("raft_small")
    fx, mags = drift.load_fixture("raft_small")
    assert (g[-1, 0] - fx).abs().max().item() < 0.1
    assert drift.epe(g[-1, 0], fx) < 1e-2
    assert abs(g[-1].norm(dim=-1).mean().item() - mags[-1]) < 1e-2 * mags[-1]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp32", "mixed"])
@pytest.mark.parametrize("arch", ["raft_large", "raft_small"])
def test_engine_drift_at_headline_config(arch, precision):
    """Engine (default settings, bf16 or the fp32 parity mode), 440x1024, 32
    iterations, batch 1: the final upsampled flow vs the committed fp32 golden fixture."""
    from jax_raft_amd.runtime.engine import RaftEngine

    fx, mags = drift.load_fixture(arch)
    m = drift.model_for(arch).cuda()
    i1, i2 = drift.inputs()
    eng = RaftEngine(m, torch.device("cuda", 0), precision=precision)
    out = eng.forward(i1.cuda(), i2.cuda(), drift.ITERS).cpu()
    torch.cuda.synchronize()
    assert out.shape == (drift.ITERS, 1, drift.H, drift.W, 2) and torch.isfinite(out).all()
    rel = drift.epe(out[-1, 0], fx) / mags[-1]
    bound = REL_BOUND_FP32 if precision == "fp32" else REL_BOUND_MIXED[arch] if precision == "mixed" else REL_BOUND[arch]
    assert rel < bound, (arch, precision, rel)
