"""Injected sub-modules on the GPU (reference ``jax_raft/model.py:636-665`` injection
kwargs, ``:702-711`` block / norm given as classes): a model the native engine cannot lower
runs op by op on the same HIP kernels (ops/functional.py: implicit-GEMM convs, correlation
pyramid, lookup) instead of raising, and matches the fp32 golden forward of the same weights."""
import pytest
import torch
from torch import nn

from jax_raft_amd import raft_large, raft_small
from jax_raft_amd.models.layers import BottleneckBlock, FeatureEncoder, InstanceNorm, MaskPredictor, ResidualBlock

pytestmark = pytest.mark.gpu

# op-by-op bf16 convs vs the fp32 golden: the engine's bounds (tests/test_engine_gpu.py REL_EPE)
REL_EPE = {"raft_small": 0.065, "raft_large": 0.026}


class ScaleNorm(nn.Module):
    """A user norm (not one of the Flax built-ins): per-channel scale + shift."""

    def __init__(self, c):
        super().__init__()
        self.scale = nn.Parameter(torch.linspace(0.5, 1.5, c))
        self.bias = nn.Parameter(torch.linspace(-0.1, 0.1, c))

    def forward(self, x):
        return x * self.scale + self.bias


def _inputs(seed=0, H=128, W=256):
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(1, H + 8, W + 8, 3, generator=g) * 2 - 1
    return base[:, 4:4 + H, 4:4 + W].contiguous(), base[:, 2:2 + H, 6:6 + W].contiguous()


def _check(model, name, iters=3):
    i1, i2 = _inputs()
    ref = model.forward_reference(i1, i2, False, iters)
    model = model.cuda()
    out = model(i1.cuda(), i2.cuda(), num_flow_updates=iters)
    torch.cuda.synchronize()
    assert model.execution_path.startswith("op-by-op"), model.execution_path
    assert out.shape == ref.shape and torch.isfinite(out).all()
    out = out.cpu()
    mag = ref.norm(dim=-1).mean().item()
    for it in range(iters):
        e = (out[it] - ref[it]).norm(dim=-1).mean().item()
        assert e < REL_EPE[name] * mag, (it, e, mag)


def test_injected_feature_encoder_and_mask_predictor_raft_large():
    """A FeatureEncoder with non-default layers (200 output channels: outside the native
    correlation's 64-channel tiling) + a custom MaskPredictor (hidden 128, x0.5)."""
    torch.manual_seed(0)
    fe = FeatureEncoder(block=ResidualBlock, layers=(64, 64, 96, 128, 200), norm=InstanceNorm,
                        gen=torch.Generator().manual_seed(1))
    mp = MaskPredictor(128, hidden_size=128, multiplier=0.5, gen=torch.Generator().manual_seed(2))
    model, _ = raft_large(feature_encoder=fe, mask_predictor=mp)
    _check(model, "raft_large")


def test_injected_custom_norm_and_block_class_raft_small():
    """The context encoder with a user norm class and the block given as a class."""
    torch.manual_seed(0)
    ce = FeatureEncoder(block=BottleneckBlock, layers=(32, 32, 64, 96, 160), norm=ScaleNorm,
                        gen=torch.Generator().manual_seed(3))
    model, _ = raft_small(context_encoder=ce)
    _check(model, "raft_small")


def test_lowerable_model_keeps_the_engine():
    model, _ = raft_small()
    model = model.cuda()
    i1, i2 = _inputs()
    model(i1.cuda(), i2.cuda(), num_flow_updates=2)
    assert model.execution_path == "engine"
