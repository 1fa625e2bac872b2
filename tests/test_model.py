"""Model API on the CPU golden path (BASELINE config 1: raft_small, 2x128x128x3, 3 iters)."""
import numpy as np
import pytest
import torch

from jax_raft_amd import RAFT, raft_large, raft_small
from jax_raft_amd.models.layers import CorrBlock
from jax_raft_amd.utils import checkpoint as C


def _pair(B=1, H=128, W=128, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, H, W, 3, generator=g) * 2 - 1, torch.rand(B, H, W, 3, generator=g) * 2 - 1


def test_config1_raft_small_cpu():
    model, variables = raft_small()
    i1, i2 = _pair(2)
    out = model.apply(variables, i1, i2, train=False, num_flow_updates=3)
    assert out.shape == (3, 2, 128, 128, 2)
    assert torch.isfinite(out).all()


def test_raft_large_cpu_shapes_default_iters():
    model, variables = raft_large()
    i1, i2 = _pair(1, 128, 136)
    out = model.apply(variables, i1, i2)
    assert out.shape == (12, 1, 128, 136, 2)


def test_apply_accepts_numpy_and_foreign_variables():
    model, variables = raft_small(seed=0)
    other, ov = raft_small(seed=7)
    i1, i2 = _pair()
    ref = other.apply(ov, i1, i2, num_flow_updates=2)
    npvars = {"params": {k: v for k, v in ov["params"].items()}}
    npvars = {"params": C.unflatten_tree({k: v.detach().numpy() for k, v in C.flatten_tree(ov["params"]).items()})}
    out = model.apply(npvars, i1.numpy(), i2.numpy(), num_flow_updates=2)
    assert torch.allclose(out, ref, atol=1e-5)


def test_input_assertions():
    model, v = raft_small()
    a, b = _pair(1, 128, 128)
    with pytest.raises(AssertionError):
        model.apply(v, a[:, :124], b[:, :124])
    with pytest.raises(AssertionError):
        model.apply(v, a, b[:, :120])
    small = torch.zeros(1, 64, 64, 3)
    with pytest.raises(AssertionError):
        model.apply(v, small, small)


def test_train_mode_updates_batch_stats_and_grads():
    model, v = raft_large()
    model.train()
    a, b = _pair(2, 128, 128)
    before = v["batch_stats"]["context_encoder"]["convnormrelu"]["layers_1"]["mean"].clone()
    out, new = model.apply(v, a, b, train=True, num_flow_updates=2, mutable=["batch_stats"])
    after = new["batch_stats"]["context_encoder"]["convnormrelu"]["layers_1"]["mean"]
    assert not torch.equal(before, after)
    loss = out.abs().mean()
    loss.backward()
    g = model.feature_encoder.convnormrelu.layers_0.kernel.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0


def test_submodule_injection():
    model, v = raft_small(corr_block=CorrBlock(num_levels=2, radius=2))
    assert model.corr_block.num_levels == 2
    assert tuple(v["params"]["update_block"]["motion_encoder"]["convcorr1"]["layers_0"]["kernel"].shape) == (1, 1, 50, 96)
    out = model.apply(v, *_pair(), num_flow_updates=1)
    assert out.shape == (1, 1, 128, 128, 2)
    with pytest.raises(TypeError):
        raft_small(bogus=1)


def test_deterministic_init():
    _, a = raft_small(seed=0)
    _, b = raft_small(seed=0)
    _, c = raft_small(seed=1)
    fa, fb, fc = (C.flatten_tree(x["params"]) for x in (a, b, c))
    k = "update_block.flow_head.conv1.kernel"
    assert torch.equal(fa[k], fb[k]) and not torch.equal(fa[k], fc[k])
    # truncated-normal init stays within 2 std
    kern = fa["feature_encoder.convnormrelu.layers_0.kernel"]
    std = np.sqrt(2.0 / (7 * 7 * 32)) / 0.87962566103423978
    assert kern.abs().max() <= 2 * std + 1e-6


def test_final_only_output_cpu():
    model, variables = raft_small()
    g = torch.Generator().manual_seed(0)
    i1 = torch.rand(1, 128, 128, 3, generator=g) * 2 - 1
    i2 = torch.rand(1, 128, 128, 3, generator=g) * 2 - 1
    full = model.apply(variables, i1, i2, num_flow_updates=3)
    last = model.apply(variables, i1, i2, num_flow_updates=3, return_all_iters=False)
    assert last.shape == (1, 1, 128, 128, 2)
    assert torch.allclose(last[0], full[-1])


def test_apply_rejects_mismatched_variable_tree():
    model, v = raft_small(seed=0)
    i1, i2 = _pair()
    flat = {k: t.detach().clone() for k, t in C.flatten_tree(v["params"]).items()}
    renamed = dict(flat)
    k0 = "update_block.flow_head.conv2.bias"
    renamed["update_block.flow_head.conv2.bias_typo"] = renamed.pop(k0)
    with pytest.raises(KeyError):
        model.apply({"params": C.unflatten_tree(renamed)}, i1, i2, num_flow_updates=1)
    missing = dict(flat)
    missing.pop(k0)
    with pytest.raises(KeyError):
        model.apply({"params": C.unflatten_tree(missing)}, i1, i2, num_flow_updates=1)
    with pytest.raises(KeyError):
        model.apply({"params": {"typo_encoder": flat[k0]}}, i1, i2, num_flow_updates=1)
    bad = dict(flat)
    bad[k0] = torch.zeros(3)
    with pytest.raises(ValueError):
        model.apply({"params": C.unflatten_tree(bad)}, i1, i2, num_flow_updates=1)


def test_apply_foreign_variables_leave_module_untouched():
    model, v = raft_small(seed=0)
    _, ov = raft_small(seed=3)
    before = {k: t.detach().clone() for k, t in C.flatten_tree(v["params"]).items()}
    i1, i2 = _pair()
    foreign = {"params": C.unflatten_tree({k: t.detach().numpy().copy()
                                           for k, t in C.flatten_tree(ov["params"]).items()})}
    out_f = model.apply(foreign, i1, i2, num_flow_updates=2)
    for k, t in C.flatten_tree(model.variables()["params"]).items():
        assert torch.equal(t, before[k]), k
    out_own = model.apply(v, i1, i2, num_flow_updates=2)
    assert not torch.allclose(out_f, out_own)


def test_apply_foreign_batch_stats_returned_not_written():
    model, v = raft_large(seed=0)
    model.train()
    i1, i2 = _pair(2)
    foreign = {c: C.unflatten_tree({k: t.detach().numpy().copy() for k, t in C.flatten_tree(v[c]).items()})
               for c in ("params", "batch_stats")}
    key = ("context_encoder", "convnormrelu", "layers_1", "mean")
    arr = foreign["batch_stats"]
    for p in key:
        arr = arr[p]
    snapshot = arr.copy()
    own_before = model.context_encoder.convnormrelu.layers_1.mean.detach().clone()
    _, new = model.apply(foreign, i1, i2, train=True, num_flow_updates=1, mutable=["batch_stats"])
    upd = new["batch_stats"]
    for p in key:
        upd = upd[p]
    assert np.array_equal(arr, snapshot)            # caller's arrays not written
    assert torch.equal(model.context_encoder.convnormrelu.layers_1.mean, own_before)
    assert not torch.allclose(upd.cpu(), torch.as_tensor(snapshot))


def test_block_and_norm_as_classes_or_callables():
    """Reference ``model.py:702-711`` passes the residual unit and the norm as classes: the
    built-in classes map to the engine-lowerable kinds, any other callable is a custom
    module (its parameters appear under ``layers_1`` like a Flax norm)."""
    from torch import nn

    from jax_raft_amd.models.layers import (BatchNorm, BottleneckBlock, FeatureEncoder, InstanceNorm,
                                            ResidualBlock, norm_kind)

    assert norm_kind(BatchNorm) == "batch" and norm_kind(InstanceNorm) == "instance" and norm_kind(None) is None

    class Affine(nn.Module):
        def __init__(self, c):
            super().__init__()
            self.scale = nn.Parameter(torch.ones(c))

        def forward(self, x):
            return x * self.scale

    fe = FeatureEncoder(block=ResidualBlock, layers=(32, 32, 48, 64, 128), norm=InstanceNorm)
    assert fe.block == "residual" and fe.norm_kind == "instance"
    ce = FeatureEncoder(block=BottleneckBlock, layers=(32, 32, 64, 96, 160), norm=Affine)
    assert ce.block == "bottleneck" and ce.norm_kind == "custom"
    model, variables = raft_small(feature_encoder=fe, context_encoder=ce)
    assert "layers_1" in variables["params"]["context_encoder"]["convnormrelu"]
    x = torch.rand(1, 128, 128, 3) * 2 - 1
    out = model(x, x, num_flow_updates=2)
    assert out.shape == (2, 1, 128, 128, 2) and torch.isfinite(out).all()
