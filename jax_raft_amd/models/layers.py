"""RAFT building blocks as ``torch.nn.Module``s whose parameter tree mirrors the
reference Flax tree exactly.

Parameters are stored in the Flax layouts -- conv ``kernel`` as HWIO
``(kh, kw, cin, cout)``, ``bias``; BatchNorm ``scale``/``bias`` parameters and
``mean``/``var`` buffers (the Flax ``batch_stats`` collection) -- so a Flax
msgpack checkpoint maps 1:1 onto ``state_dict`` keys ('/' -> '.').

The ``forward`` methods implement the reference semantics with the golden
pure-PyTorch primitives (:mod:`jax_raft_amd.models.reference`); they form the
CPU execution path and the autograd path.  The GPU inference path does not
call these forwards: :mod:`jax_raft_amd.runtime.engine` lowers the same
parameters onto the HIP kernels.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Sequence, Tuple

import torch
from torch import nn

from . import reference as R
from ..ops import functional as OF

# --------------------------------------------------------------------------- init

_TRUNC_CORR = 0.87962566103423978  # stddev of a unit normal truncated to [-2, 2]


def _variance_scaling_(t: torch.Tensor, scale: float, mode: str, gen: Optional[torch.Generator]) -> torch.Tensor:
    """flax ``variance_scaling(scale, mode, 'truncated_normal')`` for HWIO kernels."""
    kh, kw, cin, cout = t.shape
    rf = kh * kw
    fan = rf * (cin if mode == "fan_in" else cout)
    std = math.sqrt(scale / fan) / _TRUNC_CORR
    with torch.no_grad():
        # inverse-CDF truncated normal on [-2, 2] (deterministic under `gen`)
        u = torch.rand(t.shape, generator=gen, dtype=torch.float64)
        lo = 0.5 * (1 + math.erf(-2 / math.sqrt(2)))
        hi = 0.5 * (1 + math.erf(2 / math.sqrt(2)))
        p = lo + u * (hi - lo)
        z = math.sqrt(2) * torch.erfinv(2 * p - 1)
        t.copy_((z * std).to(t.dtype))
    return t


def kaiming_fan_out_(t, gen=None):
    """``Conv`` factory init, reference ``model.py:101-104``."""
    return _variance_scaling_(t, 2.0, "fan_out", gen)


def lecun_normal_(t, gen=None):
    """flax ``nn.Conv`` default kernel init (plain convs at ``model.py:304-310,347-349,394``)."""
    return _variance_scaling_(t, 1.0, "fan_in", gen)


# ------------------------------------------------------------------------ modules


class Conv(nn.Module):
    """A Flax ``nn.Conv`` leaf: ``kernel`` (kh, kw, cin, cout) + ``bias``."""

    def __init__(self, cin: int, cout: int, kernel_size: Tuple[int, int], stride=(1, 1), padding=None,
                 init: str = "kaiming", gen: Optional[torch.Generator] = None):
        super().__init__()
        kh, kw = kernel_size
        self.kernel_size = (kh, kw)
        self.stride = tuple(stride)
        if padding is None:
            padding = ((kh - 1) // 2, (kw - 1) // 2)  # model.py:137-141
        self.padding = tuple(padding)
        self.cin, self.cout = cin, cout
        self.kernel = nn.Parameter(torch.empty(kh, kw, cin, cout))
        self.bias = nn.Parameter(torch.zeros(cout))
        (kaiming_fan_out_ if init == "kaiming" else lecun_normal_)(self.kernel.data, gen)

    def forward(self, x):
        return OF.conv2d_nhwc(x, self.kernel, self.bias, self.stride, self.padding)


class BatchNorm(nn.Module):
    """Flax ``nn.BatchNorm`` (momentum 0.99, eps 1e-5): params scale/bias,
    batch_stats mean/var.  ``sync_group`` (set by
    :func:`jax_raft_amd.parallel.dp.convert_sync_batchnorm`) synchronises the
    training-mode batch statistics across data-parallel ranks."""

    def __init__(self, c: int, momentum: float = 0.99, eps: float = 1e-5):
        super().__init__()
        self.momentum, self.eps = momentum, eps
        self.sync_group = None
        self.scale = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("mean", torch.zeros(c))
        self.register_buffer("var", torch.ones(c))

    def forward(self, x, train: bool):
        y, nm, nv = R.batch_norm_nhwc(x, self.scale, self.bias, self.mean, self.var, train, self.eps, self.momentum,
                                      sync_group=self.sync_group)
        if train:
            with torch.no_grad():
                self.mean.copy_(nm)
                self.var.copy_(nv)
        return y


class InstanceNorm(nn.Module):
    """Flax ``nn.InstanceNorm(epsilon=1e-5, use_bias=False, use_scale=False)``:
    parameter-free (absent from the checkpoint tree)."""

    def __init__(self, eps: float = 1e-5):
        super().__init__()
        self.eps = eps

    def forward(self, x, train: bool = False):
        return R.instance_norm_nhwc(x, self.eps)


NORM_BATCH = "batch"
NORM_INSTANCE = "instance"
NORM_CUSTOM = "custom"


def norm_kind(norm) -> Optional[str]:
    """A norm given like the reference's ``norm_layer`` (``model.py:702-711``: a class or a
    partial of one) or by name: "batch" / "instance" / None for the built-in Flax norms
    (:class:`BatchNorm` / :class:`InstanceNorm` classes map to them), "custom" for any other
    callable ``norm(channels) -> module`` (``module(x, train)`` or ``module(x)``), which runs
    on the op-by-op path (the native engine lowers the built-in norms only)."""
    if norm is None or norm in (NORM_BATCH, NORM_INSTANCE):
        return norm
    if norm is BatchNorm:
        return NORM_BATCH
    if norm is InstanceNorm:
        return NORM_INSTANCE
    if callable(norm):
        return NORM_CUSTOM
    raise ValueError(f"unknown norm layer {norm!r}")


def _call_norm(m: nn.Module, x, train: bool):
    import inspect

    try:
        n = len(inspect.signature(m.forward).parameters)
    except (TypeError, ValueError):
        n = 1
    return m(x, train) if n >= 2 else m(x)


class ConvNormActivation(nn.Module):
    """Conv -> optional norm -> optional relu; children ``layers_0``/``layers_1``.
    Reference ``model.py:120-159``.  ``norm``: see :func:`norm_kind`."""

    def __init__(self, cin, cout, kernel_size=(3, 3), stride=(1, 1), padding=None,
                 norm=NORM_BATCH, relu: bool = True, gen=None):
        super().__init__()
        self.layers_0 = Conv(cin, cout, kernel_size, stride, padding, init="kaiming", gen=gen)
        kind = norm_kind(norm)
        self.norm = kind
        if kind == NORM_BATCH:
            self.layers_1 = BatchNorm(cout)
        elif kind == NORM_INSTANCE:
            self._in = InstanceNorm()
        elif kind == NORM_CUSTOM:
            self.layers_1 = norm(cout)
        self.relu = relu

    def forward(self, x, train: bool):
        x = self.layers_0(x)
        if self.norm == NORM_BATCH:
            x = self.layers_1(x, train)
        elif self.norm == NORM_INSTANCE:
            x = self._in(x)
        elif self.norm == NORM_CUSTOM:
            x = _call_norm(self.layers_1, x, train)
        if self.relu:
            x = torch.relu(x)
        return x


class ResidualBlock(nn.Module):
    """Reference ``model.py:162-184``."""

    def __init__(self, cin, cout, norm, stride=(1, 1), gen=None):
        super().__init__()
        self.convnormrelu1 = ConvNormActivation(cin, cout, (3, 3), stride, norm=norm, gen=gen)
        self.convnormrelu2 = ConvNormActivation(cout, cout, (3, 3), (1, 1), norm=norm, gen=gen)
        self.stride = tuple(stride)
        if self.stride != (1, 1):
            self.downsample = ConvNormActivation(cin, cout, (1, 1), stride, norm=norm, relu=False, gen=gen)

    def forward(self, x, train: bool):
        y = self.convnormrelu1(x, train)
        y = self.convnormrelu2(y, train)
        if self.stride != (1, 1):
            x = self.downsample(x, train)
        return torch.relu(x + y)


class BottleneckBlock(nn.Module):
    """Reference ``model.py:187-216``."""

    def __init__(self, cin, cout, norm, stride=(1, 1), gen=None):
        super().__init__()
        self.convnormrelu1 = ConvNormActivation(cin, cout // 4, (1, 1), norm=norm, gen=gen)
        self.convnormrelu2 = ConvNormActivation(cout // 4, cout // 4, (3, 3), stride, norm=norm, gen=gen)
        self.convnormrelu3 = ConvNormActivation(cout // 4, cout, (1, 1), norm=norm, gen=gen)
        self.stride = tuple(stride)
        if self.stride != (1, 1):
            self.downsample = ConvNormActivation(cin, cout, (1, 1), stride, norm=norm, relu=False, gen=gen)

    def forward(self, x, train: bool):
        y = self.convnormrelu1(x, train)
        y = self.convnormrelu2(y, train)
        y = self.convnormrelu3(y, train)
        if self.stride != (1, 1):
            x = self.downsample(x, train)
        return torch.relu(x + y)


BLOCKS = {"residual": ResidualBlock, "bottleneck": BottleneckBlock}


def block_factory(block):
    """A residual unit given like the reference's ``block`` (``model.py:702-711``: the class
    itself) or by name ("residual" / "bottleneck"); any other callable
    ``block(cin, cout, norm, stride, gen) -> module`` (``module(x, train)``) is accepted too
    and runs on the op-by-op path."""
    if isinstance(block, str):
        return BLOCKS[block]
    if callable(block):
        return block
    raise ValueError(f"unknown block {block!r}")


class Sequential(nn.Module):
    """Registered sequential: children ``layers_0``, ``layers_1`` (``model.py:107-117``)."""

    def __init__(self, *layers):
        super().__init__()
        for i, l in enumerate(layers):
            setattr(self, f"layers_{i}", l)
        self.n = len(layers)

    def forward(self, x, train: bool):
        for i in range(self.n):
            x = getattr(self, f"layers_{i}")(x, train)
        return x


class FeatureEncoder(nn.Module):
    """Feature / context encoder, downsamples x8.  Reference ``model.py:219-257``."""

    def __init__(self, block="residual", layers=(64, 64, 96, 128, 256),
                 strides=((2, 2), (1, 1), (2, 2), (2, 2)), norm=NORM_BATCH, in_channels: int = 3,
                 gen=None):
        super().__init__()
        assert len(layers) == 5
        B = block_factory(block)
        self.block = next((k for k, v in BLOCKS.items() if v is B), "custom")
        self.layers, self.strides, self.norm_kind = tuple(layers), tuple(strides), norm_kind(norm)
        self.convnormrelu = ConvNormActivation(in_channels, layers[0], (7, 7), strides[0], norm=norm, gen=gen)
        self.layer1 = Sequential(B(layers[0], layers[1], norm, strides[1], gen), B(layers[1], layers[1], norm, (1, 1), gen))
        self.layer2 = Sequential(B(layers[1], layers[2], norm, strides[2], gen), B(layers[2], layers[2], norm, (1, 1), gen))
        self.layer3 = Sequential(B(layers[2], layers[3], norm, strides[3], gen), B(layers[3], layers[3], norm, (1, 1), gen))
        self.conv = Conv(layers[3], layers[4], (1, 1), init="kaiming", gen=gen)

    @property
    def out_channels(self):
        return self.layers[4]

    def forward(self, x, train: bool):
        x = self.convnormrelu(x, train)
        x = self.layer1(x, train)
        x = self.layer2(x, train)
        x = self.layer3(x, train)
        return self.conv(x)


class MotionEncoder(nn.Module):
    """Reference ``model.py:260-290``."""

    def __init__(self, in_channels_corr: int, corr_layers=(256, 192), flow_layers=(128, 64), out_channels=128, gen=None):
        super().__init__()
        assert len(flow_layers) == 2
        assert len(corr_layers) in (1, 2)
        self.corr_layers, self.flow_layers, self.out_channels = tuple(corr_layers), tuple(flow_layers), out_channels
        self.convcorr1 = ConvNormActivation(in_channels_corr, corr_layers[0], (1, 1), norm=None, gen=gen)
        if len(corr_layers) == 2:
            self.convcorr2 = ConvNormActivation(corr_layers[0], corr_layers[1], (3, 3), norm=None, gen=gen)
        self.convflow1 = ConvNormActivation(2, flow_layers[0], (7, 7), norm=None, gen=gen)
        self.convflow2 = ConvNormActivation(flow_layers[0], flow_layers[1], (3, 3), norm=None, gen=gen)
        self.conv = ConvNormActivation(corr_layers[-1] + flow_layers[-1], out_channels - 2, (3, 3), norm=None, gen=gen)

    def forward(self, flow, corr_features, train: bool = False):
        corr = self.convcorr1(corr_features, train)
        if len(self.corr_layers) == 2:
            corr = self.convcorr2(corr, train)
        flow_orig = flow
        flow = self.convflow1(flow, train)
        flow = self.convflow2(flow, train)
        corr_flow = torch.cat([corr, flow], dim=-1)
        corr_flow = self.conv(corr_flow, train)
        return torch.cat([corr_flow, flow_orig], dim=-1)


class ConvGRU(nn.Module):
    """Reference ``model.py:293-312`` (plain nn.Conv, Flax default init)."""

    def __init__(self, input_size: int, hidden_size: int, kernel_size, padding, gen=None):
        super().__init__()
        self.hidden_size, self.kernel_size, self.padding = hidden_size, tuple(kernel_size), tuple(padding)
        c = hidden_size + input_size
        self.convz = Conv(c, hidden_size, kernel_size, padding=padding, init="lecun", gen=gen)
        self.convr = Conv(c, hidden_size, kernel_size, padding=padding, init="lecun", gen=gen)
        self.convq = Conv(c, hidden_size, kernel_size, padding=padding, init="lecun", gen=gen)

    def forward(self, h, x):
        hx = torch.cat([h, x], dim=-1)
        z = torch.sigmoid(self.convz(hx))
        r = torch.sigmoid(self.convr(hx))
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=-1)))
        return (1 - z) * h + z * q


class RecurrentBlock(nn.Module):
    """Reference ``model.py:315-334``."""

    def __init__(self, input_size: int, hidden_size: int, kernel_size=((1, 5), (5, 1)), padding=((0, 2), (2, 0)), gen=None):
        super().__init__()
        assert len(kernel_size) == len(padding) and len(kernel_size) in (1, 2)
        self.hidden_size = hidden_size
        self.kernel_size, self.padding = tuple(map(tuple, kernel_size)), tuple(map(tuple, padding))
        self.convgru1 = ConvGRU(input_size, hidden_size, kernel_size[0], padding[0], gen)
        if len(kernel_size) == 2:
            self.convgru2 = ConvGRU(input_size, hidden_size, kernel_size[1], padding[1], gen)

    def forward(self, h, x):
        h = self.convgru1(h, x)
        if len(self.kernel_size) == 2:
            h = self.convgru2(h, x)
        return h


class FlowHead(nn.Module):
    """Reference ``model.py:337-350``."""

    def __init__(self, in_channels: int, hidden_size: int, gen=None):
        super().__init__()
        self.hidden_size = hidden_size
        self.conv1 = Conv(in_channels, hidden_size, (3, 3), padding=(1, 1), init="lecun", gen=gen)
        self.conv2 = Conv(hidden_size, 2, (3, 3), padding=(1, 1), init="lecun", gen=gen)

    def forward(self, x):
        return self.conv2(torch.relu(self.conv1(x)))


class UpdateBlock(nn.Module):
    """Reference ``model.py:353-374``."""

    def __init__(self, motion_encoder: MotionEncoder, recurrent_block: RecurrentBlock, flow_head: FlowHead):
        super().__init__()
        self.motion_encoder = motion_encoder
        self.recurrent_block = recurrent_block
        self.flow_head = flow_head

    @property
    def hidden_state_size(self):
        return self.recurrent_block.hidden_size

    def forward(self, hidden_state, context, corr_features, flow, train: bool = False):
        motion = self.motion_encoder(flow, corr_features, train)
        x = torch.cat([context, motion], dim=-1)
        hidden_state = self.recurrent_block(hidden_state, x)
        return hidden_state, self.flow_head(hidden_state)


class MaskPredictor(nn.Module):
    """Reference ``model.py:377-400`` (x0.25 multiplier)."""

    def __init__(self, in_channels: int, hidden_size: int = 256, multiplier: float = 0.25, gen=None):
        super().__init__()
        self.hidden_size, self.multiplier = hidden_size, multiplier
        self.convrelu = ConvNormActivation(in_channels, hidden_size, (3, 3), norm=None, gen=gen)
        self.conv = Conv(hidden_size, 8 * 8 * 9, (1, 1), padding=(0, 0), init="lecun", gen=gen)

    def forward(self, x, train: bool = False):
        return self.multiplier * self.conv(self.convrelu(x, train))


class CorrBlock:
    """All-pairs correlation pyramid + lookup.  Plain Python object like the
    reference (``model.py:403-481``): it owns no parameters."""

    def __init__(self, num_levels: int = 4, radius: int = 4):
        self.num_levels = num_levels
        self.radius = radius
        self.out_channels = num_levels * (2 * radius + 1) ** 2

    def build_pyramid(self, fmap1, fmap2):
        return OF.build_pyramid(fmap1, fmap2, self.num_levels)

    def index_pyramid(self, corr_pyramid, centroids_coords):
        out = OF.index_pyramid(corr_pyramid, centroids_coords, self.radius)
        assert out.shape[-1] == self.out_channels
        return out
