"""RAFT top-level model, ``raft_large`` / ``raft_small`` factories and the
Flax-style ``apply`` API.

Reference: ``jax_raft/model.py:484-767`` (UpdateCell, RAFT, _raft, raft_large,
raft_small).  API parity:

* ``raft_large(pretrained=False, **kwargs)`` / ``raft_small(...)`` return
  ``(model, variables)``; sub-modules can be injected with the same kwargs
  (``feature_encoder``, ``context_encoder``, ``corr_block``, ``update_block``,
  ``mask_predictor``).
* ``model.apply(variables, image1, image2, train=False, num_flow_updates=12)``
  returns all ``num_flow_updates`` upsampled flows, shape (N, B, H, W, 2),
  NHWC float inputs in [-1, 1].
* ``model(image1, image2, ...)`` is the idiomatic ``nn.Module`` call.

Execution: one implementation per device.  CPU tensors run the golden
PyTorch forward (:mod:`.layers`, :mod:`.reference`); GPU tensors in inference
run the native HIP engine (:mod:`jax_raft_amd.runtime.engine`), and GPU
training runs the autograd path built from the native ops
(:mod:`jax_raft_amd.ops.autograd`).
"""
from __future__ import annotations

from typing import Any, Dict, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from . import reference as R
from .layers import (
    NORM_BATCH,
    NORM_INSTANCE,
    CorrBlock,
    FeatureEncoder,
    FlowHead,
    MaskPredictor,
    MotionEncoder,
    RecurrentBlock,
    UpdateBlock,
)
from ..utils import checkpoint as ckpt

_BASE_URL = "https://github.com/alebeck/jax-raft/releases/download/checkpoints/"
_MODELS_URLS = {
    "raft_large": _BASE_URL + "raft_large_C_T_SKHT_V2-ff5fadd5.msgpack",
    "raft_small": _BASE_URL + "raft_small_C_T_V2-01064c6d.msgpack",
}


def _as_tensor(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x
    a = np.asarray(x)
    if a.dtype == np.uint8:   # raw frames (normalised + padded by the engine / forward)
        return torch.from_numpy(np.ascontiguousarray(a))
    return torch.as_tensor(np.asarray(x, dtype=np.float32))


class RAFT(nn.Module):
    """RAFT (Recurrent All-Pairs Field Transforms), reference ``model.py:513-605``."""

    def __init__(self, feature_encoder: FeatureEncoder, context_encoder: FeatureEncoder, corr_block: CorrBlock,
                 update_block: UpdateBlock, mask_predictor: Optional[MaskPredictor] = None):
        super().__init__()
        self.feature_encoder = feature_encoder
        self.context_encoder = context_encoder
        self.corr_block = corr_block
        self.update_block = update_block
        self.mask_predictor = mask_predictor
        self._engines: Dict[Any, Any] = {}
        self._lowering_error: Optional[str] = None
        self.arch: Optional[str] = None

    # ------------------------------------------------------------ API surface
    def variables(self) -> Dict[str, Dict[str, Any]]:
        return ckpt.variables_from_module(self)

    def forward(self, image1, image2, train: bool = False, num_flow_updates: int = 12, return_all_iters: bool = True,
                **engine_kw):
        """Upsampled flows of every refinement iteration, (num_flow_updates, B, H, W, 2)
        (reference semantics, ``model.py:605``).  ``return_all_iters=False`` (inference
        serving mode) upsamples and returns only the final flow, shape (1, B, H, W, 2)."""
        image1, image2 = _as_tensor(image1), _as_tensor(image2)
        B, H, W, _ = image1.shape
        assert (H, W) == tuple(image2.shape[-3:-1]), "input images should have the same shape"
        if image1.dtype == torch.uint8:
            return self._forward_u8(image1, image2, train, num_flow_updates, return_all_iters, engine_kw)
        assert (H % 8 == 0) and (W % 8 == 0), "input image H and W should be divisible by 8"
        dev = self._param_device()
        if dev.type == "cuda" and not image1.is_cuda:   # host arrays / tensors for a model on the GPU
            image1, image2 = image1.to(dev), image2.to(dev)
        autograd = engine_kw.pop("autograd", False)
        fused = engine_kw.pop("fused", None)
        if image1.is_cuda:
            if train or autograd:
                from ..ops.autograd import raft_forward_autograd

                out = raft_forward_autograd(self, image1, image2, train, num_flow_updates, fused=fused)
                return out if return_all_iters else out[-1:]
            eng = None if self._lowering_error is not None else self._try_engine(image1.device, engine_kw)
            if eng is not None:
                return eng.forward(image1, image2, num_flow_updates, return_all_iters=return_all_iters)
            # a model the engine cannot lower (injected sub-modules, custom blocks / norms, channel
            # counts outside the fused kernels' tiling): op by op on the same native kernels
            # (convs, correlation pyramid, lookup: ops/functional.py), no graph
            with torch.no_grad():
                return self.forward_reference(image1, image2, False, num_flow_updates, return_all_iters)
        return self.forward_reference(image1, image2, train, num_flow_updates, return_all_iters)

    def _forward_u8(self, image1, image2, train, num_flow_updates, return_all_iters, engine_kw):
        """Raw uint8 NHWC frames of any size: the reference's input protocol
        (``scripts/validate_sintel.py:177-191``: x / 255 * 2 - 1, InputPadder('sintel') replicate
        padding to /8, unpad of the flows) -- on the GPU inside the engine's prep kernel, elsewhere
        (CPU golden path, training, models the engine cannot lower) with framework ops."""
        dev = self._param_device()
        if dev.type == "cuda" and not (train or engine_kw.get("autograd")) and self._lowering_error is None:
            # host frames go straight into the plan's uint8 input buffers (one H2D copy of 1/4 the
            # bytes of normalised fp32 frames)
            eng = self._try_engine(dev, {k: v for k, v in engine_kw.items() if k not in ("autograd", "fused")})
            if eng is not None:
                return eng.forward(image1, image2, num_flow_updates, return_all_iters=return_all_iters)
        if dev.type == "cuda" and not image1.is_cuda:
            image1, image2 = image1.to(dev), image2.to(dev)
        from ..runtime.engine import sintel_pad, u8_table

        H0, W0 = image1.shape[1:3]
        pt, pb, pl, pr = sintel_pad(H0, W0)
        lut = u8_table(image1.device)

        def prep(x):
            x = lut[x.long()].permute(0, 3, 1, 2)
            return torch.nn.functional.pad(x, [pl, pr, pt, pb], mode="replicate").permute(0, 2, 3, 1).contiguous()

        out = self.forward(prep(image1), prep(image2), train, num_flow_updates, return_all_iters, **engine_kw)
        return out[:, :, pt:pt + H0, pl:pl + W0]

    def _param_device(self) -> torch.device:
        p = next(self.parameters(), None)
        return p.device if p is not None else torch.device("cpu")

    def _try_engine(self, device, engine_kw):
        """The native engine, or None (remembering why) when it cannot lower this model."""
        try:
            return self.engine(device, **engine_kw)
        except NotImplementedError as e:
            self._lowering_error = str(e)
            return None

    @property
    def execution_path(self) -> str:
        """"engine" (native plan / hipGraph) or "op-by-op: <why the engine cannot lower it>"."""
        return "engine" if self._lowering_error is None else f"op-by-op: {self._lowering_error}"

    def apply(self, variables: Mapping[str, Any], image1, image2, train: bool = False, num_flow_updates: int = 12,
              mutable=False, **kw):
        """Flax-style ``model.apply(variables, image1, image2, train, num_flow_updates)``.

        With ``mutable=['batch_stats']`` (and ``train=True``) returns
        ``(flows, {'batch_stats': updated})`` like Flax."""
        own = self.variables()
        if _same_leaves(own, variables):
            out = self(image1, image2, train=train, num_flow_updates=num_flow_updates, **kw)
            if mutable:
                return out, {"batch_stats": ckpt.variables_from_module(self)["batch_stats"]}
            return out
        # Foreign variables (numpy / torch leaves): validated like Flax's apply
        # (every param present, no unexpected leaf, shapes equal; an absent
        # 'batch_stats' collection keeps the module's own statistics) and bound
        # functionally for this call only -- the module's tensors are untouched.
        # Leaves are copied, so a train-mode BatchNorm update never writes into
        # the caller's arrays; it is returned through ``mutable`` like Flax.
        bound = ckpt.variables_as_tensors(self, variables)
        out = torch.func.functional_call(
            self, bound, (image1, image2), dict(train=train, num_flow_updates=num_flow_updates, **kw))
        if mutable:
            stats = {k: v for k, v in bound.items() if k.endswith(".mean") or k.endswith(".var")}
            if not stats:
                stats = {k: v for k, v in ckpt.flatten_tree(own["batch_stats"]).items()}
            return out, {"batch_stats": ckpt.unflatten_tree(stats)}
        return out

    # ------------------------------------------------------- golden execution
    def forward_reference(self, image1, image2, train: bool, num_flow_updates: int, return_all_iters: bool = True):
        """Reference-semantics forward (``model.py:557-605`` with the scan body
        ``UpdateCell.__call__``, ``model.py:495-510``)."""
        B, H, W, _ = image1.shape
        fmaps = self.feature_encoder(torch.cat([image1, image2], dim=0), train)
        fmap1, fmap2 = torch.chunk(fmaps, 2, dim=0)
        assert tuple(fmap1.shape[1:3]) == (H // 8, W // 8), "The feature encoder should downsample H and W by 8"
        pyramid = self.corr_block.build_pyramid(fmap1, fmap2)
        ctx = self.context_encoder(image1, train)
        assert tuple(ctx.shape[1:3]) == (H // 8, W // 8), "The context encoder should downsample H and W by 8"
        hs = self.update_block.hidden_state_size
        assert ctx.shape[-1] - hs > 0, (
            f"The context encoder outputs {ctx.shape[-1]} channels, but it should have at "
            f"strictly more than hidden_state={hs} channels")
        hidden, context = ctx[..., :hs], ctx[..., hs:]
        hidden = torch.tanh(hidden)
        context = torch.relu(context)
        coords0 = R.make_coords_grid(B, H // 8, W // 8, device=image1.device)
        coords1 = coords0.clone()
        preds = []
        for it in range(num_flow_updates):
            coords1 = coords1.detach()  # stop_gradient, model.py:498
            corr = self.corr_block.index_pyramid(pyramid, coords1)
            flow = coords1 - coords0
            hidden, delta = self.update_block(hidden, context, corr, flow, train)
            coords1 = coords1 + delta
            if not return_all_iters and it + 1 < num_flow_updates:
                continue
            up_mask = None if self.mask_predictor is None else self.mask_predictor(hidden, train)
            preds.append(R.upsample_flow(coords1 - coords0, up_mask))
        return torch.stack(preds, dim=0)

    # -------------------------------------------------------- native engine
    def engine(self, device, **kw):
        """The cached native inference engine for ``device`` (built lazily)."""
        from ..runtime.engine import RaftEngine

        key = (str(device), tuple(sorted(kw.items())))
        eng = self._engines.get(key)
        if eng is None:
            eng = RaftEngine(self, device, **kw)
            eng._hold_model_weakly()   # no model <-> engine cycle: the plans die with the model
            self._engines[key] = eng
        return eng

    def _apply(self, fn, *args, **kwargs):  # drop engines when moved / cast
        self._engines = {}
        self._lowering_error = None
        return super()._apply(fn, *args, **kwargs)

    def __setattr__(self, name, value):
        # a replaced sub-module may make the model lowerable again (or not): re-decide
        if name in ("feature_encoder", "context_encoder", "corr_block", "update_block", "mask_predictor"):
            self.__dict__["_lowering_error"] = None
            if "_engines" in self.__dict__:
                self.__dict__["_engines"] = {}
        super().__setattr__(name, value)


def _same_leaves(a: Mapping[str, Any], b: Mapping[str, Any]) -> bool:
    fa = {}
    for coll in ("params", "batch_stats"):
        fa.update({f"{coll}.{k}": v for k, v in ckpt.flatten_tree(a.get(coll, {}) or {}).items()})
    fb = {}
    for coll in ("params", "batch_stats"):
        if isinstance(b, Mapping) and coll in b and b[coll]:
            fb.update({f"{coll}.{k}": v for k, v in ckpt.flatten_tree(b[coll]).items()})
    if set(fb) - set(fa):
        return False
    return all(isinstance(v, torch.Tensor) and v is fa[k] for k, v in fb.items())


def _raft(*, feature_encoder_layers, feature_encoder_block, feature_encoder_norm_layer, context_encoder_layers,
          context_encoder_block, context_encoder_norm_layer, corr_block_num_levels, corr_block_radius,
          motion_encoder_corr_layers, motion_encoder_flow_layers, motion_encoder_out_channels,
          recurrent_block_hidden_state_size, recurrent_block_kernel_size, recurrent_block_padding,
          flow_head_hidden_size, use_mask_predictor, pretrained_arch=None, weights: Optional[str] = None,
          seed: int = 0, **kwargs) -> Tuple[RAFT, Dict[str, Any]]:
    """Reference ``_raft``, ``model.py:608-691``."""
    gen = torch.Generator().manual_seed(seed)
    feature_encoder = kwargs.pop("feature_encoder", None) or FeatureEncoder(
        block=feature_encoder_block, layers=feature_encoder_layers, norm=feature_encoder_norm_layer, gen=gen)
    context_encoder = kwargs.pop("context_encoder", None) or FeatureEncoder(
        block=context_encoder_block, layers=context_encoder_layers, norm=context_encoder_norm_layer, gen=gen)
    corr_block = kwargs.pop("corr_block", None) or CorrBlock(num_levels=corr_block_num_levels, radius=corr_block_radius)
    update_block = kwargs.pop("update_block", None)
    if update_block is None:
        hidden = recurrent_block_hidden_state_size
        context_ch = context_encoder.out_channels - hidden
        motion_encoder = MotionEncoder(corr_block.out_channels, corr_layers=motion_encoder_corr_layers,
                                       flow_layers=motion_encoder_flow_layers,
                                       out_channels=motion_encoder_out_channels, gen=gen)
        recurrent_block = RecurrentBlock(context_ch + motion_encoder_out_channels, hidden,
                                         kernel_size=recurrent_block_kernel_size, padding=recurrent_block_padding,
                                         gen=gen)
        flow_head = FlowHead(hidden, flow_head_hidden_size, gen=gen)
        update_block = UpdateBlock(motion_encoder, recurrent_block, flow_head)
    mask_predictor = kwargs.pop("mask_predictor", None)
    if mask_predictor is None and use_mask_predictor:
        mask_predictor = MaskPredictor(update_block.hidden_state_size, hidden_size=256, multiplier=0.25, gen=gen)
    if kwargs:
        raise TypeError(f"unexpected keyword arguments: {sorted(kwargs)}")
    model = RAFT(feature_encoder, context_encoder, corr_block, update_block, mask_predictor)
    model.eval()
    if pretrained_arch is not None or weights is not None:
        arch = pretrained_arch or "raft_large"
        data = ckpt.resolve_pretrained(arch, _MODELS_URLS[arch], weights)
        ckpt.load_variables_into(model, ckpt.msgpack_restore(data), strict=True)
    return model, model.variables()


def raft_large(*, pretrained: bool = False, **kwargs):
    """RAFT large (``model.py:694-729``)."""
    model, variables = _raft(
        feature_encoder_layers=(64, 64, 96, 128, 256),
        feature_encoder_block="residual",
        feature_encoder_norm_layer=NORM_INSTANCE,
        context_encoder_layers=(64, 64, 96, 128, 256),
        context_encoder_block="residual",
        context_encoder_norm_layer=NORM_BATCH,
        corr_block_num_levels=4,
        corr_block_radius=4,
        motion_encoder_corr_layers=(256, 192),
        motion_encoder_flow_layers=(128, 64),
        motion_encoder_out_channels=128,
        recurrent_block_hidden_state_size=128,
        recurrent_block_kernel_size=((1, 5), (5, 1)),
        recurrent_block_padding=((0, 2), (2, 0)),
        flow_head_hidden_size=256,
        use_mask_predictor=True,
        pretrained_arch="raft_large" if pretrained else None,
        **kwargs,
    )
    model.arch = "raft_large"
    return model, variables


def raft_small(*, pretrained: bool = False, **kwargs):
    """RAFT small (``model.py:732-767``)."""
    model, variables = _raft(
        feature_encoder_layers=(32, 32, 64, 96, 128),
        feature_encoder_block="bottleneck",
        feature_encoder_norm_layer=NORM_INSTANCE,
        context_encoder_layers=(32, 32, 64, 96, 160),
        context_encoder_block="bottleneck",
        context_encoder_norm_layer=None,
        corr_block_num_levels=4,
        corr_block_radius=3,
        motion_encoder_corr_layers=(96,),
        motion_encoder_flow_layers=(64, 32),
        motion_encoder_out_channels=82,
        recurrent_block_hidden_state_size=96,
        recurrent_block_kernel_size=((3, 3),),
        recurrent_block_padding=((1, 1),),
        flow_head_hidden_size=128,
        use_mask_predictor=False,
        pretrained_arch="raft_small" if pretrained else None,
        **kwargs,
    )
    model.arch = "raft_small"
    return model, variables
