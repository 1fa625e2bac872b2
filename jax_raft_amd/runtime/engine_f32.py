"""fp32 parity mode of the native engine (``RaftEngine(..., precision="fp32")``).

The reference runs fp32 end to end (``jax_raft/model.py:101-104,304-310``;
SURVEY.md 5.6).  This engine lowers the same model onto fp32 kernels only:

* every conv -- and the level-0 all-pairs correlation GEMM, as a 1x1 "conv"
  whose weight rows are fmap2's pixels -- on the f32-input MFMA
  (``csrc/kernels/conv_f32.hip``: exact fp32 products, fp32 accumulation);
* fp32 activations, instance-norm statistics, correlation pyramid (2x2 floor
  pooling), lookups, hidden state, flow and x8 upsampling
  (``csrc/kernels/f32.hip``).

It exists to bisect the bf16 engine's numerics on the device (profiles/r5_drift.md:
the bf16 drift vs this engine vs the fp32 CPU golden) and for users who need the
reference's own precision; the bf16 engine is the throughput path.  One lane,
no deferral: each iteration runs in the reference's order (lookup, motion
encoder, 2 x ConvGRU, FlowHead, coords update, mask head + upsampling).  The
loop-invariant context share of the ConvGRU gates is folded into a per-pixel
bias map in the prologue, as in the bf16 engine (``engine.py`` module doc).
"""
from __future__ import annotations

from typing import Tuple

import torch

from ..models.layers import NORM_INSTANCE, BottleneckBlock, FeatureEncoder
from ..ops import native as nat
from ..ops.native import ACT_NONE, ACT_RELU, ACT_SPLIT_TANH_RELU, EPI_GRU_A, EPI_GRU_B, conv_f32_args, round_up
from .engine import RaftEngine, _PlanState

F32 = torch.float32


class RaftEngineF32(RaftEngine):
    """See the module docstring.  Same API as :class:`RaftEngine` (``forward``,
    ``pipelined`` / ``flush``, ``op_names``); ``split`` / ``streams`` /
    ``autotune`` / ``corr_dtype`` / ``gate_dtype`` do not apply."""

    precision = "fp32"
    _native_u8 = False   # uint8 frames: normalised + padded by framework ops, then the fp32 prep

    def _analyse(self):
        super()._analyse()
        # fp32 rows in 16-byte chunks: channel strides / offsets in multiples of 4
        self.hx_cs = round_up(self.hx_real, 4)
        self.corr_cs = round_up(self.corr_ch, 4)
        self.gate_cs = round_up(3 * self.hidden, 4)
        self.split = 1

    def _define_specs(self):
        super()._define_specs()
        fh = self.model.update_block.flow_head
        c = fh.conv2
        self._reg("fh2", lambda: (c.kernel.detach().float(), c.bias.detach().float(), c.stride, c.padding, None))

    def _cin4(self, name: str, cin: int) -> int:
        if name.startswith("gru") and (name.endswith(".a") or name.endswith(".b")):
            return self.hx_cs
        if name == "me.convcorr1":
            return self.corr_cs
        return round_up(cin, 4)

    def _pack(self):
        """(Re)pack every conv as fp32 [cout, K]; BN folded (eval mode); packed
        tensors are updated in place so captured graphs stay valid."""
        if not self._sources:
            self._define_specs()
        for name, fn in self._sources.items():
            if name in ("fh1", "fh2.taps") and self.has_mask:
                continue   # bf16-engine fusions (FlowHead conv1 || mask conv, conv2 as taps)
            if name == "fh2.taps" or name.endswith(".stem_s2d"):
                continue   # bf16-engine forms
            k, b, stride, pad, _ = fn()
            k = k.to(self.device)
            cin4 = self._cin4(name, k.shape[2])
            if name in self._specs:
                sp = self._specs[name]
                sp.w.copy_(nat.pack_weight_f32(k, cin4))
                sp.b.copy_(b.float().to(self.device))
            else:
                self._specs[name] = nat.make_spec_f32(k, b.to(self.device), stride, pad, cin4=cin4, device=self.device)
        self._snap = self._snapshot()

    def uses_lanes(self, B: int, all_iters: bool = True) -> bool:
        return False

    def _conv(self, plan, spec, x, N, H, W, y, **kw):
        plan.add_conv_f32(*conv_f32_args(spec, x, N, H, W, y, **kw))

    # ------------------------------------------------------------- lowering
    def _encoder_f32(self, st: _PlanState, plan, tag: str, enc: FeatureEncoder, x: torch.Tensor, N: int, H: int,
                     W: int) -> Tuple[torch.Tensor, int, int]:
        """FeatureEncoder up to (not including) its final 1x1 conv
        (``model.py:179-232``): convs with fused bias / ReLU / residual;
        instance norms as statistics + normalise(+residual)+ReLU passes; batch
        norms (eval) folded into the conv weights."""
        inorm = enc.norm_kind == NORM_INSTANCE
        sp = self._specs
        bufs = st.bufs

        def alloc(name, shape):
            t = torch.zeros(shape, dtype=F32, device=self.device)
            bufs[name] = t
            return t

        def conv_raw(name, x, H, W, act=ACT_NONE, res=None, res_post=0):
            s = sp[name]
            OH, OW = s.out_hw(H, W)
            y = alloc(name + ".y", (N, OH, OW, s.cout))
            self._conv(plan, s, x, N, H, W, y, act=act, res=res, res_post=res_post)
            return y, OH, OW

        def stats(name, y):
            t = alloc(name + ".stats", (N, y.shape[-1], 2))
            plan.add_stats_f32([y, t], [N, y.shape[1] * y.shape[2], y.shape[-1]])
            return t

        def norm_act(name, x, sx, res=None, sr=None, mode_r=0, relu=3):
            y = alloc(name + ".n", tuple(x.shape))
            plan.add_norm_act_f32([x, sx, res, sr, y], [1, mode_r, N, x.shape[1] * x.shape[2], x.shape[-1], relu], 1e-5)
            return y

        if inorm:
            y, H, W = conv_raw(f"{tag}.stem", x, H, W)
            x = norm_act(f"{tag}.stem", y, stats(f"{tag}.stem", y), relu=2)
        else:
            x, H, W = conv_raw(f"{tag}.stem", x, H, W, act=ACT_RELU)
        for li in (1, 2, 3):
            layer = getattr(enc, f"layer{li}")
            for bi in range(layer.n):
                blk = getattr(layer, f"layers_{bi}")
                pre = f"{tag}.l{li}.b{bi}"
                names = ["convnormrelu1", "convnormrelu2"] + (["convnormrelu3"] if isinstance(blk, BottleneckBlock) else [])
                has_ds = blk.stride != (1, 1)
                h_, w_ = H, W
                if inorm:
                    y = x
                    for j, nm in enumerate(names):
                        yr, h_, w_ = conv_raw(f"{pre}.{nm}", y, h_, w_)
                        s = stats(f"{pre}.{nm}", yr)
                        if j + 1 < len(names):
                            y = norm_act(f"{pre}.{nm}", yr, s, relu=2)
                        else:
                            last, last_s = yr, s
                    if has_ds:
                        dr, _, _ = conv_raw(f"{pre}.downsample", x, H, W)
                        x = norm_act(f"{pre}.out", last, last_s, res=dr, sr=stats(f"{pre}.downsample", dr), mode_r=1)
                    else:
                        x = norm_act(f"{pre}.out", last, last_s, res=x, mode_r=0)
                else:
                    res = x
                    if has_ds:
                        res, _, _ = conv_raw(f"{pre}.downsample", x, H, W)
                    y = x
                    for j, nm in enumerate(names):
                        last = j + 1 == len(names)
                        y, h_, w_ = conv_raw(f"{pre}.{nm}", y, h_, w_, act=ACT_RELU, res=res if last else None,
                                             res_post=1 if last else 0)
                    x = y
                H, W = h_, w_
        return x, H, W

    def _build(self, B: int, H: int, W: int, n_iters: int, all_iters: bool = True, src=None) -> _PlanState:
        assert src is None, "fp32 engine: uint8 frames are prepared by RaftEngine._host_u8"
        m = self.model
        dev = self.device
        sp = self._specs
        h, w = H // 8, W // 8
        L = self.num_levels
        min_sz = 2 * (2 ** (L - 1))
        assert h >= min_sz and w >= min_sz, (
            f"Feature maps are too small to be down-sampled by the correlation pyramid: need >= {min_sz}, got {(h, w)}; "
            f"input images should be at least {8 * min_sz}.")
        hw = h * w
        if hw % 4:
            raise NotImplementedError("fp32 engine: the feature map's pixel count h*w must be a multiple of 4")
        if self.radius > 4:
            raise NotImplementedError("fp32 engine: lookup radius <= 4")
        M = B * hw
        plan = nat.new_plan()
        st = _PlanState(plan=plan, plans=[plan], n_iters=n_iters)
        bufs = st.bufs

        def alloc(name, shape):
            t = torch.zeros(shape, dtype=F32, device=dev)
            bufs[name] = t
            return t

        st.inp1 = torch.zeros((B, H, W, 3), dtype=F32, device=dev)
        st.inp2 = torch.zeros((B, H, W, 3), dtype=F32, device=dev)
        st.out = torch.zeros((n_iters if all_iters else 1, B, H, W, 2), dtype=F32, device=dev)
        st.slot_ptr = st.out.data_ptr()
        st.out_slot = torch.tensor([st.slot_ptr], dtype=torch.int64, device=dev)
        out_stride = B * H * W * 2

        # ---------------- prologue (model.py:557-587)
        plan.set_segment(0)
        plan.set_lane(0)
        hx = alloc("hx", (M, self.hx_cs))      # [h | motion | flow]
        qx = alloc("qx", (M, self.hx_cs))      # [r*h | motion | flow]
        h32 = alloc("h32", (M, self.hidden))
        zb = alloc("z", (M, self.hidden))
        flow4 = alloc("flow4", (M, 4))
        coords = alloc("coords", (M, 2))
        flow32 = alloc("flow32", (M, 2))
        for t in (hx, qx, flow4, flow32):
            plan.add_memset([t])
        x0 = alloc("x0", (2 * B, H, W, 4))
        plan.add_prep_f32([st.inp1, st.inp2, x0], [B, H, W])
        feat, fh_, fw_ = self._encoder_f32(st, plan, "fe", m.feature_encoder, x0, 2 * B, H, W)
        assert (fh_, fw_) == (h, w), "The feature encoder should downsample H and W by 8"
        fmap = alloc("fmap", (2 * B, h, w, self.fmap_ch))
        self._conv(plan, sp["fe.conv"], feat, 2 * B, h, w, fmap)
        ctxf, _, _ = self._encoder_f32(st, plan, "ce", m.context_encoder, x0[:B], B, H, W)
        ce_out = alloc("ce_out", (M, round_up(self.hidden + self.ctx_ch, 4)))
        self._conv(plan, sp["ce.conv"], ctxf, B, h, w, ce_out, act=ACT_SPLIT_TANH_RELU, split=self.hidden,
                   h32=h32, hidden=self.hidden)
        plan.add_copy_channels_f32([ce_out, hx], [0, 0, M, self.hidden])
        gbias = []
        for gi in range(len(m.update_block.recurrent_block.kernel_size)):
            gb = alloc(f"gru{gi}.cbias", (M, self.gate_cs))
            self._conv(plan, sp[f"gru{gi}.ctx"], ce_out, B, h, w, gb, x_coff=self.hidden)
            gbias.append(gb)
        plan.add_init_coords([coords], [B, h, w])
        # correlation pyramid (model.py:418-446, 472-481): level 0 = fmap1 . fmap2^T / sqrt(C)
        # per image on the fp32 MFMA GEMM, then 2x2 floor average pooling per level; with
        # context parallelism only this rank's query rows [r0, r1)
        slabs = self._cp_slabs(h) if self.cp else [(0, h)]
        r0, r1 = slabs[self.cp_rank]
        nq = (r1 - r0) * w
        levels = []
        hl, wl = h, w
        for lv in range(L):
            levels.append(alloc(f"corr.l{lv}", (B * nq, hl, wl)))
            hl //= 2
            wl //= 2
        zero_b = alloc("corr.bias", (hw,))
        C = self.fmap_ch
        for b in range(B):
            wspec = nat.ConvSpecF32(fmap[B + b].reshape(hw, C), zero_b, 1, 1, 1, 1, 0, 0, C, C, hw)
            self._conv(plan, wspec, fmap[b, r0:r1], 1, r1 - r0, w, levels[0][b * nq:(b + 1) * nq].view(nq, hw),
                       alpha=1.0 / float(C) ** 0.5)
        hl, wl = h, w
        for lv in range(1, L):
            plan.add_corr_pool_f32([levels[lv - 1], levels[lv]], [B * nq, hl, wl])
            hl //= 2
            wl //= 2

        # ---------------- loop body (model.py:495-510)
        me = m.update_block.motion_encoder
        cl, fl = me.corr_layers, me.flow_layers
        corr = alloc("corr", (M, self.corr_cs))
        cf = alloc("cf", (M, round_up(cl[-1] + fl[-1], 4)))
        f1 = alloc("f1", (M, round_up(fl[0], 4)))
        c1 = alloc("c1", (M, round_up(cl[0], 4))) if len(cl) == 2 else None
        s1 = sp["fh1.flow"] if self.has_mask else sp["fh1"]
        fm = alloc("fm", (M, round_up(s1.cout, 4)))
        delta = alloc("delta", (M, 4))
        if self.has_mask:
            mfeat = alloc("mfeat", (M, round_up(sp["mask.convrelu"].cout, 4)))
            mask = alloc("mask", (M, round_up(sp["mask"].cout, 4)))

        def upsample(stride):
            if not self.has_mask:
                plan.add_upsample_bilinear([flow32, st.out, st.out_slot], [B, h, w, stride, 0])
                return
            self._conv(plan, sp["mask.convrelu"], hx, B, h, w, mfeat, act=ACT_RELU)
            self._conv(plan, sp["mask"], mfeat, B, h, w, mask, alpha=m.mask_predictor.multiplier)
            plan.add_upsample_convex_f32([mask, flow32, st.out, st.out_slot], [B, h, w, stride, 0])

        plan.set_segment(1)
        if self.cp:
            # this rank's lookups; the engine all-gathers them into `corr` (_gather_corr)
            # before segment 3, the rest of the iteration (replicated)
            local = alloc("corr.local", (B, max(b_ - a_ for a_, b_ in slabs) * w, self.corr_cs))
            for b in range(B):
                plan.add_lookup_f32([coords[b * hw + r0 * w:b * hw + r1 * w], local[b]]
                                    + [v[b * nq:(b + 1) * nq] for v in levels] + [None] * (4 - L),
                                    [L, 1, h, w, self.radius, nq])
            st.cp = dict(slabs=slabs, local=local, corr=corr, w=w)
            plan.set_segment(3)
        else:
            plan.add_lookup_f32([coords, corr] + levels + [None] * (4 - L), [L, B, h, w, self.radius])
        if c1 is not None:
            self._conv(plan, sp["me.convcorr1"], corr, B, h, w, c1, act=ACT_RELU)
            self._conv(plan, sp["me.convcorr2"], c1, B, h, w, cf, act=ACT_RELU)
        else:
            self._conv(plan, sp["me.convcorr1"], corr, B, h, w, cf, act=ACT_RELU)
        self._conv(plan, sp["me.convflow1"], flow4, B, h, w, f1, act=ACT_RELU)
        self._conv(plan, sp["me.convflow2"], f1, B, h, w, cf, y_coff=cl[-1], act=ACT_RELU)
        self._conv(plan, sp["me.conv"], cf, B, h, w, hx, y_coff=self.mot_off, act=ACT_RELU, y2=qx,
                   y2_coff=self.mot_off)
        for gi in range(len(m.update_block.recurrent_block.kernel_size)):
            self._conv(plan, sp[f"gru{gi}.a"], hx, B, h, w, qx, zbuf=zb, h32=h32, hidden=self.hidden,
                       epi=EPI_GRU_A, bmap=gbias[gi], bmap_coff=0)
            self._conv(plan, sp[f"gru{gi}.b"], qx, B, h, w, hx, h32=h32, zbuf=zb, hidden=self.hidden,
                       epi=EPI_GRU_B, bmap=gbias[gi], bmap_coff=2 * self.hidden)
        self._conv(plan, s1, hx, B, h, w, fm, act=ACT_RELU)
        self._conv(plan, sp["fh2"], fm, B, h, w, delta)
        plan.add_flow_update_f32([delta, coords, flow32, hx, qx, flow4], [B, h, w, self.flow_off, self.flow_off])
        if all_iters:
            upsample(out_stride)
        plan.set_segment(2)
        if not all_iters:
            upsample(0)
        return st


class RaftEngineMixed(RaftEngine):
    """``RaftEngine(..., precision="mixed")``: the feature encoder in fp32 (this module's fp32
    lowering, one plan of its own), everything else on the bf16 engine.

    raft_small's bf16 drift at 32 iterations (4.2 % relative EPE vs the fp32 golden against
    1.7 % for raft_large, profiles/r5_drift.md) comes from its feature encoder's high-resolution
    layers (profiles/r5_precision_bisect.md): 32 / 64 channels at 1/2 and 1/4 resolution, whose
    instance norms amplify the bf16 rounding of the correlation features.  Here the feature maps
    come from the fp32 encoder (fp32 convs, statistics and norms) and are rounded to bf16 once,
    as the correlation pyramid's input; the context encoder, the pyramid and the refinement loop
    are the bf16 engine's.  Per forward: the fp32 plan (prep, encoder, final 1x1 conv), one
    cast of the feature maps into the bf16 plan's buffer, then the bf16 plan without its feature
    encoder.  Cost and drift: profiles/r6_drift_mixed.md.  One-lane prologue, no
    :meth:`pipelined`, no batch split."""

    precision = "mixed"
    fe_external = True
    _native_u8 = False   # uint8 frames: normalised + padded by framework ops (the fp32 prep reads fp32)

    def __init__(self, model, device, use_graph: bool = True, copy_output: bool = True, **kw):
        kw.pop("precision", None)
        kw["split"] = 1
        super().__init__(model, device, use_graph=use_graph, copy_output=copy_output, **kw)
        self._f32 = RaftEngineF32(model, device, use_graph=use_graph, copy_output=False, precision="fp32")

    def _hold_model_weakly(self) -> None:
        super()._hold_model_weakly()
        self._f32._hold_model_weakly()

    def _build(self, B: int, H: int, W: int, n_iters: int, all_iters: bool = True, src=None) -> _PlanState:
        assert src is None, "mixed engine: uint8 frames are prepared by RaftEngine._host_u8"
        st = super()._build(B, H, W, n_iters, all_iters, src)
        f = self._f32
        if f._stale():
            f._pack()
        h, w = H // 8, W // 8
        plan = nat.new_plan()
        plan.set_segment(0)
        plan.set_lane(0)
        fst = _PlanState(plan=plan, plans=[plan], n_iters=0)
        x0 = torch.zeros((2 * B, H, W, 4), dtype=F32, device=self.device)
        fst.bufs["x0"] = x0
        plan.add_prep_f32([st.inp1, st.inp2, x0], [B, H, W])
        feat, fh_, fw_ = f._encoder_f32(fst, plan, "fe", self.model.feature_encoder, x0, 2 * B, H, W)
        assert (fh_, fw_) == (h, w), "The feature encoder should downsample H and W by 8"
        fmap32 = torch.zeros((2 * B, h, w, self.fmap_ch), dtype=F32, device=self.device)
        fst.bufs["fmap32"] = fmap32
        f._conv(plan, f._specs["fe.conv"], feat, 2 * B, h, w, fmap32)
        plan.set_segment(2)
        st.fe32 = (plan, fst, fmap32, st.bufs["p0.fmap"])
        return st

    def _pre_launch(self, st: _PlanState) -> None:
        f = self._f32
        if f._stale():
            f._pack()
        plan, _, fmap32, fmap = st.fe32
        if self.use_graph:
            if plan.captured_iters() != 0:
                plan.capture(0)
            plan.replay()
        else:
            plan.run(0)
        fmap.copy_(fmap32)   # the one bf16 rounding of the feature maps (the pyramid's input)
