"""Fused native training path of the RAFT refinement loop (forward + backward).

The unfused training path (:mod:`jax_raft_amd.ops.autograd`) runs the update
block as PyTorch autograd glue around native convolutions: every concat,
gate, activation, residual and gradient accumulation is its own framework
kernel, and each of the ``N`` iterations re-derives its weight gradients.
This module replaces the whole loop (``jax_raft/model.py:484-510`` scanned
``num_flow_updates`` times, ``model.py:589-603``) by ONE autograd node whose
forward and backward are native plans:

* **forward** -- the inference engine's fused kernels (lookup, implicit-GEMM
  convs writing straight into the persistent ``[h | motion | flow]`` GRU input
  buffers, the ConvGRU gate epilogues with the loop-invariant context share
  folded into a per-pixel bias map, the flow-head coordinate update, the mask
  conv + convex x8 upsampling), with every activation the backward needs
  written to per-iteration buffers (one ``[T, M, C]`` tensor per site);
* **backward** -- hand-written BPTT: per iteration (last to first) the
  upsampling adjoints (``train.hip``), then each conv's data gradient as the
  same implicit-GEMM kernel over flipped / transposed weights with the
  ``EPI_BWD`` epilogue, which applies the ReLU masks, accumulates the motion
  and hidden-state gradients in fp32 and performs the ConvGRU gate backward
  (``h' = (1-z) h + z q``, ``model.py:301-312``) in registers, and the
  pyramid-lookup scatter (``corr.hip``);
* **weight gradients** -- deferred to the end of the backward and computed
  ONCE per weight over all iterations stacked along K (``T * M`` rows): the
  update block's weights are shared by every iteration, so ``dW = sum_t
  X_t^T dY_t`` is one long-K GEMM instead of ``T`` small ones plus ``T - 1``
  fp32 adds.  The context share of the ConvGRU gates is linear in the
  (loop-invariant) context, so its weight and data gradients need only the
  iteration sum of the gate gradients: one conv each per step.

Both plans are recorded once per (shape, iterations) with every pointer,
shape and tile config resolved, and replayed as captured hipGraphs.  The
saved activations live in persistent buffers owned by :class:`FusedLoop`
(~3 GB for raft_large at 6 x 384 x 512, 12 iterations): a forward must be
followed by its backward before the next forward of the same loop (checked).
"""
from __future__ import annotations

import contextlib
import weakref
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ..models.layers import FeatureEncoder
from .. import knobs
from ..ops import native as nat
from ..ops.native import ACT_NONE, ACT_RELU, EPI_GRU_A, EPI_GRU_B, EPI_STD, round_up
from ..runtime import tunedb

BF16, F32 = torch.bfloat16, torch.float32
EPI_BWD = 5


@dataclass
class Seg:
    """One channel segment of an EPI_BWD conv (csrc/kernels/kernels.h:BwdSeg)."""
    mode: int = 0
    gin: Optional[torch.Tensor] = None
    gin_coff: int = 0
    mask: Optional[torch.Tensor] = None
    mask_coff: int = 0
    valid: int = 0
    out: Optional[torch.Tensor] = None
    out_coff: int = 0


def _tx(rbuf=None, qbuf=None, h32o=None, gz=None, gr=None, gq=None, ghp=None, gdq=None, gdzr=None,
        s0: Optional[Seg] = None, s1: Optional[Seg] = None):
    s0, s1 = s0 or Seg(), s1 or Seg()
    tx = [rbuf, qbuf, h32o, gz, gr, gq, ghp, gdq, gdzr, s0.gin, s0.mask, s0.out, s1.gin, s1.mask, s1.out]
    ix = [s0.mode, s0.gin_coff, s0.mask_coff, s0.valid, s0.out_coff,
          s1.mode, s1.gin_coff, s1.mask_coff, s1.valid, s1.out_coff]
    return tx, ix


def _flip_t(k: torch.Tensor) -> torch.Tensor:
    """HWIO kernel -> the kernel of its data gradient (flipped taps, in/out swapped)."""
    return torch.flip(k, dims=(0, 1)).permute(0, 1, 3, 2)


def _pad_last(k: torch.Tensor, n: int) -> torch.Tensor:
    if k.shape[-1] == n:
        return k
    out = k.new_zeros(k.shape[:-1] + (n,))
    out[..., : k.shape[-1]] = k
    return out


_CFG_CACHE: Dict[tuple, int] = {}


class GradArena:
    """One flat fp32 buffer holding the gradients of a parameter list (HWIO
    views the native weight-gradient kernels write into).  :meth:`snapshot`
    hands autograd a fresh copy in ONE kernel, so a later step's in-place
    writes never alias a gradient a caller still holds."""

    def __init__(self, params, device, model=None):
        self.params = list(params)
        # (module, attribute) -> the parameter recorded here: the backward assembles
        # gradients by module slot, so it needs no live module attribute (under
        # torch.func.functional_call the slots hold other tensors than after it)
        self.slots: Dict[tuple, int] = {}
        if model is not None:
            for mod in model.modules():
                for name, t in mod._parameters.items():
                    if t is not None:
                        self.slots[(id(mod), name)] = id(t)
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=F32, device=device)
        self.views: Dict[int, torch.Tensor] = {}
        self._off: Dict[int, int] = {}
        off = 0
        for p in self.params:
            self.views[id(p)] = self.flat[off:off + p.numel()].view(p.shape)
            self._off[id(p)] = off
            off += p.numel()

    def __getitem__(self, p) -> torch.Tensor:
        return self.views[id(p)]

    def of(self, module, name: str) -> torch.Tensor:
        """The gradient view of ``module.<name>`` as recorded at construction."""
        return self.views[self.slots[(id(module), name)]]

    def snapshot(self) -> Dict[int, torch.Tensor]:
        c = self.flat.clone()
        self.last_snapshot = c   # the flat copy the returned views alias (data-parallel reduction)
        return {id(p): c[self._off[id(p)]:self._off[id(p)] + p.numel()].view(p.shape) for p in self.params}


def record_wgrad(plan, x, n_img, H, W, x_coff, cin8, kernel_shape, stride, pad, dy, yoff, dw, db=None):
    """Native implicit-GEMM weight (+ bias) gradient of one conv (wgrad.hip)
    into the fp32 HWIO ``dw`` (+ ``db``); ``plan=None`` launches it now."""
    kh, kw, cin, cout = kernel_shape
    OH = (H + 2 * pad[0] - kh) // stride[0] + 1
    OW = (W + 2 * pad[1] - kw) // stride[1] + 1
    args = ([x, dy, dw, db], [n_img, H, W, x_coff, cin8, kh, kw, stride[0], stride[1], pad[0], pad[1], yoff, OH, OW,
                              cout, cin])
    if plan is None:
        nat.ops().wgrad(*args)
    else:
        plan.add_wgrad(*args)


class Packer:
    """Table of rectangular weight pieces repacked by ONE native launch
    (csrc/kernels/train.hip:pack_pieces_kernel) from the fp32 HWIO parameters
    into the bf16 GEMM layouts of the training plans' conv specs -- recorded as
    the first op of a forward plan, so a training step repacks every weight the
    optimizer changed without any per-parameter framework op."""

    def __init__(self):
        self.rows: List[List[int]] = []
        self.srcs: List[torch.Tensor] = []
        self.dsts: List[torch.Tensor] = []

    def _src(self, t: torch.Tensor) -> torch.Tensor:
        assert t.dtype == F32 and t.is_contiguous() and t.is_cuda, "pack source: contiguous fp32 GPU parameter"
        self.srcs.append(t)
        return t

    def piece(self, src, spec, mode: int, co, ci, so_co: int = 0, so_ci: int = 0):
        """dst output channels co = (co0, co1), input channels ci = (ci0, ci1) of
        ``spec`` from ``src`` (mode 0 forward, 1 data gradient, 2 flow-head taps; 4 / 5: the
        forward / data-gradient weights in the halo conv's stream layout, ``spec.wh``)."""
        src = self._src(src.data)
        kh, kw = spec.kh, spec.kw
        dst = spec.wh if mode >= 4 else spec.w
        self.dsts.append(dst)
        self.rows.append([src.data_ptr(), dst.data_ptr(), kh, kw, src.shape[2], src.shape[3], spec.cin8,
                          spec.w.shape[1], co[0], co[1], ci[0], ci[1], so_co, so_ci, mode, 0])

    def bias(self, src, dst: torch.Tensor, co, so: int = 0):
        src = self._src(src.data)
        assert dst.dtype == F32 and dst.is_contiguous()
        self.dsts.append(dst)
        self.rows.append([src.data_ptr(), dst.data_ptr(), 1, 1, 1, 1, 1, 1, co[0], co[1], 0, 1, so, 0, 3, 0])

    def stale(self) -> bool:
        return any(s.data_ptr() != r[0] for s, r in zip(self.srcs, self.rows))

    def record(self, plan):
        dev = self.dsts[0].device
        self.table = torch.tensor(self.rows, dtype=torch.int64).to(dev).contiguous()
        max_el = max(max(1, (r[9] - r[8]) * r[2] * r[3] * (r[11] - r[10])) for r in self.rows)
        args = ([self.table] + self.srcs + self.dsts, [len(self.rows), max_el])
        if plan is None:
            nat.ops().pack(*args)
        else:
            plan.add_pack(*args)


def record_conv(plan, spec, x, N, H, W, y, *, tx=None, ix=None, extra=None, **kw):
    """Append one conv to ``plan`` (``plan=None``: launch it now) with its tile
    config autotuned once per problem signature; returns the config.  ``extra`` = [OH, OW, log2
    dil_h, log2 dil_w] selects the input-dilation (strided data-gradient) mode.  The halo
    kernel's fused norm operands (``stats_part``: output statistics partials; ``in_stats`` /
    ``in_res`` / ``xn``: the input normalised on load, conv_halo.hip) restrict the candidates
    to halo configs.  Timing runs the same problem with the plain epilogue into a scratch
    output, so epilogues that accumulate into their buffers are never re-run."""
    x_coff = kw.get("x_coff", 0)
    fused_norm = any(kw.get(k) is not None for k in ("stats_part", "in_stats", "xn"))
    OH, OW = (extra[0], extra[1]) if extra else spec.out_hw(H, W)
    arch = tunedb.gpu_arch(x.device)
    key = ("train", N, H, W, OH, OW, spec.kh, spec.kw, spec.sh, spec.sw, spec.ph, spec.pw, spec.cin8, spec.cout,
           x.shape[-1], tuple(extra) if extra else None)
    # plain-epilogue 3x3 convs may also run on the halo kernel (conv_halo.hip); keyed apart from
    # decisions made before it was a candidate
    halo = nat.halo_cfgs_for(spec, dict(kw, y=y)) if tx is None and not extra and x_coff == 0 else ()
    cands = tuple(nat.TUNE_CFGS) + tuple(halo)
    if fused_norm:
        if not halo:
            raise ValueError("fused norm operands need a halo-kernel conv")
        cands, key = tuple(halo), key + ("halo_norm",)
    elif halo:
        key = key + ("halo",)
    cfg = _CFG_CACHE.get(key + (str(x.device),))
    if cfg is None:
        cfg = tunedb.lookup(arch, key, cands)   # persisted decision (runtime/tunedb.py)
    ops = nat.ops()
    if cfg is None:
        scratch = torch.empty(N * OH * OW, round_up(spec.cout, 8), dtype=BF16, device=x.device)
        # fused-norm convs are timed as the kernel that will run (the normalising loader / the
        # statistics epilogue have their own occupancy and ring depth): the real read-only norm
        # operands, scratch copies of what the conv writes (statistics partials, xn)
        tkw = {}
        if fused_norm:
            tkw = {k: kw[k] for k in ("in_stats", "in_relu", "in_hw", "in_res", "in_res_stats") if k in kw}
            if kw.get("stats_part") is not None:
                tkw["stats_part"] = torch.zeros_like(kw["stats_part"])
            if kw.get("xn") is not None:
                tkw["xn"] = torch.empty_like(kw["xn"])
        best = None
        for c in cands:
            t, i, a = nat.conv_args(spec, x, N, H, W, scratch, x_coff=x_coff, cfg=c, **tkw)
            if extra:
                i = i + list(extra)
            ops.conv(t, i, a)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                ops.conv(t, i, a)
            e1.record()
            e1.synchronize()
            el = e0.elapsed_time(e1)
            if best is None or el < best[0]:
                best = (el, c)
        cfg = best[1]
        tunedb.record(arch, key, cfg)
    _CFG_CACHE[key + (str(x.device),)] = cfg
    t, i, a = nat.conv_args(spec, x, N, H, W, y, cfg=cfg, **kw)
    if extra:
        if len(i) > 22:
            raise ValueError("input dilation with a bias map / iteration stride is not supported")
        i = i + list(extra)
    if tx is None:
        (plan.add_conv if plan is not None else ops.conv)(t, i, a)
    else:
        (plan.add_conv_train if plan is not None else ops.conv_train)(t, i, a, tx, ix)
    return cfg


def supported(model) -> bool:
    """Whether :class:`FusedLoop` can lower ``model``'s refinement loop."""
    ub = model.update_block
    me, rb = ub.motion_encoder, ub.recurrent_block
    if not isinstance(model.feature_encoder, FeatureEncoder) or not isinstance(model.context_encoder, FeatureEncoder):
        return False
    if any(e.block == "custom" or e.norm_kind not in (None, "batch", "instance")
           for e in (model.feature_encoder, model.context_encoder)):
        return False
    hd = rb.hidden_size
    ctx = model.context_encoder.out_channels - hd
    if hd % 16 or ctx <= 0 or me.out_channels < 3 or model.feature_encoder.out_channels % 64:
        return False
    if model.mask_predictor is not None and (model.mask_predictor.conv.cout != 576 or
                                             model.mask_predictor.convrelu.layers_0.cout % 8):
        return False
    if any(s != (1, 1) for s in (me.convflow1.layers_0.stride, me.conv.layers_0.stride)):
        return False
    return True


class FusedLoop:
    """Native forward/backward of ``num_flow_updates`` refinement iterations for
    one model at one (batch, image size); see the module docstring."""

    LANES = False       # motion-encoder backward on a side lane (slower, see __init__)
    FWD_LANES = False   # the forward's flow-feature / mask-head lane (slower, see __init__)

    def __init__(self, model, B: int, H: int, W: int, T: int, device, use_graph: bool = True):
        nat.require()
        self._model_ref = weakref.ref(model)   # weak: the plan cache (_LOOPS) must not keep the model alive
        self.B, self.H, self.W, self.T = B, H, W, T
        self.h, self.w = H // 8, W // 8
        self.M = B * self.h * self.w
        self.device = torch.device(device)
        self.use_graph = use_graph
        # side lanes of the plans (LANES / FWD_LANES class attributes, off): the motion encoder's
        # backward on a side lane measured 183 pairs/s vs 267 on one in-order stream (config 5);
        # the forward's two-edge flow-feature / mask-head lane 189-196 vs 288, although the same
        # schedule speeds up the inference engine by 4 %: in the training step the multi-lane
        # graphs' replays stall the launch queue around them
        self.lanes = 1 if self.LANES else 0
        self.fwd_lanes = 1 if self.FWD_LANES else 0
        self.gen = 0            # forward generation (a backward must match the latest forward)
        self.done_gen = -1
        self._w_pending = False  # weight-gradient plans in flight on the side stream (finish_weights joins)
        self._analyse()
        self._params()
        self._alloc()
        self._specs: Dict[str, nat.ConvSpec] = {}
        self._pack()
        self.packer = self._pieces()
        self.arena = GradArena(self.params, self.device, model=self.model)
        self._halo_tiles = [self._halo_tile(g) for g in range(self.G)] if self.gru_halo else None
        self.plan_f = self._build_fwd()
        self.plan_b = self._build_bwd()

    # ------------------------------------------------------------ structure
    def _analyse(self):
        m = self.model
        ub = m.update_block
        me, rb, fh = ub.motion_encoder, ub.recurrent_block, ub.flow_head
        self.me, self.rb, self.fh, self.mp = me, rb, fh, m.mask_predictor
        self.hd = rb.hidden_size
        self.ctx_ch = m.context_encoder.out_channels - self.hd
        self.ctx_cs = round_up(self.ctx_ch, 8)
        self.G = len(rb.kernel_size)
        self.grus = [getattr(rb, f"convgru{g + 1}") for g in range(self.G)]
        self.L = m.corr_block.num_levels
        self.radius = m.corr_block.radius
        S = 2 * self.radius + 1
        self.corr_ch = self.L * S * S
        self.corr_cs = round_up(self.corr_ch, 8)
        self.cl, self.fl = me.corr_layers, me.flow_layers
        self.mot_out = me.out_channels
        self.hx_real = self.hd + self.mot_out
        self.hx_cs = round_up(self.hx_real, 8)
        self.mot_cs = self.hx_cs - self.hd
        self.flow_off = self.hd + self.mot_out - 2
        self.cf_ch = self.cl[-1] + self.fl[-1]
        self.cf_cs = round_up(self.cf_ch, 8)
        self.fh_hidden = fh.hidden_size
        self.has_mask = self.mp is not None
        self.mask_hidden = self.mp.hidden_size if self.has_mask else 0
        self.fm_cs = round_up(self.fh_hidden + self.mask_hidden, 8)
        self.gate_cs = round_up(3 * self.hd, 8)
        self.fmap_ch = m.feature_encoder.out_channels
        # the forward's ConvGRU stages on gru_halo.hip (one launch per stage instead of EPI_GRU_A / B):
        # raft_large's 1x5 / 5x1 stages over [h | motion | flow] = 2 hd loop channels
        # (profiles/r4_train_bench.txt)
        ks = [tuple(g.convz.kernel.shape[:2]) for g in self.grus]
        self.gru_halo = (self.device.type == "cuda" and self.hd == 128 and self.hx_cs == 2 * self.hd and ks == [(1, 5), (5, 1)])

    def _params(self):
        me, fh, mp = self.me, self.fh, self.mp
        convs = [me.convcorr1.layers_0]
        if len(self.cl) == 2:
            convs.append(me.convcorr2.layers_0)
        convs += [me.convflow1.layers_0, me.convflow2.layers_0, me.conv.layers_0]
        for gru in self.grus:
            convs += [gru.convz, gru.convr, gru.convq]
        convs += [fh.conv1, fh.conv2]
        if self.has_mask:
            convs += [mp.convrelu.layers_0, mp.conv]
        self.convs = convs
        self.params: List[torch.nn.Parameter] = []
        for c in convs:
            self.params += [c.kernel, c.bias]

    def _alloc(self):
        T, G, M, hd, dev = self.T, self.G, self.M, self.hd, self.device
        h, w = self.h, self.w

        def z(*shape, dtype=BF16):
            return torch.zeros(shape, dtype=dtype, device=dev)

        self.ctx_in = z(M, self.ctx_cs)
        self.fm = z(2 * self.B, h, w, self.fmap_ch)   # feature-encoder output [img1 batch | img2 batch]
        self.fm1, self.fm2 = self.fm[: self.B], self.fm[self.B:]
        self.ctx_raw = z(self.B, h, w, self.hd + self.ctx_ch)  # context-encoder output (full-model path)
        self.gbias = [z(M, self.gate_cs, dtype=F32) for _ in range(G)]
        self.gbias_bf = [z(M, self.gate_cs) for _ in range(G)] if self.gru_halo else None
        # [g][t]: GRU g's inputs at iteration t; hx[0][t + 1] / hf[0][t + 1] = output of the last GRU
        self.hx = z(G, T + 1, M, self.hx_cs)
        self.qx = z(G, T + 1, M, self.hx_cs)
        self.hf = z(G, T + 1, M, hd, dtype=F32)
        self.zg = z(G, T, M, hd)
        self.rg = z(G, T, M, hd)
        self.qg = z(G, T, M, hd)
        self.corr = z(T, M, self.corr_cs)
        self.c1 = z(T, M, self.cl[0]) if len(self.cl) == 2 else None
        self.cf = z(T, M, self.cf_cs)
        self.f1 = z(T, M, self.fl[0])
        self.flow8 = z(T + 1, M, 8)
        self.coords = z(T + 1, M, 2, dtype=F32)
        nat.ops().init_coords([self.coords[0]], [self.B, h, w])
        self.flow32 = z(T, M, 2, dtype=F32)
        self.fmm = z(T, M, self.fm_cs)
        self.taps = z(M, 24, dtype=F32)
        self.mask = z(T, M, 576) if self.has_mask else None
        self.out = z(T, self.B, self.H, self.W, 2, dtype=F32)
        # forward pyramid: bf16 levels, 0 / 1 in the blocked layout when the maps are /16
        # wide (as in the inference engine: whole-line pyramid writes, 2 x 2 blocks per
        # lookup window); the lookup output feeding the convs is bf16 anyway.  Its
        # gradients accumulate in fp32 row-major maps (lookup backward, pyramid backward).
        self.blocked = int(w % 16 == 0 and (h * w) % 8 == 0)
        levels, lv_grads = [], []
        hl, wl = h, w
        for l in range(self.L):
            shape = (M, -(-h // 8) * (8 >> l), -(-w // 16) * (16 >> l)) if self.blocked and l < 2 else (M, hl, wl)
            levels.append(z(*shape))
            lv_grads.append(z(M, hl, wl, dtype=F32))
            hl //= 2
            wl //= 2
        self.levels = levels
        self.lv_grads = lv_grads
        # backward
        self.gout = z(T, self.B, self.H, self.W, 2, dtype=F32)
        self.dmask = z(T, M, 576) if self.has_mask else None
        self.utaps = z(T * M, 18, dtype=F32)
        self.ddelta = z(T, M, 8)
        self.dfmm = z(T, M, self.fm_cs)
        self.dq = z(G, T, M, hd)
        self.dzr = z(G, T, M, 2 * hd)
        self.dh = [z(M, hd, dtype=F32) for _ in range(G)]
        self.dh_next = z(M, hd, dtype=F32)
        self.dmot = z(M, self.mot_cs, dtype=F32)
        self.dm = z(T, M, self.mot_cs)
        self.dcf = z(T, M, self.cf_cs)
        self.dc1 = z(T, M, self.cl[0]) if len(self.cl) == 2 else None
        self.dcorr = z(T, M, self.corr_cs)
        self.df1 = z(T, M, self.fl[0])
        self.dctx = z(M, self.ctx_cs, dtype=F32)

    # --------------------------------------------------------------- weights
    def _sources(self):
        """name -> () -> (HWIO fp32 kernel, fp32 bias, padding, cin8).  Forward
        specs mirror runtime/engine.py; names ending in T are data-gradient specs
        (flipped, in/out-swapped kernels, padding k-1-p, zero bias, output
        channels padded to the buffer they are written into)."""
        me, fh, mp, hd, C = self.me, self.fh, self.mp, self.hd, self.ctx_ch
        # the sources are kept (self._src): they must not capture self, or every FusedLoop would be
        # a reference cycle that only a full garbage collection frees (with its device buffers)
        dev, hx_cs, ctx_cs = self.device, self.hx_cs, self.ctx_cs
        src = {}

        def kb(c):
            return c.kernel.detach().float(), c.bias.detach().float()

        def fwd(c, cin8=None):
            return lambda: (*kb(c), c.padding, cin8)

        def bwd(k_fn, pad, cin8, cout_pad):
            def f():
                k = k_fn()
                kh, kw = k.shape[:2]
                kt = _pad_last(_flip_t(k), cout_pad)
                return kt, torch.zeros(cout_pad, device=k.device), (kh - 1 - pad[0], kw - 1 - pad[1]), cin8
            return f

        c1, cf1, cf2, mc = me.convcorr1.layers_0, me.convflow1.layers_0, me.convflow2.layers_0, me.conv.layers_0
        src["cc1"] = fwd(c1, self.corr_cs)
        src["cc1T"] = bwd(lambda: c1.kernel.detach().float(), c1.padding, round_up(c1.cout, 8), self.corr_cs)
        if len(self.cl) == 2:
            c2 = me.convcorr2.layers_0
            src["cc2"] = fwd(c2)
            src["cc2T"] = bwd(lambda: c2.kernel.detach().float(), c2.padding, round_up(c2.cout, 8), round_up(c2.cin, 8))
        src["cf1"] = fwd(cf1, 8)
        src["cf2"] = fwd(cf2)
        src["cf2T"] = bwd(lambda: cf2.kernel.detach().float(), cf2.padding, round_up(cf2.cout, 8), round_up(cf2.cin, 8))
        src["mc"] = fwd(mc)
        src["mcT"] = bwd(lambda: mc.kernel.detach().float(), mc.padding, round_up(mc.cout, 8), self.cf_cs)

        def loop_part(k):  # input channels [h | context | motion] -> [h | motion] (hx layout, padded)
            k = k.detach().float()
            kk = torch.cat([k[:, :, :hd], k[:, :, hd + C:]], dim=2)
            out = k.new_zeros(k.shape[:2] + (hx_cs, k.shape[3]))
            out[:, :, : kk.shape[2]] = kk
            return out

        for g, gru in enumerate(self.grus):
            pad = gru.padding

            def ga(gru=gru):
                return torch.cat([loop_part(gru.convz.kernel), loop_part(gru.convr.kernel)], dim=3)

            def gb(gru=gru):
                return loop_part(gru.convq.kernel)

            def gc(gru=gru):
                return torch.cat([c.kernel.detach()[:, :, hd:hd + C] for c in (gru.convz, gru.convr, gru.convq)],
                                 dim=3).float()

            def gcb(gru=gru):
                return torch.cat([c.bias.detach() for c in (gru.convz, gru.convr, gru.convq)]).float()

            src[f"gA{g}"] = (lambda ga=ga, pad=pad: (ga(), torch.zeros(2 * hd, device=dev), pad, hx_cs))
            src[f"gB{g}"] = (lambda gb=gb, pad=pad: (gb(), torch.zeros(hd, device=dev), pad, hx_cs))
            src[f"gC{g}"] = (lambda gc=gc, gcb=gcb, pad=pad: (gc(), gcb(), pad, ctx_cs))
            src[f"gAT{g}"] = bwd(ga, pad, 2 * hd, self.hx_cs)
            src[f"gBT{g}"] = bwd(gb, pad, hd, self.hx_cs)
            src[f"gCT{g}"] = bwd(gc, pad, 3 * hd, self.ctx_cs)
        if self.has_mask:
            mr = mp.convrelu.layers_0

            def fh1():
                return torch.cat([fh.conv1.kernel.detach(), mr.kernel.detach()], dim=3).float()

            src["fh1"] = lambda: (fh1(), torch.cat([fh.conv1.bias.detach(), mr.bias.detach()]).float(), (1, 1), None)
            src["fh1T"] = bwd(fh1, (1, 1), self.fm_cs, hd)
            src["mask"] = fwd(mp.conv)
            src["maskT"] = bwd(lambda: mp.conv.kernel.detach().float(), (0, 0), 576, self.mask_hidden)
        else:
            src["fh1"] = fwd(fh.conv1)
            src["fh1T"] = bwd(lambda: fh.conv1.kernel.detach().float(), (1, 1), self.fm_cs, hd)

        def taps():  # (3,3,cin,2) -> (1,1,cin,18): out channel tap*2 + o
            k = fh.conv2.kernel.detach().float()
            cin = k.shape[2]
            return k.reshape(9, cin, 2).permute(1, 0, 2).reshape(1, 1, cin, 18)

        src["fh2t"] = lambda: (taps(), torch.zeros(18, device=dev), (0, 0), None)
        src["fh2T"] = bwd(lambda: fh.conv2.kernel.detach().float(), (1, 1), 8, self.fh_hidden)
        return src

    def _pack(self):
        """(Re)pack every spec in place (pointers stay valid for the recorded plans)."""
        if not hasattr(self, "_src"):
            self._src = self._sources()
        for name, fn in self._src.items():
            k, b, pad, cin8 = fn()
            k = k.to(self.device)
            sp = self._specs.get(name)
            if sp is None:
                sp = self._specs[name] = nat.make_spec(k, b.to(self.device), (1, 1), tuple(pad), cin8=cin8,
                                                       device=self.device)
                if self.gru_halo and name[:2] in ("gA", "gB") and name[2:].isdigit():
                    sp.wh = nat.pack_gru_halo(k, sp.cin8)   # gru_halo.hip weight stream (repacked by the plan)
            else:
                nat.pack_weight(k, sp.cin8, out=sp.w)
                sp.b.copy_(b)
                if sp.wh is not None:   # the halo kernels' weight streams (gru_halo / conv_halo)
                    if name[:2] in ("gA", "gB") and name[2:].isdigit():
                        nat.pack_gru_halo(k, sp.cin8, out=sp.wh)
                    else:
                        nat.pack_halo_conv(k, sp.cin8, out=sp.wh)
        fb = self.fh.conv2.bias.detach().float().to(self.device)
        if not hasattr(self, "_fh2_bias"):
            self._fh2_bias = fb.contiguous()
        else:
            self._fh2_bias.copy_(fb)

    def _pieces(self) -> "Packer":
        """The pack table of every spec (mirrors :meth:`_sources`)."""
        pk, sp, hd, C = Packer(), self._specs, self.hd, self.ctx_ch
        me, fh, mp = self.me, self.fh, self.mp

        def modes(name):
            # 4: the halo-kernel weight stream too -- record_conv may run a plain-epilogue 3x3 conv on
            # conv_halo.hip, which reads spec.wh (left out before round 5: those convs ran on the
            # weights of the plan's first step after every optimizer update)
            return (0, 4) if sp[name].wh is not None else (0,)

        def fwd(name, c, co=None, ci=None):
            kh, kw, cin, cout = c.kernel.shape
            for mode in modes(name):
                pk.piece(c.kernel, sp[name], mode, co or (0, cout), ci or (0, cin))
            pk.bias(c.bias, sp[name].b, (0, cout))

        def bwd(name, c):
            kh, kw, cin, cout = c.kernel.shape
            pk.piece(c.kernel, sp[name + "T"], 1, (0, cin), (0, cout))

        c1 = me.convcorr1.layers_0
        fwd("cc1", c1)
        bwd("cc1", c1)
        if len(self.cl) == 2:
            fwd("cc2", me.convcorr2.layers_0)
            bwd("cc2", me.convcorr2.layers_0)
        fwd("cf1", me.convflow1.layers_0)
        fwd("cf2", me.convflow2.layers_0)
        bwd("cf2", me.convflow2.layers_0)
        fwd("mc", me.conv.layers_0)
        bwd("mc", me.conv.layers_0)
        mot = self.mot_out
        for g, gru in enumerate(self.grus):
            for j, c in enumerate((gru.convz, gru.convr)):   # loop part [h | motion] of the z / r gates
                co = (j * hd, (j + 1) * hd)
                for mode in ((0, 4) if sp[f"gA{g}"].wh is not None else (0,)):   # 4: the gru_halo stream
                    pk.piece(c.kernel, sp[f"gA{g}"], mode, co, (0, hd))
                    pk.piece(c.kernel, sp[f"gA{g}"], mode, co, (hd, hd + mot), so_ci=hd + C)
                pk.piece(c.kernel, sp[f"gAT{g}"], 1, (0, hd), co)
                pk.piece(c.kernel, sp[f"gAT{g}"], 1, (hd, hd + mot), co, so_co=hd + C)
            q = gru.convq
            for mode in ((0, 4) if sp[f"gB{g}"].wh is not None else (0,)):
                pk.piece(q.kernel, sp[f"gB{g}"], mode, (0, hd), (0, hd))
                pk.piece(q.kernel, sp[f"gB{g}"], mode, (0, hd), (hd, hd + mot), so_ci=hd + C)
            pk.piece(q.kernel, sp[f"gBT{g}"], 1, (0, hd), (0, hd))
            pk.piece(q.kernel, sp[f"gBT{g}"], 1, (hd, hd + mot), (0, hd), so_co=hd + C)
            for j, c in enumerate((gru.convz, gru.convr, gru.convq)):   # context share + gate biases
                co = (j * hd, (j + 1) * hd)
                pk.piece(c.kernel, sp[f"gC{g}"], 0, co, (0, C), so_ci=hd)
                pk.bias(c.bias, sp[f"gC{g}"].b, co)
                pk.piece(c.kernel, sp[f"gCT{g}"], 1, (0, C), co, so_co=hd)
        if self.has_mask:
            mr = mp.convrelu.layers_0
            fh_, mh = self.fh_hidden, self.mask_hidden
            for mode in modes("fh1"):
                pk.piece(fh.conv1.kernel, sp["fh1"], mode, (0, fh_), (0, hd))
                pk.piece(mr.kernel, sp["fh1"], mode, (fh_, fh_ + mh), (0, hd))
            pk.bias(fh.conv1.bias, sp["fh1"].b, (0, fh_))
            pk.bias(mr.bias, sp["fh1"].b, (fh_, fh_ + mh))
            pk.piece(fh.conv1.kernel, sp["fh1T"], 1, (0, hd), (0, fh_))
            pk.piece(mr.kernel, sp["fh1T"], 1, (0, hd), (fh_, fh_ + mh))
            fwd("mask", mp.conv)
            pk.piece(mp.conv.kernel, sp["maskT"], 1, (0, mh), (0, 576))
        else:
            fwd("fh1", fh.conv1)
            pk.piece(fh.conv1.kernel, sp["fh1T"], 1, (0, hd), (0, self.fh_hidden))
        pk.piece(fh.conv2.kernel, sp["fh2t"], 2, (0, 18), (0, self.fh_hidden))
        pk.piece(fh.conv2.kernel, sp["fh2T"], 1, (0, self.fh_hidden), (0, 2))
        pk.bias(fh.conv2.bias, self._fh2_bias, (0, 2))
        return pk

    @property
    def model(self):
        m = self._model_ref()
        if m is None:
            raise ReferenceError("FusedLoop: its model has been garbage-collected")
        return m

    def stale(self) -> bool:
        return self.packer.stale()

    def _halo_tile(self, g: int):
        """(mode, axis, tile) of GRU stage g on gru_halo: the fastest of the candidate tilings
        (ops/native.py:gru_halo_candidates), timed once on this loop's own buffers (the first
        forward overwrites everything the trial launches write)."""
        axis = 0 if tuple(self.grus[g].convz.kernel.shape[:2]) == (1, 5) else 1
        cands = nat.gru_halo_candidates(self.hd, 0, axis, self.B, self.h, self.w)
        if len(cands) == 1:
            return 0, axis, cands[0]
        t = [self.hx[g, 0], self.hx[g, 0], self._specs[f"gA{g}"].wh, self._specs[f"gB{g}"].wh, self.gbias_bf[g],
             self.hf[g, 1] if g + 1 < self.G else self.hf[0, 1], self.hx[g + 1, 0] if g + 1 < self.G else self.hx[0, 1],
             None, None, None, None, self.hf[g, 0], self.zg[g, 0], self.rg[g, 0], self.qg[g, 0], self.qx[g, 0]]
        base = [self.B, self.h, self.w, 0, axis]
        best = None
        for tile in cands:
            nat.ops().gru_halo(t, base + list(tile))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                nat.ops().gru_halo(t, base + list(tile))
            e1.record()
            e1.synchronize()
            el = e0.elapsed_time(e1)
            if best is None or el < best[0]:
                best = (el, tile)
        return 0, axis, best[1]

    # ----------------------------------------------------------- recording
    def _conv(self, plan, name, x, y, *, x_coff=0, tx=None, ix=None, N=None, **kw):
        record_conv(plan, self._specs[name], x, N or self.B, self.h, self.w, y, x_coff=x_coff, tx=tx, ix=ix, **kw)

    def _bconv(self, plan, name, x, *, x_coff=0, split=0, s0=None, s1=None, N=None, **gru):
        """Data-gradient conv with the EPI_BWD epilogue (N images, default the batch)."""
        tx, ix = _tx(s0=s0, s1=s1, **gru)
        y = (s1.out if s1 is not None and s1.out is not None else s0.out)
        self._conv(plan, name, x, y, x_coff=x_coff, tx=tx, ix=ix, epi=EPI_BWD, hidden=split, N=N)

    def _build_fwd(self):
        P = nat.new_plan()
        P.set_segment(0)
        P.set_lane(0)
        T, G, hd, B, h, w = self.T, self.G, self.hd, self.B, self.h, self.w
        cl, fl = self.cl, self.fl
        # lanes (fwd_lanes): 0 = critical path (lookup -> correlation convs -> motion conv ->
        # GRUs -> flow head -> coordinate update); 1 = after iteration t's coordinate update,
        # the flow-feature convs of iteration t+1 (they need only that update), then iteration
        # t's mask head + x8 upsampling (read only per-iteration buffers; joined at the end).
        # Two cross-lane edges per iteration: E_FH (update -> lane 1), E_FLOW (flow features
        # -> motion conv), as in the inference engine's mask-lane schedule.
        E_PACK, E_FLOW, E_FH = 0, 2, 3
        fl = self.fwd_lanes
        self.packer.record(P)   # this step's weights -> every spec (forward and data-gradient layouts)
        P.add_corr([self.fm1, self.fm2] + self.levels + [None] * (4 - self.L),
                   [B, h, w, self.fmap_ch, self.L, h * w, self.blocked],
                   1.0 / float(self.fmap_ch) ** 0.5)
        P.add_record(E_PACK)
        for g in range(G):  # loop-invariant context share of every gate (+ biases), fp32 (+ bf16 for gru_halo)
            self._conv(P, f"gC{g}", self.ctx_in, self.gbias[g], y2=self.gbias_bf[g] if self.gru_halo else None)

        def flow_features(t):
            self._conv(P, "cf1", self.flow8[t], self.f1[t], act=ACT_RELU)
            self._conv(P, "cf2", self.f1[t], self.cf[t], y_coff=cl[-1], act=ACT_RELU)

        def mask_head(t):
            if self.has_mask:
                self._conv(P, "mask", self.fmm[t], self.mask[t], x_coff=self.fh_hidden,
                           alpha=self.mp.multiplier)
                P.add_upsample_convex([self.mask[t], self.flow32[t], self.out[t]], [B, h, w, 0])
            else:
                P.add_upsample_bilinear([self.flow32[t], self.out[t]], [B, h, w, 0])

        if fl:
            P.set_lane(1)
            P.add_wait(E_PACK)
            flow_features(0)
            P.add_record(E_FLOW)
            P.set_lane(0)
        for t in range(T):
            hx0, qx0 = self.hx[0, t], self.qx[0, t]
            if not fl:
                flow_features(t)
            P.add_lookup([self.coords[t], self.corr[t]] + self.levels + [None] * (4 - self.L),
                         [self.L, B, h, w, self.radius, h * w, self.blocked])
            if len(cl) == 2:
                self._conv(P, "cc1", self.corr[t], self.c1[t], act=ACT_RELU)
                self._conv(P, "cc2", self.c1[t], self.cf[t], act=ACT_RELU)
            else:
                self._conv(P, "cc1", self.corr[t], self.cf[t], act=ACT_RELU)
            if fl:
                P.add_wait(E_FLOW)
            self._conv(P, "mc", self.cf[t], hx0, y_coff=hd, act=ACT_RELU, y2=qx0, y2_coff=hd)
            for g in range(1, G):  # [motion | flow] into the other GRUs' inputs
                P.add_copy_channels([hx0, self.hx[g, t]], [hd, hd, self.M, self.mot_cs])
                P.add_copy_channels([hx0, self.qx[g, t]], [hd, hd, self.M, self.mot_cs])
            for g in range(G):
                last = g + 1 == G
                nh = self.hx[0, t + 1] if last else self.hx[g + 1, t]
                nhf = self.hf[0, t + 1] if last else self.hf[g + 1, t]
                if self.gru_halo:
                    # one gru_halo launch per stage (csrc/kernels/gru_halo.hip), saving z, r, q and r*h
                    # for the backward; h read from hf[g, t], h' written to the next state buffers
                    mode, axis, tile = self._halo_tiles[g]
                    P.add_gru_halo([self.hx[g, t], self.hx[g, t], self._specs[f"gA{g}"].wh, self._specs[f"gB{g}"].wh,
                                    self.gbias_bf[g], nhf, nh, None, None, None, None, self.hf[g, t], self.zg[g, t],
                                    self.rg[g, t], self.qg[g, t], self.qx[g, t]],
                                   [B, h, w, mode, axis] + list(tile))
                    continue
                tx, ix = _tx(rbuf=self.rg[g, t])
                self._conv(P, f"gA{g}", self.hx[g, t], self.qx[g, t], zbuf=self.zg[g, t], h32=self.hf[g, t],
                           hidden=hd, epi=EPI_GRU_A, bmap=self.gbias[g], bmap_coff=0, tx=tx, ix=ix)
                tx, ix = _tx(qbuf=self.qg[g, t], h32o=nhf)
                self._conv(P, f"gB{g}", self.qx[g, t], nh, zbuf=self.zg[g, t], h32=self.hf[g, t], hidden=hd,
                           epi=EPI_GRU_B, bmap=self.gbias[g], bmap_coff=2 * hd, tx=tx, ix=ix)
            hn = self.hx[0, t + 1]
            self._conv(P, "fh1", hn, self.fmm[t], act=ACT_RELU)
            self._conv(P, "fh2t", self.fmm[t], self.taps)
            P.add_copy([self.coords[t], self.coords[t + 1]])
            P.add_flow_taps([self.taps, self._fh2_bias, self.coords[t + 1], self.flow32[t], hn, self.qx[0, t + 1],
                             self.flow8[t + 1]], [B, h, w, self.flow_off, self.flow_off])
            if fl:
                P.add_record(E_FH)
                P.set_lane(1)
                P.add_wait(E_FH)
                if t + 1 < T:
                    flow_features(t + 1)
                    P.add_record(E_FLOW)
                mask_head(t)
                P.set_lane(0)
        if not fl:
            # the output heads of every iteration (nothing in the recurrence reads them) as
            # T-stacked launches after the loop (M = T * B * h * w)
            TB = T * B
            if self.has_mask:
                self._conv(P, "mask", self.fmm, self.mask, x_coff=self.fh_hidden, alpha=self.mp.multiplier, N=TB)
                P.add_upsample_convex([self.mask, self.flow32, self.out.view(TB, self.H, self.W, 2)], [TB, h, w, 0])
            else:
                P.add_upsample_bilinear([self.flow32, self.out.view(TB, self.H, self.W, 2)], [TB, h, w, 0])
        return P

    def _build_bwd(self):
        P = nat.new_plan()
        P.set_segment(0)
        P.set_lane(0)
        T, G, hd, B, h, w = self.T, self.G, self.hd, self.B, self.h, self.w
        cl = self.cl
        E_DM, E_ME = 0, 1
        for g_ in self.lv_grads:
            P.add_memset([g_])
        # The output heads' backward of every iteration at once (T * B images): the x8
        # upsampling, the mask conv and FlowHead conv2 data gradients depend only on that
        # iteration's loss gradient and forward activations -- the coordinates are
        # detached between iterations (model.py:498), so no gradient reaches delta_t
        # through later iterations -- not on the recurrence, so they leave the serial
        # per-iteration chain and run as T-stacked launches (M = T * B * h * w).
        TB = T * B
        if self.has_mask:
            P.add_upsample_convex_bwd([self.mask, self.flow32, self.gout, self.dmask, self.utaps],
                                      [TB, h, w], self.mp.multiplier)
            P.add_flow_gather_bwd([self.utaps, self.ddelta], [TB, h, w])
            self._bconv(P, "maskT", self.dmask, N=TB,
                        s1=Seg(mask=self.fmm, mask_coff=self.fh_hidden, out=self.dfmm, out_coff=self.fh_hidden))
        else:
            P.add_upsample_bilinear_bwd([self.gout, self.ddelta], [TB, h, w])
        self._bconv(P, "fh2T", self.ddelta, N=TB, s1=Seg(mask=self.fmm, out=self.dfmm))
        # the heads' weight gradients need only what ran so far: their own plan, replayed on the
        # weight-gradient stream while the (latency-bound) BPTT chain runs (see backward)
        self.plan_b1 = P
        self.plan_w1 = nat.new_plan()
        self.plan_w1.set_segment(0)
        self.plan_w1.set_lane(0)
        self._record_head_wgrads(self.plan_w1)
        P = nat.new_plan()
        P.set_segment(0)
        P.set_lane(0)
        for t in reversed(range(T)):
            # flow head (+ mask) conv1 data gradient -> blend backward of the last GRU
            gl = G - 1
            self._bconv(P, "fh1T", self.dfmm[t], split=hd,
                        s0=Seg(mode=1, gin=self.dh_next if t + 1 < T else None, out=self.dh[gl]),
                        gz=self.zg[gl, t], gq=self.qg[gl, t], ghp=self.hf[gl, t], gdq=self.dq[gl, t],
                        gdzr=self.dzr[gl, t])
            for g in reversed(range(G)):
                self._bconv(P, f"gBT{g}", self.dq[g, t], split=hd, s0=Seg(mode=2, out=self.dh[g]),
                            s1=Seg(gin=None if g == gl else self.dmot, out=self.dmot),
                            gr=self.rg[g, t], ghp=self.hf[g, t], gdzr=self.dzr[g, t])
                if g > 0:
                    self._bconv(P, f"gAT{g}", self.dzr[g, t], split=hd,
                                s0=Seg(mode=1, gin=self.dh[g], out=self.dh[g - 1]),
                                s1=Seg(gin=self.dmot, out=self.dmot),
                                gz=self.zg[g - 1, t], gq=self.qg[g - 1, t], ghp=self.hf[g - 1, t],
                                gdq=self.dq[g - 1, t], gdzr=self.dzr[g - 1, t])
                else:
                    self._bconv(P, "gAT0", self.dzr[0, t], split=hd, s0=Seg(gin=self.dh[0], out=self.dh_next),
                                s1=Seg(gin=self.dmot, mask=self.hx[0, t], mask_coff=hd, valid=self.mot_out - 2,
                                       out=self.dm[t]))
        # The motion encoder's backward (-> pyramid lookup scatter) only feeds the weight
        # and pyramid gradients, never the recurrence: after the BPTT chain, as T-stacked
        # launches (M = T * B * h * w), the lookup scatter per iteration (its level maps
        # are per query pixel of one iteration).
        TB = T * B
        P.add_record(E_DM)
        P.set_lane(self.lanes)
        P.add_wait(E_DM)
        self._bconv(P, "mcT", self.dm, N=TB, s1=Seg(mask=self.cf, out=self.dcf))
        if len(cl) == 2:
            self._bconv(P, "cc2T", self.dcf, N=TB, s1=Seg(mask=self.c1, out=self.dc1))
            self._bconv(P, "cc1T", self.dc1, N=TB, s1=Seg(out=self.dcorr, valid=self.corr_ch))
        else:
            self._bconv(P, "cc1T", self.dcf, N=TB, s1=Seg(out=self.dcorr, valid=self.corr_ch))
        self._bconv(P, "cf2T", self.dcf, N=TB, x_coff=cl[-1], s1=Seg(mask=self.f1, out=self.df1))
        for t in reversed(range(T)):   # the BPTT chain's accumulation order
            P.add_lookup_bwd([self.coords[t], self.dcorr[t]] + self.lv_grads + [None] * (4 - self.L),
                             [self.L, B, h, w, self.radius])
        P.add_record(E_ME)
        P.set_lane(0)
        P.add_wait(E_ME)
        # the stacked weight gradients: their own plan, replayed on a side stream so that they
        # overlap the pyramid and encoder backward (independent of them; joined by _finish_weights)
        self.plan_w = nat.new_plan()
        self.plan_w.set_segment(0)
        self.plan_w.set_lane(0)
        self._record_wgrads(self.plan_w)
        return P

    def _record_wgrads(self, P):
        """Weight gradients of the loop's convs over all iterations stacked
        (n_img = T * B images): one implicit-GEMM launch per weight."""
        T, G, hd, B, h, w = self.T, self.G, self.hd, self.B, self.h, self.w
        nT = T * B
        me, fh, mp, A = self.me, self.fh, self.mp, self.arena
        dev = self.device

        def wb(conv, x, x_coff, cin8, dy, yoff=0):
            record_wgrad(P, x, nT, h, w, x_coff, cin8, tuple(conv.kernel.shape), (1, 1), conv.padding, dy, yoff,
                         A.of(conv, "kernel"), A.of(conv, "bias"))

        c1 = me.convcorr1.layers_0
        if len(self.cl) == 2:
            wb(c1, self.corr, 0, self.corr_cs, self.dc1)
            wb(me.convcorr2.layers_0, self.c1, 0, self.cl[0], self.dcf)
        else:
            wb(c1, self.corr, 0, self.corr_cs, self.dcf)
        wb(me.convflow1.layers_0, self.flow8, 0, 8, self.df1)
        wb(me.convflow2.layers_0, self.f1, 0, self.fl[0], self.dcf, yoff=self.cl[-1])
        wb(me.conv.layers_0, self.cf, 0, self.cf_cs, self.dm)
        self.gAw, self.gBw = [], []
        for g, gru in enumerate(self.grus):
            kh, kw = gru.convz.kernel.shape[:2]
            ga = torch.zeros(kh, kw, self.hx_cs, 2 * hd, device=dev)
            gb = torch.zeros(kh, kw, self.hx_cs, hd, device=dev)
            record_wgrad(P, self.hx[g], nT, h, w, 0, self.hx_cs, tuple(ga.shape), (1, 1), gru.padding, self.dzr[g], 0, ga)
            record_wgrad(P, self.qx[g], nT, h, w, 0, self.hx_cs, tuple(gb.shape), (1, 1), gru.padding, self.dq[g], 0, gb)
            self.gAw.append(ga)
            self.gBw.append(gb)

    def _record_head_wgrads(self, P):
        """Weight gradients of the output heads (FlowHead conv1 + the mask head's 3x3 conv,
        FlowHead conv2, the mask 1x1 conv): inputs from the forward, output gradients from
        the heads' backward -- nothing from the BPTT chain."""
        T, hd, B, h, w = self.T, self.hd, self.B, self.h, self.w
        nT = T * B
        mp, A = self.mp, self.arena
        dev = self.device
        fm_out = self.fh_hidden + self.mask_hidden
        self.fh1w = torch.zeros(3, 3, hd, fm_out, device=dev)
        self.fh1b = torch.zeros(fm_out, device=dev)
        record_wgrad(P, self.hx[0, 1:], nT, h, w, 0, hd, tuple(self.fh1w.shape), (1, 1), (1, 1), self.dfmm, 0,
                     self.fh1w, self.fh1b)
        # flow-head output conv (256 -> 2): computed as the weight gradient of the 3x3 conv
        # ddelta -> fm with the taps flipped (K = 9 x 8 instead of 9 x 256)
        self.fh2w = torch.zeros(3, 3, 2, self.fh_hidden, device=dev)
        record_wgrad(P, self.ddelta, nT, h, w, 0, 8, tuple(self.fh2w.shape), (1, 1), (1, 1), self.fmm, 0, self.fh2w)
        if self.has_mask:
            record_wgrad(P, self.fmm, nT, h, w, self.fh_hidden, self.mask_hidden, tuple(mp.conv.kernel.shape), (1, 1),
                         mp.conv.padding, self.dmask, 0, A.of(mp.conv, "kernel"), A.of(mp.conv, "bias"))

    def _run(self, plan):
        _run_plan(plan, self.use_graph)

    # --------------------------------------------------------------- steps
    def forward(self, fmap1: torch.Tensor, fmap2: torch.Tensor, ctx_raw: torch.Tensor) -> torch.Tensor:
        """fmap1 / fmap2: feature-encoder outputs (B, h, w, C); ctx_raw:
        context-encoder output (B, h, w, hidden + ctx).  Returns the
        (T, B, H, W, 2) upsampled flows of every iteration."""
        self.fm1.copy_(fmap1.detach())
        self.fm2.copy_(fmap2.detach())
        return self.forward_prepared(ctx_raw)

    def forward_prepared(self, ctx_raw: torch.Tensor) -> torch.Tensor:
        """As :meth:`forward` with the feature maps already in :attr:`fm`."""
        hd = self.hd
        c = ctx_raw.detach().reshape(self.M, -1).float()
        h0 = torch.tanh(c[:, :hd])
        self.hf[0, 0].copy_(h0)
        self.hx[0, 0, :, :hd].copy_(h0)
        self.ctx_in[:, : self.ctx_ch].copy_(torch.relu(c[:, hd:]))
        self._run(self.plan_f)
        self.gen += 1
        return self.out.clone()

    def backward(self, gout: torch.Tensor, gen: int, fe_dy=None, defer_weights: bool = False, on_dctx=None):
        """The loop's backward: (dfmap1, dfmap2, d context-encoder output, parameter
        gradients); ``defer_weights``: the parameter gradients are None here and come from
        :meth:`finish_weights` (their kernels overlap whatever the caller enqueues meanwhile);
        ``on_dctx(dc)``: called with the context-encoder output gradient as soon as it is
        enqueued, before the pyramid backward (the caller's context-encoder backward can then
        overlap it)."""
        if gen != self.gen or self.done_gen == gen:
            raise RuntimeError("fused refinement loop: this backward's saved activations were overwritten by a "
                               "later forward of the same loop (run backward before the next forward) or it "
                               "already ran (retain_graph is not supported by the fused loop)")
        self.done_gen = gen
        self.gout.copy_(gout)
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_wstream", None) is None:
            self._wstream = torch.cuda.Stream(device=self.device)
        ws = self._wstream
        # the heads' backward, then their weight gradients on the side stream next to the BPTT chain
        self._run(self.plan_b1)
        ws.wait_stream(cur)
        with torch.cuda.stream(ws):
            self._run(self.plan_w1)
        self._run(self.plan_b)
        ws.wait_stream(cur)
        with torch.cuda.stream(ws):   # the stacked weight gradients: they overlap the caller's encoder backward
            self._run(self.plan_w)
        self._w_pending = True
        data = self._finish_data(fe_dy, on_dctx)
        # the gate / flow-head kernel assembly (~30 small copies) on the weight-gradient stream too,
        # after the context-share weight gradients of _finish_data: off the critical path
        with torch.cuda.stream(ws):
            ws.wait_event(self._ev_gc)
            self._assemble()
        if defer_weights:
            return data + (None,)
        return data + (self.finish_weights(),)

    def finish_weights(self):
        """Join the weight-gradient stream (stacked weight gradients + the kernel assembly):
        the loop parameters' gradients (after :meth:`backward`)."""
        if self._w_pending:
            torch.cuda.current_stream(self.device).wait_stream(self._wstream)
            self._w_pending = False
        grads = self.arena.snapshot()
        self.last_snapshot = self.arena.last_snapshot
        return [grads[id(p)] for p in self.params]

    def _assemble(self):
        """The gate kernels ([h | context | motion] from the loop-part and context-share
        weight gradients) and the flow-head / mask kernels into the gradient arena."""
        A = self.arena
        hd, C, fh, mp = self.hd, self.ctx_ch, self.fh, self.mp
        mot = self.mot_out
        for g, gru in enumerate(self.grus):
            gC, db = self._gC[g]
            for j, conv in enumerate((gru.convz, gru.convr, gru.convq)):
                full = A.of(conv, "kernel")
                src = self.gAw[g][..., j * hd:(j + 1) * hd] if j < 2 else self.gBw[g]
                full[:, :, :hd] = src[:, :, :hd]
                full[:, :, hd + C:] = src[:, :, hd: hd + mot]
                full[:, :, hd:hd + C] = gC[..., j * hd:(j + 1) * hd]
                A.of(conv, "bias").copy_(db[j * hd:(j + 1) * hd])
        fhn, mh = self.fh_hidden, self.mask_hidden
        A.of(fh.conv1, "kernel").copy_(self.fh1w[..., :fhn])
        A.of(fh.conv1, "bias").copy_(self.fh1b[:fhn])
        if self.has_mask:
            mr = mp.convrelu.layers_0
            A.of(mr, "kernel").copy_(self.fh1w[..., fhn:fhn + mh])
            A.of(mr, "bias").copy_(self.fh1b[fhn:fhn + mh])
        A.of(fh.conv2, "kernel").copy_(torch.flip(self.fh2w, dims=(0, 1)).permute(0, 1, 3, 2))
        A.of(fh.conv2, "bias").copy_(self.ddelta.reshape(-1, 8)[:, :2].sum(0, dtype=F32))

    def _pyramid_backward(self, out1=None, out2=None):
        """Correlation pyramid backward: the pooling adjoints of all levels as one
        native pass to a bf16 volume gradient dC (with the 1/sqrt(C) scale), then
        dfmap1 = dC fmap2 and dfmap2 = dC^T fmap1 as batched bf16 GEMMs with fp32
        accumulation (written straight into ``out1`` / ``out2`` when given): the native
        batched MFMA GEMM (csrc/kernels/bgemm.hip, dC read row-major for dfmap1 and as
        dC^T -- k-major -- for dfmap2, no transposed copy), torch.bmm only for shapes
        outside its tiling (h*w or C not a multiple of 128)."""
        B, h, w, C = self.B, self.h, self.w, self.fmap_ch
        hw = h * w
        if getattr(self, "_dC", None) is None:
            self._dC = torch.empty(B, hw, hw, dtype=BF16, device=self.device)
        nat.ops().pyr_bwd_dc([self._dC] + self.lv_grads + [None] * (4 - self.L), [self.L, self.M, h, w],
                             1.0 / float(C) ** 0.5)
        f1 = self.fm1.reshape(B, hw, C)
        f2 = self.fm2.reshape(B, hw, C)
        # the GEMMs write through reshape views of out1 / out2: a non-contiguous output would make
        # reshape return a copy and the gradient would be lost -- such outputs take the bmm path
        outs_ok = out1 is None or (out1.is_contiguous() and out2.is_contiguous())
        if hw % 128 == 0 and C % 128 == 0 and f1.is_contiguous() and f2.is_contiguous() and outs_ok:
            if out1 is None:
                out1 = torch.empty(B, h, w, C, dtype=F32, device=self.device)
                out2 = torch.empty(B, h, w, C, dtype=F32, device=self.device)
            nat.ops().bgemm([self._dC, f2, out1.reshape(B, hw, C)], [hw, C, hw, 0], 1.0)   # dC . fmap2
            nat.ops().bgemm([self._dC, f1, out2.reshape(B, hw, C)], [hw, C, hw, 1], 1.0)   # dC^T . fmap1
            return out1, out2
        if out1 is not None:
            g1 = torch.bmm(self._dC, f2).float()
            g2 = torch.bmm(self._dC.transpose(1, 2), f1).float()
            out1.copy_(g1.reshape(out1.shape))
            out2.copy_(g2.reshape(out2.shape))
            return out1, out2
        try:
            g1 = torch.bmm(self._dC, f2, out_dtype=F32)
            g2 = torch.bmm(self._dC.transpose(1, 2), f1, out_dtype=F32)
        except (RuntimeError, TypeError):
            g1 = torch.bmm(self._dC, f2).float()
            g2 = torch.bmm(self._dC.transpose(1, 2), f1).float()
        return g1.reshape(B, h, w, C), g2.reshape(B, h, w, C)

    # ---------------------------------------------------- weight gradients
    def _finish_data(self, fe_dy=None, on_dctx=None):
        """After the backward plan: the context share of the ConvGRU gates (iteration sums,
        weight gradient kept for :meth:`finish_weights`), the pyramid and context-encoder
        input gradients."""
        T, G, M, hd, C = self.T, self.G, self.M, self.hd, self.ctx_ch
        dctx = self.dctx
        self._gC = []
        for g, gru in enumerate(self.grus):
            kh, kw = gru.convz.kernel.shape[:2]
            # iteration sums of [dzr | dq] (M, 3 hd), fp32 accumulation, one bf16 rounding (train.hip)
            Sb = torch.empty(M, 3 * hd, dtype=BF16, device=self.device)
            nat.ops().sum_iters([self.dzr[g], self.dq[g], Sb], [T, M])
            gC = torch.empty(kh, kw, C, 3 * hd, device=self.device)
            db = torch.empty(3 * hd, device=self.device)
            record_wgrad(None, self.ctx_in, self.B, self.h, self.w, 0, self.ctx_cs, tuple(gC.shape), (1, 1),
                         gru.padding, Sb, 0, gC, db)
            self._gC.append((gC, db))
            # context data gradient of this GRU's gates (accumulated over the GRUs)
            tx, ix = _tx(s1=Seg(gin=dctx if g > 0 else None, out=dctx))
            self._conv(None, f"gCT{g}", Sb, dctx, tx=tx, ix=ix, epi=EPI_BWD, hidden=0)
        self._ev_gc = torch.cuda.Event()   # the context-share weight gradients are done (_assemble)
        self._ev_gc.record()
        # context-encoder output gradient: [tanh'(h0) dh | relu'(ctx) dctx] -- complete before the
        # pyramid backward, which does not touch it
        h0 = self.hf[0, 0]
        dc = torch.empty(M, hd + C, device=self.device, dtype=F32)
        dc[:, :hd] = self.dh_next * (1 - h0 * h0)
        dc[:, hd:] = dctx[:, :C] * (self.ctx_in[:, :C] > 0)
        dc = dc.reshape(self.B, self.h, self.w, hd + C)
        if on_dctx is not None:
            on_dctx(dc)
        if fe_dy is not None:   # whole-model path: straight into the feature encoder's bf16 output gradient
            g1, g2 = self._pyramid_backward(fe_dy[: self.B], fe_dy[self.B:])
        else:
            g1, g2 = self._pyramid_backward()
        return g1, g2, dc


class FusedRefine(torch.autograd.Function):
    """Autograd node of the correlation pyramid + the whole refinement loop
    (see :class:`FusedLoop`): inputs fmap1, fmap2, the context-encoder output
    and the loop's parameters; output the stacked upsampled flows."""

    @staticmethod
    def forward(ctx, loop: FusedLoop, fmap1, fmap2, ctx_raw, *params):
        out = loop.forward(fmap1, fmap2, ctx_raw)
        ctx.loop, ctx.gen = loop, loop.gen
        ctx.dtypes = (fmap1.dtype, fmap2.dtype, ctx_raw.dtype)
        return out

    @staticmethod
    def backward(ctx, gout):
        loop: FusedLoop = ctx.loop
        g1, g2, dctx, pgrads = loop.backward(gout.contiguous(), ctx.gen)
        d1, d2, d3 = ctx.dtypes
        return (None, g1.to(d1), g2.to(d2), dctx.to(d3)) + tuple(pgrads)


class FusedModel:
    """The whole RAFT training forward / backward as native plans: the
    feature and context encoders (:class:`~jax_raft_amd.train.fused_encoder.EncoderTrain`)
    write straight into the loop's feature-map / context buffers, and the
    loop's input gradients are handed back to the encoders' backward plans
    without leaving the device or the persistent buffers."""

    # the context encoder's forward / backward plans on a side stream next to the feature
    # encoder's (False: both on the caller's stream, in order -- A/B switch)
    SIDE_ENCODER = True
    # the context encoder's backward launched as soon as the loop has its gradient, next to the
    # pyramid backward (False: after the whole loop backward -- A/B switch)
    EARLY_CE = True

    def __init__(self, model, B: int, H: int, W: int, T: int, device, use_graph: bool = True):
        from .fused_encoder import EncoderTrain

        self._model_ref = weakref.ref(model)
        self.B, self.H, self.W = B, H, W
        self.loop = FusedLoop(model, B, H, W, T, device, use_graph)
        dev = self.loop.device
        self.img1 = torch.zeros(B, H, W, 3, device=dev)
        self.img2 = torch.zeros(B, H, W, 3, device=dev)
        self.x0 = torch.zeros(2 * B, H, W, 8, dtype=BF16, device=dev)
        self.fe = EncoderTrain(model.feature_encoder, self.x0, self.loop.fm, record_conv, use_graph)
        self.ce = EncoderTrain(model.context_encoder, self.x0[:B], self.loop.ctx_raw, record_conv, use_graph)
        self.params = [p for p in model.parameters()]

    @property
    def model(self):
        m = self._model_ref()
        if m is None:
            raise ReferenceError("FusedModel: its model has been garbage-collected")
        return m

    def stale(self) -> bool:
        """Parameters re-allocated (e.g. moved) since the plans were recorded."""
        return self.loop.stale() or self.fe.packer.stale() or self.ce.packer.stale()

    def _side(self):
        """The context encoder's stream: its plans overlap the feature encoder's
        (independent branches, model.py:562 vs :569)."""
        if getattr(self, "_side_stream", None) is None:
            self._side_stream = torch.cuda.Stream(device=self.loop.device)
        return self._side_stream

    def forward(self, image1, image2, train: bool) -> torch.Tensor:
        self.img1.copy_(image1)
        self.img2.copy_(image2)
        nat.ops().prep([self.img1, self.img2, self.x0], [self.B, self.H, self.W])
        cur = torch.cuda.current_stream(self.loop.device)
        side = self._side() if self.SIDE_ENCODER else cur
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self.ce.forward(update_stats=train)
        self.fe.forward(update_stats=train)
        cur.wait_stream(side)
        return self.loop.forward_prepared(self.loop.ctx_raw)

    def backward(self, gout, gen: int):
        comm = _ACTIVE_COMM.get(id(self.model))
        # the loop's stacked weight gradients run on their own stream, overlapping the encoders'
        # backward (bandwidth-bound norm passes next to MFMA-bound GEMMs)
        cur = torch.cuda.current_stream(self.loop.device)
        side = self._side() if self.SIDE_ENCODER else cur

        def ce_backward(dctx):   # as soon as the loop has the context gradient: next to the pyramid backward
            self.ce.dy_out.copy_(dctx)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self.ce.run_backward()

        if self.EARLY_CE:
            self.loop.backward(gout, gen, fe_dy=self.fe.dy_out, defer_weights=True, on_dctx=ce_backward)
        else:
            ce_backward(self.loop.backward(gout, gen, fe_dy=self.fe.dy_out, defer_weights=True)[2])
        self.fe.run_backward()
        pgrads = self.loop.finish_weights()
        if comm is not None:   # data parallel: the loop's gradients reduce while the encoders' snapshot
            comm.start(self.loop.last_snapshot)
        cur.wait_stream(side)
        grads = {id(p): g for p, g in zip(self.loop.params, pgrads)}
        for enc in (self.fe, self.ce):
            snap = enc.arena.snapshot()
            if comm is not None:
                comm.start(enc.arena.last_snapshot)
            grads.update(snap)
        if comm is not None:
            comm.finish(self.params)
        return [grads.get(id(p)) for p in self.params]


class FusedRAFT(torch.autograd.Function):
    """Autograd node of the whole model (encoders + pyramid + loop); inputs
    the images (no gradient) and every model parameter."""

    @staticmethod
    def forward(ctx, fm: FusedModel, image1, image2, train: bool, *params):
        out = fm.forward(image1, image2, train)
        ctx.fm, ctx.gen = fm, fm.loop.gen
        return out

    @staticmethod
    def backward(ctx, gout):
        grads = ctx.fm.backward(gout.contiguous(), ctx.gen)
        return (None, None, None, None) + tuple(grads)


# Native training plans per model: model -> {(kind, B, H, W, T, device): FusedLoop / FusedModel}.
# Weakly keyed, and the plans hold their model weakly, so a model's plans (hipGraphs, events,
# streams, arenas, activation buffers) are freed with the model instead of living for the process.
_LOOPS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
# Gradient communicators of the models whose Trainer step is running: set only
# inside :func:`grad_comm` (around one step's backward), keyed by the model, so a
# backward outside a training step, or of another model, never starts a collective.
_ACTIVE_COMM: Dict[int, object] = {}


def _run_plan(plan, use_graph: bool) -> None:
    """Replay a plan's own hipGraph, or enqueue it eagerly -- inline (lane 0 =
    the caller's stream) inside an outer stream capture (the trainer's
    optional whole-step graph), which records the plan's launches into it."""
    if torch.cuda.is_current_stream_capturing():
        plan.run_inline(0)
    elif use_graph:
        if plan.captured_iters() != 0:
            plan.capture(0)
        plan.replay()
    else:
        plan.run(0)


@contextlib.contextmanager
def grad_comm(model, comm):
    """Within this block, the whole-model fused backward of ``model`` all-reduces
    its flat gradient arenas through ``comm`` (``parallel.dp.FlatGradComm``) as
    they are produced.  ``comm=None`` is a no-op.  The registration is per model
    and ends with the block (the Trainer wraps each step's backward in it)."""
    if comm is None:
        yield
        return
    prev = _ACTIVE_COMM.get(id(model))
    _ACTIVE_COMM[id(model)] = comm
    try:
        yield
    finally:
        if prev is None:
            _ACTIVE_COMM.pop(id(model), None)
        else:
            _ACTIVE_COMM[id(model)] = prev


# Module switches (measured choices; tests flip them with monkeypatch.setattr -- see knobs.py):
FUSED_TRAIN = True      # native fused loop / model nodes (False: the per-op autograd path)
FUSED_ENCODERS = True   # the whole-model node (encoders + pyramid + loop); False: only the loop
FUSED_GRAPH = True      # replay the fused plans as hipGraphs (JR_PLAN_CHECK=1 forces eager plans)


def enabled() -> bool:
    return FUSED_TRAIN


def full_model_ok(model, train: bool) -> bool:
    """The whole-model node needs train-mode (batch-statistics) BatchNorm without
    cross-rank synchronisation; otherwise only the loop is fused."""
    from ..models.layers import BatchNorm

    bns = [m for m in model.modules() if isinstance(m, BatchNorm)]
    if bns and (not train or any(b.sync_group is not None for b in bns)):
        return False
    return FUSED_ENCODERS


def _tensor_sig(model) -> tuple:
    """Identity + storage of every parameter and buffer the module tree holds
    RIGHT NOW.  The plans pack / differentiate / update the tensors they were
    recorded with, so any swap -- ``torch.func.functional_call`` (the Flax-style
    ``RAFT.apply`` with foreign variables), a new ``nn.Parameter``, ``p.data =
    ...``, ``.to()`` -- must rebuild them.  (Comparing the recorded tensors with
    their own pointers cannot see a swap: they are still alive and unchanged.)"""
    sig = []
    for mod in model.modules():
        for t in mod._parameters.values():
            if t is not None:
                sig.append((id(t), t.data_ptr()))
        for t in mod._buffers.values():
            if t is not None:
                sig.append((id(t), t.data_ptr()))
    return tuple(sig)


def _cached(kind, model, B, H, W, T, device):
    key = (kind, B, H, W, T, str(device))
    plans = _LOOPS.get(model)
    obj = plans.get(key) if plans is not None else None
    sig = _tensor_sig(model)
    if obj is None or getattr(obj, "_sig", None) != sig or obj.stale():
        # one plan set per model: drop other shapes / kinds first (their buffers), then build --
        # after the device has finished their replays (Plan::~Plan destroys graph execs / streams)
        if plans and torch.device(device).type == "cuda" and not torch.cuda.is_current_stream_capturing():
            torch.cuda.synchronize(device)
        _LOOPS.pop(model, None)
        obj = None
        g = FUSED_GRAPH and not knobs.flag("JR_PLAN_CHECK")
        obj = (FusedModel if kind == "model" else FusedLoop)(model, B, H, W, T, device, use_graph=g)
        obj._sig = sig
        _LOOPS[model] = {key: obj}
    return obj


def get_loop(model, B, H, W, T, device) -> FusedLoop:
    return _cached("loop", model, B, H, W, T, device)


def forward_train(model, image1, image2, train: bool, num_flow_updates: int):
    """Training forward on the fused native path: the whole model as one
    :class:`FusedRAFT` node when :func:`full_model_ok`, else the encoders on
    the native autograd Functions and the correlation pyramid + refinement
    loop as one :class:`FusedRefine` node."""
    B, H, W, _ = image1.shape
    h, w = H // 8, W // 8
    min_sz = 2 * (2 ** (model.corr_block.num_levels - 1))
    assert h >= min_sz and w >= min_sz, (
        "Feature maps are too small to be down-sampled by the correlation pyramid. "
        f"H and W of feature maps should be at least {min_sz}; got: {(h, w)}.")
    if full_model_ok(model, train):
        fm = _cached("model", model, B, H, W, num_flow_updates, image1.device)
        return FusedRAFT.apply(fm, image1.float().contiguous(), image2.float().contiguous(), bool(train), *fm.params)
    fmaps = model.feature_encoder(torch.cat([image1, image2], dim=0), train)
    fmap1, fmap2 = torch.chunk(fmaps, 2, dim=0)
    assert tuple(fmap1.shape[1:3]) == (h, w), "The feature encoder should downsample H and W by 8"
    ctx_out = model.context_encoder(image1, train)
    assert tuple(ctx_out.shape[1:3]) == (h, w), "The context encoder should downsample H and W by 8"
    loop = get_loop(model, B, H, W, num_flow_updates, image1.device)
    return FusedRefine.apply(loop, fmap1, fmap2, ctx_out, *loop.params)
