"""Native MI355X inference engine: lowers a :class:`~jax_raft_amd.models.raft.RAFT`
onto the gfx950 kernels as one :class:`Plan` (prologue = encoders + correlation
pyramid, loop body = one refinement iteration) and runs it eagerly from C++
or as a single captured hipGraph.

Mapping to the reference forward (``jax_raft/model.py:557-605``):

=====================================  ==============================================
reference                              engine
=====================================  ==============================================
concat images, feature encoder :562    prep kernel -> implicit-GEMM convs (+IN stats/apply)
build_pyramid :567, :418-446           ``corr`` (MFMA GEMM, pooling fused, all levels)
context encoder :569 (BN eval)         convs with BN folded into weights, fused relu/residual
split/tanh/relu :582-584               final 1x1 conv epilogue writes tanh(h)|relu(ctx)
                                       straight into the persistent GRU input buffers
scan body :495-510                     loop segment: lookup, 5 motion convs, 2x GRU (A/B),
                                       flow head (+mask), coords update, x8 upsample
=====================================  ==============================================

Persistent buffers replace every concat of the reference:
``hx = [h | motion | flow]`` (GRU z/r input, ``model.py:303,366,290``) and
``qx = [r*h | motion | flow]`` (GRU q input, ``model.py:308``).  The context
features -- the third part of the GRU input ``[h | context | motion]`` -- are
loop-invariant, so their share of every ConvGRU gate (z, r and q, plus the
gate biases) is computed ONCE in the prologue (one conv per GRU over the
context, fp32 output) and added per pixel in the loop convs' epilogues (the
``bmap`` bias map).  That removes a third of the GRU GEMMs' K from every
iteration: K = 5 x 256 instead of 5 x 384 for raft_large.
"""
from __future__ import annotations

import itertools
import operator
import weakref
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from ..models.layers import (
    NORM_BATCH,
    NORM_CUSTOM,
    NORM_INSTANCE,
    BottleneckBlock,
    ConvNormActivation,
    CorrBlock,
    FeatureEncoder,
    FlowHead,
    MaskPredictor,
    MotionEncoder,
    RecurrentBlock,
    ResidualBlock,
    UpdateBlock,
)
from .. import knobs
from ..ops import native as nat
from . import tunedb
from ..ops.native import (
    ACT_NONE,
    ACT_RELU,
    ACT_SPLIT_TANH_RELU,
    EPI_GRU_A,
    EPI_GRU_B,
    EPI_STD,
    EPI_TAPS,
    ConvSpec,
    conv_args,
    round_up,
)

BF16 = torch.bfloat16
F32 = torch.float32

_TUNE_CACHE: Dict[tuple, int] = {}


def _tune(spec: ConvSpec, x, N, H, W, y, kw, reps: int = 5) -> int:
    """Time every tile config of one conv problem; return the fastest."""
    ops = nat.ops()
    best, best_t = None, None
    for cfg in _candidates(spec, kw, y):
        args = conv_args(spec, x, N, H, W, y, **dict(kw, cfg=cfg))
        ops.conv(*args)  # warm (and JIT-free: all configs are precompiled)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ops.conv(*args)
        e.record()
        e.synchronize()
        t = s.elapsed_time(e)
        if best_t is None or t < best_t:
            best, best_t = cfg, t
    return best


def _fused_norm(kw) -> bool:
    """The conv writes channel-statistics partials or normalises its input on load: only the
    halo kernel (conv_halo.hip) does either."""
    return kw.get("stats_part") is not None or kw.get("in_stats") is not None


def _candidates(spec: ConvSpec, kw, y) -> Tuple[int, ...]:
    """Tile configs that can run this conv: the taps-epilogue configs, or the implicit-GEMM
    autotune set plus the halo 3x3 configs (halo only when a norm is fused into the conv)."""
    if kw.get("epi") == nat.EPI_TAPS:
        return nat.TAPS_CFGS
    halo = nat.halo_cfgs_for(spec, dict(kw, y=y))
    return halo if _fused_norm(kw) else nat.TUNE_CFGS + halo


def _fold_bn(cna: ConvNormActivation) -> Tuple[torch.Tensor, torch.Tensor]:
    """Conv kernel/bias with an eval-mode BatchNorm folded in."""
    k = cna.layers_0.kernel.detach().float()
    b = cna.layers_0.bias.detach().float()
    if cna.norm == NORM_BATCH:
        bn = cna.layers_1
        s = bn.scale.detach().float() * torch.rsqrt(bn.var.detach().float() + bn.eps)
        k = k * s  # broadcast over cout (last dim)
        b = (b - bn.mean.detach().float()) * s + bn.bias.detach().float()
    return k, b


@dataclass
class _Shape:
    B: int
    H: int
    W: int
    N: int


@dataclass
class _PlanState:
    plan: object                      # plans[0]
    plans: List[object] = field(default_factory=list)   # one native Plan (one hipGraph) per batch part
    bufs: Dict[str, torch.Tensor] = field(default_factory=dict)
    inp1: Optional[torch.Tensor] = None
    inp2: Optional[torch.Tensor] = None
    out: Optional[torch.Tensor] = None
    n_iters: int = 0
    # Output indirection: every output writer (convex head / bilinear
    # upsampling) reads its destination base from this device int64, so a
    # replay can write into a fresh tensor (forward with copy_output) instead
    # of the captured buffer + a clone of it.  slot_ok: all writers use it.
    out_slot: Optional[torch.Tensor] = None
    slot_ok: bool = True
    slot_ptr: int = 0
    # context parallelism: {slabs, nq (padded slab pixels per image), local, corr} (see _gather_corr)
    cp: Optional[dict] = None
    # raw uint8 frames (K14): (H0, W0, pt, pl) of the frames inside the padded plan size, else None
    src: Optional[Tuple[int, int, int, int]] = None


_VERSION = operator.attrgetter("_version")


def sintel_pad(H0: int, W0: int) -> Tuple[int, int, int, int]:
    """InputPadder('sintel') of the reference (``scripts/validate_sintel.py:23-31``): the rows /
    columns (top, bottom, left, right) that replicate-pad an H0 x W0 frame to multiples of 8."""
    ph = (((H0 // 8) + 1) * 8 - H0) % 8
    pw = (((W0 // 8) + 1) * 8 - W0) % 8
    return ph // 2, ph - ph // 2, pw // 2, pw - pw // 2


_U8_LUT: Dict[str, torch.Tensor] = {}


def u8_table(device) -> torch.Tensor:
    """x / 255 * 2 - 1 for x = 0..255, evaluated on the host in fp32 exactly as the reference's
    input protocol (validate_sintel.py:177-178, demo.py:9) -- the device kernel looks values up."""
    key = str(device)
    t = _U8_LUT.get(key)
    if t is None:
        t = _U8_LUT[key] = (torch.arange(256, dtype=torch.float32) / 255.0 * 2.0 - 1.0).to(device)
    return t


class RaftEngine:
    """Inference engine bound to one model and one GPU.

    Args:
        use_graph: capture the whole forward (prologue + N iterations) into one
            hipGraph and replay it (default); otherwise launch from C++ eagerly.
        copy_output: return a fresh tensor (default) instead of the engine's
            static output buffer (which the next call overwrites).
        corr_dtype: storage dtype of the correlation pyramid (bf16 default:
            the lookup output feeding the bf16 MFMA convs is bf16 anyway;
            fp32 for bit-closer parity with the fp32 reference).
        gate_dtype: storage dtype of the ConvGRU z gate and of the folded
            context bias map (bf16 default, fp32 for bit-closer parity); the
            hidden state itself is always carried in fp32.
        autotune: pick every conv's tile config from the persisted table
            (runtime/tunedb.py) or, on a miss, by timing the candidates on the
            real buffers when a plan is built; ``False``: a size heuristic.
        streams: (True / False / "auto") run the model's independent branches
            on concurrent lanes of the plan (parallel branches of the captured
            hipGraph): context encoder || the two feature-encoder halves ||
            correlation pyramid in the prologue; in the loop, iteration i+1's
            flow-feature convs and iteration i's mask head + upsampling on a
            side lane while the critical lane runs lookup -> correlation convs
            -> motion conv -> ConvGRU -> flow head.  "auto" (default) = on at
            batch >= 4 per plan with every iteration upsampled and a
            256 -> 576 mask head (raft_large), where it measured faster.
        split: run the batch as this many independent part-forwards captured
            into ONE hipGraph with no edge between them (when the batch
            divides evenly), so one part's kernels fill CUs another part's
            leave idle.
        cfg_override: fixed tile configs per conv spec name (e.g. {"gru0.b": 27},
            tools/schedule_tune.py); ``JR_CFG_OVERRIDE="name=cfg,..."`` adds entries.
        cp_group: context parallelism of the correlation volume:
            a torch.distributed process group (``True``: the default group) whose
            ranks each hold the pyramid of one slab of query rows
            (``parallel/cp.py:row_slabs``) and all-gather the looked-up
            correlation features every iteration (RCCL over xGMI); the rest of
            the update block runs replicated.  Pyramid memory per rank / world.
            One lane, eager from C++ (the collective sits between the two
            halves of the loop body, ``Plan.run_segment``).
        precision: "bf16" (default: bf16 MFMA operands and activations, fp32
            accumulation, fp32 hidden state / flow / upsampled output) or "fp32"
            (the reference's own precision end to end on the f32 MFMA:
            :class:`~jax_raft_amd.runtime.engine_f32.RaftEngineF32`).

    Schedules (chosen per plan, see :meth:`_build_part`): the lane schedule
    above; one in-order lane with every iteration upsampled (batch < 4,
    raft_small); and the final-only serving mode.  In all of them the flow
    update of iteration i runs inside iteration i+1's lookup kernel and the
    FlowHead's second conv is an MFMA epilogue of its first (raft_large) or a
    skinny taps GEMM (raft_small).  Variants measured and removed in round 3
    (kept in the history): double-buffered flow-head outputs, the 3x3 EPI_FLOW
    and halo-tiled flow heads, the EPI_CONVEX conv epilogue, the side-lane and
    main-lane flow-feature placements, the mask lane forking after convcorr1,
    separate per-part graphs on separate streams, and submit() (the two phases
    as separate graphs on two streams, which serialise on this ROCm).
    """

    def __new__(cls, *args, precision: str = "bf16", **kwargs):
        if precision not in ("bf16", "fp32", "mixed"):
            raise ValueError(f"precision must be 'bf16', 'fp32' or 'mixed', got {precision!r}")
        if precision == "fp32" and cls is RaftEngine:
            from .engine_f32 import RaftEngineF32
            cls = RaftEngineF32
        elif precision == "mixed" and cls is RaftEngine:
            from .engine_f32 import RaftEngineMixed
            cls = RaftEngineMixed
        return super().__new__(cls)

    precision = "bf16"
    fe_external = False   # the feature encoder runs outside the plan (RaftEngineMixed: fp32), fmap filled before it

    # Lowering choices.  Each is the measured winner of an A/B (the profile is cited where the
    # choice is used); they are class attributes rather than environment switches so that tests
    # can cover the alternative lowering against the same oracle (monkeypatch.setattr on the
    # class, before the plan is built).  Operational environment variables: jax_raft_amd/knobs.py.
    GRU = "auto"          # ConvGRU stage lowering: "auto" | "halo" | "fused" | "unfused" (_gru_path)
    PRO_LANES = "auto"    # prologue branches on lanes at one-lane loops: "auto" | "on" | "off"
    HALO_NORM = True      # encoder instance norms fused into the halo 3x3 convs
    MERGED_UP = True      # one-lane loop: 7x7 flow conv merged with the x8 upsampling (merged.hip)
    CONV_GROUP = True     # one-lane loop: last correlation conv + convflow2 as one grouped grid
    MASK_PARITY = False   # lane schedule: parity-buffered h copy for the mask lane (slower at b4)
    CORR_PERSIST_B1 = True   # the persistent blocked pyramid kernel at batch 1 too (plans outside pipelined slots)
    HOST_GATE = True      # host gate of long replays (see GATE_MIN_ITERS)

    def __init__(self, model, device, use_graph: bool = True, copy_output: bool = True,
                 corr_dtype: torch.dtype = torch.bfloat16, gate_dtype: torch.dtype = torch.bfloat16,
                 autotune: bool = True, streams="auto", split: int = 1,
                 cfg_override: Optional[Dict[str, int]] = None, precision: str = "bf16", cp_group=None):
        nat.require()
        self._init_cp(cp_group)
        assert streams in (True, False, "auto"), streams
        self.streams_mode = streams
        self.streams = bool(streams)
        # instance norms of the encoders fused into halo 3x3 convs (statistics partials in the
        # producer's epilogue, normalise + relu in the consumer's footprint load; a residual
        # block's output built -- residual + its norm -- inside the next block's first halo conv;
        # profiles/r4_in_fusion_ab.txt); HALO_NORM = False: the separate statistics / norm_act passes
        self.halo_norm = bool(self.HALO_NORM)
        self.halo_res = self.halo_norm
        self.mask_head = "split"      # per plan: "split" (mask lane) | "fused" (one lane, 128 -> 512 conv)
        self.gate_dtype = gate_dtype
        self.split = split
        self.cfg_override = dict(cfg_override or {})
        self.cfg_override.update(knobs.cfg_override())
        self._cf1_w = self._cf1_b = None
        self._fh2_b = None
        self._convex_w = self._convex_b = None
        self._taps_w = None
        self._taps_epi_w = None
        self._cc1_w = self._cc1_b = None
        self._halo_w: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}   # GRU gi -> gru_halo (wa, wb)
        # the model: held strongly by an engine built directly, weakly by one the model caches itself
        # (RAFT.engine -> _hold_model_weakly): model._engines -> engine -> model would be a reference
        # cycle, and every plan of a cycle-held engine (hipGraphs, 64 events, lane streams, pyramid
        # buffers) would outlive the model until a full garbage collection
        self._model_strong = model
        self._model_ref = None
        self.device = torch.device(device)
        self.use_graph = use_graph
        self.copy_output = copy_output
        # host gate: the graph replay of a forward with >= GATE_MIN_ITERS iterations is launched
        # only after the previous call's work has finished (the host waits on its completion
        # event).  A long replay enqueued behind a still-running one runs slower on this ROCm:
        # batch 1 raft_large 32 it 208-213 -> 261 pairs/s, raft_small 32 it 334-337 -> 435-436,
        # batch 4 387-393 -> 401-402; short forwards lose (raft_small 12 it 713-754 -> 646-698),
        # where the exposed host launch is a larger share.  profiles/r4_host_gate.txt
        self.host_gate = bool(self.HOST_GATE)
        self._done_ev: Optional[torch.cuda.Event] = None
        self.corr_dtype = corr_dtype
        self.autotune = autotune
        self._specs: Dict[str, ConvSpec] = {}
        self.arch = tunedb.gpu_arch(self.device)
        self.chosen_cfgs: Dict[str, Optional[int]] = {}   # conv spec name -> tile config of the last plan built
        self._sources: Dict[str, callable] = {}
        # built plans, least recently used first; at most max_plans key groups (a forward's plan and
        # its pipelined() slots are one group) -- a long-lived serving / eval process over many input
        # shapes keeps a bounded set; release() drops them all
        self._states: "OrderedDict[tuple, _PlanState]" = OrderedDict()
        self._snap = None    # parameter / module snapshot of the last repack (_snapshot / _stale)
        self._pp = None   # pipelined(): {key, n, pending slot}
        self._analyse()
        self._pack()

    @property
    def model(self):
        m = self._model_strong if self._model_strong is not None else self._model_ref()
        if m is None:
            raise ReferenceError("RaftEngine: its model has been garbage-collected")
        return m

    def _hold_model_weakly(self) -> None:
        """Called by the model that caches this engine (``RAFT.engine``): keep a weak reference."""
        if self._model_strong is not None:
            self._model_ref = weakref.ref(self._model_strong)
            self._model_strong = None

    # ------------------------------------------------------------ plan cache
    max_plans = 8   # key groups kept (an instance attribute may lower / raise it)

    @staticmethod
    def _group(key: tuple) -> tuple:
        return key[:-2] if len(key) > 2 and key[-2] == "pslot" else key

    # raw uint8 frames are prepared on the device by the plan's prep kernel (an engine without that
    # path normalises + pads them with framework ops first: the fp32 engine)
    _native_u8 = True

    def _key(self, image1: torch.Tensor, image2: torch.Tensor, n_iters: int, all_iters: bool) -> tuple:
        """Plan key of one call: (B, H, W, n, all) for float NHWC images in [-1, 1] with H, W % 8 == 0;
        + ("u8", H0, W0, pt, pl) for uint8 NHWC frames of any size, whose plan runs at the padded
        size (InputPadder 'sintel' semantics) and returns the flows cropped back to H0 x W0."""
        B, H, W, C = image1.shape
        assert C == 3, "images must be NHWC with 3 channels"
        assert tuple(image2.shape) == tuple(image1.shape), "input images should have the same shape"
        if image1.dtype == torch.uint8:
            assert image2.dtype == torch.uint8, "both frames must be uint8"
            pt, pb, pl, pr = sintel_pad(H, W)
            return (B, H + pt + pb, W + pl + pr, n_iters, bool(all_iters), "u8", H, W, pt, pl)
        assert H % 8 == 0 and W % 8 == 0, "input image H and W should be divisible by 8"
        return (B, H, W, n_iters, bool(all_iters))

    def _build_key(self, key: tuple) -> _PlanState:
        src = tuple(key[6:10]) if len(key) >= 10 and key[5] == "u8" else None
        return self._build(*key[:5], src=src)

    @staticmethod
    def _crop(st: _PlanState, out: torch.Tensor) -> torch.Tensor:
        if st.src is None:
            return out
        H0, W0, pt, pl = st.src
        return out[:, :, pt:pt + H0, pl:pl + W0]

    def _host_u8(self, image1, image2):
        """uint8 frames -> float [-1, 1], replicate-padded to /8 with framework ops on the device
        (engines without the native u8 prep); returns (img1, img2, crop)."""
        B, H0, W0, _ = image1.shape
        pt, pb, pl, pr = sintel_pad(H0, W0)
        lut = u8_table(self.device)

        def one(x):
            x = lut[x.to(self.device).long()].permute(0, 3, 1, 2)
            return torch.nn.functional.pad(x, [pl, pr, pt, pb], mode="replicate").permute(0, 2, 3, 1).contiguous()

        return one(image1), one(image2), (H0, W0, pt, pl)

    def _plan_state(self, key: tuple, build) -> _PlanState:
        """The plan of ``key`` (built by ``build()`` on a miss), marked most recently used; a miss
        first evicts the least recently used key groups beyond ``max_plans`` (never the group of a
        batch :meth:`pipelined` left pending)."""
        st = self._states.get(key)
        if st is not None:
            for k in [k for k in self._states if self._group(k) == self._group(key)]:
                self._states.move_to_end(k)
            return st
        self._evict(self._group(key))
        st = build()
        self._states[key] = st
        return st

    def _evict(self, incoming: tuple) -> None:
        groups = list(OrderedDict.fromkeys(self._group(k) for k in self._states))
        pend = self._pp["key"] if self._pp is not None and self._pp["pending"] is not None else None
        n = len(groups) + (incoming not in groups)
        cap = max(1, int(self.max_plans))
        for g in groups:
            if n <= cap:
                break
            if g == incoming or g == pend:
                continue
            self._drop_group(g)
            n -= 1

    def _quiesce(self) -> None:
        """Wait for this engine's launched work before plans are destroyed: Plan::~Plan destroys
        graph execs, events and lane streams, and HIP does not document that destroying a graph
        exec still running is deferred until it finishes.  Eviction / release are rare."""
        if self.device.type == "cuda" and self._states and not torch.cuda.is_current_stream_capturing():
            torch.cuda.synchronize(self.device)

    def _drop_group(self, g: tuple) -> None:
        # a plan's pipelined graph holds the other slot's kernel nodes (its buffers): the whole
        # group goes at once
        self._quiesce()
        for k in [k for k in self._states if self._group(k) == g]:
            del self._states[k]
        if self._pp is not None and self._pp["key"] == g:
            self._pp = None

    def release(self) -> None:
        """Drop every built plan: their hipGraphs, events, lane streams and device buffers are freed
        now (the next forward rebuilds).  Not while a :meth:`pipelined` batch is pending."""
        if self._pp is not None and self._pp["pending"] is not None:
            raise RuntimeError("release(): flush() the pending pipelined batch first")
        self._quiesce()
        self._states.clear()
        self._pp = None
        self._done_ev = None

    def num_plans(self) -> int:
        return len(self._states)

    # ----------------------------------------------------------- structure
    def _analyse(self):
        m = self.model
        fe, ce = m.feature_encoder, m.context_encoder
        for enc in (fe, ce):
            if not isinstance(enc, FeatureEncoder):
                raise NotImplementedError("native engine supports FeatureEncoder encoders only")
            if enc.block == "custom" or enc.norm_kind == NORM_CUSTOM:
                raise NotImplementedError("native engine lowers residual / bottleneck blocks with batch / "
                                          "instance / no norm only")
        ub = m.update_block
        if not (isinstance(ub, UpdateBlock) and isinstance(ub.motion_encoder, MotionEncoder)
                and isinstance(ub.recurrent_block, RecurrentBlock) and isinstance(ub.flow_head, FlowHead)
                and isinstance(m.corr_block, CorrBlock)
                and (m.mask_predictor is None or isinstance(m.mask_predictor, MaskPredictor))):
            raise NotImplementedError("native engine lowers the reference update block / correlation block / "
                                      "mask predictor classes only")
        me, rb, fh = ub.motion_encoder, ub.recurrent_block, ub.flow_head
        self.hidden = rb.hidden_size
        self.ctx_ch = ce.out_channels - self.hidden
        self.num_levels = m.corr_block.num_levels
        self.radius = m.corr_block.radius
        S = 2 * self.radius + 1
        self.corr_ch = self.num_levels * S * S
        self.corr_cs = round_up(self.corr_ch, 8)
        self.mot_out = me.out_channels
        # loop buffers hold [h | motion | flow]; the context part of the GRU input is folded (see module doc)
        self.hx_real = self.hidden + self.mot_out
        # padded to a multiple of 64 channels when that costs <= 16 zero channels
        # (raft_small: 178 -> 192): the GRU convs' 64-deep K stages then lie inside
        # one tap and take the FAST im2col loader (conv_igemm.h:FastRow)
        hx64 = round_up(self.hx_real, 64)
        self.hx_cs = hx64 if hx64 - self.hx_real <= 16 else round_up(self.hx_real, 8)
        self.mot_off = self.hidden
        self.flow_off = self.mot_off + self.mot_out - 2
        self.gate_cs = round_up(3 * self.hidden, 8)   # fp32 context bias map: [z | r | q] per GRU
        if self.hidden % 16:
            raise NotImplementedError("native engine needs hidden % 16 == 0")
        self.fh_hidden = fh.hidden_size
        self.has_mask = m.mask_predictor is not None
        self.fmap_ch = fe.out_channels
        if self.fmap_ch % 64:
            raise NotImplementedError("native correlation needs feature channels % 64 == 0")

    def _snapshot(self):
        """What a repack saw: every parameter / buffer with its version counter, and every
        module's child list.  Holds the modules' dicts and tensors, never the root module
        itself (a weakly held model stays collectable)."""
        root = self.model
        mods = [root] + [m for n, m in root.named_modules() if n]
        dicts = [d for mod in mods for d in (mod._parameters, mod._buffers, mod._modules)]
        lens = list(map(len, dicts))
        pdicts = [d for mod in mods for d in (mod._parameters, mod._buffers)]
        keys = [(d, k) for d in pdicts for k, t in d.items() if t is not None]
        tensors = [d[k] for d, k in keys]
        kid_dicts = [mod._modules for mod in mods]
        kids = list(itertools.chain.from_iterable(map(dict.values, kid_dicts)))
        return (dicts, lens, [d for d, _ in keys], [k for _, k in keys], tensors,
                list(map(_VERSION, tensors)), kid_dicts, kids)

    def _stale(self) -> bool:
        """Whether any parameter / buffer changed in place (version counter) or was replaced,
        or a submodule was replaced, since the last repack -- checked on every forward with
        C-level map() walks over the snapshot: the tuple signature it replaces cost 0.2-0.7 ms of
        host time per call, which the batch-1 12-iteration stream (~1.2 ms of GPU time per
        pair) pays directly."""
        snap = self._snap
        if snap is None:
            return True
        dicts, lens, pds, pks, tensors, versions, kid_dicts, kids = snap
        if list(map(len, dicts)) != lens or list(map(_VERSION, tensors)) != versions:
            return True
        if not all(map(operator.is_, map(dict.get, pds, pks), tensors)):
            return True
        return not all(map(operator.is_, itertools.chain.from_iterable(map(dict.values, kid_dicts)), kids))

    def _reg(self, name: str, fn):
        """Register a conv spec source: fn() -> (kernel HWIO, bias, stride, padding, cin8)."""
        self._sources[name] = fn

    def _pack(self):
        """(Re)pack every conv into bf16 GEMM layout; BN folded (eval mode).  Packed
        tensors are updated in place so captured graphs stay valid."""
        if not self._sources:
            self._define_specs()
        for name, fn in self._sources.items():
            k, b, stride, pad, cin8 = fn()
            k = k.to(self.device)
            if name in self._specs:
                sp = self._specs[name]
                nat.pack_weight(k, sp.cin8, out=sp.w)
                if sp.wh is not None:
                    nat.pack_halo_conv(k, sp.cin8, out=sp.wh)
                sp.b.copy_(b.float().to(self.device))
            else:
                self._specs[name] = nat.make_spec(k, b.to(self.device), stride, pad, cin8=cin8, device=self.device)
        fh2 = self.model.update_block.flow_head.conv2
        bf = fh2.bias.detach().float().to(self.device).contiguous()
        if self._fh2_b is None:
            self._fh2_b = bf
        else:
            self._fh2_b.copy_(bf)
        # the correlation features' first 1x1 conv on the LDS-resident-weight kernel (conv1x1.hip)
        cc1 = self.model.update_block.motion_encoder.convcorr1.layers_0
        kpad = next((k for k in nat.CONV1X1_KPADS if k >= self.corr_cs), None)
        if kpad is not None and cc1.kernel.shape[:2] == (1, 1) and cc1.kernel.shape[3] % 64 == 0:
            wc = nat.pack_conv1x1(cc1.kernel.to(self.device), kpad)
            bc = cc1.bias.detach().float().to(self.device).contiguous()
            if self._cc1_w is None:
                self._cc1_w, self._cc1_b, self._cc1_kpad = wc, bc, kpad
            else:
                self._cc1_w.copy_(wc)
                self._cc1_b.copy_(bc)
        if fh2.kernel.shape[2] in (128, 256):
            wt = nat.pack_taps(fh2.kernel.to(self.device))
            if self._taps_w is None:
                self._taps_w = wt
            else:
                self._taps_w.copy_(wt)
        if tuple(fh2.kernel.shape) == (3, 3, 256, 2):
            wt = nat.pack_taps_epi(fh2.kernel.to(self.device))
            if self._taps_epi_w is None:
                self._taps_epi_w = wt
            else:
                self._taps_epi_w.copy_(wt)
        mp = self.model.mask_predictor
        if mp is not None and tuple(mp.conv.kernel.shape) == (1, 1, 256, 576):
            wc, bc = nat.pack_convex_head(mp.conv.kernel.to(self.device), mp.conv.bias.to(self.device))
            if self._convex_w is None:
                self._convex_w, self._convex_b = wc, bc
            else:
                self._convex_w.copy_(wc)
                self._convex_b.copy_(bc)
        if self._halo_geom() is not None:   # the halo-tiled fused ConvGRU's weight streams
            for gi in range(len(self.model.update_block.recurrent_block.kernel_size)):
                ka = self._sources[f"gru{gi}.a"]()[0].to(self.device)
                kb = self._sources[f"gru{gi}.b"]()[0].to(self.device)
                old = self._halo_w.get(gi)
                self._halo_w[gi] = (nat.pack_gru_halo(ka, self.hx_cs, out=old[0] if old else None),
                                    nat.pack_gru_halo(kb, self.hx_cs, out=old[1] if old else None))
        cf1 = self.model.update_block.motion_encoder.convflow1.layers_0
        if nat.direct_conv_ok(cf1.kernel, cf1.stride):
            wd = nat.pack_direct_weight(cf1.kernel).to(self.device)
            bd = cf1.bias.detach().float().to(self.device).contiguous()
            if self._cf1_w is None:
                self._cf1_w, self._cf1_b = wd, bd
            else:
                self._cf1_w.copy_(wd)
                self._cf1_b.copy_(bd)
        self._snap = self._snapshot()

    def _define_specs(self):
        m = self.model

        def cna_src(cna: ConvNormActivation, cin8=None):
            def f():
                k, b = _fold_bn(cna)
                c = cna.layers_0
                return k, b, c.stride, c.padding, cin8
            return f

        def conv_src(c, cin8=None):
            return lambda: (c.kernel.detach().float(), c.bias.detach().float(), c.stride, c.padding, cin8)

        def s2d_src(cna: ConvNormActivation):
            def f():
                k, b = _fold_bn(cna)
                return nat.s2d_stem_kernel(k), b, (1, 1), (2, 2), 16
            return f

        for tag, enc in (("fe", m.feature_encoder), ("ce", m.context_encoder)):
            self._reg(f"{tag}.stem", cna_src(enc.convnormrelu, 8))
            c0 = enc.convnormrelu.layers_0
            if tuple(c0.kernel.shape[:3]) == (7, 7, 3) and tuple(c0.stride) == (2, 2) and tuple(c0.padding) == (3, 3):
                # the stem as a 4x4 conv over the 2x2 space-to-depth input (ops/native.py:s2d_stem_kernel)
                self._reg(f"{tag}.stem_s2d", s2d_src(enc.convnormrelu))
            for li in (1, 2, 3):
                layer = getattr(enc, f"layer{li}")
                for bi in range(layer.n):
                    blk = getattr(layer, f"layers_{bi}")
                    names = ["convnormrelu1", "convnormrelu2"] + (["convnormrelu3"] if isinstance(blk, BottleneckBlock) else [])
                    if blk.stride != (1, 1):
                        names.append("downsample")
                    for nm in names:
                        self._reg(f"{tag}.l{li}.b{bi}.{nm}", cna_src(getattr(blk, nm)))
            self._reg(f"{tag}.conv", conv_src(enc.conv))
        ub = m.update_block
        me, rb, fh = ub.motion_encoder, ub.recurrent_block, ub.flow_head
        self._reg("me.convcorr1", cna_src(me.convcorr1, self.corr_cs))
        if len(me.corr_layers) == 2:
            self._reg("me.convcorr2", cna_src(me.convcorr2))
        self._reg("me.convflow1", cna_src(me.convflow1, 8))
        self._reg("me.convflow2", cna_src(me.convflow2))
        self._reg("me.conv", cna_src(me.conv))
        hx_cs = self.hx_cs   # the sources below must not capture the engine (no self-cycle: plans die by refcount)
        for gi in range(len(rb.kernel_size)):
            gru = getattr(rb, f"convgru{gi + 1}")

            H_, C_ = self.hidden, self.ctx_ch

            def loop_part(k):  # input channels [h | context | motion] -> [h | motion]
                k = k.detach().float()
                return torch.cat([k[:, :, :H_], k[:, :, H_ + C_:]], dim=2)

            def gru_a(gru=gru):
                k = torch.cat([loop_part(gru.convz.kernel), loop_part(gru.convr.kernel)], dim=3)
                return k, torch.zeros(2 * H_), (1, 1), gru.padding, hx_cs

            def gru_b(gru=gru):
                return loop_part(gru.convq.kernel), torch.zeros(H_), (1, 1), gru.padding, hx_cs

            def gru_ctx(gru=gru):  # context share of [z | r | q] + the gate biases (prologue, once)
                k = torch.cat([c.kernel.detach()[:, :, H_:H_ + C_] for c in (gru.convz, gru.convr, gru.convq)], dim=3)
                b = torch.cat([c.bias.detach() for c in (gru.convz, gru.convr, gru.convq)])
                return k.float(), b.float(), (1, 1), gru.padding, None

            self._reg(f"gru{gi}.a", gru_a)
            self._reg(f"gru{gi}.b", gru_b)
            self._reg(f"gru{gi}.ctx", gru_ctx)
        if self.has_mask:
            mp = m.mask_predictor

            def fh1():
                k = torch.cat([fh.conv1.kernel.detach(), mp.convrelu.layers_0.kernel.detach()], dim=3).float()
                b = torch.cat([fh.conv1.bias.detach(), mp.convrelu.layers_0.bias.detach()]).float()
                return k, b, (1, 1), (1, 1), None

            self._reg("fh1", fh1)
            self._reg("fh1.flow", conv_src(fh.conv1))  # final-only mode / split mask head: flow head alone
            self._reg("mask.convrelu", cna_src(mp.convrelu))
            self._reg("mask", conv_src(mp.conv))
        else:
            self._reg("fh1", conv_src(fh.conv1))

        def fh2_taps():  # (3,3,cin,2) -> (1,1,cin,18): out channel tap*2 + o
            k = fh.conv2.kernel.detach().float()
            cin = k.shape[2]
            k = k.reshape(9, cin, 2).permute(1, 0, 2).reshape(1, 1, cin, 18)
            return k, torch.zeros(18), (1, 1), (0, 0), None

        self._reg("fh2.taps", fh2_taps)

    # ------------------------------------------------------------- autotune
    def _conv(self, plan, spec: ConvSpec, x, N, H, W, y, x_alt=None, **kw):
        """Append one conv to ``plan``, choosing its tile config (autotuned).  ``x_alt``: the
        input of odd loop iterations (a state that ping-pongs between two buffers)."""
        args = conv_args(spec, x, N, H, W, y, **self._conv_kw(spec, x, N, H, W, y, kw))
        if x_alt is not None:
            plan.add_conv_alt(*args, x_alt)
        else:
            plan.add_conv(*args)

    def _conv_group(self, plan, a: tuple, b: tuple) -> bool:
        """Two independent STD-epilogue convs ``(spec, x, N, H, W, y, kw)`` as ONE grid
        (conv_igemm.h:conv_grouped_kernel) in the tile config tuned for the first, when a
        grouped launch serves that config; returns False (nothing added) otherwise."""
        kwa = self._conv_kw(*a[:6], a[6])
        cfg = kwa.get("cfg")
        if a[6].get("cfg") is None and self.autotune:
            # a measured config for the PAIR (tuned DB key "group" + both problems) beats the
            # first conv's own: profiles/r3_grouped_cfg_ab.txt
            (sa, xa, N, H, W, _), (sb, xb) = a[:6], b[:2]
            gkey = ("group", N * H * W, sa.cout, sa.kh, sa.kw, sa.cin8, xa.shape[-1], sb.cout, sb.kh, sb.kw, sb.cin8,
                    xb.shape[-1])
            gcfg = tunedb.peek(self.arch, gkey)
            name_a = next((k for k, v in self._specs.items() if v is sa), None)
            if gcfg in nat.GROUPED_CFGS and name_a not in self.cfg_override:
                cfg = gcfg
                kwa = dict(kwa, cfg=cfg)
                if name_a is not None:
                    self.chosen_cfgs[name_a] = cfg
        def fast(sp):   # binding.cpp build_conv: the FAST im2col loader (both convs must share it)
            taps = sp.kh * sp.kw
            return taps <= 32 and (taps == 1 or sp.cin8 % 64 == 0)

        if cfg not in nat.GROUPED_CFGS or fast(a[0]) != fast(b[0]):
            return False
        kwb = dict(b[6], cfg=cfg)
        name = next((k for k, v in self._specs.items() if v is b[0]), None)
        if name is not None:
            self.chosen_cfgs[name] = cfg
        ta, ia, aa = conv_args(*a[:6], **kwa)
        tb, ib, ab = conv_args(*b[:6], **kwb)
        plan.add_conv_group(ta, ia, aa, tb, ib, ab)
        return True

    def _conv_kw(self, spec: ConvSpec, x, N, H, W, y, kw):
        """``kw`` with the tile config of this conv (override / persisted / autotuned)."""
        if self.cfg_override and kw.get("cfg") is None:
            name = next((k for k, v in self._specs.items() if v is spec), None)
            if name in self.cfg_override:
                kw = dict(kw, cfg=self.cfg_override[name])
        if kw.get("epi") == EPI_TAPS and not self.autotune and kw.get("cfg") is None:
            kw = dict(kw, cfg=nat.TAPS_CFGS[0])
        if _fused_norm(kw) and not self.autotune and kw.get("cfg") is None:
            kw = dict(kw, cfg=_candidates(spec, kw, y)[0])
        if self.autotune and kw.get("cfg") is None:
            OH, OW = kw["out_hw"] if kw.get("out_hw") is not None else spec.out_hw(H, W)
            valid = _candidates(spec, kw, y)
            key = (N * OH * OW, spec.cout, spec.kh, spec.kw, spec.sh, spec.sw, spec.cin8, x.shape[-1],
                   kw.get("epi", EPI_STD), kw.get("bmap") is not None)
            # problems the halo kernel can run are keyed apart (decisions made before it existed
            # never timed it); a fused norm restricts the choice to the halo configs
            if any(c >= nat.HALO_CFG0 for c in valid):
                key = key + ("halo-norm" if _fused_norm(kw) else "halo",)
            cfg = _TUNE_CACHE.get(key + (str(self.device),))
            if cfg is None:
                cfg = tunedb.lookup(self.arch, key, valid)   # persisted decision (runtime/tunedb.py)
                if cfg is None:
                    cfg = _tune(spec, x, N, H, W, y, kw)
                    tunedb.record(self.arch, key, cfg)
                cfg = self._agree(cfg)
                _TUNE_CACHE[key + (str(self.device),)] = cfg
            kw = dict(kw, cfg=cfg)
        name = next((k for k, v in self._specs.items() if v is spec), None)
        if name is not None:
            self.chosen_cfgs[name] = kw.get("cfg")
        return kw

    # ------------------------------------------------------------- lowering
    def _encoder(self, st: _PlanState, plan, tag: str, enc: FeatureEncoder, x: torch.Tensor, N: int, H: int,
                 W: int, bt: str = ""):
        """Lower a FeatureEncoder up to (not including) its final 1x1 conv.  ``tag``
        names the conv specs ("fe"/"ce"), ``bt`` prefixes the buffers (batch part).
        Instance norms: a two-pass statistics op, then normalise + activation
        (+ residual).  Measured and dropped: the statistics fused into the conv
        kernels (per-tile partials re-read from L2 after the epilogue, only
        configs with one channel tile / image-aligned pixel tiles): 319-320 vs
        321-323 pairs/s; a one-launch statistics kernel with a last-block
        reduction: 0.9 ms/step slower (profiles/r2_pipelined_graph_ab.txt)."""
        inorm = enc.norm_kind == NORM_INSTANCE
        sp = self._specs
        bufs = st.bufs

        def alloc(name, shape, dtype=BF16):
            t = torch.zeros(shape, dtype=dtype, device=self.device)
            bufs[bt + name] = t
            return t

        def conv_raw(name, x, N, H, W, act=ACT_NONE, res=None, res_post=0, out_hw=None):
            s = sp[name]
            OH, OW = out_hw if out_hw is not None else s.out_hw(H, W)
            y = alloc(name + ".y", (N, OH, OW, s.cout))
            self._conv(plan, s, x, N, H, W, y, act=act, res=res, res_post=res_post, out_hw=out_hw)
            return y, OH, OW

        def halo_fusable(name) -> bool:
            return self.halo_norm and bool(nat.halo_cfgs_for(sp[name], {}))

        def conv_stats(name, x, N, H, W, in_stats=None, in_res=None, in_res_stats=None, xn=None):
            """A halo 3x3 conv that writes its output's channel-statistics partials (reduced
            by one small launch) and, given ``in_stats``, instance-normalises + relus its raw
            input as it loads it (no channel_stats pass over the output, no norm_act pass
            over the input); with ``in_res`` (+ its stats) the input is a residual block's
            output relu(IN(x) + [IN](res)), built on the fly and written to ``xn``."""
            s = sp[name]
            y = alloc(name + ".y", (N, H, W, s.cout))
            nb_max = nat.halo_max_blocks(s.cin8, H, W)
            part = alloc(name + ".part", (N, nb_max, s.cout, 2), F32)
            # a residual block's output: relu(res + relu(IN(raw))) (model.py:171-180), in_relu bits 0 + 1
            kw = dict(stats_part=part, in_stats=in_stats, in_relu=3 if in_res is not None else 1, in_hw=H * W,
                      in_res=in_res, in_res_stats=in_res_stats, xn=xn)
            kw = self._conv_kw(s, x, N, H, W, y, kw)
            if kw.get("cfg") is None or kw["cfg"] < nat.HALO_CFG0:   # an override chose another kernel
                return None
            plan.add_conv(*conv_args(s, x, N, H, W, y, **kw))
            c = nat.halo_cfg(kw["cfg"])
            nb = -(-H // c[4]) * -(-W // c[5]) * c[2]
            st_ = alloc(name + ".stats", (N, s.cout, 2), F32)
            plan.add_stats_final([part, st_], [N, nb, s.cout])
            return y, st_

        def stem(act=ACT_NONE):
            if x.shape[-1] == 16:   # space-to-depth input (prep s2d): the 4x4 / stride-1 form of the stem
                return conv_raw(f"{tag}.stem_s2d", x, N, H // 2, W // 2, act=act, out_hw=(H // 2, W // 2))
            return conv_raw(f"{tag}.stem", x, N, H, W, act=act)

        def stats(name, y, N, HW, C):
            t = alloc(name + ".stats", (N, C, 2), F32)
            plan.add_stats([y, t], [N, HW, C])
            return t

        def norm_act(name, x, sx, res=None, sr=None, mode_r=0, relu=3):
            N_, H_, W_, C = x.shape
            y = alloc(name + ".n", (N_, H_, W_, C))
            plan.add_norm_act([x, sx, None, None, res, sr, None, None, y],
                              [1, mode_r, N_, H_ * W_, C, relu], 1e-5)
            return y

        # Instance-norm encoders keep a block's output lazy -- (raw, stats, residual, its stats)
        # -- and build it inside the next block's first conv when that is a stride-1 halo conv
        # (which also writes it out for the next residual); otherwise one norm_act pass
        # materialises it (RaftEngine.HALO_NORM = False: always).
        pend = None

        def materialise(p_):
            return norm_act(p_["name"], p_["raw"], p_["s"], res=p_["res"], sr=p_["rs"],
                            mode_r=1 if p_["rs"] is not None else 0, relu=3 if p_["res"] is not None else 2)

        if inorm:
            y, H, W = stem()
            pend = dict(name=f"{tag}.stem", raw=y, s=stats(f"{tag}.stem", y, N, H * W, y.shape[-1]), res=None, rs=None)
            x = None
        else:
            x, H, W = stem(act=ACT_RELU)
        for li in (1, 2, 3):
            layer = getattr(enc, f"layer{li}")
            for bi in range(layer.n):
                blk = getattr(layer, f"layers_{bi}")
                pre = f"{tag}.l{li}.b{bi}"
                names = ["convnormrelu1", "convnormrelu2"] + (["convnormrelu3"] if isinstance(blk, BottleneckBlock) else [])
                has_ds = blk.stride != (1, 1)
                if inorm:
                    h_, w_ = H, W
                    y, ys = x, None   # ys: stats of a raw conv output y still to be normalised
                    j0 = 0
                    c1 = f"{pre}.{names[0]}"
                    if (pend is not None and self.halo_res and not has_ds and halo_fusable(c1) and sp[c1].out_hw(h_, w_) == (h_, w_)
                            and pend["raw"].shape[-1] == sp[c1].cin8):
                        xb = alloc(f"{pre}.x", tuple(pend["raw"].shape))
                        fused = conv_stats(c1, pend["raw"], N, h_, w_, in_stats=pend["s"], in_res=pend["res"],
                                           in_res_stats=pend["rs"], xn=xb)
                        if fused is not None:
                            x, pend = xb, None
                            (y, ys), j0 = fused, 1
                    if pend is not None:
                        x, pend = materialise(pend), None
                        y = x
                    for j in range(j0, len(names)):
                        nm = names[j]
                        cname = f"{pre}.{nm}"
                        fused = None
                        if halo_fusable(cname) and sp[cname].out_hw(h_, w_) == (h_, w_):
                            fused = conv_stats(cname, y, N, h_, w_, in_stats=ys)
                        if fused is not None:
                            yr, s = fused
                        else:
                            if ys is not None:
                                y = norm_act(f"{pre}.{names[j - 1]}", y, ys, relu=2)
                            yr, h_, w_ = conv_raw(cname, y, N, h_, w_)
                            s = stats(cname, yr, N, h_ * w_, yr.shape[-1])
                        if j + 1 < len(names):
                            y, ys = yr, s
                        else:
                            last, last_s = yr, s
                    if has_ds:
                        dr, _, _ = conv_raw(f"{pre}.downsample", x, N, H, W)
                        ds = stats(f"{pre}.downsample", dr, N, h_ * w_, dr.shape[-1])
                        pend = dict(name=f"{pre}.out", raw=last, s=last_s, res=dr, rs=ds)
                    else:
                        pend = dict(name=f"{pre}.out", raw=last, s=last_s, res=x, rs=None)
                    x = None
                    if not self.halo_norm:
                        x, pend = materialise(pend), None
                    H, W = h_, w_
                else:
                    res = x
                    if has_ds:
                        res, _, _ = conv_raw(f"{pre}.downsample", x, N, H, W)
                    y = x
                    h_, w_ = H, W
                    for j, nm in enumerate(names):
                        if j + 1 < len(names):
                            y, h_, w_ = conv_raw(f"{pre}.{nm}", y, N, h_, w_, act=ACT_RELU)
                        else:
                            y, h_, w_ = conv_raw(f"{pre}.{nm}", y, N, h_, w_, act=ACT_RELU, res=res, res_post=1)
                    x, H, W = y, h_, w_
        if pend is not None:
            x = materialise(pend)
        return x, H, W

    # lanes pay off once the per-iteration kernels fill the chip: measured on
    # MI355X (raft_large, 440x1024, 32 iters) the lane schedule is 17-21 % slower
    # at batch 1, equal at batch 2 and 2 % faster at batch 4 than one in-order
    # lane.  In final-only mode the loop has no mask head to overlap, only the
    # flow-feature convs: one lane measured 13.1 vs 12.7-24.9 ms (lanes,
    # schedule-dependent run to run) at batch 4.  Without a mask predictor
    # (raft_small) one lane measured 562 vs 528 pairs/s at batch 4.
    AUTO_STREAMS_MIN_BATCH = 4

    def _init_cp(self, cp_group) -> None:
        self.cp = cp_group is not None and cp_group is not False
        self.cp_group = None if cp_group is True else cp_group
        self.cp_rank, self.cp_world = 0, 1
        if self.cp:
            import torch.distributed as dist

            if dist.is_available() and dist.is_initialized():
                self.cp_rank = dist.get_rank(self.cp_group)
                self.cp_world = dist.get_world_size(self.cp_group)

    def _agree(self, v: int) -> int:
        """Context-parallel ranks build the same plan, so every tuning decision is taken
        from rank 0: ranks timing the candidates themselves (on a shared GPU, or on GPUs
        of different clocks) could pick different tile configs, i.e. flows that differ in
        bf16 rounding between ranks."""
        if not self.cp or self.cp_world == 1:
            return v
        import torch.distributed as dist

        dev = self.device if dist.get_backend(self.cp_group) == "nccl" else torch.device("cpu")
        t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        src = dist.get_global_rank(self.cp_group, 0) if self.cp_group is not None else 0
        dist.broadcast(t, src=src, group=self.cp_group)
        return int(t.item())

    def _cp_slabs(self, h: int):
        from ..parallel.cp import row_slabs

        return row_slabs(h, self.cp_world)

    def _gather_corr(self, st: _PlanState) -> None:
        """All-gather every rank's looked-up correlation features ``local``
        (B, nq, C) into the full-map ``corr`` (B*h*w, C) (stream-ordered with
        the plan: the eager plan forks from / joins to the current stream)."""
        cp = st.cp
        local, corr, slabs, w = cp["local"], cp["corr"], cp["slabs"], cp["w"]
        B = local.shape[0]
        full = corr.view(B, -1, corr.shape[-1])
        if self.cp_world == 1:
            full[:, : local.shape[1]].copy_(local)
            return
        import torch.distributed as dist

        parts = cp.get("parts")
        if parts is None:
            parts = cp["parts"] = [torch.empty_like(local) for _ in slabs]
        dist.all_gather(parts, local, group=self.cp_group)
        for (r0, r1), part in zip(slabs, parts):
            full[:, r0 * w:r1 * w].copy_(part[:, : (r1 - r0) * w])

    def _forward_cp(self, st: _PlanState, n_iters: int) -> None:
        plan = st.plan
        plan.run_segment(0, 0)
        for it in range(n_iters):
            plan.run_segment(1, it)
            self._gather_corr(st)
            plan.run_segment(3, it)
        plan.run_segment(2, n_iters)

    def _lanes_ok(self, all_iters: bool) -> bool:
        """The lane schedule needs a mask head to overlap (every iteration
        upsampled) and the FlowHead taps epilogue (a 256-channel conv1)."""
        return (all_iters and self.has_mask and self._taps_epi_w is not None and self._convex_w is not None
                and self._specs["fh1.flow"].cout == 256)

    def _halo_geom(self):
        """(hd, [(mode, axis) per ConvGRU stage]) when the halo-tiled fused ConvGRU
        (gru_halo.hip) serves this update block, else None: raft_large's 1x5 + 5x1 stages
        (hidden 128, [h | motion | flow] = 256 loop channels) or raft_small's single 3x3
        GRU (hidden 96, 192 loop channels); bf16 bias map (``gate_dtype``)."""
        rb = self.model.update_block.recurrent_block
        ks = [tuple(k) for k in rb.kernel_size]
        if self.gate_dtype != torch.bfloat16 or self.gate_cs < 3 * self.hidden:
            return None
        if self.hidden == 128 and self.hx_cs == 256 and ks == [(1, 5), (5, 1)]:
            return 128, [(0, 0), (0, 1)]
        if self.hidden == 96 and self.hx_cs == 192 and ks == [(3, 3)]:
            return 96, [(1, 0)]
        return None

    def _gru_path(self, B: int, h: int, w: int) -> str:
        """ConvGRU lowering of a plan: "halo" (gru_halo.hip: one launch per stage, any map
        size and batch), "fused" (gru_fused.hip: whole-row tiles, raft_large at >= 3/4 of
        the CUs' worth of rows) or "unfused" (two implicit-GEMM launches per stage).
        The class attribute ``GRU = "halo" | "fused" | "unfused"`` forces one (where it applies)."""
        env = self.GRU
        assert env in ("auto", "halo", "fused", "unfused"), env
        if env == "unfused":
            return "unfused"
        # auto: the whole-row kernel where it fills the GPU (its own >= 3/4-of-the-CUs rule:
        # raft_large at batch >= 4 on Sintel frames, measured 339 vs 317-334 pairs/s for the
        # halo kernel in the lane schedule, profiles/r4_gru_lowering_ab.txt), the halo kernel
        # everywhere else (batch 1: 215 vs 191 FPS; raft_small; any map size)
        if env in ("auto", "fused") and self._gru_fused_ok(B, h, w):
            return "fused"
        if env in ("auto", "halo") and self._halo_geom() is not None:
            return "halo"
        return "unfused"

    def _halo_tile(self, gi: int, mode: int, axis: int, B: int, h: int, w: int, ops_args) -> Tuple[int, int, int, int]:
        """Tile of one gru_halo stage: the persisted decision (tuned DB key "gru_halo") or
        the fastest candidate (ops/native.py:gru_halo_candidates) timed on the plan's own
        buffers (the prologue re-initialises everything the trial launches write)."""
        cands = nat.gru_halo_candidates(self.hidden, mode, axis, B, h, w)
        enc = {c[0] * 1000000 + c[1] * 1000 + c[2] * 10 + c[3]: c for c in cands}
        key = ("gru_halo", self.hidden, mode, axis, B, h, w)
        if not self.autotune or len(cands) == 1 or self.device.type != "cuda":
            return cands[0]
        code = _TUNE_CACHE.get(key + (str(self.device),))
        if code is None:
            code = tunedb.lookup(self.arch, key, set(enc))
        if code is None:
            t, base = ops_args
            best = None
            for c, tile in enc.items():
                nat.ops().gru_halo(t, base + list(tile))
                s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s_.record()
                for _ in range(5):
                    nat.ops().gru_halo(t, base + list(tile))
                e_.record()
                e_.synchronize()
                el = s_.elapsed_time(e_)
                if best is None or el < best[0]:
                    best = (el, c)
            code = best[1]
            tunedb.record(self.arch, key, code)
        code = self._agree(code)
        _TUNE_CACHE[key + (str(self.device),)] = code
        self.chosen_cfgs[f"gru{gi}.halo"] = code
        return enc[code]

    def _gru_fused_ok(self, B: int, h: int, w: int) -> bool:
        """The fused ConvGRU kernel (gru_fused.hip) serves raft_large's update block:
        hidden 128, [h | motion | flow] = 256 loop channels, a 1x5 then a 5x1 stage,
        and tiles (image rows / column pairs) that fit 128 pixels.  It launches one
        workgroup per tile, so it is used when both stages have >= 3/4 as many tiles
        as the GPU has CUs: measured on MI355X at 440x1024, batch 4 (220 / 256 tiles)
        333-335 vs 320 pairs/s; batch 1 (55 / 64 tiles) 139 vs 158 FPS for the
        two-launch implicit-GEMM path (profiles/r3_gru_fused_ab.txt).
        ``GRU = "fused"`` forces it where it fits."""
        env = "1" if self.GRU == "fused" else "auto"
        rb = self.model.update_block.recurrent_block
        ks = [tuple(k) for k in rb.kernel_size]
        if (self.hidden != 128 or self.hx_cs != 256 or self.gate_cs < 384 or ks != [(1, 5), (5, 1)]
                or self.gate_dtype != torch.bfloat16):
            return False
        tiles = min(nat.gru_fused_tiles(B, h, w, 0), nat.gru_fused_tiles(B, h, w, 1))
        return tiles > 0 and (env == "1" or tiles >= 3 * nat.NUM_CUS // 4)

    def uses_lanes(self, B: int, all_iters: bool = True) -> bool:
        """Whether the plan for batch ``B`` runs the model's branches on several
        lanes (``streams`` / its "auto" rule).  Graph-pipelined steps
        (:meth:`pipelined`) measured faster only on one-lane plans: batch 1
        145 -> 157 pairs/s, raft_small batch 4 559 -> 602, final-only 326 -> 346;
        with lanes (raft_large batch 4) 319 -> 289 (profiles/r2_pipelined_graph_ab.txt)."""
        if self.cp or not self._lanes_ok(all_iters):
            return False
        if self.streams_mode != "auto":
            return bool(self.streams_mode)
        nb = B // self.split if (self.split > 1 and B % self.split == 0) else B
        return nb >= self.AUTO_STREAMS_MIN_BATCH

    def _build(self, B: int, H: int, W: int, n_iters: int, all_iters: bool = True,
               src: Optional[Tuple[int, int, int, int]] = None) -> _PlanState:
        on = self.uses_lanes(B, all_iters)
        self.streams = on
        self.mask_head = "split" if on else "fused"
        h, w = H // 8, W // 8
        L = self.num_levels
        min_sz = 2 * (2 ** (L - 1))
        assert h >= min_sz and w >= min_sz, (
            f"Feature maps are too small to be down-sampled by the correlation pyramid: need >= {min_sz}, got {(h, w)}; "
            f"input images should be at least {8 * min_sz}.")
        dev = self.device
        parts = self.split if (self.split > 1 and B % self.split == 0 and not self.cp) else 1
        nb = B // parts
        # Each part is an independent forward with its own Plan; with use_graph
        # their captures are copied into ONE hipGraph (Plan.merge_*), so the
        # parts' kernels fill each other's idle CUs.
        plans = [nat.new_plan() for _ in range(parts)]
        st = _PlanState(plan=plans[0], plans=plans, n_iters=n_iters, src=src)
        if src is not None:   # raw frames: the prep kernel normalises + pads them (K14)
            st.inp1 = torch.zeros((B, src[0], src[1], 3), dtype=torch.uint8, device=dev)
            st.inp2 = torch.zeros((B, src[0], src[1], 3), dtype=torch.uint8, device=dev)
        else:
            st.inp1 = torch.zeros((B, H, W, 3), dtype=F32, device=dev)
            st.inp2 = torch.zeros((B, H, W, 3), dtype=F32, device=dev)
        st.out = torch.zeros((n_iters if all_iters else 1, B, H, W, 2), dtype=F32, device=dev)
        st.slot_ptr = st.out.data_ptr()
        st.out_slot = torch.tensor([st.slot_ptr], dtype=torch.int64, device=dev)
        lanes = (0, 1, 2) if on else (0, 0, 0)
        for part, plan in enumerate(plans):
            self._build_part(st, plan, part * nb, nb, H, W, n_iters, f"p{part}.", lanes, 0, all_iters)
            plan.set_lane(0)
            plan.set_segment(2)
        return st

    def _build_part(self, st: _PlanState, plan, b0: int, B: int, H: int, W: int, n_iters: int, pt: str,
                    lanes: Tuple[int, int, int], ev0: int, all_iters: bool = True):
        """Lower one forward over images [b0, b0 + B) onto ``plan`` using lanes
        (main, side, side2) and events ev0 .. ev0 + 8.

        Three loop schedules (``model.py:495-510`` per iteration):

        * lanes (``main != side``): the critical lane runs lookup (+ the
          previous iteration's flow update) -> convcorr1/2 -> motion conv ->
          2 x ConvGRU -> FlowHead conv1 with the taps epilogue; the mask lane,
          forked after the lookup, runs the flow-feature convs of this
          iteration and the mask head + convex upsampling of the previous one
          (deferred ops, skipped in iteration 0).  Three cross-lane edges per
          iteration (E_FH, E_FLOW, E_MASK): each costs ~6-12 us in a captured
          graph on this ROCm.
        * one lane, every iteration upsampled: the same deferral in order:
          lookup (+ update), flow features, upsampling of iteration i-1,
          correlation / motion / GRU convs, FlowHead conv1 (fused with the mask
          predictor's 3x3 conv as one 128 -> 512 GEMM when there is a mask
          head) + the taps GEMM.
        * final-only (``all_iters=False``, serving): the loop runs the flow head
          alone; the mask head + x8 upsampling run once in the epilogue on the
          final hidden state and flow."""
        m = self.model
        dev = self.device
        bufs = st.bufs
        sp = self._specs
        h, w = H // 8, W // 8
        M = B * h * w
        L = self.num_levels

        def alloc(name, shape, dtype=BF16):
            t = torch.zeros(shape, dtype=dtype, device=dev)
            bufs[pt + name] = t
            return t

        inp1 = st.inp1[b0:b0 + B]
        inp2 = st.inp2[b0:b0 + B]
        out = st.out[:, b0:b0 + B]
        out_off = (out.data_ptr() - st.out.data_ptr()) // 4   # in floats, from the slot's base

        # ---------------- prologue: encoders + correlation pyramid
        # lanes: 0 = feature encoder (image 1) + correlation pyramid, 1 = context
        # encoder, 2 = feature encoder (image 2)
        E_PREP, E_CTX, E_FLOW, E_FH, E_MASK, E_FE2 = range(ev0, ev0 + 6)
        main, side, side2 = lanes
        lanes_on = main != side
        # the prologue's branches (context encoder, feature encoder per image) run on their own
        # lanes even when the loop runs on one, up to Sintel-size batch 4 worth of pixels.  At
        # batch 1 ("auto") the feature encoder runs as ONE batch-2 chain next to the context
        # encoder's lane (round 6, profiles/r6_prolanes_ab.txt, r6_ce_lane_b1_ab.txt): per-image
        # lanes of its ~70 short kernels only added dispatch cost (the replayed branches ran one
        # after another, r6_graph_branches.txt); raft_small sync 297 -> 330-344 pairs/s, its
        # 12-iteration stream 662-758 -> 782-805, raft_large sync 216 -> 218-223.  (1088x1920
        # frames: 67.6 -> 63.7 with lanes, round 4, so off there.)
        # PRO_LANES = "off": never, "on": always (per-image feature-encoder lanes at batch 1 too).
        pl = self.PRO_LANES
        assert pl in ("auto", "on", "off"), pl
        pro_on = pl == "on" or (pl == "auto" and B * h * w <= 4 * 55 * 128)
        p_main, p_side, p_side2 = lanes if lanes_on or self.cp or not pro_on else (main, 1, 2)
        p_on = p_main != p_side
        # the per-image feature-encoder split (lane 2) -- never at batch 1 under "auto", also not in
        # a pipelined slot's multi-lane plan, so that its kernels (tile configs of the batch-2
        # chain) and results equal the synchronous forward's bit for bit
        fe_split = p_on and not (pl == "auto" and B == 1)

        def lane(l):
            plan.set_lane(l)

        plan.set_segment(0)
        lane(p_main)
        hx = alloc("hx", (M, self.hx_cs))
        qx = alloc("qx", (M, self.hx_cs))
        h32 = alloc("h32", (M, self.hidden), F32)
        zb = alloc("z", (M, self.hidden), self.gate_dtype)
        # bf16 flow for the flow branch: compact 2 channels for the 2-channel conv
        # kernel (4 taps = one 16-B load), 8-channel rows for the implicit GEMM
        flow8 = alloc("flow8", (M, 2 if self._cf1_w is not None else 8))
        coords = alloc("coords", (M, 2), F32)
        flow32 = alloc("flow32", (M, 2), F32)
        for t in (hx, qx, flow8, flow32):
            plan.add_memset([t])
        s2d = "fe.stem_s2d" in sp and "ce.stem_s2d" in sp and H % 2 == 0 and W % 2 == 0
        x0 = alloc("x0", (2 * B, H // 2, W // 2, 16) if s2d else (2 * B, H, W, 8))
        if st.src is not None:   # uint8 frames: normalise + replicate pad + layout in one kernel (K14)
            H0, W0, pad_t, pad_l = st.src   # (pt is this part's buffer prefix)
            plan.add_prep([inp1, inp2, x0, u8_table(dev)], [B, H, W, int(s2d), H0, W0, pad_t, pad_l])
        elif s2d:   # 2x2 space-to-depth images for the 4x4 form of the 7x7 / stride-2 stems
            plan.add_prep([inp1, inp2, x0], [B, H, W, 1])
        else:
            plan.add_prep([inp1, inp2, x0], [B, H, W])
        plan.add_record(E_PREP)

        lane(p_side)
        plan.add_wait(E_PREP)
        ctxf, ch_, cw_ = self._encoder(st, plan, "ce", m.context_encoder, x0[:B], B, H, W, bt=pt)
        assert (ch_, cw_) == (h, w), "The context encoder should downsample H and W by 8"
        # [tanh(h) | relu(context)] (model.py:582-584); h also as fp32 state
        ce_out = alloc("ce_out", (M, round_up(self.hidden + self.ctx_ch, 8)))
        self._conv(plan, sp["ce.conv"], ctxf, B, h, w, ce_out, act=ACT_SPLIT_TANH_RELU, split=self.hidden,
                   h32=h32, hidden=self.hidden)
        plan.add_copy_channels([ce_out, hx], [0, 0, M, self.hidden])
        # loop-invariant context share of every GRU gate (+ gate biases)
        gbias = []
        for gi in range(len(m.update_block.recurrent_block.kernel_size)):
            gb = alloc(f"gru{gi}.cbias", (M, self.gate_cs), self.gate_dtype)
            self._conv(plan, sp[f"gru{gi}.ctx"], ce_out, B, h, w, gb, x_coff=self.hidden)
            gbias.append(gb)
        plan.add_init_coords([coords], [B, h, w])
        plan.add_record(E_CTX)

        fmap = alloc("fmap", (2 * B, h, w, self.fmap_ch))
        if self.fe_external:
            lane(p_main)   # fmap is written before each replay (RaftEngineMixed._pre_launch)
        elif fe_split:
            # the feature encoder of image2 on a third lane, concurrent with image1's
            # (and the context encoder): per-image instance norms, so the halves are
            # exact, and the sequential encoder chain that gates the correlation
            # pyramid is half as long
            lane(p_side2)
            plan.add_wait(E_PREP)
            featb, _, _ = self._encoder(st, plan, "fe", m.feature_encoder, x0[B:], B, H, W, bt=pt + "fe2.")
            self._conv(plan, sp["fe.conv"], featb, B, h, w, fmap[B:])
            plan.add_record(E_FE2)
            lane(p_main)
            feat, fh_, fw_ = self._encoder(st, plan, "fe", m.feature_encoder, x0[:B], B, H, W, bt=pt)
            assert (fh_, fw_) == (h, w), "The feature encoder should downsample H and W by 8"
            self._conv(plan, sp["fe.conv"], feat, B, h, w, fmap[:B])
            plan.add_wait(E_FE2)
        else:
            lane(p_main)
            feat, fh_, fw_ = self._encoder(st, plan, "fe", m.feature_encoder, x0, 2 * B, H, W, bt=pt)
            assert (fh_, fw_) == (h, w), "The feature encoder should downsample H and W by 8"
            self._conv(plan, sp["fe.conv"], feat, 2 * B, h, w, fmap)
        # bf16 levels of /16-wide maps: levels 0 / 1 in the blocked layout (one
        # pyramid tile per block: whole-line writes, 2 x 2 blocks per lookup window)
        blocked = int(self.corr_dtype == BF16 and w % 16 == 0 and (h * w) % 8 == 0 and not self.cp)
        self.corr_blocked = bool(blocked)
        # context parallelism: this rank's pyramid holds the query rows [r0, r1) only
        slabs = self._cp_slabs(h) if self.cp else [(0, h)]
        r0, r1 = slabs[self.cp_rank]
        nq = (r1 - r0) * w
        levels = []
        hl, wl = h, w
        for l in range(L):
            shape = (M, -(-h // 8) * (8 >> l), -(-w // 16) * (16 >> l)) if blocked and l < 2 else (B * nq, hl, wl)
            levels.append(alloc(f"corr.l{l}", shape, self.corr_dtype))
            hl //= 2
            wl //= 2
        scale = 1.0 / float(self.fmap_ch) ** 0.5
        if self.cp:
            for b in range(B):
                plan.add_corr([fmap[b, r0:r1], fmap[B + b]] + [v[b * nq:(b + 1) * nq] for v in levels] + [None] * (4 - L),
                              [1, h, w, self.fmap_ch, L, nq, 0], scale)
        else:
            # blocked 2: the persistent pyramid kernel (corr_pyr.hip) also at batch 1 -- not in a
            # pipelined slot, whose graph runs it next to the previous pair's loop (there the
            # short-lived tiles interleave better: b1 stream 227 vs 200-204 FPS, round 4)
            bl = 2 if (blocked and self.CORR_PERSIST_B1 and not getattr(self, "_slot_build", False)) else blocked
            plan.add_corr([fmap[:B], fmap[B:]] + levels + [None] * (4 - L), [B, h, w, self.fmap_ch, L, h * w, bl],
                          scale)
        plan.add_wait(E_CTX)

        # ---------------- loop body: one refinement iteration (model.py:495-510)
        me = m.update_block.motion_encoder
        cl, fl = me.corr_layers, me.flow_layers
        corr = alloc("corr", (M, self.corr_cs))
        cf = alloc("cf", (M, cl[-1] + fl[-1]))
        f1 = alloc("f1", (M, fl[0]))
        c1 = alloc("c1", (M, cl[0])) if len(cl) == 2 else None
        taps = alloc("fh2.taps", (M, 24), F32)
        stride = st.out.shape[1] * H * W * 2  # one iteration of the full-batch output
        # mask predictor's 3x3 conv on its own (mask lane / context parallel), else fused into FlowHead conv1
        split_mask = lanes_on or self.cp
        # FlowHead conv1 of the loop: alone (lanes / final-only / no mask head) or
        # fused with the mask predictor's 3x3 conv (one lane, every iteration upsampled)
        s1 = sp["fh1"] if (self.has_mask and all_iters and not split_mask) else sp["fh1.flow"] if self.has_mask else sp["fh1"]
        # the taps epilogue: the 256 FlowHead features never leave the CU
        taps_epi = self._taps_epi_w is not None and s1.cout == 256
        fm = None if taps_epi else alloc("fm", (M, round_up(s1.cout, 8)))
        mfeat = (alloc("mfeat", (M, round_up(sp["mask.convrelu"].cout, 8)))
                 if self.has_mask and (split_mask or not all_iters) else None)
        mask = alloc("mask", (M, 576)) if self.has_mask and self._convex_w is None else None
        # ConvGRU lowering: "halo" (gru_halo.hip, one launch per stage at any size / batch),
        # "fused" (gru_fused.hip, whole-row tiles) or "unfused" (EPI_GRU_A / EPI_GRU_B convs)
        gru_path = self._gru_path(B, h, w)
        if gru_path == "fused" and self.cp:
            gru_path = "unfused"
        self.gru_path = gru_path
        ngru = len(m.update_block.recurrent_block.kernel_size)
        # the halo kernel cannot update h in place (neighbouring tiles read it): raft_large's
        # stage 1 writes h' into qx, stage 2 reads it there and writes hx; raft_small's single
        # stage ping-pongs h between hx (read on even iterations) and qx (odd), and its FlowHead
        # reads the buffer the stage just wrote
        halo_pp = gru_path == "halo" and ngru == 1
        # qx's [motion | flow] part is read only by the unfused GRU-B and the ping-pong
        qx_x = gru_path != "halo" or halo_pp
        # with the mask lane, the mask head reads h from its own copy `hm` (written by the last
        # stage), so the first stage can replace h in hx while the mask lane still runs
        # raft_small's ping-pong stage with a mask head (an injected MaskPredictor) also writes the copy:
        # its h' alternates between qx and hx, so the mask head (final-only epilogue, context parallel,
        # mask lane) reads hm instead of a buffer that holds h' only on every other iteration
        hm = (alloc("hm", (M, self.hidden))
              if gru_path != "unfused" and self.has_mask and (lanes_on or halo_pp) else None)
        # Parity-buffered mask-lane operands (gru_fused + convex head, MASK_PARITY = True): the last
        # GRU stage writes h into hm / hm2 and the update writes the flow into flow32 / flow32b by
        # iteration parity, so iteration i+1 never overwrites what the lane still reads for iteration
        # i; the lane's next read of a buffer is ordered by the E_FLOW join of the iteration after,
        # and the per-iteration E_MASK join (a ~10 us cross-stream graph edge) goes away.  Measured
        # slower at batch 4 (359-365 vs 372 pairs/s, profiles/r4_mask_parity_ab.txt): unjoined, the
        # mask head overlaps the ConvGRU stages (48 -> 54-56 us each) instead of the motion encoder.
        parity = (hm is not None and gru_path == "fused" and self._convex_w is not None
                  and self.MASK_PARITY)
        hm2 = alloc("hm2", (M, self.hidden)) if parity else None
        flow32b = alloc("flow32b", (M, 2), F32) if parity else None

        # one-lane schedule: the flow conv + the previous iteration's upsampling as one grid (merged.hip)
        c1k = me.convflow1.layers_0.kernel
        merged_up = (self._cf1_w is not None and tuple(c1k.shape[:2]) == (7, 7) and not self.cp
                     and (not self.has_mask or (self._convex_w is not None and fm is not None))
                     and self.MERGED_UP)

        def flow_features():
            if self._cf1_w is not None:
                c = me.convflow1.layers_0
                kh, kw_, _, co = c.kernel.shape
                plan.add_conv_direct([flow8, self._cf1_w, self._cf1_b, f1],
                                     [B, h, w, 2, kh, kw_, c.padding[0], c.padding[1], co, 1, 0])
            else:
                self._conv(plan, sp["me.convflow1"], flow8, B, h, w, f1, act=ACT_RELU)
            self._conv(plan, sp["me.convflow2"], f1, B, h, w, cf, y_coff=cl[-1], act=ACT_RELU)

        def flow_head():
            """FlowHead conv1 (+ conv2 as per-pixel tap partials into ``taps``)."""
            if taps_epi:
                self._conv(plan, s1, hx, B, h, w, taps, act=ACT_RELU, epi=EPI_TAPS, tapw=self._taps_epi_w)
                return
            if halo_pp:   # h' of even iterations is in qx, of odd ones in hx
                self._conv(plan, s1, qx, B, h, w, fm, x_alt=hx, act=ACT_RELU)
            else:
                self._conv(plan, s1, hx, B, h, w, fm, act=ACT_RELU)
            if self._taps_w is not None:   # skinny GEMM kernel (flowhead.hip), N = 18
                plan.add_taps_gemm([fm, self._taps_w, taps], [M, self.fh_hidden, 0])
            else:
                self._conv(plan, sp["fh2.taps"], fm, B, h, w, taps)

        def flow_update():
            """``coords1 += delta`` (model.py:505) from the taps; flow into hx / qx / flow8."""
            plan.add_flow_taps([taps, self._fh2_b, coords, flow32, hx, qx if qx_x else None, flow8]
                               + ([flow32b] if parity else []), [B, h, w, self.flow_off, self.flow_off])

        def upsample(stride, mask_from_fm: bool):
            """x8 upsampling of flow32 into the output (model.py:508): convex with
            the mask head (its 3x3 conv from hx, or the fused FlowHead conv1's
            second half in ``fm``), else bilinear."""
            if not self.has_mask:
                plan.add_upsample_bilinear([flow32, out, st.out_slot], [B, h, w, stride, out_off])
                return
            if mask_from_fm:
                feat_, coff = fm, self.fh_hidden
            else:
                self._conv(plan, sp["mask.convrelu"], hm if hm is not None else hx, B, h, w, mfeat, act=ACT_RELU,
                           x_alt=hm2)
                feat_, coff = mfeat, 0
            if self._convex_w is not None:
                plan.add_convex_head([feat_, self._convex_w, self._convex_b, flow32, out, st.out_slot]
                                     + ([flow32b] if parity else []),
                                     [B, h, w, coff, stride, 0, out_off], m.mask_predictor.multiplier)
            else:   # generic mask head (an injected MaskPredictor): 1x1 conv + convex upsampling
                st.slot_ok = False
                self._conv(plan, sp["mask"], feat_, B, h, w, mask, x_coff=coff, alpha=m.mask_predictor.multiplier)
                plan.add_upsample_convex([mask, flow32, out], [B, h, w, stride])

        def lookup(with_update: bool):
            upd = [taps, self._fh2_b, flow32, hx, qx if qx_x else None, flow8] if with_update else []
            if with_update and parity:
                upd.append(flow32b)   # t[12]: the odd iterations' flow
            extra = [self.flow_off, self.flow_off] if with_update else []
            plan.add_lookup([coords, corr] + levels + [None] * (4 - L) + upd,
                            [L, B, h, w, self.radius, h * w, blocked] + extra)

        # the one-lane merged grid also runs convcorr1 (1x1, K 324 -> 352; merged.hip)
        c1_merged = (merged_up and self.has_mask and len(cl) == 2 and self._cc1_w is not None
                     and self._cc1_kpad == 352)

        def motion_and_gru(wait_flow: bool, wait_mask: bool, flow2: bool = False):
            """``flow2``: convflow2 (the flow branch's second conv) is added here, as one grid
            with the last correlation conv when a grouped launch serves its tile config
            (conv_grouped_kernel; CONV_GROUP = False keeps them separate launches)."""
            if len(cl) == 2:
                if flow2 and c1_merged:
                    pass                      # ran in the flow conv's merged grid
                elif self._cc1_w is not None:   # LDS-resident-weight 1x1 kernel (conv1x1.hip)
                    plan.add_conv1x1([corr, self._cc1_w, self._cc1_b, c1],
                                     [M, self.corr_cs, self._cc1_kpad, cl[0], ACT_RELU, 0])
                else:
                    self._conv(plan, sp["me.convcorr1"], corr, B, h, w, c1, act=ACT_RELU)
                last = (sp["me.convcorr2"], c1, B, h, w, cf, dict(act=ACT_RELU))
            else:
                last = (sp["me.convcorr1"], corr, B, h, w, cf, dict(act=ACT_RELU))
            fl2 = (sp["me.convflow2"], f1, B, h, w, cf, dict(y_coff=cl[-1], act=ACT_RELU))
            if not (flow2 and self.CONV_GROUP and self._conv_group(plan, last, fl2)):
                if flow2:
                    self._conv(plan, *fl2[:6], **fl2[6])
                self._conv(plan, *last[:6], **last[6])
            if wait_flow:
                plan.add_wait(E_FLOW)
            self._conv(plan, sp["me.conv"], cf, B, h, w, hx, y_coff=self.mot_off, act=ACT_RELU,
                       y2=qx if qx_x else None, y2_coff=self.mot_off)
            if gru_path == "halo":
                _, stages = self._halo_geom()
                for gi, (mode, axis) in enumerate(stages):
                    wa_, wb_ = self._halo_w[gi]
                    last = gi == ngru - 1
                    if halo_pp:
                        t = [hx, hx, wa_, wb_, gbias[gi], h32, qx, hm, qx, qx, hx]
                    else:
                        t = [hx if gi == 0 else qx, hx, wa_, wb_, gbias[gi], h32, qx if gi == 0 else hx,
                             hm if last else None]
                    if wait_mask and last:
                        plan.add_wait(E_MASK)  # the previous iteration's mask head has read hm (and flow32)
                    base = [B, h, w, mode, axis]
                    tile = self._halo_tile(gi, mode, axis, B, h, w, (t, base))
                    plan.add_gru_halo(t, base + list(tile))
                return
            for gi in range(ngru):
                if gru_path == "fused":
                    last = gi == ngru - 1
                    if wait_mask and not parity and (last if hm is not None else gi == 0):
                        plan.add_wait(E_MASK)  # the previous iteration's mask head has read hm / h (and flow32)
                    ks = m.update_block.recurrent_block.kernel_size[gi]
                    plan.add_gru_fused([hx, sp[f"gru{gi}.a"].w, sp[f"gru{gi}.b"].w, gbias[gi], h32, hx,
                                        hm if last else None] + ([None, hm2] if last and parity else []),
                                       [B, h, w, int(ks[0] > 1)])
                    continue
                # r*h from the bf16 h of the conv's own input hx (no fp32 state read)
                self._conv(plan, sp[f"gru{gi}.a"], hx, B, h, w, qx, zbuf=zb, hidden=self.hidden,
                           epi=EPI_GRU_A, bmap=gbias[gi], bmap_coff=0)
                if gi == 0 and wait_mask:
                    plan.add_wait(E_MASK)  # the previous iteration's mask head has read h (and flow32)
                self._conv(plan, sp[f"gru{gi}.b"], qx, B, h, w, hx, h32=h32, zbuf=zb, hidden=self.hidden,
                           epi=EPI_GRU_B, bmap=gbias[gi], bmap_coff=2 * self.hidden)

        if self.cp:
            # segment 1: this rank's lookups; the engine all-gathers them into `corr`
            # (_gather_corr); segment 3: the rest of the iteration, replicated
            hw = h * w
            local = alloc("corr.local", (B, max(b_ - a_ for a_, b_ in slabs) * w, self.corr_cs))
            plan.set_segment(1)
            for b in range(B):
                plan.add_lookup([coords[b * hw + r0 * w:b * hw + r1 * w], local[b]]
                                + [v[b * nq:(b + 1) * nq] for v in levels] + [None] * (4 - L),
                                [L, 1, h, w, self.radius, nq, 0])
            plan.set_segment(3)
            flow_features()
            motion_and_gru(wait_flow=False, wait_mask=False)
            flow_head()
            flow_update()
            if all_iters:
                upsample(stride, mask_from_fm=False)
            plan.set_segment(2)
            if not all_iters:
                upsample(0, mask_from_fm=False)
            st.cp = dict(slabs=slabs, local=local, corr=corr, w=w)
        elif lanes_on:
            # iteration 0's flow features (zero flow) run once in the prologue
            plan.set_segment(0)
            lane(main)
            flow_features()
            plan.set_segment(1)
            lane(main)
            lookup(with_update=True)      # + iteration i-1's flow update
            plan.add_record(E_FH)
            lane(side2)
            plan.set_defer(1)             # skipped in iteration 0
            plan.add_wait(E_FH)
            flow_features()
            plan.add_record(E_FLOW)
            upsample(stride, mask_from_fm=False)   # iteration i-1 (h intact: GRU-B waits E_MASK)
            plan.add_record(E_MASK)
            plan.set_defer(0)
            lane(main)
            motion_and_gru(wait_flow=True, wait_mask=True)
            flow_head()
            plan.set_segment(2)           # epilogue: the last iteration's update, mask head and upsampling
            lane(main)
            flow_update()
            plan.set_defer(1)
            upsample(stride, mask_from_fm=False)
            plan.set_defer(0)
        elif all_iters:
            plan.set_segment(1)
            lane(main)
            lookup(with_update=True)
            if merged_up:
                # the 7x7 flow conv and iteration i-1's x8 upsampling in ONE grid (merged.hip):
                # both read the flow the lookup just updated, and at batch 1 neither fills the GPU
                c = me.convflow1.layers_0
                kh, kw_, _, co = c.kernel.shape
                ints = [B, h, w, 2, kh, kw_, c.padding[0], c.padding[1], co, 1, 0]
                if self.has_mask:
                    t_ = [flow8, self._cf1_w, self._cf1_b, f1, flow32, out, st.out_slot, fm, self._convex_w,
                          self._convex_b]
                    i_ = ints + [2, stride, out_off, self.fh_hidden]
                    if c1_merged:   # + convcorr1 (LDS-weight 1x1 kernel) in the same grid
                        t_ += [corr, self._cc1_w, self._cc1_b, c1]
                        i_ += [M, self.corr_cs, self._cc1_kpad, cl[0], ACT_RELU, 0]
                    plan.add_flowin_dual(t_, i_, m.mask_predictor.multiplier)
                else:
                    plan.add_flowin_dual([flow8, self._cf1_w, self._cf1_b, f1, flow32, out, st.out_slot],
                                         ints + [1, stride, out_off, 0], 1.0)
            else:
                flow_features()
                plan.set_defer(1)
                upsample(stride, mask_from_fm=fm is not None and self.has_mask)   # iteration i-1
                plan.set_defer(0)
            motion_and_gru(wait_flow=False, wait_mask=False, flow2=merged_up)
            flow_head()
            plan.set_segment(2)
            flow_update()
            plan.set_defer(1)
            upsample(stride, mask_from_fm=fm is not None and self.has_mask)
            plan.set_defer(0)
        elif self._cf1_w is not None and tuple(c1k.shape[:2]) == (7, 7) and B < self.AUTO_STREAMS_MIN_BATCH:
            # final-only below batch 4, the one-lane order of the all-iterations loop: the flow update
            # fused into the next lookup, the 7x7 flow conv in the merged grid (its bilinear half
            # writes the single output slot every iteration; the epilogue's upsampling overwrites
            # it), convflow2 grouped with convcorr2.  Batch 1: 239.5 -> 244.6 pairs/s; batch 4
            # loses (414.8 -> 402.7), keeps the order below (profiles/r4_host_gate.txt)
            plan.set_segment(1)
            lane(main)
            lookup(with_update=True)
            c = me.convflow1.layers_0
            kh, kw_, _, co = c.kernel.shape
            plan.add_flowin_dual([flow8, self._cf1_w, self._cf1_b, f1, flow32, out, st.out_slot],
                                 [B, h, w, 2, kh, kw_, c.padding[0], c.padding[1], co, 1, 0, 1, 0, out_off, 0], 1.0)
            motion_and_gru(wait_flow=False, wait_mask=False, flow2=True)
            flow_head()
            plan.set_segment(2)           # epilogue: the last update, then the final flow upsampled once
            flow_update()
            upsample(0, mask_from_fm=False)
        else:
            plan.set_segment(1)
            lane(main)
            flow_features()
            lookup(with_update=False)
            motion_and_gru(wait_flow=False, wait_mask=False)
            flow_head()
            flow_update()
            plan.set_segment(2)           # epilogue: upsample the final flow once (out has one iteration)
            upsample(0, mask_from_fm=False)
        lane(main)

    # --------------------------------------------------------------- forward
    @torch.no_grad()
    def forward(self, image1: torch.Tensor, image2: torch.Tensor, num_flow_updates: int = 12,
                return_all_iters: bool = True) -> torch.Tensor:
        """All ``num_flow_updates`` upsampled flows (N, B, H, W, 2), as the reference
        returns; ``return_all_iters=False`` returns only the final one, (1, B, H, W, 2)."""
        if self._stale():
            self._pack()
        if image1.dtype == torch.uint8 and not self._native_u8:
            a, b, src = self._host_u8(image1, image2)
            out = self.forward(a, b, num_flow_updates, return_all_iters)
            H0, W0, pt, pl = src
            return out[:, :, pt:pt + H0, pl:pl + W0]
        key = self._key(image1, image2, num_flow_updates, return_all_iters)
        st = self._plan_state(key, lambda: self._build_key(key))
        st.inp1.copy_(image1)
        st.inp2.copy_(image2)
        self._pre_launch(st)
        fresh = self.copy_output and st.slot_ok
        out = torch.empty_like(st.out) if fresh else st.out
        self._point_slot(st, out)
        self._gate(num_flow_updates)   # after the host-side preparation: only the launch waits
        if st.cp is not None:
            self._forward_cp(st, num_flow_updates)
        elif len(st.plans) == 1 or not self.use_graph:
            for plan in st.plans:
                self._launch(plan, num_flow_updates)
        else:
            # the parts' captures copied into ONE graph (Plan.merge_*): their chains
            # interleave with no cross-stream edge (separate graphs serialise)
            p0 = st.plans[0]
            if p0.merged_iters() != num_flow_updates:
                p0.merge_reset()
                for plan in st.plans:
                    p0.merge_add(plan, num_flow_updates)
                p0.merge_finish(num_flow_updates)
            p0.replay_pipelined()
        self._mark()
        if fresh:
            return self._crop(st, out)
        return self._crop(st, st.out.clone() if self.copy_output else st.out)

    def _pre_launch(self, st: _PlanState) -> None:
        """Work a forward runs before replaying its plan (RaftEngineMixed: the fp32 feature encoder)."""

    GATE_MIN_ITERS = 20

    def _gate(self, n_iters: int) -> None:
        """Wait (host) for the previous forward / pipelined call (see ``host_gate``)."""
        if self.host_gate and self._done_ev is not None and n_iters >= self.GATE_MIN_ITERS:
            self._done_ev.synchronize()

    def _mark(self) -> None:
        if self.host_gate and self.device.type == "cuda":
            if self._done_ev is None:
                self._done_ev = torch.cuda.Event()
            self._done_ev.record()

    @staticmethod
    def _point_slot(st: _PlanState, out: torch.Tensor) -> None:
        """Aim the plan's output writers at ``out`` (stream-ordered: the
        update is a tiny copy on the current stream, before the launch)."""
        if st.slot_ptr != out.data_ptr():
            st.out_slot.fill_(out.data_ptr())
            st.slot_ptr = out.data_ptr()

    # ------------------------------------- software-pipelined graphs (throughput)
    def _slot_state(self, key, slot: int) -> _PlanState:
        def build():
            saved, self.split = self.split, 1
            self._slot_build = True
            try:
                return self._build_key(key)
            finally:
                self.split = saved
                self._slot_build = False

        return self._plan_state(key + ("pslot", slot), build)

    @torch.no_grad()
    def pipelined(self, image1: torch.Tensor, image2: torch.Tensor, num_flow_updates: int = 12,
                  return_all_iters: bool = True) -> Optional[torch.Tensor]:
        """Software-pipelined forward for throughput (batch inference, serving):
        returns the flows of the PREVIOUS call's images (``None`` on the first
        call); :meth:`flush` returns the last pending batch's flows.

        Each call replays ONE hipGraph (``Plan.capture_pipelined``) whose
        independent branches are the previous batch's refinement loop +
        epilogue and this batch's prologue (encoders + correlation pyramid).
        The loop kernels are latency-bound (one workgroup per CU on ~220 of
        256 CUs at batch 4), the encoder convs throughput-bound, so the
        prologue mostly fills SIMD slots the loop leaves idle.  Two plan slots
        (own buffers, own graphs) alternate; every call does one prologue and
        one loop, i.e. one forward's work.  (:meth:`submit` replays the two
        phases as separate graphs on two streams, which serialise on this
        ROCm.)  The result of each batch is bitwise equal to :meth:`forward`
        (tests/test_engine_gpu.py)."""
        if self._stale():
            if self._pp is not None and self._pp["pending"] is not None:
                # the pending batch's encoders + pyramid ran with the old weights; its loop
                # would run with the new ones (a result matching neither forward)
                raise RuntimeError("pipelined(): the weights changed while a batch is pending; flush() it first")
            self._pack()
        assert self.use_graph, "pipelined() replays captured graphs (use_graph=True)"
        if self.fe_external:
            raise NotImplementedError("pipelined(): not with precision='mixed' (its fp32 encoder runs before the plan)")
        assert not self.cp, "pipelined(): not with context parallelism (a host-driven loop)"
        if image1.dtype == torch.uint8 and not self._native_u8:
            a, b, src = self._host_u8(image1, image2)
            r = self.pipelined(a, b, num_flow_updates, return_all_iters)
            return None if r is None else r[:, :, src[2]:src[2] + src[0], src[3]:src[3] + src[1]]
        n = num_flow_updates
        key = self._key(image1, image2, n, return_all_iters)
        pp = self._pp
        if pp is not None and pp["key"] != key and pp["pending"] is not None:
            raise RuntimeError("pipelined(): flush() the pending batch before changing the input shape / iterations")
        if pp is None or pp["key"] != key:
            pp = self._pp = dict(key=key, n=0, pending=None)
        slot = pp["n"] & 1
        st = self._slot_state(key, slot)
        st.inp1.copy_(image1)
        st.inp2.copy_(image2)
        prev = pp["pending"]
        result = None
        if prev is None:
            if st.plan.captured_part_iters(0) != n:
                st.plan.capture_part(0, n)
            self._gate(n)
            st.plan.replay_part(0)
        else:
            pst = self._slot_state(key, prev)
            fresh = self.copy_output and pst.slot_ok
            out = torch.empty_like(pst.out) if fresh else pst.out
            self._point_slot(pst, out)
            if pst.plan.pipelined_iters(st.plan) != n:
                pst.plan.capture_pipelined(st.plan, n)
            self._gate(n)
            pst.plan.replay_pipelined()
            result = self._crop(pst, out if fresh else (pst.out.clone() if self.copy_output else pst.out))
        self._mark()
        pp["pending"] = slot
        pp["n"] += 1
        return result

    @torch.no_grad()
    def flush(self) -> Optional[torch.Tensor]:
        """Finish the batch :meth:`pipelined` left pending (its refinement loop
        + epilogue as one graph); returns its flows, or ``None`` if none."""
        pp = self._pp
        if pp is None or pp["pending"] is None:
            return None
        key = pp["key"]
        st = self._slot_state(key, pp["pending"])
        n = key[3]
        fresh = self.copy_output and st.slot_ok
        out = torch.empty_like(st.out) if fresh else st.out
        self._point_slot(st, out)
        if st.plan.captured_part_iters(1) != n:
            st.plan.capture_part(1, n)
        st.plan.replay_part(1)
        pp["pending"] = None
        pp["n"] = 0
        return self._crop(st, out if fresh else (st.out.clone() if self.copy_output else st.out))

    def _launch(self, plan, n_iters: int) -> None:
        if self.use_graph:
            if plan.captured_iters() != n_iters:
                plan.capture(n_iters)
            plan.replay()
        else:
            plan.run(n_iters)

    def op_names(self, B: int, H: int, W: int, n_iters: int, return_all_iters: bool = True):
        st = self._plan_state((B, H, W, n_iters, return_all_iters),
                              lambda: self._build(B, H, W, n_iters, return_all_iters))
        return [st.plan.op_names(s) for s in range(3)]
