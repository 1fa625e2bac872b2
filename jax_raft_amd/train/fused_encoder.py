"""Native training forward / backward of a RAFT feature or context encoder
(``FeatureEncoder``, reference ``jax_raft/model.py:219-257`` with the
Residual / Bottleneck blocks of ``model.py:162-216``).

Every conv unit is lowered as ``conv (implicit-GEMM MFMA, bias) -> per-(n, c)
statistics -> normalise (+ relu) [+ residual (+ its norm)] -> relu`` -- the
inference engine's encoder lowering (runtime/engine.py:_encoder) with
InstanceNorm (``model.py:706-707``), train-mode BatchNorm with batch
statistics and affine parameters (``model.py:147,157``) or no norm -- and
every raw conv output, statistic and activation is kept for the backward.

The backward walks the blocks in reverse: the norm backward
(``train.hip:jr_norm_bwd``: ReLU / residual-output masks, the closed-form
instance / batch-norm adjoint, the residual-branch gradient) and each conv's
data gradient as the implicit-GEMM kernel over flipped weights (input
dilation for the strided convs, the residual gradient added in the fp32
epilogue of the block's first conv).  Weight gradients are one im2col GEMM
per conv after the plan; BatchNorm's scale / bias gradients are the norm
backward's per-channel reductions.

Forward and backward are native :class:`Plan` s recorded once per shape and
replayed (as hipGraphs by default).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from ..models.layers import NORM_BATCH, NORM_INSTANCE, BottleneckBlock, FeatureEncoder
from ..ops import native as nat
from ..ops.native import ACT_NONE, round_up

BF16, F32 = torch.bfloat16, torch.float32
EPI_BWD = 5
EPS = 1e-5
# The inference engine's encoder fusions in the training forward (instance-norm encoders,
# stride-1 3x3 convs on the halo kernel, conv_halo.hip): the conv writes its output's channel-
# statistics partials in its epilogue (no statistics pass) and normalises (+ residual, relu) its
# raw input while loading it, writing the activation the backward keeps (xn) -- no norm_act
# pass.  False: the separate statistics / norm_act passes (tests compare both).
HALO_NORM = True


def _log2(s: int) -> int:
    if s not in (1, 2, 4, 8):
        raise NotImplementedError(f"stride {s}")
    return int(math.log2(s))


class _Unit:
    """One conv -> norm (-> relu) unit and its training buffers."""

    def __init__(self, conv, norm_mod, mode: int, x: torch.Tensor, N: int, H: int, W: int):
        self.conv, self.norm_mod, self.mode = conv, norm_mod, mode
        self.x, self.N, self.H, self.W = x, N, H, W
        kh, kw = conv.kernel_size
        self.OH = (H + 2 * conv.padding[0] - kh) // conv.stride[0] + 1
        self.OW = (W + 2 * conv.padding[1] - kw) // conv.stride[1] + 1
        self.cout = conv.cout
        self.cin8 = x.shape[-1]


class EncoderTrain:
    """Training plans of one :class:`FeatureEncoder` over ``N`` images.

    ``x``: persistent bf16 input [N, H, W, cin8]; ``y_out``: bf16 [N, h, w, C]
    the final 1x1 conv writes; ``dy_out``: bf16 gradient of ``y_out`` (filled by
    the caller before :meth:`backward`)."""

    def __init__(self, enc: FeatureEncoder, x: torch.Tensor, y_out: torch.Tensor, tuner, use_graph: bool = True):
        self.enc = enc
        self.x = x
        self.y_out = y_out
        self.dy_out = torch.zeros_like(y_out)
        self.device = x.device
        self.tuner = tuner
        self.use_graph = use_graph
        self.mode = {NORM_INSTANCE: 1, NORM_BATCH: 2, None: 0}[enc.norm_kind]
        self._specs: Dict[int, nat.ConvSpec] = {}
        self._tspecs: Dict[int, nat.ConvSpec] = {}
        self.units: List[_Unit] = []
        self.blocks = []
        self.bufs: List[torch.Tensor] = []
        self.plan_f = nat.new_plan()
        self.plan_b = nat.new_plan()
        for P in (self.plan_f, self.plan_b):
            P.set_segment(0)
            P.set_lane(0)
        self._pack()
        from .fused import GradArena

        self.arena = GradArena([p for c in self._convs() for p in (c.kernel, c.bias)] +
                               [p for m in enc.modules() if getattr(m, "scale", None) is not None
                                for p in (m.scale, m.bias)], self.device)
        self.packer = self._pieces()
        self.packer.record(self.plan_f)   # first op of the forward plan: repack this step's weights
        self._record_fwd()
        self._record_bwd()

    # ------------------------------------------------------------ helpers
    def _z(self, *shape, dtype=BF16):
        t = torch.zeros(shape, dtype=dtype, device=self.device)
        self.bufs.append(t)
        return t

    def _convs(self):
        enc = self.enc
        out = [enc.convnormrelu.layers_0]
        for li in (1, 2, 3):
            layer = getattr(enc, f"layer{li}")
            for bi in range(layer.n):
                blk = getattr(layer, f"layers_{bi}")
                names = ["convnormrelu1", "convnormrelu2"] + (["convnormrelu3"] if isinstance(blk, BottleneckBlock) else [])
                if blk.stride != (1, 1):
                    names.append("downsample")
                out += [getattr(blk, n).layers_0 for n in names]
        out.append(enc.conv)
        return out

    def _pack(self):
        """(Re)pack forward and data-gradient weights in place."""
        for c in self._convs():
            k, b = c.kernel.detach().float(), c.bias.detach().float()
            kh, kw, cin, cout = k.shape
            cin8 = 8 if c is self.enc.convnormrelu.layers_0 else round_up(cin, 8)
            kt = torch.flip(k, dims=(0, 1)).permute(0, 1, 3, 2)
            if cin8 != cin:
                kt = torch.cat([kt, kt.new_zeros(kh, kw, cout, cin8 - cin)], dim=3)
            sp = self._specs.get(id(c))
            if sp is None:
                self._specs[id(c)] = nat.make_spec(k, b, c.stride, c.padding, cin8=cin8, device=self.device)
                self._tspecs[id(c)] = nat.make_spec(kt, torch.zeros(cin8, device=self.device), (1, 1),
                                                    (kh - 1 - c.padding[0], kw - 1 - c.padding[1]),
                                                    cin8=round_up(cout, 8), device=self.device)
            else:
                nat.pack_weight(k, sp.cin8, out=sp.w)
                sp.b.copy_(b)
                tp = self._tspecs[id(c)]
                nat.pack_weight(kt, tp.cin8, out=tp.w)

    def _pieces(self):
        from .fused import Packer

        pk = Packer()
        for c in self._convs():
            kh, kw, cin, cout = c.kernel.shape
            sp, tp = self._specs[id(c)], self._tspecs[id(c)]
            pk.piece(c.kernel, sp, 0, (0, cout), (0, cin))
            pk.bias(c.bias, sp.b, (0, cout))
            pk.piece(c.kernel, tp, 1, (0, cin), (0, cout))
            if sp.wh is not None:   # halo-kernel weight streams of the stride-1 3x3 convs
                pk.piece(c.kernel, sp, 4, (0, cout), (0, cin))
            if tp.wh is not None and c.stride == (1, 1):
                pk.piece(c.kernel, tp, 5, (0, cin), (0, cout))
        return pk

    def _affine(self, unit):
        if self.mode == 2:
            bn = unit.norm_mod
            return bn.scale.data, bn.bias.data
        return None, None

    # ------------------------------------------------------------ forward
    def _halo_ok(self, sp) -> bool:
        return HALO_NORM and self.device.type == "cuda" and bool(nat.halo_cfgs_for(sp, {}))

    def _conv_unit(self, conv, norm_mod, xin, N, H, W) -> _Unit:
        """One conv unit.  ``xin``: a tensor or a pending activation (:meth:`_norm_act`) that
        this conv normalises while loading when it runs on the halo kernel, else materialised
        first by a norm_act pass."""
        sp = self._specs[id(conv)]
        halo = self._halo_ok(sp)
        pend = xin if isinstance(xin, dict) else None
        fuse_in = (halo and pend is not None and not pend["done"] and self.mode == 1
                   and pend["u"].cout == sp.cin8 and self._affine(pend["u"])[0] is None)
        if pend is not None and not fuse_in:
            self._materialise(pend)
        x = pend["out"] if pend is not None else xin
        u = _Unit(conv, norm_mod, self.mode, x, N, H, W)
        u.y = self._z(N, u.OH, u.OW, u.cout)
        u.st = self._z(N, u.cout, 2, dtype=F32) if self.mode else None
        if halo and (self.mode or fuse_in):
            kw = {}
            if self.mode:
                nb_max = nat.halo_max_blocks(sp.cin8, u.OH, u.OW)
                kw["stats_part"] = part = self._z(N, nb_max, u.cout, 2, dtype=F32)
            src = x
            if fuse_in:
                p = pend["u"]
                has_res = pend["res"] is not None or pend["ru"] is not None
                r = pend["relu"]
                # norm_act's relu bits (0: on the normalised value, 1: on the sum) -> the halo
                # loader's (1: before the residual add, 0: after it)
                in_relu = (((r & 1) << 1) | ((r >> 1) & 1)) if has_res else (1 if r else 0)
                res = pend["res"]
                if isinstance(res, dict):
                    assert res["done"], "a residual must be materialised before its consumer"
                    res = res["out"]
                kw.update(in_stats=p.st, in_relu=in_relu, in_hw=p.OH * p.OW, xn=pend["out"],
                          in_res=pend["ru"].y if pend["ru"] is not None else res,
                          in_res_stats=pend["ru"].st if pend["ru"] is not None else None)
                src = p.y
                pend["done"] = True
            cfg = self.tuner(self.plan_f, sp, src, N, H, W, u.y, act=ACT_NONE, **kw)
            if self.mode:
                c = nat.halo_cfg(cfg)
                self.plan_f.add_stats_final([part, u.st], [N, -(-u.OH // c[4]) * -(-u.OW // c[5]) * c[2], u.cout])
        else:
            self.tuner(self.plan_f, sp, x, N, H, W, u.y, act=ACT_NONE)
            if self.mode:
                self.plan_f.add_stats([u.y, u.st], [N, u.OH * u.OW, u.cout])
        self.units.append(u)
        return u

    def _norm_act(self, u: _Unit, relu: int, res=None, ru: Optional[_Unit] = None) -> dict:
        """The unit's normalised (+ residual, relu) output, pending: materialised by its first
        consumer (a halo conv's loader or :meth:`_materialise`)."""
        return dict(u=u, relu=relu, res=res, ru=ru, out=self._z(u.N, u.OH, u.OW, u.cout), done=False)

    def _materialise(self, pend) -> torch.Tensor:
        if isinstance(pend, torch.Tensor):
            return pend
        if not pend["done"]:
            u, relu, res, ru, a = pend["u"], pend["relu"], pend["res"], pend["ru"], pend["out"]
            g, b = self._affine(u)
            if ru is not None:
                gr, br = self._affine(ru)
                self.plan_f.add_norm_act([u.y, u.st, g, b, ru.y, ru.st, gr, br, a],
                                         [self.mode, self.mode, u.N, u.OH * u.OW, u.cout, relu], EPS)
            else:
                self.plan_f.add_norm_act([u.y, u.st, g, b, None if res is None else self._materialise(res), None,
                                          None, None, a],
                                         [self.mode, 0, u.N, u.OH * u.OW, u.cout, relu], EPS)
            pend["done"] = True
        return pend["out"]

    def _record_fwd(self):
        enc = self.enc
        N, H, W = self.x.shape[:3]
        stem = self._conv_unit(enc.convnormrelu.layers_0, getattr(enc.convnormrelu, "layers_1", None), self.x, N, H, W)
        x = self._norm_act(stem, relu=1)
        stem.a = x["out"]
        self.stem = stem
        H, W = stem.OH, stem.OW
        for li in (1, 2, 3):
            layer = getattr(enc, f"layer{li}")
            for bi in range(layer.n):
                blk = getattr(layer, f"layers_{bi}")
                names = ["convnormrelu1", "convnormrelu2"] + (["convnormrelu3"] if isinstance(blk, BottleneckBlock) else [])
                units = []
                h_in, w_in, xin = H, W, x
                y = x
                hh, ww = H, W
                for j, nm in enumerate(names):
                    cna = getattr(blk, nm)
                    u = self._conv_unit(cna.layers_0, getattr(cna, "layers_1", None), y, N, hh, ww)
                    units.append(u)
                    hh, ww = u.OH, u.OW
                    if j + 1 < len(names):
                        y = self._norm_act(u, relu=1)
                        u.a = y["out"]
                ds = None
                if blk.stride != (1, 1):
                    cna = blk.downsample
                    ds = self._conv_unit(cna.layers_0, getattr(cna, "layers_1", None), xin, N, h_in, w_in)
                last = units[-1]
                xin_t = self._materialise(xin)   # (the block's first conv materialised it already)
                if ds is not None:
                    out = self._norm_act(last, relu=3, ru=ds)
                else:
                    out = self._norm_act(last, relu=3, res=xin_t)
                last.a = out["out"]
                self.blocks.append(dict(units=units, ds=ds, x=xin_t, out=out["out"], H=h_in, W=w_in))
                x, H, W = out, hh, ww
        x = self._materialise(x)
        self.tuner(self.plan_f, self._specs[id(enc.conv)], x, N, H, W, self.y_out, act=ACT_NONE)
        self.final_x = x
        if self.mode == 2:   # BatchNorm running statistics (Flax momentum semantics), one launch
            self._bn_table(self.plan_f, [(u.st, u.norm_mod.mean, u.norm_mod.var, u.N, u.cout, u.N * u.OH * u.OW,
                                          u.norm_mod.momentum, 0) for u in self.units])

    # ----------------------------------------------------------- backward
    def _dgrad(self, u: _Unit, dy: torch.Tensor, out: torch.Tensor, gin: Optional[torch.Tensor] = None):
        """Data gradient of unit u's conv: dy [N, OH, OW, cout] -> out [N, H, W, cin8] (bf16 or
        fp32), gin fp32 [N, H, W, cin8] added in the epilogue."""
        from .fused import Seg, _tx

        tp = self._tspecs[id(u.conv)]
        s = u.conv.stride
        if gin is None and s == (1, 1) and out.dtype == BF16:
            # nothing to accumulate: a plain conv over the flipped weights (halo-kernel candidate)
            self.tuner(self.plan_b, tp, dy, u.N, u.OH, u.OW, out, act=ACT_NONE)
            return
        tx, ix = _tx(s1=Seg(gin=gin, out=out))
        extra = None if s == (1, 1) else [u.H, u.W, _log2(s[0]), _log2(s[1])]
        self.tuner(self.plan_b, tp, dy, u.N, u.OH, u.OW, out, tx=tx, ix=ix, epi=EPI_BWD, hidden=0, extra=extra)

    def _norm_bwd(self, u: _Unit, gout, dy, om=None, relu=1, gres=None, norm_mod=None):
        g, b = self._affine(u)
        if self.mode:
            u.red = self._z(u.N, u.cout, 2, dtype=F32)
        else:
            u.red = None
        part = None  # the plan op allocates (and keeps) its reduction workspace
        self.plan_b.add_norm_bwd([gout, om, u.y, u.st, g, b, u.red, part, dy, gres],
                                 [self.mode, relu, u.N, u.OH * u.OW, u.cout], EPS)

    def _record_bwd(self):
        enc = self.enc
        N = self.x.shape[0]
        last_blk = self.blocks[-1]
        # final 1x1 conv: dL/d(last block output)
        fin = _Unit(enc.conv, None, 0, self.final_x, N, self.final_x.shape[1], self.final_x.shape[2])
        self.fin = fin
        fin.dy = self.dy_out
        dout = self._z(*last_blk["out"].shape)
        self._dgrad(fin, self.dy_out, dout)
        for bi in reversed(range(len(self.blocks))):
            blk = self.blocks[bi]
            units, ds = blk["units"], blk["ds"]
            last = units[-1]
            last.dy = self._z(*last.y.shape)
            res_g = None
            if ds is None:
                # dL/dx through the identity shortcut: gout * [block output > 0], exact in bf16
                res_g = self._z(*blk["x"].shape)
                self._norm_bwd(last, dout, last.dy, om=blk["out"], relu=1, gres=res_g)
            else:
                self._norm_bwd(last, dout, last.dy, om=blk["out"], relu=1)
                ds.dy = self._z(*ds.y.shape)
                self._norm_bwd(ds, dout, ds.dy, om=blk["out"], relu=0)
                res_g = self._z(*blk["x"].shape, dtype=F32)
                self._dgrad(ds, ds.dy, res_g)
            # chain back through the block's units
            g = last.dy
            for j in reversed(range(len(units))):
                u = units[j]
                if j > 0:
                    da = self._z(*units[j - 1].a.shape)
                    self._dgrad(u, g, da)
                    p = units[j - 1]
                    p.dy = self._z(*p.y.shape)
                    self._norm_bwd(p, da, p.dy, relu=1)
                    g = p.dy
                else:
                    dx = self._z(*blk["x"].shape)
                    self._dgrad(u, g, dx, gin=res_g)
                    dout = dx
        # stem: dL/d(stem activation) = dout of the first block's input
        self.stem.dy = self._z(*self.stem.y.shape)
        self._norm_bwd(self.stem, dout, self.stem.dy, relu=1)
        # weight (+ bias) gradients: one implicit-GEMM launch per conv
        from .fused import record_wgrad

        for u in self.units + [fin]:
            c = u.conv
            record_wgrad(self.plan_b, u.x, u.N, u.H, u.W, 0, u.cin8, tuple(c.kernel.shape), c.stride, c.padding,
                         u.dy, 0, self.arena[c.kernel], self.arena[c.bias])
        if self.mode == 2:   # BatchNorm scale / bias gradients from the norm backward's reductions
            self._bn_table(self.plan_b, [(u.red, self.arena[u.norm_mod.scale], self.arena[u.norm_mod.bias], u.N,
                                          u.cout, 1, 0.0, 1) for u in self.units])

    def _bn_table(self, plan, rows):
        import struct

        tab = []
        for src, d0, d1, n, c, cnt, mom, mode in rows:
            bits = struct.unpack("<i", struct.pack("<f", float(mom)))[0]
            tab.append([src.data_ptr(), d0.data_ptr(), d1.data_ptr(), n, c, cnt, bits, mode])
        t = torch.tensor(tab, dtype=torch.int64).to(self.device).contiguous()
        self.bufs.append(t)
        keep = [t] + [v for r in rows for v in r[:3]]
        plan.add_bn_table(keep, [len(tab), max(r[4] for r in rows)])

    # ---------------------------------------------------------------- run
    def _run(self, plan):
        from .fused import _run_plan

        _run_plan(plan, self.use_graph)

    def forward(self, update_stats: bool = True):
        """Runs the forward plan; with BatchNorm it also updates the running
        statistics (the fused path trains with batch statistics only)."""
        if self.mode == 2 and not update_stats:
            raise ValueError("the fused encoder plans update BatchNorm statistics (train mode only)")
        self._run(self.plan_f)

    def run_backward(self) -> None:
        """Runs the backward plan (``dy_out`` must be filled): data gradients,
        then every conv's weight / bias gradient into :attr:`arena`."""
        self._run(self.plan_b)

    def backward(self) -> Dict[int, torch.Tensor]:
        """:meth:`run_backward`, then {id(param): grad} (a fresh copy)."""
        self.run_backward()
        return self.arena.snapshot()
