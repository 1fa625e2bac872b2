"""Loader and thin Python front-end for the gfx950 native library (``_C.so``).

The library is built in-tree by :mod:`jax_raft_amd._build`.  On a GPU machine
the native path is the only GPU implementation: if the library cannot be
loaded, GPU execution fails loudly instead of silently falling back to
PyTorch ops.
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import torch

from .. import knobs
from .._build import SO_PATH as _DEFAULT_SO

# JR_NATIVE_SO: load another build of the library (e.g. the host-sanitizer
# build _C_san.so, jax_raft_amd/_build.py --sanitize); default: the in-tree _C.so
SO_PATH = Path(knobs.get("JR_NATIVE_SO")).resolve() if knobs.get("JR_NATIVE_SO") else _DEFAULT_SO

_lock = threading.Lock()
_loaded = False
_load_error: Optional[BaseException] = None

# activation / epilogue codes (csrc/kernels/common.h, kernels.h)
ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH, ACT_SPLIT_TANH_RELU = 0, 1, 2, 3, 4
EPI_STD, EPI_GRU_A, EPI_GRU_B = 0, 1, 2   # 3, 4: retired epilogues (kernels.h)
EPI_BWD, EPI_TAPS = 5, 6
# tile configs with the EPI_TAPS epilogue (256 channels in one N tile, 16 waves of 64 x 32)
TAPS_CFGS = (34, 22, 35, 38)
# tile configs of conv_igemm.hip: (BCO, BP)
CFG_TILES = {0: (128, 128), 1: (64, 128), 2: (128, 64), 3: (16, 256), 4: (64, 64), 5: (16, 64)}
# configs 6..11: LDS-DMA kernel D2 (csrc/kernels/conv_igemm.hip)
CFG_TILES.update({6: (128, 128), 7: (64, 128), 8: (128, 64), 9: (128, 256), 10: (64, 64), 11: (256, 128)})
# configs 12..15: 32x32x16-MFMA kernel (kernel M32)
CFG_TILES.update({12: (128, 128), 13: (64, 128), 14: (128, 64), 15: (64, 64)})
# configs 16/17: kernel R at 256-wide block tiles (128x64 / 64x128 wave tiles, one block per CU)
CFG_TILES.update({16: (256, 128), 17: (128, 256)})
# configs 18..20: kernel R with 8 waves per block (64x32, 32x64, 64x64 wave tiles)
CFG_TILES.update({18: (128, 128), 19: (128, 128), 20: (256, 128)})
# configs 21/22: 16 waves per block (32x32 / 64x32 wave tiles); 23/24: 8 waves at 128x64 / 64x128
CFG_TILES.update({21: (128, 128), 22: (256, 128), 23: (128, 64), 24: (64, 128)})
# configs 25..28: kernel M32 with 8 waves (64x64 / 64x64 / 64x32 / 64x32 wave tiles)
CFG_TILES.update({25: (256, 128), 26: (128, 256), 27: (128, 128), 28: (64, 256)})
# configs 33/34: kernel P (register double-buffered fragments), 8 / 16 waves
CFG_TILES.update({33: (128, 128), 34: (256, 128)})
# configs 35..41: kernel D2 (LDS-DMA ring) at 8 / 16 waves with the FAST loader
CFG_TILES.update({35: (256, 128), 36: (128, 128), 37: (128, 128), 38: (256, 128), 39: (256, 128), 40: (128, 256),
                  41: (64, 128), 42: (256, 128), 43: (256, 128)})
# Autotune candidates: configs that win at least one RAFT conv on MI355X
# (tools/microbench.py, profiles/r1_microbench_conv_cfgs.txt); the others stay
# compiled and tested but are not timed at plan build.
# Of the D2 configs 35..43 only the 16-wave 64x32 ones (35, 38) come within a few
# percent of kernel P on a loop conv (profiles/r2_conv_d2_microbench.txt).
TUNE_CFGS = (0, 1, 2, 3, 4, 5, 12, 13, 14, 15, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 33, 34,
             35, 38)
NUM_CUS = 256
# tile configs served by the grouped two-conv launch (csrc/kernels/conv_fam_grp.hip)
GROUPED_CFGS = frozenset((2, 4, 5, 23, 24, 12, 14, 15))


def gru_fused_tiles(N: int, H: int, W: int, vertical: int) -> int:
    """Workgroups of the fused ConvGRU stage (csrc/kernels/gru_fused.hip; mirrors
    binding.cpp:gru_fused_fits): image rows (1x5, W <= 128) or pairs / singles of
    image columns (5x1, J * H <= 128); 0 when the geometry does not fit a tile."""
    if not vertical:
        return N * H if 1 <= W <= 128 else 0
    J = 2 if 2 * H <= 128 and W % 2 == 0 else 1
    return N * (W // J) if 1 <= H and J * H <= 128 and J * (H + 4) <= 136 and W % J == 0 else 0


def _m32_chan(r: torch.Tensor) -> torch.Tensor:
    """Channel held by row r of a 32-row MFMA A block whose accumulator register i of lane
    half h is channel 16 h + i (row (i & 3) + 8 (i >> 2) + 4 h of the 32x32x16 tile)."""
    return 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3)


def pack_gru_halo(kernel: torch.Tensor, cin_pad: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ConvGRU gate kernel (kh, kw, cin, cout) HWIO -> the weight stream of gru_halo.hip:
    bf16 [cout/32][kh*kw*cin_pad/16][64][8], fragment (blk, s), lane l, element j holding
    W[k = 16 s + 8 (l >> 5) + j][co = 32 blk + _m32_chan(l & 31)] with k = tap * cin_pad + ci
    (tap row-major, input channels zero-padded to cin_pad): one contiguous 1 KB load per
    MFMA A fragment."""
    kh, kw, cin, cout = kernel.shape
    assert cout % 32 == 0 and cin <= cin_pad and cin_pad % 16 == 0, (kernel.shape, cin_pad)
    dev = kernel.device
    k = torch.zeros(kh * kw, cin_pad, cout, dtype=torch.float32, device=dev)
    k[:, :cin] = kernel.detach().float().reshape(kh * kw, cin, cout)
    k = k.reshape(kh * kw * cin_pad, cout)
    ks = kh * kw * cin_pad // 16
    blk = torch.arange(cout // 32, device=dev).view(-1, 1, 1, 1)
    s = torch.arange(ks, device=dev).view(1, -1, 1, 1)
    l = torch.arange(64, device=dev).view(1, 1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, 8)
    kk = (16 * s + 8 * (l >> 5) + j).expand(cout // 32, ks, 64, 8)
    co = (32 * blk + _m32_chan(l & 31)).expand(cout // 32, ks, 64, 8)
    w = k[kk, co].to(torch.bfloat16).contiguous()
    if out is not None:
        assert out.shape == w.shape and out.dtype == torch.bfloat16
        out.copy_(w)
        return out
    return w


# (hd, mode) -> the (nb1, nb2) block counts gru_halo.hip instantiates (JR_HALO_CASES)
GRU_HALO_BLOCKS = {(128, 0): ((1, 1), (2, 1), (2, 2), (3, 2), (3, 3), (5, 4)), (96, 1): ((2, 1), (2, 2), (3, 2))}


def gru_halo_lds(hd: int, mode: int, TR: int, TC: int, nb1: int, nb2: int) -> int:
    """LDS bytes of one gru_halo workgroup (mirrors gru_halo.hip:lds_bytes)."""
    f_rows = TC + 8 if mode == 0 else (TR + 4) * (TC + 4)
    f_elems = max(f_rows * 256, (hd // 32) * nb2 * 4 * 256 * 2)
    return (round_up(f_elems, 8) + 32 * nb1 * 128) * 2


def gru_halo_geom_ok(hd: int, mode: int, TR: int, TC: int, nb1: int, nb2: int) -> bool:
    """Host-side mirror of binding.cpp:gru_halo_geom_ok (no library needed)."""
    if (nb1, nb2) not in GRU_HALO_BLOCKS.get((hd, mode), ()) or TR < 1 or TC < 1:
        return False
    if mode == 0 and TR != 1:
        return False
    nreg = TC + 4 if mode == 0 else (TR + 2) * (TC + 2)
    return nreg <= 32 * nb1 and TR * TC <= 32 * nb2 and gru_halo_lds(hd, mode, TR, TC, nb1, nb2) <= 160 * 1024


def gru_halo_tiles(mode: int, axis: int, N: int, H: int, W: int, TR: int, TC: int) -> int:
    """Workgroups of a gru_halo stage (binding.cpp:make_gru_halo)."""
    if mode == 0:
        length, lines = (H, W) if axis else (W, H)
        return N * lines * -(-length // TC)
    return N * -(-H // TR) * -(-W // TC)


def gru_halo_candidates(hd: int, mode: int, axis: int, N: int, H: int, W: int) -> List[Tuple[int, int, int, int]]:
    """(TR, TC, nb1, nb2) tilings of one gru_halo stage worth timing: per instantiated block
    count, the largest tile that fits it, balanced so the last tile along the run / the
    block grid is not a sliver (mode 0: runs of L = ceil(len / segments) pixels)."""
    out = []
    if mode == 0:
        length = H if axis else W
        for nb1, nb2 in ((1, 1), (2, 1), (2, 2), (3, 2), (3, 3), (5, 4)):
            lmax = min(32 * nb1 - 4, 32 * nb2)
            segs = -(-length // lmax)
            L = -(-length // segs)
            if (L + 4 > 32 * (nb1 - 1) or nb1 == 1) and (L > 32 * (nb2 - 1) or nb2 == 1):
                out.append((1, L, nb1, nb2))
    else:
        for nb1, nb2, tr, tc in ((2, 1, 5, 6), (2, 1, 4, 8), (2, 2, 6, 6), (3, 2, 7, 8)):
            out.append((min(tr, H), min(tc, W), nb1, nb2))
    seen, res = set(), []
    for c in out:
        if c not in seen and gru_halo_geom_ok(hd, mode, *c):
            seen.add(c)
            res.append(c)
    return res


def load(build_if_missing: bool = True) -> None:
    """Load ``_C.so`` (building it with hipcc first if it is missing)."""
    global _loaded, _load_error
    if _loaded:
        return
    with _lock:
        if _loaded:
            return
        try:
            if not SO_PATH.exists() and build_if_missing:
                from .._build import build

                build()
            torch.ops.load_library(str(SO_PATH))
            _loaded = True
        except BaseException as e:  # pragma: no cover - reported by require()
            _load_error = e
            raise


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except BaseException:
        return False


def require() -> None:
    """Raise if the native library is not usable (GPU path must not fall back)."""
    try:
        load()
    except BaseException as e:
        raise RuntimeError(f"jax_raft_amd native library unavailable ({SO_PATH}): {e}") from e


def ops():
    require()
    return torch.ops.jax_raft_amd


def new_plan():
    require()
    return torch.classes.jax_raft_amd.Plan()


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# ------------------------------------------------------------------ conv specs


@dataclass
class ConvSpec:
    """A packed convolution ready for the implicit-GEMM kernel.

    ``w``: bf16 [cout_pad, kpad], K ordered (kh, kw, cin8) with the input
    channels zero-padded to ``cin8``; ``b``: fp32 [cout]; ``wh``: for a 3x3 /
    stride-1 / pad-1 conv with cin8 % 16 == 0, the weights of the halo kernel
    (conv_halo.hip; :func:`pack_halo_conv`), else None."""

    w: torch.Tensor
    b: torch.Tensor
    kh: int
    kw: int
    sh: int
    sw: int
    ph: int
    pw: int
    cin: int
    cin8: int
    cout: int
    wh: Optional[torch.Tensor] = None

    def out_hw(self, H: int, W: int) -> Tuple[int, int]:
        return (H + 2 * self.ph - self.kh) // self.sh + 1, (W + 2 * self.pw - self.kw) // self.sw + 1

    @property
    def halo_shape(self) -> bool:
        return self.halo_ks != 0

    @property
    def halo_ks(self) -> int:
        """3: a 3x3 / stride-1 / pad-1 conv the halo kernel runs; 4: the space-to-depth stem
        (4x4 / pad 2, output cropped to the input size, 16 input channels); else 0."""
        g = (self.kh, self.kw, self.sh, self.sw, self.ph, self.pw)
        if g == (3, 3, 1, 1, 1, 1) and self.cin8 % 16 == 0:
            return 3
        if g == (4, 4, 1, 1, 2, 2) and self.cin8 == 16:
            return 4
        return 0


# halo 3x3 conv tile configs (csrc/kernels/conv_halo.hip kCfgs; conv op cfg id = HALO_CFG0 + index):
# (cin, waves along cout, waves along pixels, 32-pixel blocks per wave, tile rows, tile cols)
HALO_CFG0 = 100
HALO_CFGS = ((64, 2, 2, 4, 16, 16), (64, 2, 2, 2, 8, 16), (96, 3, 2, 2, 8, 16), (96, 3, 1, 2, 4, 16),
             (128, 4, 2, 2, 8, 16), (128, 4, 1, 2, 4, 16), (128, 2, 2, 2, 8, 16), (128, 2, 1, 1, 4, 8),
             (256, 2, 2, 2, 8, 16), (256, 2, 1, 1, 4, 8), (128, 4, 1, 1, 4, 8), (256, 4, 1, 1, 4, 8),
             (256, 2, 1, 2, 4, 16), (256, 6, 1, 4, 8, 16), (256, 4, 1, 4, 8, 16), (128, 8, 1, 4, 8, 16),
             (128, 2, 1, 4, 8, 16), (256, 6, 1, 2, 4, 16), (256, 4, 1, 2, 4, 16), (256, 1, 2, 2, 8, 16),
             (256, 1, 4, 1, 8, 16), (128, 1, 2, 2, 8, 16), (128, 1, 4, 1, 8, 16))
# the 4x4 space-to-depth stem (kCfgs entries with ks = 4): conv op cfg id -> the same fields
HALO_STEM_CFGS = {HALO_CFG0 + len(HALO_CFGS): (16, 2, 2, 2, 8, 16), HALO_CFG0 + len(HALO_CFGS) + 1: (16, 2, 2, 4, 16, 16)}
# round-6 3x3 configs, after the stem entries of kCfgs (ids of the older configs unchanged)
HALO_CFGS_R6 = ((256, 6, 2, 2, 8, 16), (256, 4, 2, 2, 8, 16), (128, 8, 2, 2, 8, 16), (128, 4, 2, 4, 16, 16),
                (128, 2, 4, 2, 16, 16))
# every 3x3 config: cfg id -> (cin, waves along cout, waves along pixels, blocks per wave, tile rows, tile cols)
HALO_3X3 = {**{HALO_CFG0 + i: c for i, c in enumerate(HALO_CFGS)},
            **{HALO_CFG0 + len(HALO_CFGS) + len(HALO_STEM_CFGS) + i: c for i, c in enumerate(HALO_CFGS_R6)}}


def halo_cfg(cfg: int) -> Tuple[int, int, int, int, int, int]:
    """(cin, waves along cout, waves along pixels, blocks per wave, tile rows, tile cols) of a halo cfg id."""
    return HALO_STEM_CFGS[cfg] if cfg in HALO_STEM_CFGS else HALO_3X3[cfg]


def halo_max_blocks(cin8: int, H: int, W: int) -> int:
    """The most statistics-partial blocks per image any 3x3 config of ``cin8`` input channels
    writes for an H x W output (tiles x pixel waves): the size of a ``stats_part`` buffer."""
    return max(-(-H // c[4]) * -(-W // c[5]) * c[2] for c in HALO_3X3.values() if c[0] == cin8)


def pack_halo_conv(kernel: torch.Tensor, cin8: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(3, 3, cin, cout) HWIO -> the halo conv's weight stream: :func:`pack_gru_halo` with the
    input channels padded to cin8 and the output channels to a multiple of 32."""
    kh, kw, cin, cout = kernel.shape
    k = kernel.detach().float()
    if cout % 32:
        k = torch.cat([k, torch.zeros(kh, kw, cin, round_up(cout, 32) - cout, device=k.device)], dim=3)
    return pack_gru_halo(k, cin8, out=out)


def halo_cfgs_for(spec: "ConvSpec", kw: dict) -> Tuple[int, ...]:
    """Halo conv configs that can run this conv (shape, epilogue, channel count).
    """
    if spec.wh is None or not spec.halo_shape:
        return ()
    if kw.get("epi", EPI_STD) != EPI_STD or kw.get("act", ACT_NONE) not in (ACT_NONE, ACT_RELU):
        return ()
    if kw.get("alpha", 1.0) != 1.0 or kw.get("bmap") is not None or kw.get("h32") is not None:
        return ()
    if kw.get("y") is not None and kw["y"].dtype != torch.bfloat16:
        return ()
    if spec.halo_ks == 4:   # the stem: its output is the input's size (out_hw given by the caller)
        if kw.get("out_hw") is None or spec.cout > 512:
            return ()
        return tuple(HALO_STEM_CFGS)
    if kw.get("out_hw") is not None:
        return ()
    return tuple(i for i, c in HALO_3X3.items() if c[0] == spec.cin8 and spec.cout <= 512)


def _row_perm(cout_pad: int) -> torch.Tensor:
    """Storage row s -> output channel.  Within each 64-row group the rows are
    ordered so that D row (4*q + r) of the 16-row MFMA tile t is channel
    q*16 + t*4 + r: every lane of the conv epilogue then owns contiguous
    channels and both GEMM operands are read from LDS in natural row order."""
    s = torch.arange(cout_pad)
    g, i = s // 64, s % 64
    t, q, r = i // 16, (i % 16) // 4, i % 4
    return g * 64 + q * 16 + t * 4 + r


def pack_weight(kernel: torch.Tensor, cin8: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """HWIO fp32 kernel -> bf16 [cout_pad, kpad] (GEMM A operand), K ordered
    (kh, kw, cin8), rows permuted per :func:`_row_perm`, cout padded to 64."""
    kh, kw, cin, cout = kernel.shape
    cin8 = cin8 or round_up(cin, 8)
    kraw = kh * kw * cin8
    kpad = round_up(kraw, 64)
    cout_pad = round_up(cout, 64)
    k = torch.zeros(kh, kw, cin8, cout, dtype=torch.float32, device=kernel.device)
    k[:, :, :cin, :] = kernel.detach().float()
    w = torch.zeros(cout_pad, kpad, dtype=torch.float32, device=kernel.device)
    w[:cout, :kraw] = k.permute(3, 0, 1, 2).reshape(cout, kraw)
    w = w[_row_perm(cout_pad).to(w.device)].to(torch.bfloat16).contiguous()
    if out is not None:
        assert out.shape == w.shape and out.dtype == torch.bfloat16
        out.copy_(w)
        return out
    return w


def pack_direct_weight(kernel: torch.Tensor) -> torch.Tensor:
    """HWIO kernel (kh, kw, 2, cout) -> bf16 MFMA A fragments [cout/16][NKC][64][8]
    for the 2-channel conv (conv_direct.hip).  K is ordered (kh, kw padded to
    KWP = 4 | 8, c): fragment (t, kc), lane l, element e holds
    W[co = 16t + l % 16][k = 32 kc + 8 (l // 16) + e]."""
    kh, kw, cin, cout = kernel.shape
    assert cin == 2 and cout % 32 == 0, "2-channel conv with cout % 32 == 0"
    kwp = 4 if kw <= 4 else 8
    nkc = (kh * kwp * 2 + 31) // 32
    k = torch.zeros(kh, kwp, 2, cout, dtype=torch.float32, device=kernel.device)
    k[:, :kw] = kernel.detach().float()
    wk = torch.zeros(cout, nkc * 32, dtype=torch.float32, device=kernel.device)
    wk[:, : kh * kwp * 2] = k.reshape(kh * kwp * 2, cout).t()
    wk = wk.reshape(cout // 16, 16, nkc, 4, 8).permute(0, 2, 3, 1, 4)  # [t][kc][kg][i][e]
    return wk.reshape(cout // 16, nkc, 64, 8).to(torch.bfloat16).contiguous()


def direct_conv_ok(kernel: torch.Tensor, stride=(1, 1)) -> bool:
    """Shapes the direct VALU conv kernel supports (the flow branch's 7x7 / 3x3 on 2 channels)."""
    kh, kw, cin, cout = kernel.shape
    return cin == 2 and (kh, kw) in ((7, 7), (3, 3)) and tuple(stride) == (1, 1) and cout % 32 == 0


def make_spec(kernel: torch.Tensor, bias: torch.Tensor, stride=(1, 1), padding=(0, 0), cin8: Optional[int] = None,
              device=None) -> ConvSpec:
    kh, kw, cin, cout = kernel.shape
    cin8 = cin8 or round_up(cin, 8)
    k = kernel.to(device) if device is not None else kernel
    w = pack_weight(k, cin8)
    b = bias.detach().float().to(w.device).contiguous()
    spec = ConvSpec(w, b, kh, kw, stride[0], stride[1], padding[0], padding[1], cin, cin8, cout)
    if spec.halo_ks == 4 or (spec.halo_shape and any(c[0] == cin8 for c in HALO_CFGS)):
        spec.wh = pack_halo_conv(k, cin8)
    return spec


def s2d_stem_kernel(kernel: torch.Tensor) -> torch.Tensor:
    """A 7x7 / stride-2 / pad-3 conv over 3 channels (the encoders' stem, model.py:238-240)
    as the equivalent 4x4 / stride-1 conv (top / left pad 2, output H/2 x W/2) over the 2x2
    space-to-depth input (channel (sy * 2 + sx) * 3 + c, 16 with zero padding):
    W'[ty][tx][(sy, sx, c)] = W[2 ty + sy - 1][2 tx + sx - 1][c] where that tap exists."""
    kh, kw, cin, cout = kernel.shape
    assert (kh, kw, cin) == (7, 7, 3), kernel.shape
    k = kernel.detach().float()
    out = torch.zeros(4, 4, 16, cout, dtype=k.dtype, device=k.device)
    for ty in range(4):
        for tx in range(4):
            for sy in range(2):
                for sx in range(2):
                    a, b = 2 * ty + sy - 1, 2 * tx + sx - 1
                    if 0 <= a < 7 and 0 <= b < 7:
                        c0 = (sy * 2 + sx) * 3
                        out[ty, tx, c0:c0 + 3] = k[a, b]
    return out


def pick_cfg(M: int, cout: int) -> int:
    """Tile-config heuristic: minimise (waves of blocks) x (tile cost), where a
    tile's per-FLOP cost rises as it shrinks; keeps >= one wave of blocks over
    256 CUs whenever the problem allows."""
    if cout <= 16:
        return 5
    best, best_cost = 0, None
    # (cfg, relative per-FLOP efficiency of the tile); time ~ blocks per CU x tile area / eff
    for cfg, eff in ((0, 1.0), (2, 0.85), (1, 0.85), (4, 0.65)):
        bco, bp = CFG_TILES[cfg]
        nb = math.ceil(M / bp) * math.ceil(cout / bco)
        cost = math.ceil(nb / NUM_CUS) * (bco * bp) / eff
        if best_cost is None or cost < best_cost - 1e-9:
            best, best_cost = cfg, cost
    return best


def conv_args(spec: ConvSpec, x: torch.Tensor, N: int, H: int, W: int, y: torch.Tensor, *, x_coff: int = 0,
              y_coff: int = 0, act: int = ACT_NONE, split: int = 0, alpha: float = 1.0, y2=None, y2_coff: int = 0,
              res=None, res_coff: int = 0, res_post: int = 0, h32=None, zbuf=None, hidden: int = 0, coords=None,
              flow32=None, y3=None, y3_coff: int = 0, epi: int = EPI_STD, cfg: Optional[int] = None,
              bmap=None, bmap_coff: int = 0, tapw=None, out_hw: Optional[Tuple[int, int]] = None,
              stats_part=None, in_stats=None, in_relu: int = 0, in_hw: int = 0, in_res=None, in_res_stats=None,
              xn=None):
    """Build the (tensors, ints, alpha) argument triple of the ``conv`` op.
    ``bmap``: optional fp32 per-pixel bias map [M, C], channels from ``bmap_coff``.
    Halo tile configs only (cfg >= HALO_CFG0): ``stats_part`` receives per-tile channel
    (sum, sumsq) partials of the output; ``in_stats`` ([N][cin][2] sums over ``in_hw``
    pixels) normalises the input (instance norm; ``in_relu`` bit 0: relu, bit 1: relu before the
    residual add) as it is loaded;
    ``in_res`` (+ ``in_res_stats``: normalised too) is added before the relu (a residual
    block's output built on the fly) and ``xn`` receives the built input."""
    OH, OW = out_hw if out_hw is not None else spec.out_hw(H, W)
    if cfg is None:
        cfg = pick_cfg(N * OH * OW, spec.cout)
    t = [x, spec.w, spec.b, y, y2, res, h32, zbuf, coords, flow32, y3, bmap]
    if tapw is not None:
        t.append(tapw)
    elif cfg >= HALO_CFG0:   # the halo 3x3 kernel (conv_halo.hip): its own weight stream
        assert spec.wh is not None, "halo tile config for a conv without halo weights"
        t.append(spec.wh)
        if in_res is not None or in_res_stats is not None or xn is not None:
            t += [stats_part, in_stats, in_res, in_res_stats, xn]
        elif stats_part is not None or in_stats is not None:
            t += [stats_part, in_stats]
    assert (stats_part is None and in_stats is None and in_res is None and xn is None) or cfg >= HALO_CFG0, \
        "stats / input norm need a halo config"
    i = [N, H, W, x_coff, spec.cin8, spec.kh, spec.kw, spec.sh, spec.sw, spec.ph, spec.pw, spec.cout, act, split,
         y_coff, y2_coff, res_coff, hidden, y3_coff, epi, cfg, res_post]
    if bmap is not None or out_hw is not None or in_stats is not None:
        i += [OH if out_hw is not None else 0, OW if out_hw is not None else 0, 0, 0, bmap_coff]
    if in_stats is not None:
        i += [int(in_relu), int(in_hw)]
    return t, i, float(alpha)


def pack_convex_head(kernel: torch.Tensor, bias: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """MaskPredictor 1x1 conv (1, 1, 256, 576) -> the A-fragment order of
    csrc/kernels/convex_head.hip: [kstep 8][tap 9][wave 4][lane 64][8] bf16 with
    lane = 16 q + r holding W[ci = 32 kstep + 8 q + j][co = 64 tap + 16 wave + r]
    (co in the reference order k*64 + s, ``model.py:86``); bias stays fp32 [576]."""
    kh, kw, cin, c = kernel.shape
    assert (kh, kw, cin, c) == (1, 1, 256, 576), kernel.shape
    wc = kernel.detach().float().reshape(8, 4, 8, 9, 4, 16)      # (ks, q, j, k, w, r)
    wp = wc.permute(0, 3, 4, 1, 5, 2).contiguous().to(torch.bfloat16)
    return wp.reshape(-1), bias.detach().float().contiguous()


def pack_taps_epi(kernel: torch.Tensor) -> torch.Tensor:
    """FlowHead conv2 (3, 3, 256, 2) -> the A fragments of the EPI_TAPS conv
    epilogue (csrc/kernels/conv_igemm.h:taps_epilogue): [group 4][kstep 2][tile 2][lane 64][8]
    bf16 with lane = 16 q + r holding Wt[o = 16 tile + r][c = 64 group + 16 q + 8 kstep + j],
    Wt[o = 2 tap + comp][c] = W[tap // 3, tap % 3, c, comp] (rows 18..31 zero) -- the k
    order of the 16 contiguous channels each conv1 epilogue lane owns."""
    kh, kw, cin, co = kernel.shape
    assert (kh, kw, cin, co) == (3, 3, 256, 2), kernel.shape
    dev = kernel.device
    wt = torch.zeros(32, 256, dtype=torch.float32, device=dev)
    wt[:18] = kernel.detach().float().reshape(9, cin, 2).permute(0, 2, 1).reshape(18, cin)
    g = torch.arange(4, device=dev).view(4, 1, 1, 1, 1)
    s = torch.arange(2, device=dev).view(1, 2, 1, 1, 1)
    t = torch.arange(2, device=dev).view(1, 1, 2, 1, 1)
    lane = torch.arange(64, device=dev).view(1, 1, 1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, 1, 8)
    o = 16 * t + lane % 16
    c = 64 * g + 16 * (lane // 16) + 8 * s + j
    return wt[o.expand(4, 2, 2, 64, 8), c.expand(4, 2, 2, 64, 8)].to(torch.bfloat16).contiguous()


CONV1X1_KPADS = (128, 256, 352, 384)


def pack_conv1x1(kernel: torch.Tensor, kpad: int) -> torch.Tensor:
    """1x1 conv (1, 1, K, N) -> the A fragments of conv1x1.hip: per output group
    g of 64 channels [g][k-step kpad/32][row tile 4][lane 64][8] bf16, lane =
    16 q + r holding W[k = 32 ks + 8 q + j][co = 64 g + 16 (r >> 2) + 4 t + (r & 3)]
    (zero for k >= K), so that a lane's accumulators are 16 contiguous channels."""
    _, _, K, N = kernel.shape
    assert N % 64 == 0 and K <= kpad and kpad % 32 == 0, (kernel.shape, kpad)
    w = torch.zeros(kpad, N, dtype=torch.float32, device=kernel.device)
    w[:K] = kernel.detach().float().reshape(K, N)
    dev = kernel.device
    g, ks, t, l, j = torch.meshgrid(torch.arange(N // 64, device=dev), torch.arange(kpad // 32, device=dev),
                                    torch.arange(4, device=dev), torch.arange(64, device=dev),
                                    torch.arange(8, device=dev), indexing="ij")
    r = l & 15
    k = 32 * ks + 8 * (l >> 4) + j
    co = 64 * g + 16 * (r >> 2) + 4 * t + (r & 3)
    return w[k, co].to(torch.bfloat16).reshape(-1).contiguous()


def conv1x1(x: torch.Tensor, wpk: torch.Tensor, bias: torch.Tensor, kvalid: int, kpad: int, cout: int,
            act: int = ACT_NONE) -> torch.Tensor:
    """Eager pointwise conv with LDS-resident weights: x bf16 [M][cs] -> bf16 [M][cout]."""
    M = x.shape[0]
    y = torch.empty(M, cout, device=x.device, dtype=torch.bfloat16)
    ops().conv1x1([x, wpk, bias, y], [M, kvalid, kpad, cout, act, 0])
    return y


def pack_taps(kernel: torch.Tensor) -> torch.Tensor:
    """Flow head output conv (3, 3, K, 2) -> the A fragments of
    flowhead.hip:taps_gemm_kernel: rows o = tap * 2 + c (18 real of 32), packed
    [k-step K/32][row tile 2][lane 64][8] bf16 with lane = 16 q + r holding
    W[k = 32 ks + 8 q + j][o = 16 t + r]."""
    kh, kw, K, co = kernel.shape
    assert (kh, kw, co) == (3, 3, 2) and K % 32 == 0, kernel.shape
    w = kernel.detach().float().reshape(9, K, 2).permute(1, 0, 2).reshape(K, 18)     # [k][tap * 2 + c]
    a = torch.zeros(K, 32, dtype=torch.float32, device=kernel.device)
    a[:, :18] = w
    a = a.reshape(K // 32, 4, 8, 2, 16)            # (ks, q, j, t, r)
    return a.permute(0, 3, 1, 4, 2).contiguous().to(torch.bfloat16).reshape(-1)


def taps_gemm(fm: torch.Tensor, wpk: torch.Tensor, K: int, coff: int = 0) -> torch.Tensor:
    """Eager flow-head taps: fm bf16 [M][cs] -> fp32 [M][24]."""
    M = fm.shape[0]
    out = torch.empty(M, 24, device=fm.device, dtype=torch.float32)
    ops().taps_gemm([fm, wpk, out], [M, K, coff])
    return out


def convex_head(feat: torch.Tensor, wpk: torch.Tensor, bias: torch.Tensor, flow: torch.Tensor, B: int, h: int,
                w: int, alpha: float, coff: int = 0, out: Optional[torch.Tensor] = None, tiles: int = 0) -> torch.Tensor:
    """Eager fused mask head: feat bf16 [M][cs] (channels coff..coff+256), flow fp32
    [M][2] -> upsampled flow (B, 8h, 8w, 2) (csrc/kernels/convex_head.hip)."""
    if out is None:
        out = torch.empty(B, 8 * h, 8 * w, 2, device=feat.device, dtype=torch.float32)
    ops().convex_head([feat, wpk, bias, flow, out], [B, h, w, coff, 0, tiles], float(alpha))
    return out


def conv2d(spec: ConvSpec, x: torch.Tensor, act: int = ACT_NONE, out_dtype=torch.bfloat16, alpha: float = 1.0,
           res: Optional[torch.Tensor] = None, res_post: int = 0, cfg: Optional[int] = None) -> torch.Tensor:
    """Eager NHWC conv of a contiguous bf16 tensor [N, H, W, C] (C == cin8)."""
    N, H, W, C = x.shape
    assert C == spec.cin8, f"input channels {C} != packed cin8 {spec.cin8}"
    OH, OW = spec.out_hw(H, W)
    y = torch.empty(N, OH, OW, round_up(spec.cout, 8), device=x.device, dtype=out_dtype)
    t, i, a = conv_args(spec, x, N, H, W, y, act=act, alpha=alpha, res=res, res_post=res_post, cfg=cfg)
    ops().conv(t, i, a)
    return y[..., : spec.cout] if y.shape[-1] != spec.cout else y


# ------------------------------------------------------ fp32 parity mode convs


@dataclass
class ConvSpecF32:
    """A conv for the fp32 implicit-GEMM kernel (csrc/kernels/conv_f32.hip):
    ``w`` fp32 [cout, K], K ordered (kh, kw, cin4) with the input channels
    zero-padded to ``cin4`` (a multiple of 4), rows in natural channel order;
    ``b`` fp32 [cout]."""

    w: torch.Tensor
    b: torch.Tensor
    kh: int
    kw: int
    sh: int
    sw: int
    ph: int
    pw: int
    cin: int
    cin4: int
    cout: int

    def out_hw(self, H: int, W: int) -> Tuple[int, int]:
        return (H + 2 * self.ph - self.kh) // self.sh + 1, (W + 2 * self.pw - self.kw) // self.sw + 1


def pack_weight_f32(kernel: torch.Tensor, cin4: Optional[int] = None) -> torch.Tensor:
    """HWIO kernel -> fp32 [cout, kh*kw*cin4] (input channels zero-padded)."""
    kh, kw, cin, cout = kernel.shape
    cin4 = cin4 or round_up(cin, 4)
    assert cin4 >= cin and cin4 % 4 == 0
    k = torch.zeros(kh, kw, cin4, cout, dtype=torch.float32, device=kernel.device)
    k[:, :, :cin, :] = kernel.detach().float()
    return k.permute(3, 0, 1, 2).reshape(cout, kh * kw * cin4).contiguous()


def make_spec_f32(kernel: torch.Tensor, bias: torch.Tensor, stride=(1, 1), padding=(0, 0),
                  cin4: Optional[int] = None, device=None) -> ConvSpecF32:
    kh, kw, cin, cout = kernel.shape
    cin4 = cin4 or round_up(cin, 4)
    w = pack_weight_f32(kernel.to(device) if device is not None else kernel, cin4)
    b = bias.detach().float().to(w.device).contiguous()
    return ConvSpecF32(w, b, kh, kw, stride[0], stride[1], padding[0], padding[1], cin, cin4, cout)


def conv_f32_args(spec: ConvSpecF32, x: torch.Tensor, N: int, H: int, W: int, y: torch.Tensor, *, x_coff: int = 0,
                  y_coff: int = 0, act: int = ACT_NONE, split: int = 0, alpha: float = 1.0, y2=None, y2_coff: int = 0,
                  res=None, res_coff: int = 0, res_post: int = 0, h32=None, zbuf=None, hidden: int = 0, bmap=None,
                  bmap_coff: int = 0, epi: int = EPI_STD, ksplit: int = 0):
    """(tensors, ints, alpha) of the ``conv_f32`` op / ``Plan.add_conv_f32``; ``ksplit`` > 0 forces
    an n-way split-K (0: the kernel's own choice)."""
    t = [x, spec.w, spec.b, y, y2, res, h32, zbuf, bmap]
    i = [N, H, W, x_coff, spec.cin4, spec.kh, spec.kw, spec.sh, spec.sw, spec.ph, spec.pw, spec.cout, act, split,
         y_coff, y2_coff, res_coff, res_post, hidden, bmap_coff, epi, ksplit]
    return t, i, float(alpha)


def conv2d_f32(spec: ConvSpecF32, x: torch.Tensor, act: int = ACT_NONE, alpha: float = 1.0, res=None,
               res_post: int = 0) -> torch.Tensor:
    """Eager fp32 NHWC conv (x: (N, H, W, C >= cin4) fp32) -> (N, OH, OW, cout)."""
    N, H, W, _ = x.shape
    OH, OW = spec.out_hw(H, W)
    y = torch.empty((N, OH, OW, spec.cout), dtype=torch.float32, device=x.device)
    ops().conv_f32(*conv_f32_args(spec, x, N, H, W, y, act=act, alpha=alpha, res=res, res_post=res_post))
    return y
