// All-pairs correlation pyramid and radius-r pyramid lookup (gfx950).
//
// Reference: CorrBlock in jax_raft/model.py:403-481 -- build_pyramid
// (matmul / sqrt(C) then 2x2 VALID avg-pool L-1 times, :418-446, :472-481) and
// index_pyramid (grid_sample of a (2r+1)^2 window around coords/2^l,
// :448-470; grid_sample itself :24-34).
//
// corr_pyramid_kernel: one MFMA GEMM tile = 128 query pixels (A operand,
// rows) x a 2-D 8x16 block of target pixels (B operand, columns).  Because
// the target tile is a spatially aligned 8x16 block, every pyramid level's
// 2x2 pooling is formed in-register (tile pairs for y, lane shuffles for x)
// and all L levels are written by the same kernel: the level-0 volume is
// never re-read to build the pyramid.  Floor semantics: only cells whose
// full 2^l x 2^l footprint is inside the map are emitted.
//
// corr_lookup_kernel: one wave per query pixel; lane = (level, window
// column).  All (2r+1)^2 samples of a level share one fractional offset, so
// each lane loads one (2r+2)-tall column of the level map, interpolates
// vertically, and takes the horizontal neighbour column from lane+1 via a
// shuffle.  Output channels follow the reference order
// l*(2r+1)^2 + i*(2r+1) + j (x-offset i-r is the slow index), staged in LDS
// and written as 16-B vectors, zero-padded to the consumer's channel stride.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;
JR_DEVICE int swz(int row) { return (row >> 1) & 7; }

// 4 waves x (TM=2 query tiles of 16) = 128 queries; TN = 8 target rows x 16 cols.
constexpr int CQ = 128;
constexpr int TY = 8, TX = 16;
constexpr int CT = TY * TX;

template <typename T>
JR_DEVICE T cvt_out(float v);
template <>
JR_DEVICE float cvt_out<float>(float v) { return v; }
template <>
JR_DEVICE bf16 cvt_out<bf16>(float v) { return f2bf(v); }
JR_DEVICE float to_f(float v) { return v; }
JR_DEVICE float to_f(bf16 v) { return bf2f(v); }

template <typename T, bool WIDE>
__global__ __launch_bounds__(256) void corr_pyramid_kernel(const bf16* __restrict__ f1, const bf16* __restrict__ f2,
                                                           int h, int w, int nq, int C, int cs, T* __restrict__ l0,
                                                           T* __restrict__ l1, T* __restrict__ l2,
                                                           T* __restrict__ l3, int nlev, float scale, int blocked) {
  constexpr int TM = 2, TN = 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (CQ + CT) * BK];
  const int P = h * w;
  // 1-D grid, XCD-aware order: MI355X dispatches blocks round-robin over its 8
  // XCDs, so block id k runs on XCD k % 8.  Each XCD walks a contiguous run of
  // tasks, and tasks are ordered (image, query tile, target row, target tile)
  // with the target tile fastest: the 16-wide tiles that share a 128-byte
  // line of a query's level-0 / level-1 row are written back to back from one
  // L2, which then evicts whole lines instead of 32-byte pieces from 8 L2s.
  const int ntx = (w + TX - 1) / TX, nty = (h + TY - 1) / TY, nqt = (nq + CQ - 1) / CQ;
  int task = blockIdx.x;
  {
    const int nwg = gridDim.x, xcd = task & 7, qq = nwg >> 3, rr = nwg & 7;
    if (nwg > 8) task = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (task >> 3);
  }
  const int tx0 = (task % ntx) * TX;
  const int ty0 = ((task / ntx) % nty) * TY;
  const int q0 = ((task / (ntx * nty)) % nqt) * CQ;
  const int b = task / (ntx * nty * nqt);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & 7;
  const bf16* A = f1 + (long)b * nq * cs;
  const bf16* Bm = f2 + (long)b * P * cs;

  // each thread loads 4 query rows and 4 target rows (chunk ch of 8)
  long aoff[4], boff[4];
  bool aok[4], bok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int q = q0 + r;
    aok[i] = q < nq;
    aoff[i] = (long)(aok[i] ? q : 0) * cs;
    const int ty = ty0 + (r >> 4), tx = tx0 + (r & 15);
    bok[i] = ty < h && tx < w;
    boff[i] = (long)(bok[i] ? ty * w + tx : 0) * cs;
  }
  u32x4 ar[4], br[4];
  auto load = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ar[i] = aok[i] ? *(const u32x4*)(A + aoff[i] + ks * BK + ch * 8) : u32x4{0u, 0u, 0u, 0u};
      br[i] = bok[i] ? *(const u32x4*)(Bm + boff[i] + ks * BK + ch * 8) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int buf) {
    bf16* sA = smem + buf * (CQ + CT) * BK;
    bf16* sB = sA + CQ * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *(u32x4*)(sA + r * BK + ((ch ^ swz(r)) << 3)) = ar[i];
      *(u32x4*)(sB + r * BK + ((ch ^ swz(r)) << 3)) = br[i];
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int c = 0; c < TN; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nks = C / BK;
  load(0);
  store(0);
  __syncthreads();
  const int li = lane & 15, lq = lane >> 4;
  for (int ks = 0; ks < nks; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nks;
    if (more) load(ks + 1);
    const bf16* sA = smem + cur * (CQ + CT) * BK;
    const bf16* sB = sA + CQ * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + lq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wave * (TM * 16) + tm * 16 + li;
        af[tm] = *(const bf16x8*)(sA + row * BK + ((chunk ^ swz(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = tn * 16 + li;
        bfr[tn] = *(const bf16x8*)(sB + row * BK + ((chunk ^ swz(row)) << 3));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
    if (more) store(cur ^ 1);
    __syncthreads();
  }

  // Epilogue: D[query = qbase + 4*lq + r][target = (ty0 + tn, tx0 + li)]
  const int x0 = tx0 + li;
  const int h1 = h >> 1, w1 = w >> 1, h2 = h1 >> 1, w2 = w1 >> 1, h3 = h2 >> 1, w3 = w2 >> 1;
  // WIDE (bf16 levels, w % 16 == 0): the tile's level blocks (per query 8x16,
  // 4x8, 2x4, 1x2) are staged in LDS (the GEMM buffers are free now) and
  // written with 16 / 16 / 8 / 4-byte stores.  Per-lane 2-byte stores cost the
  // vector memory pipe about a cycle per lane: 452 us for the raft_large
  // batch-4 pyramid, bound by store issue, not by its 500 MB of writes.
  bf16* st0 = smem;                       // [CQ][TY][TX]
  bf16* st1 = st0 + CQ * CT;              // [CQ][TY/2][TX/2]
  bf16* st2 = st1 + CQ * CT / 4;          // [CQ][TY/4][TX/4]
  bf16* st3 = st2 + CQ * CT / 16;         // [CQ][TY/8][TX/8]
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = wave * (TM * 16) + tm * 16 + 4 * lq + r;
      const int q = q0 + qi;
      const bool qok = q < nq;
      float v[TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) v[tn] = acc[tm][tn][r] * scale;
      // level 0
      if constexpr (WIDE) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) st0[(qi * TY + tn) * TX + li] = f2bf(v[tn]);
      } else if (qok && x0 < w) {
        T* dst = l0 + ((long)b * nq + q) * P;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          if (ty0 + tn < h) dst[(ty0 + tn) * w + x0] = cvt_out<T>(v[tn]);
      }
      if (nlev < 2) continue;
      // level 1: pairs of rows (tn, tn+1), lanes (li, li^1)
      float v1[TN / 2];
#pragma unroll
      for (int t = 0; t < TN / 2; ++t) {
        const float s = v[2 * t] + v[2 * t + 1];
        v1[t] = 0.25f * (s + __shfl_xor(s, 1));
      }
      {
        const int X1 = x0 >> 1;
        if constexpr (WIDE) {
          if ((li & 1) == 0) {
#pragma unroll
            for (int t = 0; t < TN / 2; ++t) st1[(qi * (TY / 2) + t) * (TX / 2) + (li >> 1)] = f2bf(v1[t]);
          }
        } else if (qok && (li & 1) == 0 && X1 < w1) {
          T* dst = l1 + ((long)b * nq + q) * (h1 * w1);
#pragma unroll
          for (int t = 0; t < TN / 2; ++t) {
            const int Y1 = (ty0 >> 1) + t;
            if (Y1 < h1) dst[Y1 * w1 + X1] = cvt_out<T>(v1[t]);
          }
        }
      }
      if (nlev < 3) continue;
      float v2[TN / 4];
#pragma unroll
      for (int t = 0; t < TN / 4; ++t) {
        const float s = v1[2 * t] + v1[2 * t + 1];
        v2[t] = 0.25f * (s + __shfl_xor(s, 2));
      }
      {
        const int X2 = x0 >> 2;
        if constexpr (WIDE) {
          if ((li & 3) == 0) {
#pragma unroll
            for (int t = 0; t < TN / 4; ++t) st2[(qi * (TY / 4) + t) * (TX / 4) + (li >> 2)] = f2bf(v2[t]);
          }
        } else if (qok && (li & 3) == 0 && X2 < w2) {
          T* dst = l2 + ((long)b * nq + q) * (h2 * w2);
#pragma unroll
          for (int t = 0; t < TN / 4; ++t) {
            const int Y2 = (ty0 >> 2) + t;
            if (Y2 < h2) dst[Y2 * w2 + X2] = cvt_out<T>(v2[t]);
          }
        }
      }
      if (nlev < 4) continue;
      {
        const float s = v2[0] + v2[1];
        const float v3 = 0.25f * (s + __shfl_xor(s, 4));
        const int X3 = x0 >> 3;
        const int Y3 = ty0 >> 3;
        if constexpr (WIDE) {
          if ((li & 7) == 0) st3[qi * (TX / 8) + (li >> 3)] = f2bf(v3);
        } else if (qok && (li & 7) == 0 && X3 < w3 && Y3 < h3) {
          l3[((long)b * nq + q) * (h3 * w3) + Y3 * w3 + X3] = cvt_out<T>(v3);
        }
      }
    }
  }
  if constexpr (WIDE) {
    __syncthreads();
    if (blocked) {
      // levels 0 / 1: the query's block is contiguous (tile rows past h land in padding rows)
      const long blk = (long)(ty0 / TY) * ntx + tx0 / TX;
      const long qs0 = (long)nty * ntx * CT, qs1 = qs0 / 4;
#pragma unroll
      for (int i = tid; i < CQ * 16; i += 256) {
        const int qi = i >> 4, c = i & 15;
        if (q0 + qi < nq)
          *(u32x4*)((bf16*)l0 + ((long)b * nq + q0 + qi) * qs0 + blk * CT + 8 * c) = *(const u32x4*)(st0 + qi * CT + 8 * c);
      }
      if (nlev >= 2) {
        for (int i = tid; i < CQ * 4; i += 256) {
          const int qi = i >> 2, c = i & 3;
          if (q0 + qi < nq)
            *(u32x4*)((bf16*)l1 + ((long)b * nq + q0 + qi) * qs1 + blk * (CT / 4) + 8 * c) =
                *(const u32x4*)(st1 + qi * (CT / 4) + 8 * c);
        }
      }
    }
    // level 0: per query 8 rows x 2 chunks of 8; consecutive threads -> one query's chunks
#pragma unroll
    for (int i = tid; !blocked && i < CQ * TY * 2; i += 256) {
      const int qi = i >> 4, row = (i >> 1) & 7, half = i & 1;
      const int q = q0 + qi;
      if (q < nq && ty0 + row < h)
        *(u32x4*)((bf16*)l0 + ((long)b * nq + q) * P + (ty0 + row) * w + tx0 + 8 * half) =
            *(const u32x4*)(st0 + (qi * TY + row) * TX + 8 * half);
    }
    if (nlev >= 2 && !blocked) {
      for (int i = tid; i < CQ * (TY / 2); i += 256) {   // 4 rows x 8 (16 B)
        const int qi = i >> 2, row = i & 3;
        const int q = q0 + qi, Y1 = (ty0 >> 1) + row;
        if (q < nq && Y1 < h1)
          *(u32x4*)((bf16*)l1 + ((long)b * nq + q) * (h1 * w1) + Y1 * w1 + (tx0 >> 1)) =
              *(const u32x4*)(st1 + (qi * (TY / 2) + row) * (TX / 2));
      }
    }
    if (nlev >= 3) {
      for (int i = tid; i < CQ * (TY / 4); i += 256) {   // 2 rows x 4 (8 B)
        const int qi = i >> 1, row = i & 1;
        const int q = q0 + qi, Y2 = (ty0 >> 2) + row;
        if (q < nq && Y2 < h2)
          *(u32x2*)((bf16*)l2 + ((long)b * nq + q) * (h2 * w2) + Y2 * w2 + (tx0 >> 2)) =
              *(const u32x2*)(st2 + (qi * (TY / 4) + row) * (TX / 4));
      }
    }
    if (nlev >= 4) {
      for (int i = tid; i < CQ; i += 256) {               // 1 row x 2 (4 B)
        const int q = q0 + i, Y3 = ty0 >> 3;
        if (q < nq && Y3 < h3)
          *(unsigned*)((bf16*)l3 + ((long)b * nq + q) * (h3 * w3) + Y3 * w3 + (tx0 >> 3)) =
              *(const unsigned*)(st3 + i * (TX / 8));
      }
    }
  }
}

struct LevelPtrs {
  const void* p[4];
};

// Level layout.  Row-major: [hl][wl] per query.  Blocked (inference, bf16
// levels of /16-wide maps): levels 0 and 1 are stored as the correlation tile
// grid's blocks, [ceil(h/8)][ceil(w/16)] blocks of (8 >> l) x (16 >> l)
// elements (256 / 64 B), i.e. exactly what one corr_pyramid_kernel tile
// produces per query: the pyramid writes whole cache lines, and a lookup
// window (10 x 10) touches 2 x 2 blocks instead of 10 row segments.  Levels
// 2 and 3 stay row-major.
struct LvGeom {
  int blocked, nty, ntx;
};
JR_DEVICE long lv_qstride(const LvGeom& g, int l, int hl, int wl) {
  return (g.blocked && l < 2) ? (long)g.nty * g.ntx * (128 >> (2 * l)) : (long)hl * wl;
}
JR_DEVICE int lv_off(const LvGeom& g, int l, int wl, int y, int x) {  // y, x >= 0
  if (g.blocked && l < 2) {
    const int sh = 3 - l, sw = 4 - l;
    return (((y >> sh) * g.ntx + (x >> sw)) << (sh + sw)) + ((y & ((1 << sh) - 1)) << sw) + (x & ((1 << sw) - 1));
  }
  return y * wl + x;
}

// Query coordinates of a lookup wave (QPW queries q0 ..), with the optional
// fused flow update (TapsUpd): lane 18 k + 2 t + c loads tap t, component c of
// query k's 3x3 neighbour (zero outside the image); lanes 18 k + c sum bias[c]
// and the nine taps in jr_flow_taps' order, store the new coords / flow, and
// every lane receives the new coords by shuffle.  All lanes take part.
template <int QPW>
JR_DEVICE void lookup_coords(const TapsUpd& u, const float* coords, int q0, int total, int h, int w, int lane,
                             float (&cx)[QPW], float (&cy)[QPW]) {
  static_assert(QPW * 18 <= 64, "QPW");
  if (!u.on) {
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
      const int q = q0 + k;
      cx[k] = q < total ? coords[2 * (long)q] : 0.f;
      cy[k] = q < total ? coords[2 * (long)q + 1] : 0.f;
    }
    return;
  }
  const int uq = lane / 18, k = lane - uq * 18;
  const int tap = k >> 1, c = k & 1;
  const long q = (long)q0 + uq;
  const bool own = uq < QPW && q < total;
  const int hw = h * w;
  int y = 0, x = 0;
  float val = 0.f;
  if (own) {
    const int rem = (int)(q % hw);
    y = rem / w;
    x = rem - y * w;
    const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
    if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
      val = u.taps[(q - rem + (long)yy * w + xx) * u.tcs + k];
  }
  float d = u.bias[c];
#pragma unroll
  for (int t = 0; t < 9; ++t) d += __shfl(val, min(uq * 18 + 2 * t + c, 63));
  float cn = 0.f;
  if (own && k < 2) {
    cn = coords[2 * q + k] + d;
    u.coords[2 * q + k] = cn;
    const float f = cn - (float)(k == 0 ? x : y);
    u.flow32[2 * q + k] = f;
    const bf16 fb = f2bf(f);
    ((bf16*)u.hx)[q * u.hx_cs + u.hx_off + k] = fb;
    if (u.qx) ((bf16*)u.qx)[q * u.qx_cs + u.qx_off + k] = fb;
    if (u.f8) ((bf16*)u.f8)[q * u.f8_cs + k] = fb;
  }
#pragma unroll
  for (int kk = 0; kk < QPW; ++kk) {
    cx[kk] = __shfl(cn, kk * 18);
    cy[kk] = __shfl(cn, kk * 18 + 1);
  }
}

// blockDim = 256: 4 waves x QPW queries each; lane = level*16 + window column i.
// General-shape path (any level size); see corr_lookup_wide_kernel below for
// the fast path.
template <int R, typename T, int QPW>
__global__ __launch_bounds__(256) void corr_lookup_kernel(LevelPtrs lv, int nlev, int total, int h, int w,
                                                          const float* coords, bf16* __restrict__ out,
                                                          int ocs, LvGeom geo, TapsUpd upd) {
  constexpr int S = 2 * R + 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q0 = (blockIdx.x * 4 + wave) * QPW;
  bf16* st = (bf16*)dyn_smem + wave * QPW * ocs;  // [QPW][ocs]
  for (int c = lane; c < QPW * ocs; c += 64) st[c] = f2bf(0.f);
  const int lvl = lane >> 4;
  const int i = lane & 15;
  const bool on = lvl < nlev && i <= S;
  const float sc = 1.0f / (float)(1 << lvl);
  const int hl = h >> lvl, wl = w >> lvl;
  float qcx[QPW], qcy[QPW];
  lookup_coords<QPW>(upd, coords, q0, total, h, w, lane, qcx, qcy);
  float fx[QPW], fy[QPW], colv[QPW][S + 1];
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    const int q = q0 + u;
    fx[u] = fy[u] = 0.f;
#pragma unroll
    for (int j = 0; j <= S; ++j) colv[u][j] = 0.f;
    if (q < total && on) {
      const float cx = qcx[u] * sc, cy = qcy[u] * sc;
      const float flx = floorf(cx), fly = floorf(cy);
      fx[u] = cx - flx;
      fy[u] = cy - fly;
      const int col = (int)flx - R + i;
      const int row0 = (int)fly - R;
      const T* map = (const T*)lv.p[lvl] + (long)q * lv_qstride(geo, lvl, hl, wl);
      const bool colok = (unsigned)col < (unsigned)wl;
#pragma unroll
      for (int j = 0; j <= S; ++j) {
        const int rr = row0 + j;
        if (colok && (unsigned)rr < (unsigned)hl) colv[u][j] = to_f(map[lv_off(geo, lvl, wl, rr, col)]);
      }
    }
  }
  __syncthreads();  // staging zeroed
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    float vv[S];
#pragma unroll
    for (int j = 0; j < S; ++j) vv[j] = (1.f - fy[u]) * colv[u][j] + fy[u] * colv[u][j + 1];
    // horizontal interpolation with the neighbouring column (lane + 1)
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const float nb = __shfl_down(vv[j], 1);
      vv[j] = (1.f - fx[u]) * vv[j] + fx[u] * nb;
    }
    if (q0 + u < total && lvl < nlev && i < S) {
      const int base = u * ocs + lvl * S * S + i * S;
#pragma unroll
      for (int j = 0; j < S; ++j) st[base + j] = f2bf(vv[j]);
    }
  }
  __syncthreads();
  // the wave's QPW output rows are contiguous: [q0, q0 + QPW) x ocs
  const int nq = min(QPW, total - q0);
  if (nq > 0) {
    bf16* dst = out + (long)q0 * ocs;
    for (int c = lane * 8; c < nq * ocs; c += 64 * 8) *(u32x4*)(dst + c) = *(const u32x4*)(st + c);
  }
}

// Wide-load lookup (every level's row length and map size a multiple of one
// 16-byte chunk, 16-byte aligned levels: raft's /64-wide frames).  The
// per-lane 2-byte column loads above cost ~1 cycle per lane address in the
// vector memory pipe (67 cycles per load instruction measured at raft_large
// batch 4, 31 us per lookup, with only 35 MB fetched).  Here a query's window
// rows are fetched as aligned 16-byte chunks: (2r+2) rows x NCH chunks per
// level, e.g. 120 lane-loads = 2 instructions per query instead of 10, into a
// per-wave LDS window image [query][level][row][NCH * EPC]; the bilinear
// taps are then read from LDS (no shuffles).  Chunks are wholly inside or
// wholly outside a row (row length % EPC == 0), so zero padding stays exact.
template <int R, typename T, int QPW>
__global__ __launch_bounds__(256) void corr_lookup_wide_kernel(LevelPtrs lv, int nlev, int total, int h, int w,
                                                               const float* coords,
                                                               bf16* __restrict__ out, int ocs, LvGeom geo,
                                                               TapsUpd upd) {
  constexpr int S = 2 * R + 1;
  constexpr int EPC = 16 / sizeof(T);                   // elements per chunk
  constexpr int NCH = (S + 1 + EPC - 1) / EPC + 1;      // chunks per window row
  constexpr int RW = NCH * EPC;                         // image row length (elements)
  constexpr int NT = QPW * 4 * (S + 1) * NCH;           // chunk loads per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q0 = (blockIdx.x * 4 + wave) * QPW;
  T* win = (T*)dyn_smem + (long)wave * NT * EPC;                       // [QPW][4][S+1][RW]
  bf16* st = (bf16*)(dyn_smem + 4L * NT * 16) + wave * QPW * ocs;     // [QPW][ocs]
  for (int c = lane; c < QPW * ocs; c += 64) st[c] = f2bf(0.f);
  float qcx[QPW], qcy[QPW];
  lookup_coords<QPW>(upd, coords, q0, total, h, w, lane, qcx, qcy);
  u32x4 v[(NT + 63) / 64];
#pragma unroll
  for (int n = 0; n < (NT + 63) / 64; ++n) {
    const int t = n * 64 + lane;
    v[n] = u32x4{0u, 0u, 0u, 0u};
    const int k = t % NCH, j = (t / NCH) % (S + 1), l = (t / (NCH * (S + 1))) % 4, u = t / (NCH * (S + 1) * 4);
    const int q = q0 + u;
    float ucx = qcx[0], ucy = qcy[0];
#pragma unroll
    for (int kk = 1; kk < QPW; ++kk)
      if (u == kk) { ucx = qcx[kk]; ucy = qcy[kk]; }
    if (t < NT && q < total && l < nlev) {
      const float sc = 1.0f / (float)(1 << l);
      const int hl = h >> l, wl = w >> l;
      const int col0 = (int)floorf(ucx * sc) - R;
      const int rr = (int)floorf(ucy * sc) - R + j;
      const int c0 = (col0 >= 0 ? col0 / EPC : -((-col0 + EPC - 1) / EPC)) * EPC;
      const int cc = c0 + k * EPC;
      // the window row [col0, col0 + S] needs its last chunk only when it reaches into it
      // (bf16, R = 4: 1 of 8 alignments): skipping it drops ~1/3 of the fetched chunks
      const bool need = k < NCH - 1 || col0 - c0 + S >= (NCH - 1) * EPC;
      if (need && (unsigned)rr < (unsigned)hl && (unsigned)cc < (unsigned)wl)
        v[n] = *(const u32x4*)((const T*)lv.p[l] + (long)q * lv_qstride(geo, l, hl, wl) + lv_off(geo, l, wl, rr, cc));
    }
  }
#pragma unroll
  for (int n = 0; n < (NT + 63) / 64; ++n) {
    const int t = n * 64 + lane;
    if (t < NT) ((u32x4*)win)[t] = v[n];
  }
  __syncthreads();
  const int l = lane >> 4, i = lane & 15;
  if (l < nlev && i < S) {
    const float sc = 1.0f / (float)(1 << l);
#pragma unroll
    for (int u = 0; u < QPW; ++u) {
      const int q = q0 + u;
      if (q >= total) break;
      const float cx = qcx[u] * sc, cy = qcy[u] * sc;
      const float flx = floorf(cx), fly = floorf(cy);
      const float fx = cx - flx, fy = cy - fly;
      const int col0 = (int)flx - R;
      const int o = col0 - (col0 >= 0 ? col0 / EPC : -((-col0 + EPC - 1) / EPC)) * EPC;  // col0 mod EPC
      const T* wr = win + ((u * 4 + l) * (S + 1)) * RW + o + i;
      float a0 = to_f(wr[0]), a1 = to_f(wr[1]);
      const int base = u * ocs + l * S * S + i * S;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const float b0 = to_f(wr[(j + 1) * RW]), b1 = to_f(wr[(j + 1) * RW + 1]);
        const float top = (1.f - fx) * a0 + fx * a1, bot = (1.f - fx) * b0 + fx * b1;
        st[base + j] = f2bf((1.f - fy) * top + fy * bot);
        a0 = b0;
        a1 = b1;
      }
    }
  }
  __syncthreads();
  const int nq = min(QPW, total - q0);
  if (nq > 0) {
    bf16* dst = out + (long)q0 * ocs;
    for (int c = lane * 8; c < nq * ocs; c += 64 * 8) *(u32x4*)(dst + c) = *(const u32x4*)(st + c);
  }
}

// Backward of the lookup w.r.t. the pyramid levels: grad_out [q][ocs]
// (channel l*S^2 + i*S + j) -> dlevels fp32 [q][hl][wl] (accumulated).
// Lane (level, i) folds the bilinear weights of its (2r+1) samples into the
// (2r+2) cells of window columns x0+i (weight 1-fx) and x0+i+1 (weight fx);
// the x0+i+1 part is handed to lane i+1 by a shuffle, so every cell of the
// (2r+2)^2 window receives exactly one read-modify-write: no atomics, and
// each query's level map is private to that query (no cross-query races).
template <int R, typename G>
__global__ __launch_bounds__(256) void corr_lookup_bwd_kernel(LevelPtrs dlv, int nlev, int total, int h, int w,
                                                              const float* __restrict__ coords,
                                                              const G* __restrict__ gout, int gcs) {
  constexpr int S = 2 * R + 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = blockIdx.x * 4 + wave;
  if (q >= total) return;
  const int lvl = lane >> 4;
  const int i = lane & 15;
  const bool on = lvl < nlev && i <= S;
  float fx = 0.f, fy = 0.f;
  int col = 0, row0 = 0, hl = 1, wl = 1;
  if (on) {
    const float sc = 1.0f / (float)(1 << lvl);
    const float cx = coords[2 * (long)q] * sc, cy = coords[2 * (long)q + 1] * sc;
    const float flx = floorf(cx), fly = floorf(cy);
    fx = cx - flx;
    fy = cy - fly;
    hl = h >> lvl;
    wl = w >> lvl;
    col = (int)flx - R + i;
    row0 = (int)fly - R;
  }
  float a[S + 1], b[S + 1];  // contributions to column x0+i (a) and x0+i+1 (b)
#pragma unroll
  for (int j = 0; j <= S; ++j) { a[j] = 0.f; b[j] = 0.f; }
  if (on && i < S) {
    const G* g = gout + (long)q * gcs + lvl * S * S + i * S;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const float gv = to_f(g[j]);
      a[j] += (1.f - fx) * (1.f - fy) * gv;
      a[j + 1] += (1.f - fx) * fy * gv;
      b[j] += fx * (1.f - fy) * gv;
      b[j + 1] += fx * fy * gv;
    }
  }
#pragma unroll
  for (int j = 0; j <= S; ++j) {
    const float nb = __shfl_up(b[j], 1);
    if (i > 0) a[j] += nb;
  }
  if (on && (unsigned)col < (unsigned)wl) {
    float* map = (float*)dlv.p[lvl] + (long)q * (hl * wl);
#pragma unroll
    for (int j = 0; j <= S; ++j) {
      const int rr = row0 + j;
      if ((unsigned)rr < (unsigned)hl) map[rr * wl + col] += a[j];
    }
  }
}

// The wide kernel needs every level's row length and map size to be a whole
// number of 16-byte chunks and 16-byte aligned level bases.
template <typename T>
bool lookup_wide_ok(const LevelPtrs& lv, int L, int h, int w, const LvGeom& geo) {
  constexpr int EPC = 16 / sizeof(T);
  for (int l = 0; l < L; ++l) {
    const int hl = h >> l, wl = w >> l;
    if (reinterpret_cast<uintptr_t>(lv.p[l]) % 16) return false;
    if (geo.blocked && l < 2) continue;   // 16-byte chunks never cross a block row
    if (wl % EPC || (hl * wl) % EPC) return false;
  }
  return true;
}

template <typename T>
int launch_lookup(const LevelPtrs& lv, int L, int total, int h, int w, int r, const float* coords, bf16* out, int ocs,
                  const LvGeom& geo, const TapsUpd& upd, hipStream_t stream) {
  if (r <= 4 && lookup_wide_ok<T>(lv, L, h, w, geo)) {
    constexpr int QPW = 2;
    constexpr int EPC = 16 / sizeof(T);
    dim3 grid((total + 4 * QPW - 1) / (4 * QPW));
    switch (r) {
#define JR_LKW(RR)                                                                                                    \
  case RR: {                                                                                                        \
    constexpr int NT = QPW * 4 * (2 * RR + 2) * ((2 * RR + 2 + EPC - 1) / EPC + 1);                                 \
    const size_t smem = 4 * NT * 16 + 4 * QPW * ocs * sizeof(bf16);                                                 \
    hipLaunchKernelGGL((corr_lookup_wide_kernel<RR, T, QPW>), grid, dim3(256), smem, stream, lv, L, total, h, w,    \
                       coords, out, ocs, geo, upd);                                                                  \
    break;                                                                                                          \
  }
      JR_LKW(1) JR_LKW(2) JR_LKW(3) JR_LKW(4)
#undef JR_LKW
    }
    return (int)hipGetLastError();
  }
  constexpr int QPW = 1;
  dim3 grid((total + 4 * QPW - 1) / (4 * QPW));
  const size_t smem = 4 * QPW * ocs * sizeof(bf16);
  switch (r) {
#define JR_LK(RR) case RR: hipLaunchKernelGGL((corr_lookup_kernel<RR, T, QPW>), grid, dim3(256), smem, stream, lv, L, total, h, w, coords, out, ocs, geo, upd); break;
    JR_LK(1) JR_LK(2) JR_LK(3) JR_LK(4) JR_LK(5) JR_LK(6)
#undef JR_LK
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int jr_corr_pyramid(const void* f1, const void* f2, int B, int h, int w, int nq, int C, int cs, void* lvl0,
                               void* lvl1, void* lvl2, void* lvl3, int num_levels, float scale, int out_bf16,
                               int blocked, hipStream_t stream) {
  if (C % BK != 0 || cs % 8 != 0 || num_levels < 1 || num_levels > 4 || nq < 1) return (int)hipErrorInvalidValue;
  dim3 grid(((nq + CQ - 1) / CQ) * ((h + TY - 1) / TY) * ((w + TX - 1) / TX) * B);
  // wide stores: whole 16-wide tiles and 16-byte aligned rows / query maps at every level
  bool wide = out_bf16 && w % 16 == 0 && (h * w) % 8 == 0;
  void* lv[4] = {lvl0, lvl1, lvl2, lvl3};
  for (int l = 0; l < num_levels; ++l) wide = wide && reinterpret_cast<uintptr_t>(lv[l]) % 16 == 0;
  if (blocked && !wide) return (int)hipErrorInvalidValue;   // the blocked layout is written by the wide epilogue only
  // the persistent kernel (corr_pyr.hip) holds every CU for the whole build: at batch 1 the
  // pipelined graph runs the previous pair's loop concurrently, and the short-lived tiles of
  // the kernel below interleave with it (measured b1 stream 227 vs 200-204 FPS)
  // blocked == 2: the plan is never replayed next to another forward's loop (runtime/engine.py,
  // not a pipelined slot), so the persistent kernel also serves batch 1
  if (blocked && nq == h * w && (B >= 2 || blocked == 2)) {
    const int e = jr_corr_pyramid_blocked(f1, f2, B, h, w, C, cs, lvl0, lvl1, lvl2, lvl3, num_levels, scale, stream);
    if (e != (int)hipErrorNotSupported) return e;
  }
  if (wide)
    hipLaunchKernelGGL((corr_pyramid_kernel<bf16, true>), grid, dim3(256), 0, stream, (const bf16*)f1, (const bf16*)f2,
                       h, w, nq, C, cs, (bf16*)lvl0, (bf16*)lvl1, (bf16*)lvl2, (bf16*)lvl3, num_levels, scale,
                       blocked ? 1 : 0);
  else if (out_bf16)
    hipLaunchKernelGGL((corr_pyramid_kernel<bf16, false>), grid, dim3(256), 0, stream, (const bf16*)f1,
                       (const bf16*)f2, h, w, nq, C, cs, (bf16*)lvl0, (bf16*)lvl1, (bf16*)lvl2, (bf16*)lvl3,
                       num_levels, scale, 0);
  else
    hipLaunchKernelGGL((corr_pyramid_kernel<float, false>), grid, dim3(256), 0, stream, (const bf16*)f1,
                       (const bf16*)f2, h, w, nq, C, cs, (float*)lvl0, (float*)lvl1, (float*)lvl2, (float*)lvl3,
                       num_levels, scale, 0);
  return (int)hipGetLastError();
}

// h, w: the (target) level-0 map size; nq: query pixels per image (h * w
// unless the queries are a slab of rows, cp.py).
extern "C" int jr_corr_lookup(const void* const* levels, int num_levels, int B, int h, int w, int nq, int radius,
                              const float* coords, void* out, int out_cstride, int lv_bf16, int blocked,
                              hipStream_t stream, const TapsUpd* upd) {
  const int S = 2 * radius + 1;
  if (num_levels > 4 || radius < 1 || radius > 6 || out_cstride % 8 != 0 || out_cstride < num_levels * S * S)
    return (int)hipErrorInvalidValue;
  TapsUpd u{};
  if (upd && upd->on) {
    if (nq != h * w || !upd->taps || upd->tcs < 18 || !upd->bias || upd->coords != coords || !upd->flow32 || !upd->hx)
      return (int)hipErrorInvalidValue;
    u = *upd;
  }
  LevelPtrs lv;
  for (int l = 0; l < 4; ++l) lv.p[l] = l < num_levels ? levels[l] : nullptr;
  const int total = B * nq;
  const LvGeom geo{blocked, (h + TY - 1) / TY, (w + TX - 1) / TX};
  if (lv_bf16)
    return launch_lookup<bf16>(lv, num_levels, total, h, w, radius, coords, (bf16*)out, out_cstride, geo, u, stream);
  return launch_lookup<float>(lv, num_levels, total, h, w, radius, coords, (bf16*)out, out_cstride, geo, u, stream);
}

extern "C" int jr_corr_lookup_bwd(void* const* dlevels, int num_levels, int B, int h, int w, int nq, int radius,
                                  const float* coords, const void* gout, int gcs, int g_bf16, hipStream_t stream) {
  const int S = 2 * radius + 1;
  if (num_levels > 4 || radius < 1 || radius > 6 || gcs < num_levels * S * S) return (int)hipErrorInvalidValue;
  LevelPtrs lv;
  for (int l = 0; l < 4; ++l) lv.p[l] = l < num_levels ? dlevels[l] : nullptr;
  const int total = B * nq;
  dim3 grid((total + 3) / 4);
  switch (radius) {
#define JR_LB(RR)                                                                                               \
  case RR:                                                                                                      \
    if (g_bf16)                                                                                                 \
      hipLaunchKernelGGL((corr_lookup_bwd_kernel<RR, bf16>), grid, dim3(256), 0, stream, lv, num_levels, total, h, w, \
                         coords, (const bf16*)gout, gcs);                                                       \
    else                                                                                                        \
      hipLaunchKernelGGL((corr_lookup_bwd_kernel<RR, float>), grid, dim3(256), 0, stream, lv, num_levels, total, h,   \
                         w, coords, (const float*)gout, gcs);                                                   \
    break;
    JR_LB(1) JR_LB(2) JR_LB(3) JR_LB(4) JR_LB(5) JR_LB(6)
#undef JR_LB
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
