// NHWC implicit-GEMM convolution on gfx950 MFMA (bf16 in, fp32 accumulate):
// kernel templates shared by the per-family translation units conv_fam_*.hip
// (split so the tile-config instantiations compile in parallel).
//
// Replaces every convolution of the reference RAFT (flax.linen.Conv sites in
// jax_raft/model.py:101-159 (ConvNormActivation), :238-255 (encoders),
// :275-290 (MotionEncoder), :304-310 (ConvGRU), :347-349 (FlowHead),
// :389-394 (MaskPredictor)).  Design (MI355X-first, not a translation):
//
//  * "Swapped" GEMM orientation: the MFMA A operand is the packed weight
//    matrix W[co][k] and the B operand the implicit im2col X[pixel][k].  The
//    16x16x32 accumulator then holds, per lane, 4 consecutive output channels
//    of ONE pixel; with the A-row permutation below each lane owns 4*TM
//    contiguous channels, so the epilogue is pixel-local and vectorised
//    (16-32 B stores, residual/GRU-state loads as whole vectors).
//  * K = (kh, kw, cin8) flattened in 8-channel (16 B) chunks, so any kernel
//    shape (1x1, 3x3, 7x7, 1x5, 5x1, strided) runs through one loader.
//  * 64-deep K stages, double-buffered LDS, register-staged global loads
//    issued before the MFMA block of the previous stage (one barrier per
//    stage).  LDS rows are 128 B with XOR swizzles chosen so that the
//    ds_read_b128 fragment reads of both operands are bank-conflict free.
//  * Fused epilogues: bias, residual, activation (incl. the context-encoder
//    tanh/relu split), scaling, dual stores into concat buffers, the
//    ConvGRU gate/blend of the RAFT loop and the FlowHead taps (EPI_TAPS).
#pragma once
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;

JR_DEVICE int swzB(int row) { return (row >> 1) & 7; }
// A (weight) images read with the 32x32x16 row order m32_arow: a ds_read_b128 lane group
// ({0-3, 12-15, 20-27} / {4-11, 16-19, 28-31}) reads 4 row pairs 16 or 32 rows apart, which
// swzB maps two-by-two onto the same 16-B slots (2-way conflicts: profiles/r5_pmc_b4.txt,
// gru_fused 29 % / conv_m32 17-19 % of LDS cycles); xoring bit 4 of the pair index into the
// slot's top bit separates them (rows of a 64-row group; groups start at multiples of 64)
JR_DEVICE int swzA(int row) { return ((row >> 1) ^ ((row >> 5) << 2)) & 7; }

template <int NV>
JR_DEVICE void store_bf16(bf16* dst, const float* v) {
  if constexpr (NV % 8 == 0) {
#pragma unroll
    for (int c = 0; c < NV / 8; ++c) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[c * 8 + j]);
      *(bf16x8*)(dst + c * 8) = o;
    }
  } else {
    static_assert(NV == 4, "NV");
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
    *(bf16x4*)dst = o;
  }
}

template <int NV>
JR_DEVICE void load_bf16(const bf16* src, float* v) {
  if constexpr (NV % 8 == 0) {
#pragma unroll
    for (int c = 0; c < NV / 8; ++c) {
      bf16x8 o = *(const bf16x8*)(src + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c * 8 + j] = bf2f(o[j]);
    }
  } else {
    bf16x4 o = *(const bf16x4*)src;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = bf2f(o[j]);
  }
}

template <int NV>
JR_DEVICE void store_f32(float* dst, const float* v) {
#pragma unroll
  for (int c = 0; c < NV / 4; ++c) *(f32x4*)(dst + 4 * c) = f32x4{v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
}

template <int NV>
JR_DEVICE void load_f32(const float* src, float* v) {
#pragma unroll
  for (int c = 0; c < NV / 4; ++c) {
    f32x4 o = *(const f32x4*)(src + 4 * c);
    v[4 * c] = o[0]; v[4 * c + 1] = o[1]; v[4 * c + 2] = o[2]; v[4 * c + 3] = o[3];
  }
}

// EPI_BWD epilogue (training backward, see BwdSeg in kernels.h): v[NV] holds the
// data gradient of NV contiguous input channels [cbase, cbase + NV) of pixel m.
// Modes 1 / 2 need whole groups inside [0, hidden) (hidden % 16 == 0, checked
// on the host); mode 0 handles a partial last group (cbase + NV > cout).
template <int NV>
JR_DEVICE void epi_bwd(const ConvParams& p, float (&v)[NV], int m, int cbase) {
  const int s = cbase < p.hidden ? 0 : 1;
  const BwdSeg& g = p.seg[s];
  const int lc = cbase - (s ? p.hidden : 0);
  const int n = min(NV, p.cout - cbase);  // valid channels of this group
  const bool full = n == NV;
  if (g.gin && g.gin_bf16) {   // bf16 gradient input (exact when it is a masked bf16 gradient)
    const bf16* gp = (const bf16*)g.gin + (long)m * g.gin_cs + g.gin_coff + lc;
    if (full) {
      float gi[NV];
      load_bf16<NV>(gp, gi);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] += gi[j];
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j) if (j < n) v[j] += bf2f(gp[j]);
    }
  } else if (g.gin) {
    const float* gp = (const float*)g.gin + (long)m * g.gin_cs + g.gin_coff + lc;
    if (full) {
      float gi[NV];
      load_f32<NV>(gp, gi);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] += gi[j];
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j) if (j < n) v[j] += gp[j];
    }
  }
  if (g.mode == 0) {
    if (g.mask) {
      const bf16* mp = (const bf16*)g.mask + (long)m * g.mask_cs + g.mask_coff + lc;
      float mv[NV];
      if (full) load_bf16<NV>(mp, mv);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) mv[j] = j < n ? bf2f(mp[j]) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] = mv[j] > 0.f ? v[j] : 0.f;
    }
    if (g.valid > 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j) if (lc + j >= g.valid) v[j] = 0.f;
    }
    if (g.out_f32) {
      float* op = (float*)g.out + (long)m * g.out_cs + g.out_coff + lc;
      if (full) store_f32<NV>(op, v);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) if (j < n) op[j] = v[j];
      }
    } else {
      bf16* op = (bf16*)g.out + (long)m * g.out_cs + g.out_coff + lc;
      if (full) store_bf16<NV>(op, v);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) if (j < n) op[j] = f2bf(v[j]);
      }
    }
    return;
  }
  const int hd = p.hidden;
  float hp[NV];
  load_f32<NV>(p.ghp + (long)m * hd + lc, hp);
  float* dh = (float*)g.out + (long)m * g.out_cs + g.out_coff + lc;
  if (g.mode == 1) {
    float z[NV], q[NV], a[NV], b[NV];
    load_bf16<NV>((const bf16*)p.gz + (long)m * hd + lc, z);
    load_bf16<NV>((const bf16*)p.gq + (long)m * hd + lc, q);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      a[j] = v[j] * z[j] * (1.f - q[j] * q[j]);                  // dL/d(q pre-activation)
      b[j] = v[j] * (q[j] - hp[j]) * z[j] * (1.f - z[j]);        // dL/d(z pre-activation)
      v[j] *= 1.f - z[j];                                        // dL/dh (blend path)
    }
    store_bf16<NV>((bf16*)p.gdq + (long)m * hd + lc, a);
    store_bf16<NV>((bf16*)p.gdzr + (long)m * 2 * hd + lc, b);
    store_f32<NV>(dh, v);
  } else {
    float r[NV], d[NV], a[NV];
    load_bf16<NV>((const bf16*)p.gr + (long)m * hd + lc, r);
    load_f32<NV>(dh, d);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      a[j] = v[j] * hp[j] * r[j] * (1.f - r[j]);                 // dL/d(r pre-activation)
      d[j] += v[j] * r[j];                                       // dL/dh (reset path)
    }
    store_bf16<NV>((bf16*)p.gdzr + (long)m * 2 * hd + hd + lc, a);
    store_f32<NV>(dh, d);
  }
}

// Output channel base of a lane: storage rows are permuted in 64-row groups so
// that D row (4*lq + r) of 16-row MFMA tile t maps to channel G + lq*16 + t*4 + r.
template <int TM>
JR_DEVICE int chan_base(int wrow0, int lq) {
  const int G = wrow0 & ~63;
  const int t0 = (wrow0 & 63) >> 4;
  return G + lq * 16 + t0 * 4;
}

// Shared epilogue.  Lane (li, lq) of wave (wco, wp) holds, for each pixel tile
// tn, NV = 4*TM contiguous output channels starting at cbase (see the weight
// row permutation in jax_raft_amd/ops/native.py:pack_weight).
// Per-pixel epilogue: v[NV] holds the raw accumulators of NV contiguous
// output channels [cbase, cbase + NV) of output pixel m (bias not yet added).
template <int NV, int EPI>
JR_DEVICE void epi_pixel(const ConvParams& p, float (&v)[NV], int m, int cbase) {
  const bool full = cbase + NV <= p.cout;
  const int OHW = p.OH * p.OW;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] += (cbase + j < p.cout) ? p.bias[cbase + j] : 0.f;
  if (p.bmap) {
    const long bo = (long)m * p.bmap_cstride + p.bmap_coff + cbase;
    float bv[NV];
    if (p.bmap_bf16) {
      const bf16* bp = (const bf16*)p.bmap + bo;
      if (full) load_bf16<NV>(bp, bv);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) bv[j] = (cbase + j < p.cout) ? bf2f(bp[j]) : 0.f;
      }
    } else {
      const float* bp = (const float*)p.bmap + bo;
      if (full) load_f32<NV>(bp, bv);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) bv[j] = (cbase + j < p.cout) ? bp[j] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] += bv[j];
  }
  if constexpr (EPI == EPI_STD) {
    if (p.res) {
      float rv[NV];
      const bf16* rp = (const bf16*)p.res + (long)m * p.res_cstride + p.res_coff + cbase;
      if (full) {
        load_bf16<NV>(rp, rv);
      } else {
#pragma unroll
        for (int j = 0; j < NV; ++j) rv[j] = (cbase + j < p.cout) ? bf2f(rp[j]) : 0.f;
      }
      if (p.res_post) {
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = fmaxf(apply_act(v[j], p.act, cbase + j, p.split) + rv[j], 0.f);
      } else {
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = apply_act(v[j] + rv[j], p.act, cbase + j, p.split);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] = apply_act(v[j], p.act, cbase + j, p.split);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] *= p.alpha;
    if (p.y_fp32) {
      float* yp = (float*)p.y + (long)m * p.y_cstride + p.y_coff + cbase;
      if (full) store_f32<NV>(yp, v);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) if (cbase + j < p.cout) yp[j] = v[j];
      }
    } else {
      bf16* yp = (bf16*)p.y + (long)m * p.y_cstride + p.y_coff + cbase;
      if (full) store_bf16<NV>(yp, v);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) if (cbase + j < p.cout) yp[j] = f2bf(v[j]);
      }
    }
    if (p.y2) {
      bf16* yp = (bf16*)p.y2 + (long)m * p.y2_cstride + p.y2_coff + cbase;
      if (full) store_bf16<NV>(yp, v);
      else {
#pragma unroll
        for (int j = 0; j < NV; ++j) if (cbase + j < p.cout) yp[j] = f2bf(v[j]);
      }
    }
    if (p.h32) {  // fp32 copy of the channels below `split` (context-encoder hidden state)
      if (cbase < p.split) {
        float* hp = p.h32 + (long)m * p.hidden + cbase;
#pragma unroll
        for (int j = 0; j < NV; ++j) if (cbase + j < p.split) hp[j] = v[j];
      }
    }
  } else if constexpr (EPI == EPI_GRU_A) {
    // [z | r] logits -> z (fp32 / bf16) and r*h (bf16) into the q-input buffer.
    // h comes from the fp32 state when given, else from the conv's own bf16
    // input (channels [x_coff, x_coff + hidden) of the same pixel: the GRU
    // input [h | ...] at stride 1): half the bytes, usually still L2-resident.
    const int hd = p.hidden;
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = sigmoidf_(v[j]);
    if (cbase < hd) {
      if (p.z_bf16) store_bf16<NV>((bf16*)p.zbuf + (long)m * hd + cbase, v);
      else store_f32<NV>((float*)p.zbuf + (long)m * hd + cbase, v);
    } else {
      const int hc = cbase - hd;
      if (p.rbuf) store_bf16<NV>((bf16*)p.rbuf + (long)m * hd + hc, v);  // training: r for the backward
      float h[NV];
      if (p.h32) load_f32<NV>(p.h32 + (long)m * hd + hc, h);
      else load_bf16<NV>((const bf16*)p.x + (long)m * p.x_cstride + p.x_coff + hc, h);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] *= h[j];
      store_bf16<NV>((bf16*)p.y + (long)m * p.y_cstride + p.y_coff + hc, v);
    }
  } else if constexpr (EPI == EPI_GRU_B) {
    const int hd = p.hidden;
    float z[NV], h[NV];
    if (p.z_bf16) load_bf16<NV>((const bf16*)p.zbuf + (long)m * hd + cbase, z);
    else load_f32<NV>((const float*)p.zbuf + (long)m * hd + cbase, z);
    float* hp = p.h32 + (long)m * hd + cbase;
    load_f32<NV>(hp, h);
    float qv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float q = tanhf_(v[j]);
      qv[j] = q;
      v[j] = (1.0f - z[j]) * h[j] + z[j] * q;
    }
    if (p.qbuf) store_bf16<NV>((bf16*)p.qbuf + (long)m * hd + cbase, qv);  // training: q for the backward
    if (p.h32o) hp = p.h32o + (long)m * hd + cbase;
    store_f32<NV>(hp, v);
    store_bf16<NV>((bf16*)p.y + (long)m * p.y_cstride + p.y_coff + cbase, v);
    if (p.y2) store_bf16<NV>((bf16*)p.y2 + (long)m * p.y2_cstride + p.y2_coff + cbase, v);
  } else if constexpr (EPI == EPI_BWD) {
    epi_bwd<NV>(p, v, m, cbase);
  }
}

// Epilogue of the 16x16x32 kernels.  Lane (li, lq) of a wave whose first
// storage row is wrow0 holds, for each pixel tile tn and each 64-row group g
// the wave covers, 4*min(TM,4) contiguous output channels starting at
// chan_base(wrow0 + 64 g) (see the weight row permutation in
// jax_raft_amd/ops/native.py:pack_weight).
template <int I, int N, typename F>
JR_DEVICE void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int TM, int TN, int EPI>
JR_DEVICE void conv_epilogue(const ConvParams& p, f32x4 (&acc)[TM][TN], int mbase, int wrow0, int lq, int li) {
  constexpr int TG = TM > 4 ? 4 : TM;   // 16-row tiles per 64-row permutation group
  static_assert(TM % TG == 0, "TM");
  constexpr int NV = 4 * TG;
  // compile-time loops: a large epilogue body defeats `#pragma unroll`, and a
  // runtime index into acc[][] would move the accumulators to scratch
  static_for<0, TM / TG>([&](auto gc) {
    constexpr int g = decltype(gc)::value;
    const int cbase = chan_base<TG>(wrow0 + 64 * g, lq);
    if (cbase >= p.cout) return;
    static_for<0, TN>([&](auto tc) {
      constexpr int tn = decltype(tc)::value;
      const int m = mbase + tn * 16 + li;
      if (m >= p.M) return;
      float v[NV];
#pragma unroll
      for (int tm = 0; tm < TG; ++tm)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[tm * 4 + r] = acc[g * TG + tm][tn][r];
      epi_pixel<NV, EPI>(p, v, m, cbase);
    });
  });
}

// EPI_TAPS epilogue (FlowHead conv1 -> the 18 taps of conv2, model.py:347-350):
// the block holds all 256 channels of its 128 pixels (one N tile, 16 waves of
// 64 x 32).  Lane (li, lq) of wave (wco, wp) owns channels wco*64 + 16 lq + (0..15)
// of pixels wp*32 + 16 tn + li; after bias + activation those 16 values ARE the
// B fragments (k-steps s = 0, 1) of a second MFMA against the packed tap weights
// (ops/native.py:pack_taps_epi, same k order), giving each wave the 32 (18 real)
// tap partial sums of its 64 channels.  The four channel groups are summed through
// LDS (the staging buffers, free after the K loop) and written as fp32 [M][y_cstride].
JR_DEVICE void taps_epilogue(const ConvParams& p, f32x4 (&acc)[4][2], bf16* smem, int p0, int wco, int wp,
                             int lane) {
  const int li = lane & 15, lq = lane >> 4;
  const int c0 = wco * 64 + 16 * lq;
  float b[16];
  load_f32<16>(p.bias + c0, b);
  const u32x4* wt = (const u32x4*)p.tapw + wco * 4 * 64 + lane;
  u32x4 a[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) a[s][t] = wt[(s * 2 + t) * 64];
  f32x4 d[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) d[t][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tn = 0; tn < 2; ++tn)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = acc[2 * s + (j >> 2)][tn][j & 3] + b[8 * s + j];
        bf[j] = f2bf(apply_act(v, p.act, c0 + 8 * s + j, p.split));
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
        d[t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[s][t]), bf, d[t][tn], 0, 0, 0);
    }
  __syncthreads();  // every wave is done with the staging LDS
  f32x4* red = (f32x4*)smem;  // [wp 4][wco 4][t 2][tn 2][lane 64]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) red[(((wp * 4 + wco) * 2 + t) * 2 + tn) * 64 + lane] = d[t][tn];
  __syncthreads();
  if (wco != 0) return;
#pragma unroll
  for (int tn = 0; tn < 2; ++tn) {
    const int m = p0 + wp * 32 + tn * 16 + li;
    f32x4 sum[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sum[t] = red[(((wp * 4 + 0) * 2 + t) * 2 + tn) * 64 + lane];
#pragma unroll
      for (int g = 1; g < 4; ++g) {
        const f32x4 v = red[(((wp * 4 + g) * 2 + t) * 2 + tn) * 64 + lane];
        sum[t] += v;
      }
    }
    if (m >= p.M) continue;
    // lane (li, lq) holds taps o = 16 t + 4 lq + r of pixel m
    float* yp = (float*)p.y + (long)m * p.y_cstride;
    *(f32x4*)(yp + 4 * lq) = sum[0];
    if (lq == 0) *(float2*)(yp + 16) = make_float2(sum[1][0], sum[1][1]);
  }
}

// XCD-aware tile order.  MI355X dispatches workgroups round-robin over its 8
// XCDs (private L2 each), so consecutive linear ids -- neighbouring pixel
// tiles, which share the input rows of a 3x3 / 1x5 / 5x1 window -- land on
// different L2s.  Remap the linear id so every XCD walks a contiguous run of
// tiles (bijective for any grid size; dispatch placement only changes speed).
JR_DEVICE void tile_of_block(const ConvParams& p, int& bx, int& by) {
  bx = blockIdx.x;
  by = blockIdx.y;
  const int nx = gridDim.x, nwg = nx * gridDim.y;
  if (!p.xcd_remap || nwg <= 8) return;
  const int bid = by * nx + bx;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  bx = t % nx;
  by = t / nx;
}

// Per-row state of the FAST im2col loader (ConvParams::fast): the byte offset
// of the row's first tap + this lane's 16-B chunk, and a bitmask of the taps
// (kh * KW + kw) that fall inside the input.  A stage's tap and channel block
// are wave-uniform, so a stage costs per row one bit test, one add and one
// select.
struct FastRow {
  unsigned off;
  unsigned mask;
};

JR_DEVICE FastRow fast_row(const ConvParams& p, int ih0, int iw0, unsigned rbase, bool valid, int ch,
                           unsigned xrow_bytes) {
  FastRow r{0u, 0u};
  if (!valid) return r;
  r.off = rbase + (unsigned)(ih0 * p.W + iw0) * xrow_bytes + (unsigned)ch * 16u;  // may wrap; only used when a tap is valid
  for (int kh = 0; kh < p.KH; ++kh) {
    if ((unsigned)(ih0 + kh) >= (unsigned)p.H) continue;
    for (int kw = 0; kw < p.KW; ++kw)
      if ((unsigned)(iw0 + kw) < (unsigned)p.W) r.mask |= 1u << (kh * p.KW + kw);
  }
  return r;
}

// Wave-uniform stage state of the FAST loader.
struct FastStage {
  int tap = 0, kh = 0, kw = 0, cb = 0;
  JR_DEVICE void advance(const ConvParams& p, int cpb) {
    if (++cb == cpb) {
      cb = 0;
      ++tap;
      if (++kw == p.KW) { kw = 0; ++kh; }
    }
  }
};

// Body of kernels R / P for the block tile (bx_, by_) (the grid mapping is the caller's:
// conv_igemm_kernel below, or the grouped launch conv_igemm_grouped).
template <int BCO, int BP, int WCO, int EPI, bool FAST, int NW = 4, int PIPE = 0>  // PIPE 1: kernel P
JR_DEVICE void conv_igemm_body(const ConvParams& p, const int bx_, const int by_) {
  constexpr int WP = NW / WCO;
  constexpr int RP = NW * 8;              // staging rows covered by one pass of the block (8 lanes per row)
  constexpr int WTCO = BCO / WCO;
  constexpr int WTP = BP / WP;
  constexpr int TM = WTCO / 16;
  constexpr int TN = WTP / 16;
  constexpr int NV = 4 * TM;              // contiguous channels per lane
  constexpr int XR = BP / RP;             // X rows loaded per thread
  constexpr int WR = BCO >= RP ? BCO / RP : 1;
  constexpr int A_ELEMS = BCO * BK;
  constexpr int B_ELEMS = BP * BK;
  constexpr unsigned OOB = 0x80000000u;   // buffer offset past num_records -> hardware returns 0
  static_assert(TM >= 1 && TN >= 1 && WCO * WP == NW && XR >= 1, "tile");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (A_ELEMS + B_ELEMS)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wco = wave % WCO;
  const int wp = wave / WCO;
  const int p0 = bx_ * BP;
  const int co0 = by_ * BCO;
  const int ch = tid & 7;
  const int OHW = p.OH * p.OW;

  // Buffer resources: out-of-range offsets (padding taps, tail rows, K tail)
  // read as zero with no branch and no exec masking.
  const __amdgpu_buffer_rsrc_t xsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.w_bytes, 0x00020000);

  // Per-thread im2col row descriptors (fixed across the K loop); byte offsets.
  int ih0[XR], iw0[XR];
  unsigned rbase[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int m = p0 + (tid >> 3) + RP * i;
    if (m < p.M) {
      const int n = m / OHW;
      const int rem = m - n * OHW;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      ih0[i] = oh * p.SH - p.PH;
      iw0[i] = ow * p.SW - p.PW;
      rbase[i] = (unsigned)(((long)n * p.H * p.W * p.x_cstride + p.x_coff) * 2);
    } else {
      ih0[i] = -(1 << 28);
      iw0[i] = -(1 << 28);
      rbase[i] = 0;
    }
  }
  const unsigned wrow_off = (unsigned)((co0 + (tid >> 3)) * p.kpad * 2 + ch * 16);
  const unsigned wrow_lim = (unsigned)(p.cout_pad - co0 - (tid >> 3));  // rows i*RP < lim are valid

  // K-chunk state of the NEXT stage to load: kc = ks*8 + ch.
  const int cpt = p.cin8 >> 3;
  int tap = ch / cpt;
  int cc = ch - tap * cpt;
  int kh = tap / p.KW;
  int kw = tap - kh * p.KW;
  int ks_next = 0;
  const unsigned xrow_bytes = (unsigned)p.x_cstride * 2;
  [[maybe_unused]] FastRow frow[XR];
  [[maybe_unused]] FastStage fst;
  [[maybe_unused]] const int cpb = (p.KH * p.KW == 1) ? (p.kpad / BK) : (p.cin8 >> 6);
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < XR; ++i) frow[i] = fast_row(p, ih0[i], iw0[i], rbase[i], ih0[i] > -(1 << 27), ch, xrow_bytes);
  }

  struct Regs { u32x4 x[XR]; u32x4 w[WR]; };
  Regs ra, rb;

  auto issue = [&](Regs& r) {
    if constexpr (FAST) {
      const bool kin = ks_next * BK < p.kpad;
      const bool cv = kin && ch * 8 < p.cin8 - fst.cb * 64;   // channel tail of a 1x1 conv
      const unsigned soff = (unsigned)(fst.kh * p.W + fst.kw) * xrow_bytes + (unsigned)fst.cb * 128u;
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        const bool ok = cv && ((frow[i].mask >> (fst.tap & 31)) & 1u);
        r.x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, ok ? frow[i].off + soff : OOB, 0, 0));
      }
      fst.advance(p, cpb);
    } else {
    const bool kvalid = kh < p.KH;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int ihl = ih0[i] + kh, iwl = iw0[i] + kw;  // coordinates in the (dilated) input
      const int ih = ihl >> p.dsh, iw = iwl >> p.dsw;
      const bool ok = kvalid && ((ihl & ((1 << p.dsh) - 1)) | (iwl & ((1 << p.dsw) - 1))) == 0 &&
                  (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const unsigned off = rbase[i] + (unsigned)(ih * p.W + iw) * xrow_bytes + (unsigned)cc * 16u;
      r.x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, ok ? off : OOB, 0, 0));
    }
    }
    const unsigned kofs = (unsigned)ks_next * (BK * 2);
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const bool ok = ((BCO >= RP) || (tid < BCO * 8)) && (unsigned)(RP * i) < wrow_lim && ks_next * BK < p.kpad;
      const unsigned off = wrow_off + (unsigned)(RP * i) * (unsigned)p.kpad * 2u + kofs;
      r.w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wsrd, ok ? off : OOB, 0, 0));
    }
    // advance the chunk state to the following stage
    ++ks_next;
    if constexpr (!FAST) {
      cc += 8;
      while (cc >= cpt) {
        cc -= cpt;
        if (++kw == p.KW) { kw = 0; ++kh; }
      }
    }
  };
  auto store = [&](const Regs& r, int buf) {
    bf16* sA = smem + buf * (A_ELEMS + B_ELEMS);
    bf16* sB = sA + A_ELEMS;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int rr = (tid >> 3) + RP * i;
      *(u32x4*)(sB + rr * BK + ((ch ^ swzB(rr)) << 3)) = r.x[i];
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int rr = (tid >> 3) + RP * i;
      if ((BCO >= RP) || (tid < BCO * 8)) *(u32x4*)(sA + rr * BK + ((ch ^ swzB(rr)) << 3)) = r.w[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15;
  const int lq = lane >> 4;
  auto compute = [&](int buf) {
    const bf16* sA = smem + buf * (A_ELEMS + B_ELEMS);
    const bf16* sB = sA + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + lq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wco * WTCO + tm * 16 + li;
        af[tm] = *(const bf16x8*)(sA + row * BK + ((chunk ^ swzB(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wp * WTP + tn * 16 + li;
        bfr[tn] = *(const bf16x8*)(sB + row * BK + ((chunk ^ swzB(row)) << 3));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
  };

  if constexpr (PIPE == 1) {
    // Kernel P main loop: the same staging (global loads two stages ahead in
    // register sets ra/rb, LDS double-buffered, one barrier per stage), but the
    // MFMA fragments are double-buffered in registers at half-stage (32-deep K)
    // granularity, so every LDS read burst overlaps MFMAs already issued:
    //   read F_b (this stage, k 32..63) || MFMAs on F_a (k 0..31)
    //   stage the next stage into the other LDS buffer, issue its successor's loads
    //   MFMAs on F_b, barrier, read F_a of the next stage || the F_b MFMAs drain.
    // In kernel R every wave reads a whole stage right after the barrier and
    // then multiplies: the LDS burst (~768 array cycles per CU for 16 waves) and
    // the MFMAs serialise.
    auto rdfrag = [&](int buf, int kk, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
      const bf16* sA = smem + buf * (A_ELEMS + B_ELEMS);
      const bf16* sB = sA + A_ELEMS;
      const int chunk = kk * 4 + lq;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wco * WTCO + tm * 16 + li;
        af[tm] = *(const bf16x8*)(sA + row * BK + ((chunk ^ swzB(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wp * WTP + tn * 16 + li;
        bfr[tn] = *(const bf16x8*)(sB + row * BK + ((chunk ^ swzB(row)) << 3));
      }
    };
    auto mma = [&](const bf16x8 (&af)[TM], const bf16x8 (&bfr)[TN]) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    };
    bf16x8 fa[TM], fb[TN], ga[TM], gb[TN];   // F_a = (fa, fb), F_b = (ga, gb)
    const int nks = p.kpad / BK;
    issue(ra);          // stage 0
    issue(rb);          // stage 1
    store(ra, 0);
    __syncthreads();
    issue(ra);          // stage 2
    rdfrag(0, 0, fa, fb);
    const int npairs = nks >> 1;
    for (int it = 0; it < npairs; ++it) {
      // stage 2it (LDS buffer 0)
      rdfrag(0, 1, ga, gb);
      mma(fa, fb);
      store(rb, 1);     // stage 2it+1
      issue(rb);        // stage 2it+3
      mma(ga, gb);
      __syncthreads();
      rdfrag(1, 0, fa, fb);
      // stage 2it+1 (LDS buffer 1)
      rdfrag(1, 1, ga, gb);
      mma(fa, fb);
      store(ra, 0);     // stage 2it+2
      issue(ra);        // stage 2it+4
      mma(ga, gb);
      __syncthreads();
      rdfrag(0, 0, fa, fb);
    }
    if (nks & 1) {      // stage nks-1 (buffer 0, F_a already read)
      rdfrag(0, 1, ga, gb);
      mma(fa, fb);
      mma(ga, gb);
    }
    if constexpr (EPI == EPI_TAPS) {
      static_assert(TM == 4 && TN == 2 && WCO == 4 && NW == 16, "EPI_TAPS tiling");
      taps_epilogue(p, acc, smem, p0, wco, wp, lane);
    } else {
      const int wrow0 = co0 + wco * WTCO;
      conv_epilogue<TM, TN, EPI>(p, acc, p0 + wp * WTP, wrow0, lq, li);
    }
    return;
  }

  // Software pipeline: global loads run two K-stages ahead of the MFMAs
  // (register sets ra/rb alternate, LDS double-buffered, one barrier per
  // stage).  Loads past the end of K are issued with OOB offsets (zeros),
  // keeping the loop body branch-free so hipcc emits counted vmcnt waits.
  const int nks = p.kpad / BK;
  issue(ra);
  issue(rb);
  store(ra, 0);
  __syncthreads();
  const int npairs = nks >> 1;
  for (int it = 0; it < npairs; ++it) {
    issue(ra);          // stage 2it+2
    compute(0);         // stage 2it
    store(rb, 1);       // stage 2it+1 (loaded one stage ago)
    __syncthreads();
    issue(rb);          // stage 2it+3
    compute(1);         // stage 2it+1
    store(ra, 0);       // stage 2it+2
    __syncthreads();
  }
  if (nks & 1) compute(0);

  if constexpr (EPI == EPI_TAPS) {
    static_assert(TM == 4 && TN == 2 && WCO == 4 && NW == 16, "EPI_TAPS tiling");
    taps_epilogue(p, acc, smem, p0, wco, wp, lane);
  } else {
    const int wrow0 = co0 + wco * WTCO;
    conv_epilogue<TM, TN, EPI>(p, acc, p0 + wp * WTP, wrow0, lq, li);
  }
}

template <int BCO, int BP, int WCO, int EPI, bool FAST, int NW = 4, int PIPE = 0>
__global__ __launch_bounds__(NW * 64) void conv_igemm_kernel(const ConvParams p) {
  int bx, by;
  tile_of_block(p, bx, by);
  conv_igemm_body<BCO, BP, WCO, EPI, FAST, NW, PIPE>(p, bx, by);
}

// ---------------------------------------------------------------------------
// Kernel M32: as kernel R (register-staged operands, 64-deep K stages,
// 2-stage prefetch) but on v_mfma_f32_32x32x16_bf16: half the MFMA
// instructions (and MFMA issue-blocking cycles) per FLOP of the 16x16x32
// form, the loop being issue-bound.  The 32x32 accumulator gives lane
// (col = pixel, h = lane>>5) the D rows (r&3) + 8(r>>2) + 4h; the A-operand LDS
// rows are read in the permuted order below so that those 16 rows are the 16
// contiguous output channels 32t + 16h + r of the wave's 64-channel group
// (stored permuted per pack_weight), keeping the epilogue vectorised.
// ---------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

// storage row (within a 64-row group) holding channel 32t + c(rho), c(rho) = 16((rho>>2)&1) + (rho&3) + 4(rho>>3)
JR_DEVICE int m32_arow(int t, int rho) { return 16 * (rho >> 3) + 4 * (2 * t + ((rho >> 2) & 1)) + (rho & 3); }

template <int BCO, int BP, int WCO, int EPI, bool FAST, int NW = 4>
JR_DEVICE void conv_m32_body(const ConvParams& p, const int bx_, const int by_) {
  constexpr int WP = NW / WCO;
  constexpr int RP = NW * 8;   // staging rows per block pass
  constexpr int WTCO = BCO / WCO;
  constexpr int WTP = BP / WP;
  constexpr int TM = WTCO / 32;
  constexpr int TN = WTP / 32;
  constexpr int XR = BP / RP;
  constexpr int WR = BCO >= RP ? BCO / RP : 1;
  constexpr int A_ELEMS = BCO * BK;
  constexpr int B_ELEMS = BP * BK;
  constexpr unsigned OOB = 0x80000000u;
  static_assert(TM >= 1 && TN >= 1 && WCO * WP == NW && BCO >= RP && XR >= 1, "tile");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (A_ELEMS + B_ELEMS)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wco = wave % WCO;
  const int wp = wave / WCO;
  const int p0 = bx_ * BP;
  const int co0 = by_ * BCO;
  const int ch = tid & 7;
  const int OHW = p.OH * p.OW;

  const __amdgpu_buffer_rsrc_t xsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.w_bytes, 0x00020000);

  int ih0[XR], iw0[XR];
  unsigned rbase[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int m = p0 + (tid >> 3) + RP * i;
    if (m < p.M) {
      const int n = m / OHW;
      const int rem = m - n * OHW;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      ih0[i] = oh * p.SH - p.PH;
      iw0[i] = ow * p.SW - p.PW;
      rbase[i] = (unsigned)(((long)n * p.H * p.W * p.x_cstride + p.x_coff) * 2);
    } else {
      ih0[i] = -(1 << 28);
      iw0[i] = -(1 << 28);
      rbase[i] = 0;
    }
  }
  const unsigned wrow_off = (unsigned)((co0 + (tid >> 3)) * p.kpad * 2 + ch * 16);
  const unsigned wrow_lim = (unsigned)(p.cout_pad - co0 - (tid >> 3));
  const int cpt = p.cin8 >> 3;
  int tap = ch / cpt;
  int cc = ch - tap * cpt;
  int kh = tap / p.KW;
  int kw = tap - kh * p.KW;
  int ks_next = 0;
  const unsigned xrow_bytes = (unsigned)p.x_cstride * 2;
  [[maybe_unused]] FastRow frow[XR];
  [[maybe_unused]] FastStage fst;
  [[maybe_unused]] const int cpb = (p.KH * p.KW == 1) ? (p.kpad / BK) : (p.cin8 >> 6);
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < XR; ++i) frow[i] = fast_row(p, ih0[i], iw0[i], rbase[i], ih0[i] > -(1 << 27), ch, xrow_bytes);
  }

  struct Regs { u32x4 x[XR]; u32x4 w[WR]; };
  Regs ra, rb;

  auto issue = [&](Regs& r) {
    if constexpr (FAST) {
      const bool kin = ks_next * BK < p.kpad;
      const bool cv = kin && ch * 8 < p.cin8 - fst.cb * 64;   // channel tail of a 1x1 conv
      const unsigned soff = (unsigned)(fst.kh * p.W + fst.kw) * xrow_bytes + (unsigned)fst.cb * 128u;
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        const bool ok = cv && ((frow[i].mask >> (fst.tap & 31)) & 1u);
        r.x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, ok ? frow[i].off + soff : OOB, 0, 0));
      }
      fst.advance(p, cpb);
    } else {
    const bool kvalid = kh < p.KH;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int ihl = ih0[i] + kh, iwl = iw0[i] + kw;
      const int ih = ihl >> p.dsh, iw = iwl >> p.dsw;
      const bool ok = kvalid && ((ihl & ((1 << p.dsh) - 1)) | (iwl & ((1 << p.dsw) - 1))) == 0 &&
                      (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const unsigned off = rbase[i] + (unsigned)(ih * p.W + iw) * xrow_bytes + (unsigned)cc * 16u;
      r.x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, ok ? off : OOB, 0, 0));
    }
    }
    const unsigned kofs = (unsigned)ks_next * (BK * 2);
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const bool ok = (unsigned)(RP * i) < wrow_lim && ks_next * BK < p.kpad;
      const unsigned off = wrow_off + (unsigned)(RP * i) * (unsigned)p.kpad * 2u + kofs;
      r.w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wsrd, ok ? off : OOB, 0, 0));
    }
    ++ks_next;
    if constexpr (!FAST) {
      cc += 8;
      while (cc >= cpt) {
        cc -= cpt;
        if (++kw == p.KW) { kw = 0; ++kh; }
      }
    }
  };
  auto store = [&](const Regs& r, int buf) {
    bf16* sA = smem + buf * (A_ELEMS + B_ELEMS);
    bf16* sB = sA + A_ELEMS;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int rr = (tid >> 3) + RP * i;
      *(u32x4*)(sB + rr * BK + ((ch ^ swzB(rr)) << 3)) = r.x[i];
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int rr = (tid >> 3) + RP * i;
      *(u32x4*)(sA + rr * BK + ((ch ^ swzA(rr)) << 3)) = r.w[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int rho = lane & 31;
  const int hh = lane >> 5;
  const int wbase = wco * WTCO;               // wave's first storage row in the block
  const int tabs0 = ((co0 + wbase) & 63) >> 5;  // 32-row half of the 64-row group
  const int gbase = wbase - ((co0 + wbase) & 63);  // block-relative start of that 64-row group
  auto compute = [&](int buf) {
    const bf16* sA = smem + buf * (A_ELEMS + B_ELEMS);
    const bf16* sB = sA + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int chunk = kk * 2 + hh;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = gbase + 64 * ((tabs0 + tm) >> 1) + m32_arow((tabs0 + tm) & 1, rho);  // 128-row wave tiles span two groups
        af[tm] = *(const bf16x8*)(sA + row * BK + ((chunk ^ swzA(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wp * WTP + tn * 32 + rho;
        bfr[tn] = *(const bf16x8*)(sB + row * BK + ((chunk ^ swzB(row)) << 3));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
  };

  const int nks = p.kpad / BK;
  issue(ra);
  issue(rb);
  store(ra, 0);
  __syncthreads();
  const int npairs = nks >> 1;
  for (int it = 0; it < npairs; ++it) {
    issue(ra);
    compute(0);
    store(rb, 1);
    __syncthreads();
    issue(rb);
    compute(1);
    store(ra, 0);
    __syncthreads();
  }
  if (nks & 1) compute(0);

  // epilogue: tile tm of lane hh -> channels G + 32*(tabs0+tm) + 16*hh + [0,16)
  const int G = (co0 + wbase) & ~63;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int cbase = G + 32 * (tabs0 + tm) + 16 * hh;
    if (cbase >= p.cout) continue;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int m = p0 + wp * WTP + tn * 32 + rho;
      if (m >= p.M) continue;
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[tm][tn][r];
      epi_pixel<16, EPI>(p, v, m, cbase);
    }
  }
}

template <int BCO, int BP, int WCO, int EPI, bool FAST, int NW = 4>
__global__ __launch_bounds__(NW * 64) void conv_m32_kernel(const ConvParams p) {
  int bx, by;
  tile_of_block(p, bx, by);
  conv_m32_body<BCO, BP, WCO, EPI, FAST, NW>(p, bx, by);
}

// Grouped launch (one-lane schedule): two independent convs with the same tile config in ONE
// grid -- blocks [0, n1) are p1's tiles, the rest p2's (each in dispatch order) -- so at batch 1
// their small grids run side by side without a cross-stream graph edge (runtime/engine.py:
// _conv_group).  Used for the MotionEncoder's last correlation conv and its second flow conv
// (reference jax_raft/model.py:279 / 285: independent branches until the concat at :287).
template <int BCO, int BP, int WCO, bool FAST, int NW, bool M32>
__global__ __launch_bounds__(NW * 64) void conv_grouped_kernel(const ConvParams p1, const ConvParams p2, int n1,
                                                               int gx1, int gx2) {
  const int id = blockIdx.x;
  const bool first = id < n1;
  const ConvParams& p = first ? p1 : p2;
  const int t = first ? id : id - n1, gx = first ? gx1 : gx2;
  const int by = t / gx, bx = t - by * gx;
  if constexpr (M32) conv_m32_body<BCO, BP, WCO, EPI_STD, FAST, NW>(p, bx, by);
  else conv_igemm_body<BCO, BP, WCO, EPI_STD, FAST, NW, 0>(p, bx, by);
}

template <int BCO, int BP, int WCO, int NW, bool M32>
int launch_grouped(const ConvParams* p1, const ConvParams* p2, hipStream_t s) {
  if (p1->fast != p2->fast) return (int)hipErrorInvalidValue;
  auto grid_of = [](const ConvParams* p, int& gx) {
    const int rows = (p->cout + 63) / 64 * 64;
    gx = (p->M + BP - 1) / BP;
    return gx * ((rows + BCO - 1) / BCO);
  };
  int gx1, gx2;
  const int n1 = grid_of(p1, gx1), n2 = grid_of(p2, gx2);
  if (p1->fast)
    hipLaunchKernelGGL((conv_grouped_kernel<BCO, BP, WCO, true, NW, M32>), dim3(n1 + n2), dim3(NW * 64), 0, s, *p1,
                       *p2, n1, gx1, gx2);
  else
    hipLaunchKernelGGL((conv_grouped_kernel<BCO, BP, WCO, false, NW, M32>), dim3(n1 + n2), dim3(NW * 64), 0, s, *p1,
                       *p2, n1, gx1, gx2);
  return (int)hipGetLastError();
}

// LDS-DMA helpers (kernel D2)
// One 16-B-per-lane LDS-DMA (buffer_load_dwordx4 ... lds): lane i lands at lds + 16*i.
JR_DEVICE void dma16(__amdgpu_buffer_rsrc_t r, bf16* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

template <int N>
JR_DEVICE void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

JR_DEVICE void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------
// Kernel D2: LDS-DMA staging at BK = 64 with an NS-deep ring.
//
// A stage is (BCO + BP) LDS rows of 128 B (64 bf16 of K): the weight tile then
// the im2col pixel tile.  It is filled by 1-KiB LDS-DMA pieces
// (`buffer_load_dwordx4 ... lds`, lane i -> piece base + 16 i) of 8 whole
// rows, (BCO + BP) / (8 NW) pieces per wave, so every wave issues the same
// count and the ring waits are exact counted `vmcnt`s with raw barriers: stage
// ks + NS - 1 is in flight while stage ks feeds the MFMAs.  Row r keeps
// 16-B chunk c at slot c ^ (r & 6).  That swizzle depends only on the row
// inside a piece, so each DMA lane fetches one FIXED chunk
// ((lane & 7) ^ ((lane >> 3) & 6)) for every piece and stage (one im2col K
// state per lane, as in kernel R), and the ds_read_b128 fragment reads are
// bank-conflict free under the hardware's lane grouping
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (rows li and li^4.. of a group
// land on distinct (row parity, slot) pairs).  No staging VGPRs and no
// ds_write traffic: the LDS array only serves the fragment reads.
// NW = 8 / 16 waves (one block per CU at 256x128 tiles, 144 KiB ring at NS 3)
// with the FAST im2col loader (ConvParams::fast) are the configs that compete
// with kernels R / P on the refinement-loop convs (configs 35..39).
// ---------------------------------------------------------------------------
template <int BCO, int BP, int WCO, int NS, int EPI, bool FAST = false, int NW = 4>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(1, NW > 4 || (BCO + BP) * NS * 128 > 81920 ? 1 : 2))) void conv_d2_kernel(const ConvParams p) {
  constexpr int WP = NW / WCO;
  constexpr int WTCO = BCO / WCO;
  constexpr int WTP = BP / WP;
  constexpr int TM = WTCO / 16;
  constexpr int TN = WTP / 16;
  constexpr int ROWS = BCO + BP;
  constexpr int PPW = ROWS / (8 * NW);             // 8-row pieces per wave per stage
  constexpr int STAGE = ROWS * BK;                 // bf16 elements
  constexpr unsigned OOB = 0x80000000u;
  static_assert(TM >= 1 && TN >= 1 && WCO * WP == NW && ROWS % (8 * NW) == 0, "tile");
  static_assert(NS >= 2 && NS <= 4 && NS * STAGE * 2 <= 160 * 1024, "ring depth");
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wco = wave % WCO;
  const int wp = wave / WCO;
  int bx_, by_;
  tile_of_block(p, bx_, by_);
  const int p0 = bx_ * BP;
  const int co0 = by_ * BCO;
  const int OHW = p.OH * p.OW;
  const int cl = (lane & 7) ^ ((lane >> 3) & 6);   // this lane's fixed logical chunk in a stage

  const __amdgpu_buffer_rsrc_t xsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.w_bytes, 0x00020000);
  const unsigned xrow_bytes = (unsigned)p.x_cstride * 2;

  // piece j of this wave covers stage rows q*8 .. q*8+7, q = wave*PPW + j:
  // rows < BCO are weight rows, the rest pixel rows.  Per-lane row = q*8 + lane/8.
  int ih0[PPW], iw0[PPW];
  unsigned rbase[PPW];
  [[maybe_unused]] FastRow frow[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int row = (wave * PPW + j) * 8 + (lane >> 3);
    if (row < BCO) {
      // weight row: rbase = byte offset of (row, chunk cl); ih0 flags validity
      const int wr = co0 + row;
      rbase[j] = (unsigned)(wr * p.kpad * 2 + cl * 16);
      ih0[j] = wr < p.cout_pad ? 0 : -1;
      iw0[j] = 0;
    } else {
      const int m = p0 + row - BCO;
      if (m < p.M) {
        const int n = m / OHW;
        const int rem = m - n * OHW;
        const int oh = rem / p.OW;
        const int ow = rem - oh * p.OW;
        ih0[j] = oh * p.SH - p.PH;
        iw0[j] = ow * p.SW - p.PW;
        rbase[j] = (unsigned)(((long)n * p.H * p.W * p.x_cstride + p.x_coff) * 2);
      } else {
        ih0[j] = -(1 << 28);
        iw0[j] = -(1 << 28);
        rbase[j] = 0;
      }
      if constexpr (FAST) frow[j] = fast_row(p, ih0[j], iw0[j], rbase[j], m < p.M, cl, xrow_bytes);
    }
  }

  // im2col K state of the next stage to issue: global chunk kc = ks*8 + cl
  const int cpt = p.cin8 >> 3;
  int tap = cl / cpt;
  int cc = cl - tap * cpt;
  int kh = tap / p.KW;
  int kw = tap - kh * p.KW;
  int ks_next = 0;
  const int nks = p.kpad / BK;
  [[maybe_unused]] FastStage fst;
  [[maybe_unused]] const int cpb = (p.KH * p.KW == 1) ? (p.kpad / BK) : (p.cin8 >> 6);

  auto issue = [&]() {
    bf16* st = smem + (ks_next % NS) * STAGE;
    const bool kvalid = kh < p.KH;
    const bool kin = ks_next < nks;
    const unsigned kofs = (unsigned)ks_next * (BK * 2);
    [[maybe_unused]] bool cv = false;
    [[maybe_unused]] unsigned soff = 0;
    if constexpr (FAST) {
      cv = kin && cl * 8 < p.cin8 - fst.cb * 64;   // channel tail of a 1x1 conv
      soff = (unsigned)(fst.kh * p.W + fst.kw) * xrow_bytes + (unsigned)fst.cb * 128u;
    }
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int q = wave * PPW + j;               // wave-uniform
      bf16* dst = st + q * 8 * BK;
      if (q * 8 < BCO) {
        dma16(wsrd, dst, (kin && ih0[j] == 0) ? rbase[j] + kofs : OOB);
      } else if constexpr (FAST) {
        const bool ok = cv && ((frow[j].mask >> (fst.tap & 31)) & 1u);
        dma16(xsrd, dst, ok ? frow[j].off + soff : OOB);
      } else {
        const int ihl = ih0[j] + kh, iwl = iw0[j] + kw;  // coordinates in the (dilated) input
        const int ih = ihl >> p.dsh, iw = iwl >> p.dsw;
        const bool ok = kvalid && ((ihl & ((1 << p.dsh) - 1)) | (iwl & ((1 << p.dsw) - 1))) == 0 &&
                        (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        const unsigned off = rbase[j] + (unsigned)(ih * p.W + iw) * xrow_bytes + (unsigned)cc * 16u;
        dma16(xsrd, dst, ok ? off : OOB);
      }
    }
    ++ks_next;
    if constexpr (FAST) {
      fst.advance(p, cpb);
    } else {
      cc += 8;
      while (cc >= cpt) {
        cc -= cpt;
        if (++kw == p.KW) { kw = 0; ++kh; }
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15;
  const int lq = lane >> 4;
  auto compute = [&](int buf) {
    const bf16* sA = smem + buf * STAGE;
    const bf16* sB = sA + BCO * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + lq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wco * WTCO + tm * 16 + li;
        af[tm] = *(const bf16x8*)(sA + row * BK + ((chunk ^ (row & 6)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wp * WTP + tn * 16 + li;
        bfr[tn] = *(const bf16x8*)(sB + row * BK + ((chunk ^ (row & 6)) << 3));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
  };

  // prologue: stages 0 .. NS-2 in flight; wait for stage 0
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue();
  wait_vmcnt<(NS - 2) * PPW>();
  raw_barrier();
  for (int ks = 0; ks < nks; ++ks) {
    issue();                      // stage ks+NS-1 into the buffer stage ks-1 used
    compute(ks % NS);             // stage ks
    wait_vmcnt<(NS - 2) * PPW>(); // stage ks+1 has landed (stages ks+2.. may still fly)
    raw_barrier();
  }
  wait_vmcnt<0>();

  if constexpr (EPI == EPI_TAPS) {
    static_assert(TM == 4 && TN == 2 && WCO == 4 && NW == 16, "EPI_TAPS tiling");
    taps_epilogue(p, acc, smem, p0, wco, wp, lane);
  } else {
    const int wrow0 = co0 + wco * WTCO;
    conv_epilogue<TM, TN, EPI>(p, acc, p0 + wp * WTP, wrow0, lq, li);
  }
}

template <int BCO, int BP, int WCO, int KIND>
int launch_cfg(const ConvParams* p, int epi, hipStream_t s) {
  // storage rows are permuted inside 64-row groups: cover every group that holds a real channel
  const int rows = (p->cout + 63) / 64 * 64;
  dim3 grid((p->M + BP - 1) / BP, (rows + BCO - 1) / BCO);
  dim3 block(256);
#define JR_LAUNCH(E)                                                                          \
  if constexpr (KIND == 9 || KIND == 11) {                                                     \
    constexpr int NW_ = KIND == 9 ? 8 : 16;                                                      \
    if (p->fast) hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, E, true, NW_, 1>), grid, dim3(NW_ * 64), 0, s, *p); \
    else hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, E, false, NW_, 1>), grid, dim3(NW_ * 64), 0, s, *p);         \
  } else if constexpr (KIND == 6 || KIND == 7) {                                                     \
    constexpr int NW_ = KIND == 6 ? 8 : 16;                                                    \
    if (p->fast) hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, E, true, NW_>), grid, dim3(NW_ * 64), 0, s, *p); \
    else hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, E, false, NW_>), grid, dim3(NW_ * 64), 0, s, *p);         \
  } else if constexpr (KIND == 3 || KIND == 4) hipLaunchKernelGGL((conv_d2_kernel<BCO, BP, WCO, KIND - 1, E>), grid, block, 0, s, *p); \
  else if constexpr (KIND >= 12 && KIND <= 14) {                                              \
    constexpr int NW_ = KIND == 13 ? 8 : 16, NS_ = KIND == 14 ? 2 : 3;                          \
    if (p->fast) hipLaunchKernelGGL((conv_d2_kernel<BCO, BP, WCO, NS_, E, true, NW_>), grid, dim3(NW_ * 64), 0, s, *p); \
    else hipLaunchKernelGGL((conv_d2_kernel<BCO, BP, WCO, NS_, E, false, NW_>), grid, dim3(NW_ * 64), 0, s, *p);         \
  } \
  else if constexpr (KIND == 2) {                                                              \
    if (p->fast) hipLaunchKernelGGL((conv_m32_kernel<BCO, BP, WCO, E, true>), grid, block, 0, s, *p); \
    else hipLaunchKernelGGL((conv_m32_kernel<BCO, BP, WCO, E, false>), grid, block, 0, s, *p);         \
  } else if constexpr (KIND == 8) {                                                            \
    if (p->fast) hipLaunchKernelGGL((conv_m32_kernel<BCO, BP, WCO, E, true, 8>), grid, dim3(512), 0, s, *p); \
    else hipLaunchKernelGGL((conv_m32_kernel<BCO, BP, WCO, E, false, 8>), grid, dim3(512), 0, s, *p);         \
  } else {                                                                                     \
    if (p->fast) hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, E, true>), grid, block, 0, s, *p); \
    else hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, E, false>), grid, block, 0, s, *p);         \
  }
  switch (epi) {
    case EPI_STD: JR_LAUNCH(EPI_STD) break;
    case EPI_GRU_A: JR_LAUNCH(EPI_GRU_A) break;
    case EPI_GRU_B: JR_LAUNCH(EPI_GRU_B) break;
    case EPI_BWD: JR_LAUNCH(EPI_BWD) break;
    case EPI_TAPS:
      // one N tile of 256 channels, 16 waves of 64 x 32 (configs 22, 34, 35, 38)
      if constexpr (BCO == 256 && BP == 128 && WCO == 4 && (KIND == 7 || KIND == 11 || KIND == 12 || KIND == 14)) {
        if (p->cout != 256) return (int)hipErrorInvalidValue;
        JR_LAUNCH(EPI_TAPS) break;
      } else {
        return (int)hipErrorInvalidValue;
      }
    default: return (int)hipErrorInvalidValue;
  }
#undef JR_LAUNCH
  return (int)hipGetLastError();
}

}  // namespace
