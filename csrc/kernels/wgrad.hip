// Implicit-GEMM weight gradient of an NHWC convolution on gfx950 MFMA
// (training: every conv of the fused forward, reference sites as in
// conv_igemm.h).  dW[co][k] = sum_m dY[m][co] * im2col(X)[m][k], k = (tap, cin8
// chunk), m = (n, oh, ow): a long-K GEMM (K = pixels, up to 2e5 for the
// refinement loop's iteration-stacked convs) with a small output.
//
//  * No im2col in memory: each stage gathers a [64 pixel][BKK] tile of the
//    implicit im2col matrix straight from X (16-B chunks, zero padding via
//    buffer range checks) and a [64 pixel][BCO] tile of dY into LDS.
//  * Both MFMA operands reduce over the pixel dimension, which is the ROW
//    dimension of both LDS images: fragments are read with ds_read_b64_tr_b16
//    (gfx950 transposed LDS read, 4 pixels x 16 channels per 16-lane group),
//    two reads per 8-pixel fragment, on an XOR-swizzled image that keeps
//    every 32-lane half of those reads on distinct banks.
//  * Split-K over pixel ranges (grid.z): fp32 partial tiles, reduced in a
//    fixed order by a second kernel that writes the HWIO fp32 gradient
//    directly (the Flax kernel layout, no transpose copy) and the bias
//    gradient (column sums of dY, accumulated by the k-tile-0 workgroups
//    from the staged dY registers).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int WPX = 64;  // pixels per stage

// XOR swizzle (in 8-B units) of LDS image row r with U units per row, so that
// the transposed reads of a 32-lane half (rows 8g+q, g in {0,1}, q in 0..3,
// units 4a+p) hit 32 distinct bank pairs.
template <int U>
JR_DEVICE int swz(int r) {
  if constexpr (U >= 32) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
}

struct WgParams {
  const void* x; int xcs, xoff, N, H, W, cin8, KH, KW, SH, SW, PH, PW;
  const void* dy; int ycs, yoff, OH, OW, cout;
  int K, M, px_split;
  int gx, gy, S, per;               // k tiles, cout tiles, pixel splits; workgroups per XCD
  float* part; int cout_pad, kpad;  // [S][cout_pad][kpad]
  float* bpart;                     // [S][cout_pad] (bias partials) or null
  long x_bytes, y_bytes;
};

template <int BCO, int BKK, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void wgrad_kernel(const WgParams p) {
  constexpr int NT = 64 * WM * WN;                 // threads: WM x WN waves over the output tile
  constexpr int UA = BCO / 4, UB = BKK / 4;        // 8-B units per LDS row
  constexpr int A_EL = WPX * BCO, B_EL = WPX * BKK;
  constexpr int CA = BCO / 8, CB = BKK / 8;        // 16-B chunks per pixel row
  constexpr int NA = WPX * CA / NT, NB = WPX * CB / NT;    // chunks per thread
  constexpr int TM = BCO / WM / 16, TN = BKK / WN / 16;    // 16x16 tiles per wave
  static_assert(NA >= 1 && NB >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];   // 2 x (A_EL + B_EL)
  constexpr unsigned OOB = 0x80000000u;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  // XCD-aware order: hardware block L runs on XCD L % 8, so logical workgroup (L % 8) * per + L / 8
  // puts the gx * gy tiles of one pixel split -- which read the same dY rows and (tap-shifted) the
  // same X rows -- on one L2, dispatched back to back.  Padding blocks (logical id past the grid) exit.
  const int lid = (int)(blockIdx.x & 7) * p.per + (int)(blockIdx.x >> 3);
  const int tps = p.gx * p.gy;
  if (lid >= tps * p.S) return;
  const int bz = lid / tps, bt = lid - bz * tps;
  const int by = bt / p.gx, bx = bt - by * p.gx;
  const int k0 = bx * BKK, co0 = by * BCO;
  const int m_begin = bz * p.px_split;
  const int m_end = min(p.M, m_begin + p.px_split);
  const int OHW = p.OH * p.OW;
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, (int)p.y_bytes, 0x00020000);

  // fixed per-thread chunk columns: dY chunk cA = tid % CA (rows tid / CA + 256/CA * i),
  // X chunk cB = tid % CB (its tap / channel are fixed for the whole reduction)
  const int cA = tid % CA, rA = tid / CA;
  const int cB = tid % CB, rB = tid / CB;
  const bool a_ok = co0 + 8 * cA < p.cout;
  const int kk = k0 + 8 * cB;
  const int tap = kk / p.cin8, ci = kk - tap * p.cin8;
  const bool b_tap = tap < p.KH * p.KW && kk < p.K;
  const int kh = b_tap ? tap / p.KW : 0, kw = b_tap ? tap - (tap / p.KW) * p.KW : 0;

  struct Regs { u32x4 a[NA]; u32x4 b[NB]; };
  Regs ra;
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
  const bool do_bias = p.bpart != nullptr && bx == 0;

  // X rows of this thread: pixels m = stage base + rB + (256 / CB) i, tracked incrementally as
  // (n, oh, ow) (no integer division in the loop); every issue() advances them by one stage
  int xn[NB], xoh[NB], xow[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int m = m_begin + rB + (NT / CB) * i;
    xn[i] = m / OHW;
    const int rem = m - xn[i] * OHW;
    xoh[i] = rem / p.OW;
    xow[i] = rem - xoh[i] * p.OW;
  }
  int mb_next = m_begin;

  auto issue = [&](Regs& r) {
    const int mb = mb_next;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = mb + rA + (NT / CA) * i;
      const bool ok = a_ok && m < m_end;
      const unsigned off = (unsigned)(((long)m * p.ycs + p.yoff + co0 + 8 * cA) * 2);
      r.a[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ys, ok ? off : OOB, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int m = mb + rB + (NT / CB) * i;
      const int ih = xoh[i] * p.SH - p.PH + kh, iw = xow[i] * p.SW - p.PW + kw;
      const bool ok = b_tap && m < m_end && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const unsigned off = (unsigned)(((((long)xn[i] * p.H + ih) * p.W + iw) * p.xcs + p.xoff + ci) * 2);
      r.b[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xs, ok ? off : OOB, 0, 0));
      xow[i] += WPX;   // advance to the next stage's pixel
      while (xow[i] >= p.OW) {
        xow[i] -= p.OW;
        if (++xoh[i] == p.OH) { xoh[i] = 0; ++xn[i]; }
      }
    }
    mb_next = mb + WPX;
  };
  auto store = [&](const Regs& r, int buf) {
    bf16* sA = smem + buf * (A_EL + B_EL);
    bf16* sB = sA + A_EL;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = rA + (NT / CA) * i;
      const int u = (2 * cA) ^ swz<UA>(row);
      *(u32x4*)(sA + row * BCO + 4 * u) = r.a[i];
      if (do_bias) {
        const bf16x8 v = __builtin_bit_cast(bf16x8, r.a[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += bf2f(v[j]);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int row = rB + (NT / CB) * i;
      const int u = (2 * cB) ^ swz<UB>(row);
      *(u32x4*)(sB + row * BKK + 4 * u) = r.b[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto tr = [&](const bf16* img, int U, int cols, int r, int cb) -> s16x4 {
    // row r, 8-B unit of columns cb + 4 pp (the lane's part of the 4 x 16 block)
    const int u = cb / 4 + pp;
    const int sw = (U >= 32) ? (4 * ((r & 3) | (((r >> 3) & 1) << 2))) : (4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)));
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r * cols + 4 * (u ^ sw)));
  };
  auto compute = [&](int buf) {
    const bf16* sA = smem + buf * (A_EL + B_EL);
    const bf16* sB = sA + A_EL;
#pragma unroll
    for (int ks = 0; ks < WPX / 32; ++ks) {
      const int r0 = 32 * ks + 8 * g + q;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int cb = wr * (BCO / WM) + 16 * tm;
        const s16x4 lo = tr(sA, UA, BCO, r0, cb), hi = tr(sA, UA, BCO, r0 + 4, cb);
        af[tm] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int cb = wc * (BKK / WN) + 16 * tn;
        const s16x4 lo = tr(sB, UB, BKK, r0, cb), hi = tr(sB, UB, BKK, r0 + 4, cb);
        bfr[tn] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
  };

  // Register-staged pipeline: the next stage's global loads fly while this stage
  // multiplies (LDS double-buffered, one barrier per stage); loads past the split's
  // end read zeros (range-checked).  (A second register set -- loads two stages
  // ahead -- measured 10-15 % slower on the loop shapes: fewer resident waves.)
  const int nst = (m_end - m_begin + WPX - 1) / WPX;
  issue(ra);
  store(ra, 0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) issue(ra);
    compute(buf);
    if (st + 1 < nst) store(ra, buf ^ 1);
    __syncthreads();
  }

  // partial tile -> part[z][co][k]
  float* out = p.part + (long)bz * p.cout_pad * p.kpad;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + wr * (BCO / WM) + 16 * tm + 4 * g + j;
        const int k = k0 + wc * (BKK / WN) + 16 * tn + (lane & 15);
        out[(long)co * p.kpad + k] = acc[tm][tn][j];
      }
  if (do_bias) {
    // threads with the same chunk column cA hold partial sums of the same 8 channels
    __syncthreads();
    float* red = (float*)smem;
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bsum[j];
    __syncthreads();
    if (tid < BCO) {
      const int c8 = tid >> 3, j = tid & 7;
      float s = 0.f;
      for (int t = c8; t < NT; t += CA) s += red[t * 8 + j];
      p.bpart[(long)bz * p.cout_pad + co0 + tid] = s;
    }
  }
}

// dW_hwio[kh][kw][ci][co] = sum_z part[z][co][(kh*KW + kw)*cin8 + ci] (ci < cin), db[co] = sum_z bpart[z][co].
// Block = one output channel co x 32 consecutive k: thread (k lane, z group of 8) sums
// every 8th split along z with coalesced reads (k is the partials' contiguous dim),
// the 8 groups combine through LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, const float* __restrict__ bpart,
                                                           int S, int cout_pad, int kpad, int KH, int KW, int cin8,
                                                           int cin, int cout, float* __restrict__ dw,
                                                           float* __restrict__ db) {
  __shared__ float red[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int co = blockIdx.y;
  const int k = blockIdx.x * 32 + tx;
  const long zs = (long)cout_pad * kpad;
  float s = 0.f;
  if (k < kpad) {
    const float* pp = part + (long)co * kpad + k;
#pragma unroll 4
    for (int z = ty; z < S; z += 8) s += pp[z * zs];
  }
  red[ty][tx] = s;
  float b = 0.f;
  if (db && blockIdx.x == 0 && tx == 0)
    for (int z = ty; z < S; z += 8) b += bpart[(long)z * cout_pad + co];
  __syncthreads();
  if (ty == 0) {
    float v = red[0][tx];
#pragma unroll
    for (int j = 1; j < 8; ++j) v += red[j][tx];
    const int tap = k / cin8, ci = k - tap * cin8;
    if (tap < KH * KW && ci < cin) dw[((long)tap * cin + ci) * cout + co] = v;
  }
  __syncthreads();
  if (db && blockIdx.x == 0) {
    if (tx == 0) red[ty][0] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
      float v = red[0][0];
      for (int j = 1; j < 8; ++j) v += red[j][0];
      db[co] = v;
    }
  }
}

template <int BCO, int BKK, int WM = 2, int WN = 2>
int launch(const WgParams& p, int S, hipStream_t st) {
  constexpr int lds = 2 * WPX * (BCO + BKK) * 2;
  static const bool attr = hipFuncSetAttribute((const void*)wgrad_kernel<BCO, BKK, WM, WN>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!attr) return (int)hipErrorInvalidValue;
  WgParams q = p;
  q.gx = (p.K + BKK - 1) / BKK;
  q.gy = (p.cout + BCO - 1) / BCO;
  q.S = S;
  q.per = (q.gx * q.gy * S + 7) / 8;
  hipLaunchKernelGGL((wgrad_kernel<BCO, BKK, WM, WN>), dim3(8 * q.per), dim3(64 * WM * WN), lds, st, q);
  return (int)hipGetLastError();
}

// Tile of one wgrad problem.  256 x 256 for the refinement loop's wide convs (cout >= 192, K >= 1024):
// 128 FLOP per staged byte (vs 64 for 128 x 128), which the per-CU operand stream from L2 / MALL bounds,
// at one resident workgroup per CU (128 KB of LDS, the accumulators in AGPRs).
inline void wgrad_tile(int K, int cout, int* bco, int* bkk, int* slots) {
  if (cout >= 192 && K >= 1024) {
    *bco = 256; *bkk = 256; *slots = 256;
  } else {
    *bco = cout > 64 ? 128 : 64; *bkk = K > 64 ? 128 : 64; *slots = 512;
  }
}


// ---------------------------------------------------------------------------------------------
// Halo weight gradient of a 3x3 / stride-1 / pad-1 conv (every 3x3 conv of the encoders' residual
// blocks, the motion encoder, flow head and mask head; model.py:120-159, 275-289, 347-349, 389-390).
//
// The im2col kernel above re-gathers the input for every K tile: 9 shifted copies of each pixel
// row per 3x3 tap.  Here a workgroup owns a (64 output x 64 input channel) block of dW (all 9 taps:
// a 64 x 576 output tile) and walks a contiguous range of 8 x 16 pixel tiles: per tile it stages the
// tile's dY rows [128 px][64 co] and the input footprint [10 x 18 px][64 ci] in LDS once, and reads
// the B fragment of tap (u, v) from the footprint shifted by a constant -- 39 KB staged per 9.4
// MFLOP (241 FLOP per byte, vs 64 for the 128 x 128 im2col tile).
//
// MFMA v_mfma_f32_16x16x32_bf16, K = pixels: both operands are transposed LDS reads
// (ds_read_b64_tr_b16) of images whose rows are pixels, as in wgrad_kernel; each lane addresses its
// own pixel row, so the footprint rows of a tap are just (pixel row + tap offset).  Wave w computes
// the 64 co x (9 taps x 16 ci at 16 w) block: 4 x 9 accumulators (one wave per SIMD, ~480 registers).  Partials go to the same
// [split][cout_pad][kpad] layout as wgrad_kernel (k = tap * cin8 + ci), reduced by wgrad_reduce_kernel.
// ---------------------------------------------------------------------------------------------
constexpr int HTR = 8, HTC = 16, HFW = HTC + 2, HNF = (HTR + 2) * HFW;   // tile, footprint
constexpr int HPX = HTR * HTC;                                          // 128 pixels per tile
constexpr int HA_EL = HPX * 64, HB_EL = (HNF + 4) * 64;                 // LDS image elements
constexpr int HNT = 256;                                                // 4 waves, one per SIMD
constexpr int HNA = HPX * 8 / HNT, HNB = (HNF * 8 + HNT - 1) / HNT;     // 16-B chunks per thread

struct WgHaloParams {
  const void* x; int xcs, xoff, N, H, W, cin8;
  const void* dy; int ycs, yoff, cout;
  int tiles_x, tiles_y, ntiles, nco, nci, S, per, tps;   // tps: tiles per split
  float* part; int cout_pad, kpad;
  float* bpart;
  long x_bytes, y_bytes;
};

JR_DEVICE int hswz(int r) { return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }   // 64-col image

__global__ __launch_bounds__(256, 1) void wgrad_halo_kernel(const WgHaloParams p) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];   // 2 x (A image + B image)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lid = (int)(blockIdx.x & 7) * p.per + (int)(blockIdx.x >> 3);   // XCD-aware (wgrad_kernel)
  const int ncb = p.nco * p.nci;
  if (lid >= ncb * p.S) return;
  const int z = lid / ncb, cb = lid - z * ncb;
  const int cob = cb / p.nci, cib = cb - cob * p.nci;
  const int co0 = cob * 64, ci0 = cib * 64;
  const int t_begin = z * p.tps, t_end = min(p.ntiles, t_begin + p.tps);
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, (int)p.y_bytes, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const bool do_bias = p.bpart != nullptr && cib == 0;

  struct Regs { u32x4 a[HNA]; u32x4 b[HNB]; };
  Regs ra;
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
  const int ch = tid & 7;          // 16-B chunk (8 channels) of every row this thread stages
  const bool a_ok = co0 + 8 * ch < p.cout;
  const bool b_ok = ci0 + 8 * ch < p.cin8;

  auto issue = [&](Regs& r, int t) {
    const int per_img = p.tiles_x * p.tiles_y;
    const int n = t / per_img, rem = t - n * per_img;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    const int y0 = ty * HTR, x0 = tx * HTC;
#pragma unroll
    for (int i = 0; i < HNA; ++i) {
      const int row = (tid >> 3) + (HNT / 8) * i;   // pixel of the tile
      const int yy = y0 + (row >> 4), xx = x0 + (row & 15);
      const bool ok = a_ok && yy < p.H && xx < p.W;
      const unsigned off = (unsigned)(((long)((n * p.H + yy) * p.W + xx) * p.ycs + p.yoff + co0 + 8 * ch) * 2);
      r.a[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ys, ok ? off : OOB, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < HNB; ++i) {
      const int f = (tid >> 3) + (HNT / 8) * i;     // footprint pixel
      const int fy = f / HFW, fx = f - fy * HFW;
      const int yy = y0 - 1 + fy, xx = x0 - 1 + fx;
      const bool ok = b_ok && f < HNF && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      const unsigned off = (unsigned)(((long)((n * p.H + yy) * p.W + xx) * p.xcs + p.xoff + ci0 + 8 * ch) * 2);
      r.b[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xs, ok ? off : OOB, 0, 0));
    }
  };
  auto store = [&](const Regs& r, int buf) {
    bf16* sA = smem + buf * (HA_EL + HB_EL);
    bf16* sB = sA + HA_EL;
#pragma unroll
    for (int i = 0; i < HNA; ++i) {
      const int row = (tid >> 3) + (HNT / 8) * i;
      *(u32x4*)(sA + row * 64 + 4 * ((2 * ch) ^ hswz(row))) = r.a[i];
      if (do_bias) {
        const bf16x8 v = __builtin_bit_cast(bf16x8, r.a[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += bf2f(v[j]);
      }
    }
#pragma unroll
    for (int i = 0; i < HNB; ++i) {
      const int f = (tid >> 3) + (HNT / 8) * i;
      if (f < HNF) *(u32x4*)(sB + f * 64 + 4 * ((2 * ch) ^ hswz(f))) = r.b[i];
    }
  };

  // wave w: all 64 output channels x input channels ci0 + 16 w + [0, 16), all taps (measured: 8 waves of
  // 32 x 144 -- two per SIMD, B fragments read twice -- were 20-30 % slower)
  const int wco = 0, wci = wave;
  f32x4 acc[4][9];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 9; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  // transposed read of the 4 x 16 block at image row r (this lane's row), columns cb + 4 pp
  auto tr = [&](const bf16* img, int r, int cbase) -> s16x4 {
    const int u = cbase / 4 + pp;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r * 64 + 4 * (u ^ hswz(r))));
  };
  auto fpr = [](int px) { return (px >> 4) * HFW + (px & 15); };   // footprint row of pixel (tap (0, 0))
  auto compute = [&](int buf) {
    const bf16* sA = smem + buf * (HA_EL + HB_EL);
    const bf16* sB = sA + HA_EL;
#pragma unroll
    for (int ks = 0; ks < HPX / 32; ++ks) {
      const int p0 = 32 * ks + 8 * g + q;           // this lane's pixels: p0 (low half), p0 + 4 (high)
      bf16x8 af[4];
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const s16x4 lo = tr(sA, p0, 32 * wco + 16 * tm), hi = tr(sA, p0 + 4, 32 * wco + 16 * tm);
        af[tm] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      const int f0 = fpr(p0), f1 = fpr(p0 + 4);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int to = (tap / 3) * HFW + tap % 3;
        const s16x4 lo = tr(sB, f0 + to, 16 * wci), hi = tr(sB, f1 + to, 16 * wci);
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) acc[tm][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr, acc[tm][tap], 0, 0, 0);
      }
    }
  };

  if (t_begin < t_end) {
    issue(ra, t_begin);
    store(ra, 0);
    __syncthreads();
    for (int t = t_begin; t < t_end; ++t) {
      const int buf = (t - t_begin) & 1;
      if (t + 1 < t_end) issue(ra, t + 1);
      compute(buf);
      if (t + 1 < t_end) store(ra, buf ^ 1);
      __syncthreads();
    }
  }

  // partial tile -> part[z][co][tap * cin8 + ci]
  float* out = p.part + (long)z * p.cout_pad * p.kpad;
#pragma unroll
  for (int tm = 0; tm < 4; ++tm)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ci = ci0 + 16 * wci + (lane & 15);
      if (ci >= p.cin8) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + 32 * wco + 16 * tm + 4 * g + j;
        out[(long)co * p.kpad + tap * p.cin8 + ci] = acc[tm][tap][j];
      }
    }
  if (do_bias) {
    // threads with the same chunk ch hold partial sums of the same 8 channels
    __syncthreads();
    float* red = (float*)smem;
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bsum[j];
    __syncthreads();
    if (tid < 64) {
      const int c8 = tid >> 3, j = tid & 7;
      float s = 0.f;
      for (int t = c8; t < HNT; t += 8) s += red[t * 8 + j];
      p.bpart[(long)z * p.cout_pad + co0 + tid] = s;
    }
  }
}

// the halo path serves 3x3 / stride-1 / pad-1 convs; S: splits of the pixel tiles so that the
// (split x channel block) grid is about one round of resident workgroups (one per CU: ~480 registers)
inline bool wgrad_halo_ok(int KH, int KW, int SH, int SW, int PH, int PW) {
  return KH == 3 && KW == 3 && SH == 1 && SW == 1 && PH == 1 && PW == 1;
}
inline void wgrad_halo_geom(int N, int H, int W, int cin8, int cout, int* ntiles, int* nco, int* nci, int* S, int* tps) {
  const int tx = (W + HTC - 1) / HTC, ty = (H + HTR - 1) / HTR;
  *ntiles = N * tx * ty;
  *nco = (cout + 63) / 64;
  *nci = (cin8 + 63) / 64;
  const int cbs = *nco * *nci;
  int s = std::max(1, std::min(256 / cbs, (*ntiles + 3) / 4));   // one workgroup per CU, >= 4 tiles per split
  *tps = (*ntiles + s - 1) / s;
  *S = (*ntiles + *tps - 1) / *tps;
}

}  // namespace

extern "C" int jr_wgrad_plan(int M, int K, int cout, int* S, int* cout_pad, int* kpad) {
  int bco, bkk, slots;
  wgrad_tile(K, cout, &bco, &bkk, &slots);
  const int tiles = ((K + bkk - 1) / bkk) * ((cout + bco - 1) / bco);
  // one round of resident workgroups (2 per CU at 64 KB of LDS, 1 at 128 KB): S = floor(slots / tiles)
  // (rounding up left a few workgroups for a second round), >= 4 stages of pixels per split
  int s = std::max(1, std::min(slots / tiles, (M + 4 * WPX - 1) / (4 * WPX)));
  *S = s;
  *cout_pad = (cout + bco - 1) / bco * bco;
  *kpad = (K + bkk - 1) / bkk * bkk;
  return 0;
}

extern "C" int jr_wgrad_plan_geom(int N, int H, int W, int cin8, int KH, int KW, int SH, int SW, int PH, int PW,
                                  int OH, int OW, int cout, int* S, int* cout_pad, int* kpad) {
  jr_wgrad_plan(N * OH * OW, KH * KW * cin8, cout, S, cout_pad, kpad);
  if (wgrad_halo_ok(KH, KW, SH, SW, PH, PW)) {
    int nt, nco, nci, s, tps;
    wgrad_halo_geom(N, H, W, cin8, cout, &nt, &nco, &nci, &s, &tps);
    *S = s;
    *cout_pad = std::max(*cout_pad, nco * 64);
  }
  return 0;
}

extern "C" int jr_wgrad(const void* x, int xcs, int xoff, int N, int H, int W, int cin8, int KH, int KW, int SH,
                        int SW, int PH, int PW, const void* dy, int ycs, int yoff, int OH, int OW, int cout, int cin,
                        float* part, float* bpart, int S, float* dw, float* db, long x_bytes, long y_bytes,
                        hipStream_t stream) {
  if (cin8 % 8 || xcs % 8 || xoff % 8 || ycs % 8 || yoff % 8) return (int)hipErrorInvalidValue;
  WgParams p{};
  p.x = x; p.xcs = xcs; p.xoff = xoff; p.N = N; p.H = H; p.W = W; p.cin8 = cin8;
  p.KH = KH; p.KW = KW; p.SH = SH; p.SW = SW; p.PH = PH; p.PW = PW;
  p.dy = dy; p.ycs = ycs; p.yoff = yoff; p.OH = OH; p.OW = OW; p.cout = cout;
  p.K = KH * KW * cin8;
  p.M = N * OH * OW;
  int s_, cp, kp;
  jr_wgrad_plan_geom(N, H, W, cin8, KH, KW, SH, SW, PH, PW, OH, OW, cout, &s_, &cp, &kp);
  if (S <= 0) S = s_;
  if (wgrad_halo_ok(KH, KW, SH, SW, PH, PW)) {
    WgHaloParams h{};
    h.x = x; h.xcs = xcs; h.xoff = xoff; h.N = N; h.H = H; h.W = W; h.cin8 = cin8;
    h.dy = dy; h.ycs = ycs; h.yoff = yoff; h.cout = cout;
    h.tiles_x = (W + HTC - 1) / HTC; h.tiles_y = (H + HTR - 1) / HTR;
    int s;
    wgrad_halo_geom(N, H, W, cin8, cout, &h.ntiles, &h.nco, &h.nci, &s, &h.tps);
    if (S < s) return (int)hipErrorInvalidValue;   // workspace planned for another geometry
    h.S = s;
    h.per = (h.nco * h.nci * s + 7) / 8;
    h.part = part; h.cout_pad = cp; h.kpad = kp; h.bpart = db ? bpart : nullptr;
    h.x_bytes = x_bytes; h.y_bytes = y_bytes;
    constexpr int lds = 2 * (HA_EL + HB_EL) * 2;
    static const bool attr = hipFuncSetAttribute((const void*)wgrad_halo_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 lds) == hipSuccess;
    if (!attr) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(wgrad_halo_kernel, dim3(8 * h.per), dim3(HNT), lds, stream, h);
    if (const int e = (int)hipGetLastError()) return e;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((p.K + 31) / 32), (unsigned)cout), dim3(256), 0, stream, part,
                       h.bpart, s, cp, kp, KH, KW, cin8, cin, cout, dw, db);
    return (int)hipGetLastError();
  }
  const int per = (p.M + S - 1) / S;
  p.px_split = (per + WPX - 1) / WPX * WPX;
  S = (p.M + p.px_split - 1) / p.px_split;
  p.part = part; p.cout_pad = cp; p.kpad = kp; p.bpart = db ? bpart : nullptr;
  p.x_bytes = x_bytes; p.y_bytes = y_bytes;
  int bco, bkk, slots;
  wgrad_tile(p.K, cout, &bco, &bkk, &slots);
  const bool bc = cout > 64, bk = p.K > 64;
  int r;
  if (bco == 256) r = launch<256, 256, 2, 4>(p, S, stream);
  else if (bc && bk) r = launch<128, 128>(p, S, stream);
  else if (bc) r = launch<128, 64>(p, S, stream);
  else if (bk) r = launch<64, 128>(p, S, stream);
  else r = launch<64, 64>(p, S, stream);
  if (r) return r;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((p.K + 31) / 32), (unsigned)cout), dim3(256), 0, stream, part,
                     p.bpart, S, cp, kp, KH, KW, cin8, cin, cout, dw, db);
  return (int)hipGetLastError();
}
