// Convolution of the 2-channel flow: the motion encoder's flow branch
// `convflow1` (7x7, 2 -> 128 + relu, jax_raft/model.py:282-283), run every
// refinement iteration.
//
// Through the generic implicit GEMM its K is 49 taps x (2 real of 8 padded)
// channels: 392 -> 448, each 16-B im2col chunk a separate scattered load, 3/4
// of the MFMA work on zeros.  Here K is packed for 2 channels: k = (kh, kw
// padded to KWP = 4 or 8, c), so one 16x16x32 MFMA k-chunk covers 16 taps and
// a lane's 8 B-operand elements are 4 consecutive taps of one kernel row =
// four 4-B (fx, fy) loads of horizontally adjacent pixels, assembled straight
// into the fragment register: no LDS, no im2col buffer.  7x7: K = 7 x 8 x 2 =
// 112 -> 4 k-chunks (3.5x fewer MFMAs than the padded GEMM).
//
// Block = 4 waves x 32 output channels (2 co tiles of 16) over 64 pixels
// (4 pixel tiles of 16).  The weight (A) fragments of a wave's 32 channels are
// loaded once, pre-packed on the host in fragment order (one 16-B load per
// fragment per lane).  The accumulator holds 4 consecutive channels of one
// pixel per lane; bias + relu fused, 8-B bf16 stores into the consumer's
// channel slice.
#pragma once
#include "common.h"
#include "kernels.h"

namespace {


typedef unsigned u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// one block (bx: 64-pixel tile, by: 128-channel group) -- kernel body shared with the
// merged launches of merged.hip
template <int KH, int KW>
JR_DEVICE void conv_flowin_block(const bf16* __restrict__ x, int xcs, int N, int H, int W, int PH, int PW,
                                 const bf16x8* __restrict__ wp, const float* __restrict__ bias, int cout, int relu,
                                 bf16* __restrict__ y, int ycs, int ycoff, int bx, int by) {
  constexpr int KWP = KW <= 4 ? 4 : 8;
  constexpr int NKC = (KH * KWP * 2 + 31) / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int co0 = (by * 4 + wave) * 32;
  if (co0 >= cout) return;
  const int li = lane & 15, kg = lane >> 4;
  bf16x8 a[2][NKC];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) a[t][kc] = wp[((co0 / 16 + t) * NKC + kc) * 64 + lane];
  float bv[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[t][r] = bias[co0 + 16 * t + 4 * kg + r];
  const int HW = H * W;
  const int M = N * HW;
  // all B-operand taps of the 4 pixel tiles are loaded before the first MFMA
  // (16 x NKC independent 4-B loads in flight per lane), then 8 x NKC MFMAs
  u32x4 u[4][NKC];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int m = bx * 64 + pt * 16 + li;
    const bool mok = m < M;
    const int mm = mok ? m : 0;
    const int n = mm / HW;
    const int rem = mm - n * HW;
    const int oy = rem / W;
    const int ox = rem - oy * W;
    const bf16* xn = x + (long)n * HW * xcs;
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      const int tt0 = kc * 16 + 4 * kg;   // first of this lane's 4 taps
      const int kh = tt0 / KWP, kw0 = tt0 % KWP;
      const int iy = oy + kh - PH;
      const bool rok = mok && kh < KH && (unsigned)iy < (unsigned)H;
      const int ix0 = ox + kw0 - PW;
      if (xcs == 2 && rok && ix0 >= 0 && ix0 + 3 < W) {
        // compact 2-channel source: the 4 taps are 16 contiguous bytes (4-B aligned; a
        // padding tap kw >= KW reads an in-image pixel and meets a zero weight)
        u[pt][kc] = *(const u32x4_a4*)(xn + ((long)iy * W + ix0) * 2);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kw = kw0 + q;
          const int ix = ix0 + q;
          const bool ok = rok && kw < KW && (unsigned)ix < (unsigned)W;
          u[pt][kc][q] = ok ? *(const unsigned*)(xn + ((long)iy * W + ix) * xcs) : 0u;
        }
      }
    }
  }
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int m = bx * 64 + pt * 16 + li;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, u[pt][kc]);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][kc], b, acc[t], 0, 0, 0);
    }
    if (m >= M) continue;
    bf16* yp = y + (long)m * ycs + ycoff + co0 + 4 * kg;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[t][r] + bv[t][r];
        o[r] = f2bf(relu ? fmaxf(v, 0.f) : v);
      }
      *(bf16x4*)(yp + 16 * t) = o;
    }
  }
}


template <int KH, int KW>
__global__ __launch_bounds__(256) void conv_flowin_kernel(const bf16* __restrict__ x, int xcs, int N, int H, int W,
                                                          int PH, int PW, const bf16x8* __restrict__ wp,
                                                          const float* __restrict__ bias, int cout, int relu,
                                                          bf16* __restrict__ y, int ycs, int ycoff) {
  conv_flowin_block<KH, KW>(x, xcs, N, H, W, PH, PW, wp, bias, cout, relu, y, ycs, ycoff, blockIdx.x, blockIdx.y);
}
}  // namespace
