// Flow-head output conv (3x3, hidden -> 2) as per-pixel tap partials + the
// coordinate update (FlowHead.conv2, jax_raft/model.py:347-350, and
// `coords1 = coords1 + delta`, model.py:505).  (A halo-tiled direct kernel
// for the 3x3 conv was measured slower and retired in round 3.)
#include "common.h"
#include "kernels.h"

// ---------------------------------------------------------------------------
// Flow-head output conv as "1x1 GEMM + tap sum" (the default engine path).
// A 3x3 conv with 2 outputs is linear in its input, so
//   delta(p) = b + sum_{kh,kw} W[kh][kw]^T fm(p + (kh-1, kw-1))
//            = b + sum_tap t[p + d_tap][tap],   t[q][tap] = W[tap]^T fm(q)
// t (9 taps x 2 outputs per pixel) is ONE 1x1 implicit-GEMM conv over fm
// (K = cin, N = 18: fm is read once instead of 9 times), and this kernel adds
// the 9 shifted partials (zero padding = skipping out-of-map neighbours)
// and applies the update: coords += delta, flow =
// coords - grid as fp32 and as bf16 into hx / qx / flow8 (model.py:347-350,505).
// One thread per pixel; t is [M][tcs] fp32 (tcs >= 18), 2.7 MB at batch 4 and
// L2-resident right after the GEMM that wrote it.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void flow_taps_kernel(const float* __restrict__ t, int tcs, const float* __restrict__ bias,
                                                       int N, int h, int w, float* __restrict__ coords,
                                                       float* __restrict__ flow32, bf16* __restrict__ hx, int hx_cs,
                                                       int hx_off, bf16* __restrict__ qx, int qx_cs, int qx_off,
                                                       bf16* __restrict__ f8, int f8_cs) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  const long M = (long)N * h * w;
  if (m >= M) return;
  const int hw = h * w;
  const int rem = (int)(m % hw);
  const int y = rem / w, x = rem - (rem / w) * w;
  const long img0 = m - rem;
  float dx = bias[0], dy = bias[1];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int yy = y + kh - 1;
    if ((unsigned)yy >= (unsigned)h) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int xx = x + kw - 1;
      if ((unsigned)xx >= (unsigned)w) continue;
      const float2 v = *(const float2*)(t + (img0 + (long)yy * w + xx) * tcs + 2 * (kh * 3 + kw));
      dx += v.x;
      dy += v.y;
    }
  }
  const float cx = coords[2 * m] + dx;
  const float cy = coords[2 * m + 1] + dy;
  coords[2 * m] = cx;
  coords[2 * m + 1] = cy;
  const float fx = cx - (float)x, fy = cy - (float)y;
  flow32[2 * m] = fx;
  flow32[2 * m + 1] = fy;
  hx[m * hx_cs + hx_off] = f2bf(fx);
  hx[m * hx_cs + hx_off + 1] = f2bf(fy);
  if (qx) {
    qx[m * qx_cs + qx_off] = f2bf(fx);
    qx[m * qx_cs + qx_off + 1] = f2bf(fy);
  }
  if (f8) {
    f8[m * f8_cs] = f2bf(fx);
    f8[m * f8_cs + 1] = f2bf(fy);
  }
}

// ---------------------------------------------------------------------------
// Flow head output conv as per-pixel taps (the "taps" formulation above):
// taps[m][0..24) = fm[m][fcoff .. fcoff + K) . Wt[K][24] (18 real columns,
// tap * 2 + o; the rest zero).  A skinny GEMM (N = 18): the generic conv tile
// pads the 18 output rows to 64 and runs 220 one-round workgroups at batch 4
// (10.7 us, latency bound); here one wave owns 16 pixels and all 32 (padded)
// output rows as two 16x16x32 MFMA row tiles, and loads every k-step's
// fragments up front (K = 256: 8 x 16 B features + 16 x 16 B weights per
// lane), so a wave costs one memory round trip.  Weights are packed host-side
// (ops/native.py:pack_taps) as A fragments [k-step][row tile 2][lane 64][8].
// ---------------------------------------------------------------------------
template <int KS>  // K / 32
__global__ __launch_bounds__(256) void taps_gemm_kernel(const bf16* __restrict__ fm, int fcs, int fcoff,
                                                        const u32x4* __restrict__ wpk, float* __restrict__ taps,
                                                        int tcs, int M) {
  const int lane = threadIdx.x & 63;
  const int p0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  if (p0 >= M) return;  // whole wave
  const int col = lane & 15, q = lane >> 4;
  const bf16* bp = fm + (long)min(p0 + col, M - 1) * fcs + fcoff + 8 * q;
  u32x4 b[KS], a0[KS], a1[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    b[ks] = *(const u32x4*)(bp + 32 * ks);
    a0[ks] = wpk[(ks * 2) * 64 + lane];
    a1[ks] = wpk[(ks * 2 + 1) * 64 + lane];
  }
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const bf16x8 bv = __builtin_bit_cast(bf16x8, b[ks]);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a0[ks]), bv, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a1[ks]), bv, c1, 0, 0, 0);
  }
  if (p0 + col < M) {  // lane holds rows 4q .. 4q+3 of each row tile for pixel p0 + col
    float* tp = taps + (long)(p0 + col) * tcs;
    *(f32x4*)(tp + 4 * q) = c0;
    if (q < 2) *(f32x4*)(tp + 16 + 4 * q) = c1;
  }
}

extern "C" int jr_taps_gemm(const void* fm, int fcs, int fcoff, int K, const void* wpk, float* taps, int tcs, int M,
                            hipStream_t stream) {
  if (tcs < 24 || tcs % 4 || fcs % 8 || fcoff % 8) return (int)hipErrorInvalidValue;
  const dim3 grid((M + 63) / 64);
  if (K == 256)
    hipLaunchKernelGGL(taps_gemm_kernel<8>, grid, dim3(256), 0, stream, (const bf16*)fm, fcs, fcoff,
                       (const u32x4*)wpk, taps, tcs, M);
  else if (K == 128)
    hipLaunchKernelGGL(taps_gemm_kernel<4>, grid, dim3(256), 0, stream, (const bf16*)fm, fcs, fcoff,
                       (const u32x4*)wpk, taps, tcs, M);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

extern "C" int jr_flow_taps(const float* t, int tcs, const float* bias, int N, int h, int w, float* coords,
                            float* flow32, void* hx, int hx_cs, int hx_off, void* qx, int qx_cs, int qx_off, void* f8,
                            int f8_cs, hipStream_t stream) {
  const long M = (long)N * h * w;
  if (tcs < 18 || (tcs & 1)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(flow_taps_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, stream, t, tcs, bias, N, h, w,
                     coords, flow32, (bf16*)hx, hx_cs, hx_off, (bf16*)qx, qx_cs, qx_off, (bf16*)f8, f8_cs);
  return (int)hipGetLastError();
}
