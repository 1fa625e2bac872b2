// Training-only kernels of the fused refinement-loop backward (gfx950):
// the adjoints of the x8 flow upsampling (jax_raft/model.py:69-98) w.r.t. the
// mask logits and the low-res flow.  Both are deterministic gathers (no float
// atomics): the convex upsampling's flow gradient is split into per-neighbour
// partials (one wave per low-res pixel) and a shifted-partials sum, the same
// "taps" decomposition the forward flow head uses (flowhead.hip).
#include "common.h"
#include "kernels.h"

namespace {

JR_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// One wave per low-res pixel q, lane = sub-pixel s = a*8 + b (as the forward).
// up(s) = sum_k w_k(s) u_k, w = softmax_k(mask[k*64 + s]), u_k = 8 flow(q + d_k) (0 off-map).
//   dL/dmask_k(s) = w_k (g.u_k - g.up)          (g = dL/dup(s))
//   dL/du_k      = sum_s w_k(s) g(s)  ->  taps[q][2k + c] = 8 sum_s w_k(s) g_c(s)
__global__ __launch_bounds__(256) void upsample_convex_bwd_kernel(const bf16* __restrict__ mask, int mcs,
                                                                  const float* __restrict__ flow,
                                                                  const float* __restrict__ gout, int B, int h, int w,
                                                                  float alpha, bf16* __restrict__ dmask, int dcs,
                                                                  float* __restrict__ taps) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int P = h * w;
  if (p >= B * P) return;  // wave-uniform
  const int b = p / P;
  const int rem = p - b * P;
  const int y = rem / w, x = rem - y * w;
  const bf16* mp = mask + (long)p * mcs + lane;
  float wk[9], ux[9], uy[9];
  float mx = -3.0e38f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    wk[k] = bf2f(mp[k * 64]);
    mx = fmaxf(mx, wk[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    wk[k] = __expf(wk[k] - mx);
    s += wk[k];
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    ux[k] = uy[k] = 0.f;
    if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) {
      const float2 f = *(const float2*)(flow + 2 * ((long)b * P + yy * w + xx));
      ux[k] = 8.f * f.x;
      uy[k] = 8.f * f.y;
    }
  }
  const float inv = 1.f / s;
  float upx = 0.f, upy = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    wk[k] *= inv;
    upx += wk[k] * ux[k];
    upy += wk[k] * uy[k];
  }
  const int a = lane >> 3, bb = lane & 7;
  const long W8 = 8L * w;
  const float2 g = *(const float2*)(gout + 2 * (((long)b * 8 * h + 8 * y + a) * W8 + 8 * x + bb));
  const float gu = g.x * upx + g.y * upy;
  bf16* dp = dmask + (long)p * dcs + lane;
#pragma unroll
  for (int k = 0; k < 9; ++k) dp[k * 64] = f2bf(alpha * wk[k] * (g.x * ux[k] + g.y * uy[k] - gu));
  float tx[9], ty[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    tx[k] = wave_sum(8.f * wk[k] * g.x);
    ty[k] = wave_sum(8.f * wk[k] * g.y);
  }
  if (lane == 0) {
    float2* tp = (float2*)(taps + (long)p * 18);
#pragma unroll
    for (int k = 0; k < 9; ++k) tp[k] = make_float2(tx[k], ty[k]);
  }
}

// dflow(p) = sum over the in-map q = p - d_k of taps[q][2k + c].  One thread per pixel.
__global__ __launch_bounds__(256) void flow_gather_bwd_kernel(const float* __restrict__ taps, int tcs, int N, int h,
                                                              int w, bf16* __restrict__ dflow, int dcs) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  const long M = (long)N * h * w;
  if (m >= M) return;
  const int hw = h * w;
  const int rem = (int)(m % hw);
  const int y = rem / w, x = rem - (rem / w) * w;
  const long img0 = m - rem;
  float dx = 0.f, dy = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int yy = y - (kh - 1);
    if ((unsigned)yy >= (unsigned)h) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int xx = x - (kw - 1);
      if ((unsigned)xx >= (unsigned)w) continue;
      const float2 v = *(const float2*)(taps + (img0 + (long)yy * w + xx) * tcs + 2 * (kh * 3 + kw));
      dx += v.x;
      dy += v.y;
    }
  }
  bf16* o = dflow + m * dcs;
  o[0] = f2bf(dx);
  o[1] = f2bf(dy);
  for (int c = 2; c < dcs; ++c) o[c] = f2bf(0.f);
}

// Bilinear x8 (align_corners) adjoint as a gather: low-res pixel (y, x) collects
// 8 * wy(Y, y) * wx(X, x) * g(Y, X) over the high-res pixels whose 2x2 source
// window contains it (the forward's clamped x0 / x1 = min(x0 + 1, w - 1) weights).
JR_DEVICE void src_window(int X, float sc, int w, int& x0, int& x1, float& f) {
  const float xi = X * sc;
  x0 = min(max((int)floorf(xi), 0), w - 1);
  x1 = min(x0 + 1, w - 1);
  f = xi - x0;
}

__global__ __launch_bounds__(256) void upsample_bilinear_bwd_kernel(const float* __restrict__ gout, int B, int h, int w,
                                                                    bf16* __restrict__ dflow, int dcs) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  const long M = (long)B * h * w;
  if (m >= M) return;
  const int hw = h * w;
  const int b = (int)(m / hw);
  const int rem = (int)(m - (long)b * hw);
  const int y = rem / w, x = rem - (rem / w) * w;
  const int H8 = 8 * h, W8 = 8 * w;
  const float sx = (w > 1) ? (float)(w - 1) / (float)(W8 - 1) : 0.f;
  const float sy = (h > 1) ? (float)(h - 1) / (float)(H8 - 1) : 0.f;
  // candidate ranges: floor(X * sx) in [x - 1, x] (+1 margin for rounding)
  const int X0 = sx > 0.f ? max(0, (int)floorf((x - 1) / sx) - 1) : 0;
  const int X1 = sx > 0.f ? min(W8 - 1, (int)ceilf((x + 1) / sx) + 1) : W8 - 1;
  const int Y0 = sy > 0.f ? max(0, (int)floorf((y - 1) / sy) - 1) : 0;
  const int Y1 = sy > 0.f ? min(H8 - 1, (int)ceilf((y + 1) / sy) + 1) : H8 - 1;
  const float2* g = (const float2*)gout + (long)b * H8 * W8;
  float dx = 0.f, dy = 0.f;
  for (int Y = Y0; Y <= Y1; ++Y) {
    int a0, a1;
    float fy;
    src_window(Y, sy, h, a0, a1, fy);
    const float wyc = (a0 == y ? 1.f - fy : 0.f) + (a1 == y ? fy : 0.f);
    if (wyc == 0.f) continue;
    for (int X = X0; X <= X1; ++X) {
      int c0, c1;
      float fx;
      src_window(X, sx, w, c0, c1, fx);
      const float wxc = (c0 == x ? 1.f - fx : 0.f) + (c1 == x ? fx : 0.f);
      if (wxc == 0.f) continue;
      const float2 v = g[(long)Y * W8 + X];
      dx += wyc * wxc * v.x;
      dy += wyc * wxc * v.y;
    }
  }
  bf16* o = dflow + m * dcs;
  o[0] = f2bf(8.f * dx);
  o[1] = f2bf(8.f * dy);
  for (int c = 2; c < dcs; ++c) o[c] = f2bf(0.f);
}

inline unsigned nblk(long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

}  // namespace

extern "C" int jr_upsample_convex_bwd(const void* mask, int mask_cs, const float* flow, const float* gout, int B,
                                      int h, int w, float alpha, void* dmask, int dmask_cs, float* taps,
                                      hipStream_t stream) {
  const long total = (long)B * h * w;
  hipLaunchKernelGGL(upsample_convex_bwd_kernel, dim3(nblk(total, 4)), dim3(256), 0, stream, (const bf16*)mask,
                     mask_cs, flow, gout, B, h, w, alpha, (bf16*)dmask, dmask_cs, taps);
  return (int)hipGetLastError();
}

extern "C" int jr_flow_gather_bwd(const float* taps, int tcs, int N, int h, int w, void* dflow, int dcs,
                                  hipStream_t stream) {
  if (tcs < 18 || (tcs & 1) || dcs < 2) return (int)hipErrorInvalidValue;
  const long M = (long)N * h * w;
  hipLaunchKernelGGL(flow_gather_bwd_kernel, dim3(nblk(M, 256)), dim3(256), 0, stream, taps, tcs, N, h, w,
                     (bf16*)dflow, dcs);
  return (int)hipGetLastError();
}

extern "C" int jr_upsample_bilinear_bwd(const float* gout, int B, int h, int w, void* dflow, int dcs,
                                        hipStream_t stream) {
  if (dcs < 2) return (int)hipErrorInvalidValue;
  const long M = (long)B * h * w;
  hipLaunchKernelGGL(upsample_bilinear_bwd_kernel, dim3(nblk(M, 256)), dim3(256), 0, stream, gout, B, h, w,
                     (bf16*)dflow, dcs);
  return (int)hipGetLastError();
}
