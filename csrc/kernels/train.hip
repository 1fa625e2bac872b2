// Training-only kernels of the fused refinement-loop backward (gfx950):
// the adjoints of the x8 flow upsampling (jax_raft/model.py:69-98) w.r.t. the
// mask logits and the low-res flow.  Both are deterministic gathers (no float
// atomics): the convex upsampling's flow gradient is split into per-neighbour
// partials (one wave per low-res pixel) and a shifted-partials sum, the same
// "taps" decomposition the forward flow head uses (flowhead.hip).
#include <algorithm>

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

// RAFT sequence loss (original RAFT recipe; the reference returns every
// iteration's prediction for it, model.py:510,605): one pass over the N
// predictions.  Per block, partial sums of |pred_i - gt| over the valid pixels
// (valid = (|gt| < max_flow) & (valid_in >= 0.5)) for every iteration, and on
// the final prediction the EPE sum, the <1/<3/<5 px counts and the valid
// count: part[block][N + 5], reduced on the host side in fixed order.
constexpr int LOSS_MAX_N = 32;

JR_DEVICE bool loss_valid(const float* gt, const float* vin, long p, float max_flow) {
  const float2 g = *(const float2*)(gt + 2 * p);
  return sqrtf(g.x * g.x + g.y * g.y) < max_flow && (vin == nullptr || vin[p] >= 0.5f);
}

__global__ __launch_bounds__(256) void seq_loss_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                       const float* __restrict__ vin, long P, int N, float max_flow,
                                                       float* __restrict__ part) {
  __shared__ float red[LOSS_MAX_N + 5][8];
  float acc[LOSS_MAX_N + 5];
#pragma unroll
  for (int k = 0; k < LOSS_MAX_N + 5; ++k) acc[k] = 0.f;
  const long stride = (long)gridDim.x * 256;
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < P; p += stride) {
    // As the PyTorch oracle (train/loss.py:sequence_loss_reference): the L1 term
    // is valid * |d| over EVERY pixel, so a non-finite prediction (or gt) at an
    // invalid pixel still poisons the loss (0 * NaN = NaN) and reaches the
    // non-finite step guard; the metrics count valid pixels only.
    const bool ok = loss_valid(gt, vin, p, max_flow);
    const float vw = ok ? 1.f : 0.f;
    const float2 g = *(const float2*)(gt + 2 * p);
#pragma unroll
    for (int i = 0; i < LOSS_MAX_N; ++i) {
      if (i < N) {
        const float2 f = *(const float2*)(pred + 2 * ((long)i * P + p));
        acc[i] += vw * (fabsf(f.x - g.x) + fabsf(f.y - g.y));
        if (i == N - 1 && ok) {
          const float e = sqrtf((f.x - g.x) * (f.x - g.x) + (f.y - g.y) * (f.y - g.y));
          acc[LOSS_MAX_N] += e;
          acc[LOSS_MAX_N + 1] += e < 1.f ? 1.f : 0.f;
          acc[LOSS_MAX_N + 2] += e < 3.f ? 1.f : 0.f;
          acc[LOSS_MAX_N + 3] += e < 5.f ? 1.f : 0.f;
          acc[LOSS_MAX_N + 4] += 1.f;
        }
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < LOSS_MAX_N + 5; ++k) {
    float v = acc[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[k][wave] = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < LOSS_MAX_N + 5; k += 256)
    part[(long)blockIdx.x * (LOSS_MAX_N + 5) + k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
}

// grad[i][p] = scale_i * valid(p) * sign(pred_i(p) - gt(p))   (scale_i = g_out * gamma^(N-1-i) / (2P))
__global__ __launch_bounds__(256) void seq_loss_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                           const float* __restrict__ vin, long P, int N,
                                                           float max_flow, const float* __restrict__ scale,
                                                           float* __restrict__ grad) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const bool v = loss_valid(gt, vin, p, max_flow);
  const float2 g = *(const float2*)(gt + 2 * p);
  for (int i = 0; i < N; ++i) {
    const long o = 2 * ((long)i * P + p);
    const float2 f = *(const float2*)(pred + o);
    const float s = v ? scale[i] : 0.f;
    // s * sign(d) with torch's sign(NaN) = 0 (the oracle's abs backward gives 0 there;
    // the NaN reaches the step guard through the loss value, seq_loss_kernel)
    const float dx = f.x > g.x ? s : (f.x < g.x ? -s : 0.f);
    const float dy = f.y > g.y ? s : (f.y < g.y ? -s : 0.f);
    *(float2*)(grad + o) = make_float2(dx, dy);
  }
}

// ---------------------------------------------------------------------------
// Normalisation backward of the encoders' "conv -> norm -> (relu) [+ residual]"
// units (InstanceNorm model.py:706-707, BatchNorm :147,157 in train mode, or
// identity), given the forward's raw conv output y and its per-(n, c)
// (sum, sumsq) statistics (elementwise.hip:jr_channel_stats):
//   g   = gout * [om > 0] * [relu: z > 0],  z = gamma * xhat + beta
//   dy  = rstd * gamma * (g - mean(g) - xhat * mean(g * xhat))     (means over the norm set)
//   gres = gout * [om > 0]                                          (residual-branch gradient)
// mode 0 (no norm): dy = g.  Reductions are deterministic two-pass (no atomics).
// ---------------------------------------------------------------------------
constexpr int NB_ROWS = 1024;

struct NormCo {
  float mean[8], rstd[8], gam[8], bet[8];
};

// (mean, rstd) of channel c of sample n: mode 1 over the map, mode 2 over the batch and map,
// mode 0 (no norm) identity
JR_DEVICE void norm_stat(const float* st, int mode, int n, int N, int HW, int C, int c, float eps, float& m,
                         float& r) {
  m = 0.f;
  r = 1.f;
  if (mode == 1) {
    const float inv = 1.0f / (float)HW;
    m = st[((long)n * C + c) * 2] * inv;
    r = rsqrtf(fmaxf(st[((long)n * C + c) * 2 + 1] * inv - m * m, 0.f) + eps);
  } else if (mode == 2) {
    float s0 = 0.f, s1 = 0.f;
    for (int k = 0; k < N; ++k) { s0 += st[((long)k * C + c) * 2]; s1 += st[((long)k * C + c) * 2 + 1]; }
    const float inv = 1.0f / ((float)HW * (float)N);
    m = s0 * inv;
    r = rsqrtf(fmaxf(s1 * inv - m * m, 0.f) + eps);
  }
}

// Per-channel coefficients are computed ONCE per block, one channel per thread, into LDS
// (cof[k * C + c], k = mean, rstd, gamma, beta[, a, m1, m2]) and read back 8 channels at a time:
// each of the block's 256 / (C / 8) row groups evaluating them itself cost 48 scalar loads per
// thread (2 N + ... for BatchNorm, whose statistics sum over the batch), and at ~2000 blocks
// that load-instruction stream, not the bytes, bounded the small maps and the BatchNorm
// backward (dev/probes/norm_bwd_bench.py: 2.1-2.6 TB/s vs 4.5-5.2 on the large IN maps).
JR_DEVICE void norm_co_lds(float* cof, const float* st, int mode, const float* gam, const float* bet, int n, int N,
                           int HW, int C, float eps) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float m, r;
    norm_stat(st, mode, n, N, HW, C, c, eps, m, r);
    cof[c] = m;
    cof[C + c] = r;
    cof[2 * C + c] = gam ? gam[c] : 1.f;
    cof[3 * C + c] = bet ? bet[c] : 0.f;
  }
}

JR_DEVICE void norm_co(NormCo& o, const float* cof, int C, int c0) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o.mean[j] = cof[c0 + j];
    o.rstd[j] = cof[C + c0 + j];
    o.gam[j] = cof[2 * C + c0 + j];
    o.bet[j] = cof[3 * C + c0 + j];
  }
}

// raw operands of 8 channels of one row, and g / xhat from them
struct NormRow {
  bf16x8 g, o, y;
};

JR_DEVICE void norm_load(NormRow& r, const bf16* gp, const bf16* op, const bf16* yp) {
  r.g = *(const bf16x8*)gp;
  r.y = *(const bf16x8*)yp;
  if (op) r.o = *(const bf16x8*)op;
}

JR_DEVICE void norm_eval(const NormCo& co, const NormRow& r, bool has_o, int relu, float (&g)[8], float (&xh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    xh[j] = (bf2f(r.y[j]) - co.mean[j]) * co.rstd[j];
    float v = bf2f(r.g[j]);
    if (has_o && !(bf2f(r.o[j]) > 0.f)) v = 0.f;
    if ((relu & 1) && !(co.gam[j] * xh[j] + co.bet[j] > 0.f)) v = 0.f;
    g[j] = v;
  }
}

// rows per thread whose loads are issued together: the row loop is a 3-stream copy, and one row
// (48 B per thread) in flight per iteration ran both kernels at about a third of HBM bandwidth
// (profiles/r5_train_breakdown.txt: 1.34 + 0.74 ms per step for ~0.65 ms of bytes)
constexpr int NORM_U = 4;

__global__ __launch_bounds__(256) void norm_bwd_partial_kernel(const bf16* __restrict__ gout, const bf16* __restrict__ om,
                                                               const bf16* __restrict__ y, const float* __restrict__ st,
                                                               int mode, const float* __restrict__ gam,
                                                               const float* __restrict__ bet, int relu, int N, int HW,
                                                               int C, float eps, float* __restrict__ part, int rows) {
  __shared__ float red[256][17];
  extern __shared__ float cof[];   // [4][C]
  const int n = blockIdx.y;
  const int cg = C >> 3;
  const int tid = threadIdx.x;
  const int g8 = tid % cg, rg = tid / cg, nrg = 256 / cg;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(r0 + rows, HW);
  norm_co_lds(cof, st, mode, gam, bet, n, N, HW, C, eps);
  __syncthreads();
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (rg < nrg) {
    NormCo co;
    norm_co(co, cof, C, g8 * 8);
    const long base = (long)n * HW * C + g8 * 8;
    for (int r = r0 + rg; r < r1; r += NORM_U * nrg) {
      NormRow v[NORM_U];
#pragma unroll
      for (int u = 0; u < NORM_U; ++u) {   // all loads first (clamped rows; only valid ones count)
        const long off = base + (long)min(r + u * nrg, r1 - 1) * C;
        norm_load(v[u], gout + off, om ? om + off : nullptr, y + off);
      }
#pragma unroll
      for (int u = 0; u < NORM_U; ++u) {
        if (r + u * nrg >= r1) break;
        float g[8], xh[8];
        norm_eval(co, v[u], om != nullptr, relu, g, xh);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += g[j]; q[j] += g[j] * xh[j]; }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[tid][j] = s[j]; red[tid][8 + j] = q[j]; }
  __syncthreads();
  const int nb = gridDim.x;
  for (int t = tid; t < cg * 16; t += 256) {
    const int gg = t % cg, vi = t / cg;
    float acc = 0.f;
    for (int k = 0; k < nrg; ++k) acc += red[k * cg + gg][vi];
    const int c = gg * 8 + (vi & 7);
    part[(((long)n * nb + blockIdx.x) * C + c) * 2 + (vi >> 3)] = acc;
  }
}

__global__ __launch_bounds__(256) void norm_bwd_final_kernel(const float* __restrict__ part, int nb, int C,
                                                             float* __restrict__ red) {
  // block = 8 values (lane v) x 32 partial groups (g): thread (v, g) sums partials g, g + 32, ... with
  // 8 loads in flight per round trip (the loop is latency-bound: a few MB of partials), then the 32
  // groups combine in a fixed order (deterministic)
  __shared__ float red_[32][9];
  const int n = blockIdx.y;
  const int v = threadIdx.x & 7, g = threadIdx.x >> 3;
  const int vi = blockIdx.x * 8 + v;
  const int nv = 2 * C;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (vi < nv) {
    const float* p = part + (long)n * nb * nv + vi;
    for (int b = g; b < nb; b += 32 * 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int bb = b + 32 * u;
        t[u] = bb < nb ? p[(long)bb * nv] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u & 3] += t[u];
    }
  }
  red_[g][v] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (g == 0 && vi < nv) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) t += red_[k][v];
    red[(long)n * nv + vi] = t;
  }
}

__global__ __launch_bounds__(256) void norm_bwd_apply_kernel(const bf16* __restrict__ gout, const bf16* __restrict__ om,
                                                             const bf16* __restrict__ y, const float* __restrict__ st,
                                                             int mode, const float* __restrict__ gam,
                                                             const float* __restrict__ bet, int relu,
                                                             const float* __restrict__ red, int N, int HW, int C,
                                                             float eps, bf16* __restrict__ dy, void* __restrict__ gres,
                                                             int gres_bf16,
                                                             int rows) {
  extern __shared__ float cof[];   // [7][C]: mean, rstd, gamma, beta, a, m1, m2
  const int n = blockIdx.y;
  const int cg = C >> 3;
  const int tid = threadIdx.x;
  const int g8 = tid % cg, rg = tid / cg, nrg = 256 / cg;
  norm_co_lds(cof, st, mode, gam, bet, n, N, HW, C, eps);
  for (int c = tid; c < C; c += blockDim.x) {
    float S1 = 0.f, S2 = 0.f, cnt = (float)HW;
    if (mode == 1) {
      S1 = red[((long)n * C + c) * 2];
      S2 = red[((long)n * C + c) * 2 + 1];
    } else if (mode == 2) {
      for (int k = 0; k < N; ++k) { S1 += red[((long)k * C + c) * 2]; S2 += red[((long)k * C + c) * 2 + 1]; }
      cnt *= (float)N;
    }
    cof[4 * C + c] = cof[C + c] * cof[2 * C + c];
    cof[5 * C + c] = S1 / cnt;
    cof[6 * C + c] = S2 / cnt;
  }
  __syncthreads();
  if (rg >= nrg) return;
  const int c0 = g8 * 8;
  NormCo co;
  norm_co(co, cof, C, c0);
  float a[8], m1[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = cof[4 * C + c0 + j];
    m1[j] = cof[5 * C + c0 + j];
    m2[j] = cof[6 * C + c0 + j];
  }
  const long base = (long)n * HW * C + c0;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(r0 + rows, HW);
  for (int row0 = r0 + rg; row0 < r1; row0 += NORM_U * nrg) {
    NormRow v[NORM_U];
#pragma unroll
    for (int u = 0; u < NORM_U; ++u) {   // all loads first (clamped rows; only valid ones are stored)
      const long off = base + (long)min(row0 + u * nrg, r1 - 1) * C;
      norm_load(v[u], gout + off, om ? om + off : nullptr, y + off);
    }
#pragma unroll
    for (int u = 0; u < NORM_U; ++u) {
      const int row = row0 + u * nrg;
      if (row >= r1) break;
      const long off = base + (long)row * C;
      float g[8], xh[8];
      norm_eval(co, v[u], om != nullptr, relu, g, xh);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(mode == 0 ? g[j] : a[j] * (g[j] - m1[j] - xh[j] * m2[j]));
      *(bf16x8*)(dy + off) = o;
      if (gres) {
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = (om && !(bf2f(v[u].o[j]) > 0.f)) ? 0.f : bf2f(v[u].g[j]);
        if (gres_bf16) {   // exact: a masked bf16 gradient
          bf16x8 rb;
#pragma unroll
          for (int j = 0; j < 8; ++j) rb[j] = f2bf(r[j]);
          *(bf16x8*)((bf16*)gres + off) = rb;
        } else {
          *(f32x4*)((float*)gres + off) = f32x4{r[0], r[1], r[2], r[3]};
          *(f32x4*)((float*)gres + off + 4) = f32x4{r[4], r[5], r[6], r[7]};
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight packing for training: every step the optimizer changes the fp32 HWIO
// parameters, and every conv of the fused training plans needs its bf16 GEMM
// A operand ([cout_pad][kpad], K = (tap, cin8), rows permuted in 64-row groups,
// ops/native.py:pack_weight) -- forward, flipped / transposed data-gradient
// and flow-head tap layouts.  One launch repacks all of them from a table of
// rectangular pieces (blockIdx.y = piece), as the first op of the captured
// forward plan (no per-parameter framework ops).
// ---------------------------------------------------------------------------
JR_DEVICE long packed_row(long co) {   // storage row of output channel co (inverse of _row_perm)
  const long g = co >> 6, j = co & 63;
  return g * 64 + ((j & 15) >> 2) * 16 + (j >> 4) * 4 + (j & 3);
}

__global__ __launch_bounds__(256) void pack_pieces_kernel(const PackPiece* __restrict__ pieces) {
  const PackPiece pc = pieces[blockIdx.y];
  const float* src = (const float*)pc.src;
  const long nco = pc.co1 - pc.co0, nci = pc.ci1 - pc.ci0;
  const long taps = pc.mode == 3 ? 1 : pc.kh * pc.kw;
  const long total = nco * taps * (pc.mode == 3 ? 1 : nci);
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    if (pc.mode == 3) {  // bias: fp32 dst[co] = src[co - co0 + so_co]
      ((float*)pc.dst)[pc.co0 + e] = src[e + pc.so_co];
      continue;
    }
    const long ci = pc.ci0 + e % nci;
    const long r = e / nci;
    const long tap = r % taps;
    const long co = pc.co0 + r / taps;
    const long sco = co - pc.co0 + pc.so_co, sci = ci - pc.ci0 + pc.so_ci;
    float v;
    if (pc.mode == 0 || pc.mode == 4) {          // forward: W[tap][ci][co]
      v = src[(tap * pc.cin_s + sci) * pc.cout_s + sco];
    } else if (pc.mode == 1 || pc.mode == 5) {   // data gradient: W[flipped tap][src in = co][src out = ci]
      const long th = tap / pc.kw, tw = tap % pc.kw;
      const long ft = (pc.kh - 1 - th) * pc.kw + (pc.kw - 1 - tw);
      v = src[(ft * pc.cin_s + sco) * pc.cout_s + sci];
    } else {                     // flow-head taps: dst (1,1,cin,18), co = 2 * src tap + c
      v = src[((co >> 1) * pc.cin_s + sci) * pc.cout_s + (co & 1)];
    }
    if (pc.mode >= 4) {
      // halo weight stream (conv_halo.hip, ops/native.py:pack_gru_halo): fragment (co / 32,
      // k / 16), lane 32 ((k >> 3) & 1) + r with _m32_chan(r) = co % 32, element k & 7
      const long k = tap * pc.cin8 + ci, c = co & 31;
      const long r = ((c >> 2) & 3) * 8 + ((c >> 4) & 1) * 4 + (c & 3);
      const long ks = taps * pc.cin8 / 16;
      ((bf16*)pc.dst)[(((co >> 5) * ks + (k >> 4)) * 64 + ((k >> 3) & 1) * 32 + r) * 8 + (k & 7)] = f2bf(v);
    } else {
      ((bf16*)pc.dst)[packed_row(co) * pc.kpad + tap * pc.cin8 + ci] = f2bf(v);
    }
  }
}

// Correlation-pyramid backward, first half (jax_raft/model.py:443-445,472-481):
// the 2x2 floor average-pooling adjoints of every level summed into the
// full-resolution volume gradient, scaled by the 1/sqrt(C) of the volume and
// stored bf16 for the two GEMMs dfmap1 = dC fmap2, dfmap2 = dC^T fmap1.
//   dC[q][y][x] = s * sum_l g_l[q][y >> l][x >> l] / 4^l   (y < h_l 2^l, x < w_l 2^l)
__global__ __launch_bounds__(256) void pyr_bwd_dc_kernel(const float* __restrict__ g0, const float* __restrict__ g1,
                                                         const float* __restrict__ g2, const float* __restrict__ g3,
                                                         int L, long M, int h, int w, float scale,
                                                         bf16* __restrict__ dc) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long hw = (long)h * w;
  if (e >= M * hw) return;
  const long q = e / hw;
  const int r = (int)(e - q * hw);
  const int y = r / w, x = r - (r / w) * w;
  float v = g0[e];
  const float* gl[3] = {g1, g2, g3};
  int hl = h, wl = w;
#pragma unroll
  for (int l = 1; l < 4; ++l) {
    hl >>= 1;
    wl >>= 1;
    if (l < L) {
      const int yy = y >> l, xx = x >> l;
      if (yy < hl && xx < wl) v += gl[l - 1][(q * hl + yy) * wl + xx] * (1.0f / (float)(1 << (2 * l)));
    }
  }
  dc[e] = f2bf(v * scale);
}

// Same, 8 consecutive x per thread (w % 8 == 0): two 16-B g0 loads, one 16-B dC store
// (the scalar form moved 2-byte stores: 235 us for the 113 MB volume of config 5).
__global__ __launch_bounds__(256) void pyr_bwd_dc8_kernel(const float* __restrict__ g0, const float* __restrict__ g1,
                                                          const float* __restrict__ g2, const float* __restrict__ g3,
                                                          int L, long M, int h, int w, float scale,
                                                          bf16* __restrict__ dc) {
  const long e8 = (long)blockIdx.x * 256 + threadIdx.x;
  const long hw = (long)h * w;
  if (e8 * 8 >= M * hw) return;
  const long e = e8 * 8;
  const long q = e / hw;
  const int r = (int)(e - q * hw);
  const int y = r / w, x0 = r - (r / w) * w;
  const f32x4 a = *(const f32x4*)(g0 + e);
  const f32x4 b = *(const f32x4*)(g0 + e + 4);
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  const float* gl[3] = {g1, g2, g3};
  int hl = h, wl = w;
#pragma unroll
  for (int l = 1; l < 4; ++l) {
    hl >>= 1;
    wl >>= 1;
    if (l < L) {
      const int yy = y >> l;
      if (yy < hl) {
        const float* row = gl[l - 1] + (q * hl + yy) * wl;
        const float s = 1.0f / (float)(1 << (2 * l));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int xx = (x0 + j) >> l;
          if (xx < wl) v[j] += row[xx] * s;
        }
      }
    }
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] * scale);
  *(bf16x8*)(dc + e) = o;
}

// BatchNorm bookkeeping of the encoder training plans, one launch for all layers
// (blockIdx.y = layer): forward (mode 0) the Flax running statistics
// (model.py:147, momentum m: ra = m ra + (1 - m) batch, biased batch variance)
// from the per-(n, c) (sum, sumsq) of the layer's conv output; backward (mode 1)
// the scale / bias gradients (sum over n of the norm backward's (sum g xhat, sum g)).
__global__ __launch_bounds__(256) void bn_table_kernel(const BnRow* __restrict__ rows) {
  const BnRow r = rows[blockIdx.y];
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= r.C) return;
  const float* st = (const float*)r.src;
  float s0 = 0.f, s1 = 0.f;
  for (int n = 0; n < r.N; ++n) {
    s0 += st[((long)n * r.C + c) * 2];
    s1 += st[((long)n * r.C + c) * 2 + 1];
  }
  float* a = (float*)r.dst0;
  float* b = (float*)r.dst1;
  if (r.mode == 0) {
    const float mom = __builtin_bit_cast(float, (int)r.momentum_bits);
    const float cnt = (float)r.count;
    const float m = s0 / cnt;
    const float v = fmaxf(s1 / cnt - m * m, 0.f);
    a[c] = mom * a[c] + (1.f - mom) * m;
    b[c] = mom * b[c] + (1.f - mom) * v;
  } else {
    a[c] = s1;   // d scale = sum g xhat
    b[c] = s0;   // d bias  = sum g
  }
}

// Same, 32-bit indexing and vector level reads (w % 8 == 0, M * h * w / 8 < 2^31): the 8 outputs
// of a thread read 4 / 2 / 1 consecutive cells of levels 1 / 2 / 3 (one 16-B, 8-B, 4-B load each)
// instead of 24 scalar gathers, and no 64-bit divisions (config 5: 356 us at 1.2 TB/s before).
__global__ __launch_bounds__(256) void pyr_bwd_dc8v_kernel(const float* __restrict__ g0, const float* __restrict__ g1,
                                                           const float* __restrict__ g2, const float* __restrict__ g3,
                                                           int L, unsigned n8, unsigned hw8, int h, int w, float scale,
                                                           bf16* __restrict__ dc) {
  const unsigned e8 = blockIdx.x * 256u + threadIdx.x;
  if (e8 >= n8) return;
  const unsigned q = e8 / hw8;
  const unsigned r8 = e8 - q * hw8;
  const unsigned w8 = (unsigned)w >> 3;
  const int y = (int)(r8 / w8);
  const int x0 = (int)(r8 - (unsigned)y * w8) * 8;
  const long e = (long)e8 * 8;
  const f32x4 a = *(const f32x4*)(g0 + e);
  const f32x4 b = *(const f32x4*)(g0 + e + 4);
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  if (L > 1) {
    const int hl = h >> 1, wl = w >> 1, yy = y >> 1;
    if (yy < hl) {
      const f32x4 t = *(const f32x4*)(g1 + ((long)q * hl + yy) * wl + (x0 >> 1));
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j >> 1] * 0.25f;
    }
  }
  if (L > 2) {
    const int hl = h >> 2, wl = w >> 2, yy = y >> 2;
    if (yy < hl) {
      const float2 t = *(const float2*)(g2 + ((long)q * hl + yy) * wl + (x0 >> 2));
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (j < 4 ? t.x : t.y) * 0.0625f;
    }
  }
  if (L > 3) {
    const int hl = h >> 3, wl = w >> 3, yy = y >> 3;
    if (yy < hl) {
      const float t = g3[((long)q * hl + yy) * wl + (x0 >> 3)];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t * 0.015625f;
    }
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] * scale);
  *(bf16x8*)(dc + e) = o;
}

inline unsigned nblk(long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

}  // namespace

extern "C" int jr_bn_table(const void* rows, int n, int max_c, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(bn_table_kernel, dim3((unsigned)((max_c + 255) / 256), (unsigned)n), dim3(256), 0, stream,
                     (const BnRow*)rows);
  return (int)hipGetLastError();
}

extern "C" int jr_pyr_bwd_dc(const float* g0, const float* g1, const float* g2, const float* g3, int L, long M, int h,
                             int w, float scale, void* dc, hipStream_t stream) {
  if (L < 1 || L > 4) return (int)hipErrorInvalidValue;
  if (w % 8 == 0 && M * h * w / 8 < (1L << 31)) {
    const long n8 = M * h * w / 8;
    hipLaunchKernelGGL(pyr_bwd_dc8v_kernel, dim3(nblk(n8, 256)), dim3(256), 0, stream, g0, g1, g2, g3, L,
                       (unsigned)n8, (unsigned)((long)h * w / 8), h, w, scale, (bf16*)dc);
    return (int)hipGetLastError();
  }
  if (w % 8 == 0) {
    hipLaunchKernelGGL(pyr_bwd_dc8_kernel, dim3(nblk(M * h * w / 8, 256)), dim3(256), 0, stream, g0, g1, g2, g3, L, M,
                       h, w, scale, (bf16*)dc);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(pyr_bwd_dc_kernel, dim3(nblk(M * h * w, 256)), dim3(256), 0, stream, g0, g1, g2, g3, L, M, h, w,
                     scale, (bf16*)dc);
  return (int)hipGetLastError();
}

extern "C" int jr_pack_pieces(const void* table, int n, long max_elems, hipStream_t stream) {
  if (n <= 0) return 0;
  const unsigned bx = (unsigned)std::min<long>(256, std::max<long>(1, (max_elems + 255) / 256));
  hipLaunchKernelGGL(pack_pieces_kernel, dim3(bx, n), dim3(256), 0, stream, (const PackPiece*)table);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Iteration sums of the ConvGRU gate gradients (the loop-invariant context share of the gates,
// train/fused.py:_finish_data): out[m][c] = sum_t a[t][m][c] (c < Ca), then b (c >= Ca), bf16 in,
// fp32 sums, one bf16 rounding -- one pass instead of two strided framework reductions + cat + cast.
// Thread = 8 channels of one pixel (16-B loads), T loads in flight.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sum_iters_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, int T,
                                                        long M, int Ca, int Cb, bf16* __restrict__ out) {
  const int cg = (Ca + Cb) >> 3;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * cg) return;
  const long m = idx / cg;
  const int c = (int)(idx - m * cg) * 8;
  const bool fa = c < Ca;
  const bf16* src = fa ? a + m * Ca + c : b + m * Cb + (c - Ca);
  const long tstride = fa ? M * Ca : M * Cb;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int t = 0; t < T; ++t) {
    const bf16x8 v = *(const bf16x8*)(src + (long)t * tstride);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
  *(bf16x8*)(out + m * (Ca + Cb) + c) = o;
}

extern "C" int jr_sum_iters(const void* a, const void* b, int T, long M, int Ca, int Cb, void* out, hipStream_t stream) {
  if (Ca % 8 || Cb % 8 || T < 1) return (int)hipErrorInvalidValue;
  const long n = M * ((Ca + Cb) / 8);
  hipLaunchKernelGGL(sum_iters_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const bf16*)a,
                     (const bf16*)b, T, M, Ca, Cb, (bf16*)out);
  return (int)hipGetLastError();
}

// rows per partial-reduction block: enough blocks (>= ~1024 over the batch) that the small deep-layer
// maps are not latency-bound on a few dozen blocks, at most NB_ROWS, a multiple of the row groups
static int norm_bwd_rows(int N, int HW, int C) {
  const int nrg = 256 / (C / 8);
  const int nb = std::max(1, (1024 + N - 1) / N);
  const int r = (HW + nb - 1) / nb;
  return std::min(NB_ROWS, std::max(nrg, (r + nrg - 1) / nrg * nrg));
}

extern "C" int jr_norm_bwd_partials(int N, int HW, int C) {
  return N * ((HW + norm_bwd_rows(N, HW, C) - 1) / norm_bwd_rows(N, HW, C));
}

extern "C" int jr_norm_bwd(const void* gout, const void* om, const void* y, const float* stats, int mode,
                           const float* gamma, const float* beta, int relu, int N, int HW, int C, float eps,
                           float* red, float* partial, void* dy, void* gres, int gres_bf16, hipStream_t stream) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  if (mode != 0) {
    const int prow = norm_bwd_rows(N, HW, C);
    const int nb = (HW + prow - 1) / prow;
    hipLaunchKernelGGL(norm_bwd_partial_kernel, dim3(nb, N), dim3(256), 4 * C * sizeof(float), stream, (const bf16*)gout,
                       (const bf16*)om, (const bf16*)y, stats, mode, gamma, beta, relu, N, HW, C, eps, partial, prow);
    hipLaunchKernelGGL(norm_bwd_final_kernel, dim3((2 * C + 7) / 8, N), dim3(256), 0, stream, partial, nb, C, red);
  }
  const int nrg = 256 / (C / 8);
  const long want = ((long)N * HW + 2047) / 2048;
  const int rows = (int)std::max<long>(nrg, (want + nrg - 1) / nrg * nrg);
  const unsigned nbk = (unsigned)((HW + rows - 1) / rows);
  hipLaunchKernelGGL(norm_bwd_apply_kernel, dim3(nbk, N), dim3(256), 7 * C * sizeof(float), stream, (const bf16*)gout, (const bf16*)om,
                     (const bf16*)y, stats, mode, gamma, beta, relu, red, N, HW, C, eps, (bf16*)dy, gres, gres_bf16, rows);
  return (int)hipGetLastError();
}

extern "C" int jr_seq_loss_blocks(long P) { return (int)std::min<long>(1024, (P + 255) / 256); }

extern "C" int jr_seq_loss(const float* pred, const float* gt, const float* valid, long P, int N, float max_flow,
                           float* part, hipStream_t stream) {
  if (N < 1 || N > LOSS_MAX_N) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(seq_loss_kernel, dim3(jr_seq_loss_blocks(P)), dim3(256), 0, stream, pred, gt, valid, P, N,
                     max_flow, part);
  return (int)hipGetLastError();
}

extern "C" int jr_seq_loss_bwd(const float* pred, const float* gt, const float* valid, long P, int N, float max_flow,
                               const float* scale, float* grad, hipStream_t stream) {
  hipLaunchKernelGGL(seq_loss_bwd_kernel, dim3(nblk(P, 256)), dim3(256), 0, stream, pred, gt, valid, P, N, max_flow,
                     scale, grad);
  return (int)hipGetLastError();
}

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
