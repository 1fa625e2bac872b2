// Memory-bound kernels of the fp32 parity mode (engine precision="fp32"):
// instance-norm statistics / application, input staging, channel copies,
// correlation pyramid pooling and lookup, the coordinate update and the convex
// upsampling, all on fp32 tensors.  The convs (and the level-0 correlation
// GEMM) run on conv_f32.hip.
//
// Reference semantics:
//   InstanceNorm (Flax, fast variance)      jax_raft/model.py:147,157
//   avg_pool 2x2 of the correlation volume  jax_raft/model.py:433-441
//   index_pyramid / grid_sample             jax_raft/model.py:448-470, :14-35
//   coords1 + delta, flow = coords1 - coords0   model.py:505-506
//   upsample_flow (convex)                  jax_raft/model.py:69-84
#include "common.h"
#include "kernels.h"

namespace {

inline unsigned nblk(long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

// ------------------------------------------------------------- statistics
// Deterministic two-pass (sum, sumsq): pass 1 = fixed row ranges per block,
// C/4 threads per row (one float4 each), the row lanes reduced in order through
// LDS; pass 2 sums the per-block partials in order.
constexpr int STATS_ROWS = 1024;

__global__ __launch_bounds__(256) void stats_partial_f32(const float* __restrict__ x, int HW, int C,
                                                         float* __restrict__ part) {
  __shared__ float red[256][9];
  const int n = blockIdx.y, cg = C >> 2, tid = threadIdx.x;
  const int g = tid % cg, rg = tid / cg, nrg = 256 / cg;
  const int r0 = blockIdx.x * STATS_ROWS, r1 = min(r0 + STATS_ROWS, HW);
  float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  if (rg < nrg) {
    const float* base = x + (long)n * HW * C + g * 4;
    for (int r = r0 + rg; r < r1; r += nrg) {
      const float4 v = *(const float4*)(base + (long)r * C);
      const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] += f[j];
        q[j] = fmaf(f[j], f[j], q[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) { red[tid][j] = s[j]; red[tid][4 + j] = q[j]; }
  __syncthreads();
  const int nb = gridDim.x;
  for (int t = tid; t < cg * 8; t += 256) {
    const int gg = t % cg, vi = t / cg;
    float acc = 0.f;
    for (int k = 0; k < nrg; ++k) acc += red[k * cg + gg][vi];
    const int c = gg * 4 + (vi & 3);
    part[(((long)n * nb + blockIdx.x) * C + c) * 2 + (vi >> 2)] = acc;
  }
}

__global__ __launch_bounds__(256) void stats_final_f32(const float* __restrict__ part, int nb, int C,
                                                       float* __restrict__ stats) {
  const int n = blockIdx.y;
  const int vi = blockIdx.x * 256 + threadIdx.x;
  if (vi >= 2 * C) return;
  const float* p = part + (long)n * nb * 2 * C + vi;
  float acc = 0.f;
  for (int b = 0; b < nb; ++b) acc += p[(long)b * 2 * C];
  stats[(long)n * 2 * C + vi] = acc;
}

// y = act(xn + rn), xn / rn normalised with instance (mode 1) or batch (mode 2)
// statistics or raw (mode 0); relu bit 0 before the residual add, bit 1 after.
JR_DEVICE void coeffs4(float (&a)[4], float (&b)[4], const float* st, int mode, int n, int N, int HW, int C, int c0,
                       float eps) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + j;
    a[j] = 1.f;
    b[j] = 0.f;
    if (mode == 0) continue;
    float s0 = 0.f, s1 = 0.f;
    const int k0 = mode == 1 ? n : 0, k1 = mode == 1 ? n + 1 : N;
    for (int k = k0; k < k1; ++k) { s0 += st[((long)k * C + c) * 2]; s1 += st[((long)k * C + c) * 2 + 1]; }
    const float inv = 1.0f / ((float)HW * (float)(k1 - k0));
    const float m = s0 * inv;
    const float var = fmaxf(s1 * inv - m * m, 0.f);
    a[j] = 1.0f / sqrtf(var + eps);
    b[j] = -m * a[j];
  }
}

__global__ __launch_bounds__(256) void norm_act_f32(const float* __restrict__ x, const float* __restrict__ sx,
                                                    int mode_x, const float* __restrict__ r,
                                                    const float* __restrict__ sr, int mode_r, float* __restrict__ y,
                                                    int N, int HW, int C, float eps, int relu, int rows) {
  const int n = blockIdx.y, cg = C >> 2, tid = threadIdx.x;
  const int g = tid % cg, rg = tid / cg, nrg = 256 / cg;
  if (rg >= nrg) return;
  const int c0 = g * 4;
  float ax[4], bx[4], ar[4], br[4];
  coeffs4(ax, bx, sx, mode_x, n, N, HW, C, c0, eps);
  if (r) coeffs4(ar, br, sr, mode_r, n, N, HW, C, c0, eps);
  const long base = (long)n * HW * C + c0;
  const int r0 = blockIdx.x * rows, r1 = min(r0 + rows, HW);
  for (int row = r0 + rg; row < r1; row += nrg) {
    const long off = base + (long)row * C;
    const float4 v = *(const float4*)(x + off);
    float a[4] = {v.x, v.y, v.z, v.w};
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r) w = *(const float4*)(r + off);
    const float rv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = a[j] * ax[j] + bx[j];
      if (relu & 1) a[j] = fmaxf(a[j], 0.f);
      if (r) a[j] += rv[j] * ar[j] + br[j];
      if (relu & 2) a[j] = fmaxf(a[j], 0.f);
    }
    *(float4*)(y + off) = make_float4(a[0], a[1], a[2], a[3]);
  }
}

// ------------------------------------------------------------------ misc
__global__ void prep_f32(const float* __restrict__ i1, const float* __restrict__ i2, int B, long HW,
                         float* __restrict__ out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long half = (long)B * HW;
  if (idx >= 2 * half) return;
  const float* src = idx < half ? i1 + idx * 3 : i2 + (idx - half) * 3;
  *(float4*)(out + idx * 4) = make_float4(src[0], src[1], src[2], 0.f);
}

__global__ void copy_channels_f32(const float* __restrict__ src, int scs, int soff, float* __restrict__ dst, int dcs,
                                  int doff, int M, int C) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)M * C) return;
  const long m = idx / C;
  const int c = (int)(idx - m * C);
  dst[m * dcs + doff + c] = src[m * scs + soff + c];
}

// One wave per low-res pixel, lane = sub-pixel a*8 + b; mask channel k*64 + s
// (k = 3x3 neighbour), softmax over k, convex combination of 8 * flow.
__global__ __launch_bounds__(256) void upsample_convex_f32(const float* __restrict__ mask, int mcs,
                                                           const float* __restrict__ flow, int B, int h, int w,
                                                           float* __restrict__ out, const long long* __restrict__ slot,
                                                           long out_off) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int P = h * w;
  if (slot) out = (float*)(*slot) + out_off;
  if (p >= B * P) return;
  const int b = p / P, rem = p - b * P, y = rem / w, x = rem - y * w;
  const float* mp = mask + (long)p * mcs + lane;
  float lg[9], mx = -3.0e38f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lg[k] = mp[k * 64];
    mx = fmaxf(mx, lg[k]);
  }
  float s = 0.f, ux = 0.f, uy = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    const float e = expf(lg[k] - mx);
    s += e;
    if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) {
      const float* fp = flow + 2 * ((long)b * P + yy * w + xx);
      ux += e * (8.0f * fp[0]);
      uy += e * (8.0f * fp[1]);
    }
  }
  const int a = lane >> 3, bb = lane & 7;
  float* op = out + 2 * (((long)b * 8 * h + 8 * y + a) * (8L * w) + 8 * x + bb);
  *(float2*)op = make_float2(ux / s, uy / s);
}

// ------------------------------------------------------------ correlation
__global__ void corr_pool_f32(const float* __restrict__ src, long M, int hl, int wl, float* __restrict__ dst) {
  const int ho = hl >> 1, wo = wl >> 1;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)ho * wo;
  if (idx >= M * per) return;
  const long q = idx / per;
  const int rem = (int)(idx - q * per), y = rem / wo, x = rem - y * wo;
  const float* s = src + q * hl * wl + (2 * y) * wl + 2 * x;
  dst[idx] = ((s[0] + s[1]) + (s[wl] + s[wl + 1])) * 0.25f;
}

struct Lv4 {
  const float* p[4];
};

// Thread = (query, level, window column i): bilinear samples of column i at
// the S window rows (vertical interpolation first, then horizontal -- the
// order of corr.hip's lookups), zero outside the map.
template <int R>
__global__ __launch_bounds__(256) void lookup_f32(Lv4 lv, int L, long total, int h, int w,
                                                  const float* __restrict__ coords, float* __restrict__ out, int ocs) {
  constexpr int S = 2 * R + 1;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total * L * S) return;
  const long q = idx / (L * S);
  const int rem = (int)(idx - q * (L * S)), l = rem / S, i = rem - l * S;
  const int hl = h >> l, wl = w >> l;
  const float sc = 1.0f / (float)(1 << l);
  const float cx = coords[2 * q] * sc, cy = coords[2 * q + 1] * sc;
  const float flx = floorf(cx), fly = floorf(cy);
  const float fx = cx - flx, fy = cy - fly;
  const int c0 = (int)flx - R + i, r0 = (int)fly - R;
  const float* map = lv.p[l] + q * hl * wl;
  const bool ok0 = (unsigned)c0 < (unsigned)wl, ok1 = (unsigned)(c0 + 1) < (unsigned)wl;
  float a[S + 1], b[S + 1];
#pragma unroll
  for (int j = 0; j <= S; ++j) {
    const int rr = r0 + j;
    const bool rok = (unsigned)rr < (unsigned)hl;
    a[j] = rok && ok0 ? map[rr * wl + c0] : 0.f;
    b[j] = rok && ok1 ? map[rr * wl + c0 + 1] : 0.f;
  }
  float* o = out + q * ocs + l * S * S + i * S;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const float va = (1.f - fy) * a[j] + fy * a[j + 1];
    const float vb = (1.f - fy) * b[j] + fy * b[j + 1];
    o[j] = (1.f - fx) * va + fx * vb;
  }
}

__global__ void flow_update_f32(const float* __restrict__ d, int dcs, long M, int h, int w,
                                float* __restrict__ coords, float* __restrict__ flow32, float* __restrict__ hx,
                                int hx_cs, int hx_off, float* __restrict__ qx, int qx_cs, int qx_off,
                                float* __restrict__ f4) {
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const int rem = (int)(m % ((long)h * w)), y = rem / w, x = rem - y * w;
  const float cx = coords[2 * m] + d[m * dcs], cy = coords[2 * m + 1] + d[m * dcs + 1];
  coords[2 * m] = cx;
  coords[2 * m + 1] = cy;
  const float fx = cx - (float)x, fy = cy - (float)y;
  flow32[2 * m] = fx;
  flow32[2 * m + 1] = fy;
  hx[m * hx_cs + hx_off] = fx;
  hx[m * hx_cs + hx_off + 1] = fy;
  if (qx) {
    qx[m * qx_cs + qx_off] = fx;
    qx[m * qx_cs + qx_off + 1] = fy;
  }
  if (f4) *(float4*)(f4 + 4 * m) = make_float4(fx, fy, 0.f, 0.f);
}

}  // namespace

extern "C" int jr_channel_stats_f32(const float* x, int N, int HW, int C, float* stats, float* partial,
                                    hipStream_t stream) {
  if (C % 4 != 0 || C / 4 > 256) return (int)hipErrorInvalidValue;
  const int nb = (HW + STATS_ROWS - 1) / STATS_ROWS;
  hipLaunchKernelGGL(stats_partial_f32, dim3(nb, N), dim3(256), 0, stream, x, HW, C, partial);
  hipLaunchKernelGGL(stats_final_f32, dim3((2 * C + 255) / 256, N), dim3(256), 0, stream, partial, nb, C, stats);
  return (int)hipGetLastError();
}

extern "C" int jr_norm_act_f32(const float* x, const float* sx, int mode_x, const float* res, const float* sr,
                               int mode_r, float* y, int N, int HW, int C, float eps, int relu, hipStream_t stream) {
  if (C % 4 != 0 || C / 4 > 256) return (int)hipErrorInvalidValue;
  const int nrg = 256 / (C / 4);
  const long want = ((long)N * HW + 2047) / 2048;
  const int rows = (int)std::max<long>(nrg, (want + nrg - 1) / nrg * nrg);
  hipLaunchKernelGGL(norm_act_f32, dim3((unsigned)((HW + rows - 1) / rows), N), dim3(256), 0, stream, x, sx, mode_x,
                     res, sr, mode_r, y, N, HW, C, eps, relu, rows);
  return (int)hipGetLastError();
}

extern "C" int jr_prep_images_f32(const float* img1, const float* img2, int B, int H, int W, float* out,
                                  hipStream_t stream) {
  hipLaunchKernelGGL(prep_f32, dim3(nblk(2L * B * H * W, 256)), dim3(256), 0, stream, img1, img2, B, (long)H * W, out);
  return (int)hipGetLastError();
}

extern "C" int jr_copy_channels_f32(const float* src, int s_cstride, int s_coff, float* dst, int d_cstride, int d_coff,
                                    int M, int C, hipStream_t stream) {
  hipLaunchKernelGGL(copy_channels_f32, dim3(nblk((long)M * C, 256)), dim3(256), 0, stream, src, s_cstride, s_coff, dst,
                     d_cstride, d_coff, M, C);
  return (int)hipGetLastError();
}

extern "C" int jr_upsample_convex_f32(const float* mask, int mask_cstride, const float* flow, int B, int h, int w,
                                      float* out, const void* out_slot, long out_off, hipStream_t stream) {
  if (mask_cstride < 576) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(upsample_convex_f32, dim3(nblk((long)B * h * w, 4)), dim3(256), 0, stream, mask, mask_cstride,
                     flow, B, h, w, out, (const long long*)out_slot, out_off);
  return (int)hipGetLastError();
}

extern "C" int jr_corr_pool_f32(const float* src, long M, int hl, int wl, float* dst, hipStream_t stream) {
  if (hl < 2 || wl < 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(corr_pool_f32, dim3(nblk(M * (hl / 2) * (wl / 2), 256)), dim3(256), 0, stream, src, M, hl, wl,
                     dst);
  return (int)hipGetLastError();
}

extern "C" int jr_corr_lookup_f32(const float* const* levels, int num_levels, int B, int h, int w, int nq,
                                  int radius, const float* coords, float* out, int out_cstride, hipStream_t stream) {
  const int S = 2 * radius + 1;
  if (num_levels < 1 || num_levels > 4 || out_cstride < num_levels * S * S) return (int)hipErrorInvalidValue;
  Lv4 lv{};
  for (int l = 0; l < num_levels; ++l) lv.p[l] = levels[l];
  const long total = (long)B * nq;
  const dim3 grid(nblk(total * num_levels * S, 256));
  switch (radius) {
    case 1: hipLaunchKernelGGL(lookup_f32<1>, grid, dim3(256), 0, stream, lv, num_levels, total, h, w, coords, out, out_cstride); break;
    case 2: hipLaunchKernelGGL(lookup_f32<2>, grid, dim3(256), 0, stream, lv, num_levels, total, h, w, coords, out, out_cstride); break;
    case 3: hipLaunchKernelGGL(lookup_f32<3>, grid, dim3(256), 0, stream, lv, num_levels, total, h, w, coords, out, out_cstride); break;
    case 4: hipLaunchKernelGGL(lookup_f32<4>, grid, dim3(256), 0, stream, lv, num_levels, total, h, w, coords, out, out_cstride); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

extern "C" int jr_flow_update_f32(const float* delta, int dcs, int N, int h, int w, float* coords, float* flow32,
                                  float* hx, int hx_cs, int hx_off, float* qx, int qx_cs, int qx_off, float* flow4,
                                  hipStream_t stream) {
  const long M = (long)N * h * w;
  if (dcs < 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(flow_update_f32, dim3(nblk(M, 256)), dim3(256), 0, stream, delta, dcs, M, h, w, coords, flow32,
                     hx, hx_cs, hx_off, qx, qx_cs, qx_off, flow4);
  return (int)hipGetLastError();
}
