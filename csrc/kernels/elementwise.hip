// Memory-bound kernels: flow upsampling (convex + bilinear), norm statistics /
// application, input preparation and small buffer helpers (gfx950).
//
// Reference semantics:
//   upsample_flow            jax_raft/model.py:69-98
//   resize_with_aligned_corners (bilinear, align_corners)  model.py:43-66
//   InstanceNorm / BatchNorm (Flax)                         model.py:147,157,706-711
//   make_coords_grid                                        model.py:37-40
//   image normalisation / NHWC staging                      scripts/validate_sintel.py:177-183
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "upsample.h"

namespace {

// One wave per low-res pixel, lane = sub-pixel s = a*8 + b.
__global__ __launch_bounds__(256) void upsample_convex_kernel(const bf16* __restrict__ mask, int mcs,
                                                              const float* __restrict__ flow, int B, int h, int w,
                                                              float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int P = h * w;
  if (p >= B * P) return;
  const int b = p / P;
  const int rem = p - b * P;
  const int y = rem / w, x = rem - y * w;
  const bf16* mp = mask + (long)p * mcs + lane;
  float lg[9];
  float mx = -3.0e38f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lg[k] = bf2f(mp[k * 64]);
    mx = fmaxf(mx, lg[k]);
  }
  float s = 0.f, ux = 0.f, uy = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    const float e = __expf(lg[k] - mx);
    s += e;
    if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) {
      const float* fp = flow + 2 * ((long)b * P + yy * w + xx);
      ux += e * fp[0];
      uy += e * fp[1];
    }
  }
  const float inv = 8.0f / s;
  const int a = lane >> 3, bb = lane & 7;
  const long W8 = 8L * w;
  float* op = out + 2 * (((long)b * 8 * h + 8 * y + a) * W8 + 8 * x + bb);
  *(float2*)op = make_float2(ux * inv, uy * inv);
}

__global__ void upsample_bilinear_kernel(const float* __restrict__ flow, int B, int h, int w,
                                         float* __restrict__ out, const long long* __restrict__ out_slot, long out_off) {
  upsample_bilinear_elem(flow, B, h, w, out, out_slot, out_off, (long)blockIdx.x * blockDim.x + threadIdx.x);
}

// Deterministic per-(n, c) statistics: pass 1 writes one (sum, sumsq) partial
// per block (fixed row ranges), pass 2 sums the partials in order.  No float
// atomics, so eager and graph-replayed forwards are bitwise identical.
// blockDim 256; C/8 threads per row.
constexpr int STATS_ROWS = 1024;

__global__ __launch_bounds__(256) void channel_stats_partial_kernel(const bf16* __restrict__ x, int HW, int C,
                                                                    float* __restrict__ part, int rows) {
  __shared__ float red[256][17];
  const int n = blockIdx.y;
  const int cg = C >> 3;
  const int tid = threadIdx.x;
  const int g = tid % cg;
  const int rg = tid / cg;
  const int nrg = 256 / cg;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(r0 + rows, HW);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (rg < nrg) {
    const bf16* base = x + (long)n * HW * C + g * 8;
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += nrg) {
      const bf16x8 v = *(const bf16x8*)(base + (long)r * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(v[j]);
        s[j] += f;
        q[j] += f * f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[tid][j] = s[j]; red[tid][8 + j] = q[j]; }
  __syncthreads();
  // thread t < cg*16 reduces (channel group t%cg, value t/cg) over the row groups in order
  const int nb = gridDim.x;
  for (int t = tid; t < cg * 16; t += 256) {
    const int gg = t % cg, vi = t / cg;
    float acc = 0.f;
    for (int k = 0; k < nrg; ++k) acc += red[k * cg + gg][vi];
    const int c = gg * 8 + (vi & 7);
    part[(((long)n * nb + blockIdx.x) * C + c) * 2 + (vi >> 3)] = acc;
  }
}

// Deterministic final reduction of the per-block partials: block (n, value
// chunk) = 64 consecutive (channel, sum|sumsq) values x 4 partial-block lanes;
// each thread sums every 4th partial block (unrolled so several loads are in
// flight), then the 4 lanes combine through LDS in a fixed order.
__global__ __launch_bounds__(256) void channel_stats_final_kernel(const float* __restrict__ part, int N, int nb, int C,
                                                                   float* __restrict__ stats) {
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
    stats[(long)n * nv + vi] = t;
  }
}

// y = act(xn + rn).  Block = (row chunk, image n); thread = (8-channel group g,
// row lane).  The per-channel scale/shift of x (and of the residual) are derived
// from the statistics ONCE per block, one channel per thread, into LDS: each row
// lane deriving them itself was 8 x (2 .. 2N + 2) scalar loads per thread, and
// over ~2000 blocks that load stream (not the bytes) bounded the small maps and
// the BatchNorm (mode 2) form.  Rows are then visited NORM_ACT_U at a time with
// all their loads issued first; all indexing is 32-bit within one image.
constexpr int NORM_ACT_U = 4;

JR_DEVICE void norm_coeff(float& ao, float& bo, const float* st, int mode, const float* gam, const float* bet, int n,
                          int N, int HW, int C, int c, float eps) {
  float a = 1.f, b = 0.f;
  if (mode == 1) {
    const float inv = 1.0f / (float)HW;
    const float m = st[((long)n * C + c) * 2] * inv;
    const float var = fmaxf(st[((long)n * C + c) * 2 + 1] * inv - m * m, 0.f);
    a = rsqrtf(var + eps);
    b = -m * a;
  } else if (mode == 2) {
    float s0 = 0.f, s1 = 0.f;
    for (int k = 0; k < N; ++k) { s0 += st[((long)k * C + c) * 2]; s1 += st[((long)k * C + c) * 2 + 1]; }
    const float inv = 1.0f / ((float)HW * (float)N);
    const float m = s0 * inv;
    const float var = fmaxf(s1 * inv - m * m, 0.f);
    a = rsqrtf(var + eps);
    b = -m * a;
  }
  if (gam) { a *= gam[c]; b *= gam[c]; }
  if (bet) b += bet[c];
  ao = a;
  bo = b;
}

__global__ __launch_bounds__(256) void norm_act_kernel(const bf16* __restrict__ x, const float* __restrict__ sx,
                                                       int mode_x, const float* __restrict__ gx,
                                                       const float* __restrict__ bx, const bf16* __restrict__ r,
                                                       const float* __restrict__ sr, int mode_r,
                                                       const float* __restrict__ gr, const float* __restrict__ br,
                                                       bf16* __restrict__ y, int N, int HW, int C, float eps, int relu,
                                                       int rows) {
  extern __shared__ float cof[];   // [4][C]: x scale, x shift, residual scale, residual shift
  const int n = blockIdx.y;
  const int cg = C >> 3;
  const int tid = threadIdx.x;
  const int g = tid % cg, rg = tid / cg, nrg = 256 / cg;
  for (int c = tid; c < C; c += blockDim.x) {
    norm_coeff(cof[c], cof[C + c], sx, mode_x, gx, bx, n, N, HW, C, c, eps);
    if (r) norm_coeff(cof[2 * C + c], cof[3 * C + c], sr, mode_r, gr, br, n, N, HW, C, c, eps);
  }
  __syncthreads();
  if (rg >= nrg) return;
  const int c0 = g * 8;
  float xa[8], xb_[8], ra[8], rb_[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    xa[j] = cof[c0 + j];
    xb_[j] = cof[C + c0 + j];
    ra[j] = r ? cof[2 * C + c0 + j] : 0.f;
    rb_[j] = r ? cof[3 * C + c0 + j] : 0.f;
  }
  const long base = (long)n * HW * C + c0;
  const bf16* xb = x + base;
  const bf16* rb = r ? r + base : nullptr;
  bf16* yb = y + base;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(r0 + rows, HW);
  for (int row0 = r0 + rg; row0 < r1; row0 += NORM_ACT_U * nrg) {
    bf16x8 v[NORM_ACT_U], w[NORM_ACT_U];
#pragma unroll
    for (int u = 0; u < NORM_ACT_U; ++u) {   // all loads first (clamped rows; only valid ones are stored)
      const int off = min(row0 + u * nrg, r1 - 1) * C;
      v[u] = *(const bf16x8*)(xb + off);
      if (rb) w[u] = *(const bf16x8*)(rb + off);
    }
#pragma unroll
    for (int u = 0; u < NORM_ACT_U; ++u) {
      const int row = row0 + u * nrg;
      if (row >= r1) break;
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = fmaf(bf2f(v[u][j]), xa[j], xb_[j]);
        if (relu & 1) a[j] = fmaxf(a[j], 0.f);
        if (rb) a[j] += fmaf(bf2f(w[u][j]), ra[j], rb_[j]);
        if (relu & 2) a[j] = fmaxf(a[j], 0.f);
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(a[j]);
      *(bf16x8*)(yb + row * C) = o;
    }
  }
}

__global__ void prep_images_kernel(const float* __restrict__ i1, const float* __restrict__ i2, int B, long HW,
                                   bf16* __restrict__ out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = 2L * B * HW;
  if (idx >= total) return;
  const long half = (long)B * HW;
  const float* src = idx < half ? i1 + idx * 3 : i2 + (idx - half) * 3;
  bf16x8 o;
  o[0] = f2bf(src[0]); o[1] = f2bf(src[1]); o[2] = f2bf(src[2]);
#pragma unroll
  for (int j = 3; j < 8; ++j) o[j] = f2bf(0.f);
  *(bf16x8*)(out + idx * 8) = o;
}

// Space-to-depth image prep for the encoders' 7x7 / stride-2 stem (model.py:238-240):
// out[n][Y][X][(sy * 2 + sx) * 3 + c] = img[n][2Y + sy][2X + sx][c] (bf16, channels 12..15 zero),
// the input of the equivalent 4x4 / stride-1 conv (ops/native.py:s2d_stem_kernel): K = 16 x 16
// instead of 49 x 8 (8-channel padded 3-channel taps).
__global__ void prep_images_s2d_kernel(const float* __restrict__ i1, const float* __restrict__ i2, int B, int H, int W,
                                       bf16* __restrict__ out) {
  const int H2 = H >> 1, W2 = W >> 1;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)H2 * W2;
  if (idx >= 2L * B * per) return;
  const long n = idx / per;
  const int r = (int)(idx - n * per), Y = r / W2, X = r - (r / W2) * W2;
  const float* img = n < B ? i1 + n * (long)H * W * 3 : i2 + (n - B) * (long)H * W * 3;
  bf16x8 o0, o1;
#pragma unroll
  for (int sy = 0; sy < 2; ++sy) {
    const float* row = img + ((long)(2 * Y + sy) * W + 2 * X) * 3;
#pragma unroll
    for (int k = 0; k < 6; ++k) {   // (sx, c) of this row: channels sy * 6 + k
      const int ch = sy * 6 + k;
      if (ch < 8) o0[ch] = f2bf(row[k]);
      else o1[ch - 8] = f2bf(row[k]);
    }
  }
#pragma unroll
  for (int j = 4; j < 8; ++j) o1[j] = f2bf(0.f);
  *(bf16x8*)(out + idx * 16) = o0;
  *(bf16x8*)(out + idx * 16 + 8) = o1;
}

// Device-side input preparation of raw frames (the host protocol of the reference is
// validate_sintel.py:177-183 -- x / 255 * 2 - 1, InputPadder('sintel') replicate padding to /8,
// NCHW -> NHWC -- and demo.py:7-10): uint8 NHWC frames of any size H0 x W0 are normalised through
// a 256-entry fp32 table (computed on the host by the reference's own expression, so the values
// are bitwise those of the host path) and replicate-padded to the plan's H x W (pt / pl rows /
// columns before the frame: source pixel = clamp(y - pt, 0, H0 - 1), clamp(x - pl, 0, W0 - 1)),
// then written in the layout of prep_images(_s2d)_kernel above.  One thread per output pixel
// (S2D: per 2 x 2 block); the table is staged in LDS.
template <bool S2D>
__global__ void prep_u8_kernel(const unsigned char* __restrict__ i1, const unsigned char* __restrict__ i2,
                               const float* __restrict__ lut, int B, int H0, int W0, int H, int W, int pt, int pl,
                               bf16* __restrict__ out) {
  __shared__ float tab[256];
  tab[threadIdx.x] = lut[threadIdx.x];   // blockDim.x == 256
  __syncthreads();
  constexpr int R = S2D ? 2 : 1;
  const int Hq = H / R, Wq = W / R;
  const long per = (long)Hq * Wq;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2L * B * per) return;
  const long n = idx / per;
  const int r = (int)(idx - n * per), Y = r / Wq, X = r - (r / Wq) * Wq;
  const unsigned char* img = n < B ? i1 + n * (long)H0 * W0 * 3 : i2 + (n - B) * (long)H0 * W0 * 3;
  float v[12];
#pragma unroll
  for (int sy = 0; sy < R; ++sy) {
    const int y = min(max(R * Y + sy - pt, 0), H0 - 1);
#pragma unroll
    for (int sx = 0; sx < R; ++sx) {
      const int x = min(max(R * X + sx - pl, 0), W0 - 1);
      const unsigned char* px = img + ((long)y * W0 + x) * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[(sy * R + sx) * 3 + c] = tab[px[c]];
    }
  }
  if (S2D) {
    bf16x8 o0, o1;
#pragma unroll
    for (int k = 0; k < 8; ++k) o0[k] = f2bf(v[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) o1[k] = f2bf(v[8 + k]);
#pragma unroll
    for (int k = 4; k < 8; ++k) o1[k] = f2bf(0.f);
    *(bf16x8*)(out + idx * 16) = o0;
    *(bf16x8*)(out + idx * 16 + 8) = o1;
  } else {
    bf16x8 o;
    o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]);
#pragma unroll
    for (int k = 3; k < 8; ++k) o[k] = f2bf(0.f);
    *(bf16x8*)(out + idx * 8) = o;
  }
}

__global__ void init_coords_kernel(float* __restrict__ coords, int B, int h, int w) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * h * w;
  if (idx >= total) return;
  const int rem = idx % (h * w);
  coords[2 * idx] = (float)(rem % w);
  coords[2 * idx + 1] = (float)(rem / w);
}

__global__ void copy_channels_kernel(const bf16* __restrict__ src, int scs, int soff, bf16* __restrict__ dst, int dcs,
                                     int doff, int M, int C) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)M * C;
  if (idx >= total) return;
  const long m = idx / C;
  const int c = idx - m * C;
  dst[m * dcs + doff + c] = src[m * scs + soff + c];
}

// im2col in the packed-weight K order (tap-major, cin8 chunks, zero K tail):
// col[m][k], k = (kh*KW + kw)*cin8 + c.  One thread per 8 channels.
__global__ void im2col_kernel(const bf16* __restrict__ x, int H, int W, int xcs, int xoff, int cin8, int KH, int KW,
                              int SH, int SW, int PH, int PW, int OH, int OW, int kpad, long M, bf16* __restrict__ col) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int kc = kpad >> 3;
  if (idx >= M * kc) return;
  const long m = idx / kc;
  const int k = (int)(idx - m * kc) * 8;
  const int OHW = OH * OW;
  const int n = (int)(m / OHW);
  const int rem = (int)(m - (long)n * OHW);
  const int oh = rem / OW, ow = rem - (rem / OW) * OW;
  const int tap = k / cin8, c = k - tap * cin8;
  u32x4 v = {0u, 0u, 0u, 0u};
  if (tap < KH * KW) {
    const int kh = tap / KW, kw = tap - (tap / KW) * KW;
    const int ih = oh * SH - PH + kh, iw = ow * SW - PW + kw;
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
      v = *(const u32x4*)(x + (((long)n * H + ih) * W + iw) * xcs + xoff + c);
  }
  *(u32x4*)(col + m * kpad + k) = v;
}

inline unsigned nblk(long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

}  // namespace

extern "C" int jr_upsample_convex(const void* mask, int mask_cstride, const float* flow, int B, int h, int w,
                                  float* out, hipStream_t stream) {
  const int total = B * h * w;
  hipLaunchKernelGGL(upsample_convex_kernel, dim3((total + 3) / 4), dim3(256), 0, stream, (const bf16*)mask,
                     mask_cstride, flow, B, h, w, out);
  return (int)hipGetLastError();
}

extern "C" int jr_upsample_bilinear(const float* flow, int B, int h, int w, float* out, const void* out_slot,
                                    long out_off, hipStream_t stream) {
  const long total = (long)B * 64 * h * w;
  hipLaunchKernelGGL(upsample_bilinear_kernel, dim3(nblk(total, 256)), dim3(256), 0, stream, flow, B, h, w, out,
                     (const long long*)out_slot, out_off);
  return (int)hipGetLastError();
}

// rows per partial block: >= ~1024 blocks over the batch (the deep layers' small maps are otherwise
// latency-bound on a few dozen blocks), at most STATS_ROWS, a multiple of the row groups
static int stats_rows(int N, int HW, int C) {
  const int nrg = 256 / (C / 8);
  const int nb = std::max(1, (1024 + N - 1) / N);
  const int r = (HW + nb - 1) / nb;
  return std::min(STATS_ROWS, std::max(nrg, (r + nrg - 1) / nrg * nrg));
}

extern "C" int jr_channel_stats(const void* x, int N, int HW, int C, float* stats, float* partial,
                                hipStream_t stream) {
  if (C % 8 != 0 || (C / 8) > 256) return (int)hipErrorInvalidValue;
  const int rows = stats_rows(N, HW, C);
  const int nb = (HW + rows - 1) / rows;
  hipLaunchKernelGGL(channel_stats_partial_kernel, dim3(nb, N), dim3(256), 0, stream, (const bf16*)x, HW, C, partial,
                     rows);
  hipLaunchKernelGGL(channel_stats_final_kernel, dim3((2 * C + 7) / 8, N), dim3(256), 0, stream, partial, N, nb, C,
                     stats);
  return (int)hipGetLastError();
}

// an upper bound for both the bf16 path (adaptive rows) and jr_channel_stats_f32 (STATS_ROWS rows)
extern "C" int jr_channel_stats_partials(int N, int HW, int C) {
  if (C % 8 != 0 || C / 8 > 256) return N * ((HW + 3) / 4);
  return N * ((HW + stats_rows(N, HW, C) - 1) / stats_rows(N, HW, C));
}

extern "C" int jr_channel_stats_final(const float* part, int N, int nb, int C, float* stats, hipStream_t stream) {
  hipLaunchKernelGGL(channel_stats_final_kernel, dim3((2 * C + 7) / 8, N), dim3(256), 0, stream, part, N, nb, C, stats);
  return (int)hipGetLastError();
}

extern "C" int jr_norm_act(const void* x, const float* sx, int mode_x, const float* gamma, const float* beta,
                           const void* res, const float* sr, int mode_r, const float* gamma_r, const float* beta_r,
                           void* y, int N, int HW, int C, float eps, int relu, hipStream_t stream) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  if (C / 8 > 256) return (int)hipErrorInvalidValue;
  // rows per block: a multiple of the block's row lanes, sized for ~2048 blocks
  const int nrg = 256 / (C / 8);
  const long want = ((long)N * HW + 2047) / 2048;
  const int rows = (int)std::max<long>(nrg, (want + nrg - 1) / nrg * nrg);
  const unsigned nb = (unsigned)((HW + rows - 1) / rows);
  hipLaunchKernelGGL(norm_act_kernel, dim3(nb, N), dim3(256), 4 * C * sizeof(float), stream, (const bf16*)x, sx, mode_x, gamma, beta,
                     (const bf16*)res, sr, mode_r, gamma_r, beta_r, (bf16*)y, N, HW, C, eps, relu, rows);
  return (int)hipGetLastError();
}

extern "C" int jr_prep_images(const float* img1, const float* img2, int B, int H, int W, void* out,
                              hipStream_t stream) {
  const long total = 2L * B * H * W;
  hipLaunchKernelGGL(prep_images_kernel, dim3(nblk(total, 256)), dim3(256), 0, stream, img1, img2, B, (long)H * W,
                     (bf16*)out);
  return (int)hipGetLastError();
}

extern "C" int jr_prep_images_s2d(const float* img1, const float* img2, int B, int H, int W, void* out,
                                  hipStream_t stream) {
  if ((H | W) & 1) return (int)hipErrorInvalidValue;
  const long total = 2L * B * (H / 2) * (W / 2);
  hipLaunchKernelGGL(prep_images_s2d_kernel, dim3(nblk(total, 256)), dim3(256), 0, stream, img1, img2, B, H, W,
                     (bf16*)out);
  return (int)hipGetLastError();
}

extern "C" int jr_prep_u8(const void* img1, const void* img2, const float* lut, int B, int H0, int W0, int H, int W,
                          int pt, int pl, int s2d, void* out, hipStream_t stream) {
  if (H0 < 1 || W0 < 1 || H < H0 || W < W0 || pt < 0 || pl < 0 || (s2d && ((H | W) & 1))) return (int)hipErrorInvalidValue;
  const long total = 2L * B * (s2d ? (long)(H / 2) * (W / 2) : (long)H * W);
  const auto* a = (const unsigned char*)img1;
  const auto* b = (const unsigned char*)img2;
  if (s2d)
    hipLaunchKernelGGL(prep_u8_kernel<true>, dim3(nblk(total, 256)), dim3(256), 0, stream, a, b, lut, B, H0, W0, H, W,
                       pt, pl, (bf16*)out);
  else
    hipLaunchKernelGGL(prep_u8_kernel<false>, dim3(nblk(total, 256)), dim3(256), 0, stream, a, b, lut, B, H0, W0, H,
                       W, pt, pl, (bf16*)out);
  return (int)hipGetLastError();
}

extern "C" int jr_init_coords(float* coords, int B, int h, int w, hipStream_t stream) {
  const long total = (long)B * h * w;
  hipLaunchKernelGGL(init_coords_kernel, dim3(nblk(total, 256)), dim3(256), 0, stream, coords, B, h, w);
  return (int)hipGetLastError();
}

extern "C" int jr_copy_channels(const void* src, int s_cstride, int s_coff, void* dst, int d_cstride, int d_coff,
                                int M, int C, hipStream_t stream) {
  const long total = (long)M * C;
  hipLaunchKernelGGL(copy_channels_kernel, dim3(nblk(total, 256)), dim3(256), 0, stream, (const bf16*)src, s_cstride,
                     s_coff, (bf16*)dst, d_cstride, d_coff, M, C);
  return (int)hipGetLastError();
}

extern "C" int jr_im2col(const void* x, int N, int H, int W, int x_cstride, int x_coff, int cin8, int KH, int KW,
                         int SH, int SW, int PH, int PW, int OH, int OW, int kpad, void* col, hipStream_t stream) {
  if (cin8 % 8 || kpad % 8 || x_cstride % 8 || x_coff % 8) return (int)hipErrorInvalidValue;
  const long M = (long)N * OH * OW;
  hipLaunchKernelGGL(im2col_kernel, dim3(nblk(M * (kpad / 8), 256)), dim3(256), 0, stream, (const bf16*)x, H, W,
                     x_cstride, x_coff, cin8, KH, KW, SH, SW, PH, PW, OH, OW, kpad, M, (bf16*)col);
  return (int)hipGetLastError();
}

// Zero fill (plan memsets are kernels, not hipMemsetAsync nodes, so a captured
// plan is a pure kernel + event graph on every lane).
__global__ __launch_bounds__(256) void zero_fill_kernel(u32x4* __restrict__ p16, long n16, unsigned* __restrict__ p4,
                                                          long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) p16[i] = u32x4{0u, 0u, 0u, 0u};
  if (i < n4) p4[i] = 0u;
}

extern "C" int jr_zero_fill(void* p, long bytes, hipStream_t stream) {
  if (((uintptr_t)p & 15) || (bytes & 3)) return (int)hipErrorInvalidValue;
  const long n16 = bytes / 16;
  const long n4 = (bytes - n16 * 16) / 4;
  const long n = n16 > n4 ? n16 : n4;
  if (n == 0) return 0;
  hipLaunchKernelGGL(zero_fill_kernel, dim3(nblk(n, 256)), dim3(256), 0, stream, (u32x4*)p, n16,
                     (unsigned*)((char*)p + n16 * 16), n4);
  return (int)hipGetLastError();
}
