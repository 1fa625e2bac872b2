// fp32 implicit-GEMM NHWC convolution on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation -- a k-ordered
// fmaf chain, no TF32/xf32 shortcut exists on gfx950) for the engine's
// precision="fp32" parity mode: every conv of the reference (jax_raft/model.py
// :101-159, :238-255, :275-290, :304-310, :347-349, :389-394) in the reference's
// own precision, and (as a 1x1 "conv" whose weight rows are fmap2's pixels) the
// all-pairs correlation GEMM (:472-481).
//
// Design: 64 x 64 (output channel x pixel) block tile, 4 waves of 32 x 32
// (2 x 2 MFMA tiles), 32-deep K stages double-buffered in LDS, global loads
// one stage ahead in registers.  Weights are plain row-major [cout][K] with
// K = (kh, kw, cin4) -- no permutation, so the correlation uses fmap2 itself as
// the weight matrix.  Activations are fp32 NHWC with a channel stride / offset,
// channels padded to 4 (16-byte chunks).  The D fragment gives each lane 4
// consecutive output channels of one pixel: one 16-byte store per output.
// Epilogues: bias + per-pixel bias map + residual (pre / post activation) +
// activation + alpha, optional second output copy and fp32 hidden-state copy
// (EPI 0); the ConvGRU gates z, r*h (EPI 1) and q + blend (EPI 2) as in
// conv_igemm.h, all in fp32.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int FB_CO = 64, FB_P = 64, FBK = 32, FPAD = 4;   // LDS rows of 36 floats: conflict-free b32 reads

// 4 consecutive channels at p (nv < 4: the channel tail of a cout % 4 != 0 conv, scalar)
JR_DEVICE void ld4(const float* p, int nv, float (&v)[4]) {
  if (nv == 4) {
    const float4 t = *(const float4*)p;
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = j < nv ? p[j] : 0.f;
  }
}
JR_DEVICE void st4(float* p, int nv, const float (&v)[4]) {
  if (nv == 4) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) if (j < nv) p[j] = v[j];
  }
}

template <int EPI>
JR_DEVICE void f32_epilogue(const ConvF32Params& p, float (&v)[4], int m, int c0) {
  // v: raw accumulators of channels c0 .. c0 + nv - 1 of pixel m
  const int nv = min(4, p.cout - c0);
  float t[4];
  ld4(p.bias + c0, nv, t);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] += t[j];
  if (p.bmap) {
    ld4(p.bmap + (long)m * p.bmap_cs + p.bmap_coff + c0, nv, t);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += t[j];
  }
  if constexpr (EPI == 0) {
    if (p.res) {
      ld4(p.res + (long)m * p.res_cs + p.res_coff + c0, nv, t);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = p.res_post ? fmaxf(apply_act(v[j], p.act, c0 + j, p.split) + t[j], 0.f)
                          : apply_act(v[j] + t[j], p.act, c0 + j, p.split);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = apply_act(v[j], p.act, c0 + j, p.split);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= p.alpha;
    st4(p.y + (long)m * p.y_cs + p.y_coff + c0, nv, v);
    if (p.y2) st4(p.y2 + (long)m * p.y2_cs + p.y2_coff + c0, nv, v);
    if (p.h32 && c0 < p.split) st4(p.h32 + (long)m * p.hidden + c0, nv, v);
  } else if constexpr (EPI == 1) {   // [z | r] logits -> z, r*h (h from the fp32 state); hidden % 4 == 0
    const int hd = p.hidden;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = sigmoidf_(v[j]);
    if (c0 < hd) {
      st4(p.zbuf + (long)m * hd + c0, 4, v);
    } else {
      const int hc = c0 - hd;
      ld4(p.h32 + (long)m * hd + hc, 4, t);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= t[j];
      st4(p.y + (long)m * p.y_cs + p.y_coff + hc, 4, v);
    }
  } else {                           // q = tanh ; h = (1 - z) h + z q
    const int hd = p.hidden;
    float z[4];
    ld4(p.zbuf + (long)m * hd + c0, 4, z);
    float* hp = p.h32 + (long)m * hd + c0;
    ld4(hp, 4, t);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (1.0f - z[j]) * t[j] + z[j] * tanhf_(v[j]);
    st4(hp, 4, v);
    st4(p.y + (long)m * p.y_cs + p.y_coff + c0, 4, v);
    if (p.y2) st4(p.y2 + (long)m * p.y2_cs + p.y2_coff + c0, 4, v);
  }
}

template <int EPI>
__global__ __launch_bounds__(256) void conv_f32_kernel(const ConvF32Params p) {
  __shared__ float sA[2][FB_CO][FBK + FPAD];
  __shared__ float sB[2][FB_P][FBK + FPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p0 = blockIdx.x * FB_P, co0 = blockIdx.y * FB_CO;
  const int OHW = p.OH * p.OW;
  // per-thread staging: 2 chunks (4 floats) of A and of B per stage: rows tid/8 and tid/8 + 32, k-chunk tid % 8
  const int kc = tid & 7;
  int ihb[2], iwb[2];
  long xbase[2];
  bool pok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = p0 + (tid >> 3) + 32 * i;
    pok[i] = m < p.M;
    const int mm = pok[i] ? m : 0;
    const int n = mm / OHW, rem = mm - n * OHW, oh = rem / p.OW, ow = rem - oh * p.OW;
    ihb[i] = oh * p.SH - p.PH;
    iwb[i] = ow * p.SW - p.PW;
    xbase[i] = (long)n * p.H * p.W * p.x_cs + p.x_coff;
  }
  const int nks = (p.K + FBK - 1) / FBK;
  float4 ra[2], rb[2];
  auto load = [&](int ks) {
    const int k = ks * FBK + kc * 4;
    const bool kok = k < p.K;
    const int tap = kok ? k / p.cin4 : 0, ci = k - tap * p.cin4;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = co0 + (tid >> 3) + 32 * i;
      ra[i] = (kok && co < p.cout) ? *(const float4*)(p.w + (long)co * p.K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      const int ih = ihb[i] + kh, iw = iwb[i] + kw;
      const bool ok = kok && pok[i] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      rb[i] = ok ? *(const float4*)(p.x + xbase[i] + ((long)ih * p.W + iw) * p.x_cs + ci) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *(float4*)&sA[buf][r][kc * 4] = ra[i];
      *(float4*)&sB[buf][r][kc * 4] = rb[i];
    }
  };
  const int wco = (wave & 1) * 32, wp = (wave >> 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
#pragma unroll
    for (int kk = 0; kk < FBK / 4; ++kk) {
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = sA[buf][wco + 16 * t + li][4 * kk + lk];
        b[t] = sB[buf][wp + 16 * t + li][4 * kk + lk];
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[u], acc[t][u], 0, 0, 0);
    }
    if (ks + 1 < nks) store(buf ^ 1);
    __syncthreads();
  }
  // D: lane (col = pixel li, rows 4 lk .. 4 lk + 3) of tile (t, u)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c0 = co0 + wco + 16 * t + 4 * lk;
    if (c0 >= p.cout) continue;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = p0 + wp + 16 * u + li;
      if (m >= p.M) continue;
      float v[4] = {acc[t][u][0], acc[t][u][1], acc[t][u][2], acc[t][u][3]};
      f32_epilogue<EPI>(p, v, m, c0);
    }
  }
}

}  // namespace

extern "C" int jr_conv_f32(const ConvF32Params* p, int epi, hipStream_t stream) {
  if (p->M <= 0) return 0;
  // 16-byte operand chunks: every channel stride / offset a multiple of 4 floats
  const bool gru = epi == 1 || epi == 2;
  if (p->cin4 % 4 || p->x_cs % 4 || p->x_coff % 4 || p->K != p->KH * p->KW * p->cin4 || p->y_cs % 4 ||
      p->y_coff % 4 || (p->y2 && (p->y2_cs % 4 || p->y2_coff % 4)) || (p->res && (p->res_cs % 4 || p->res_coff % 4)) ||
      (p->bmap && (p->bmap_cs % 4 || p->bmap_coff % 4)) || (p->h32 && p->hidden % 4) ||
      (gru && (p->hidden % 4 || !p->h32 || !p->zbuf || p->cout != (epi == 1 ? 2 : 1) * p->hidden)))
    return (int)hipErrorInvalidValue;
  dim3 grid((p->M + FB_P - 1) / FB_P, (p->cout + FB_CO - 1) / FB_CO);
  switch (epi) {
    case 0: hipLaunchKernelGGL(conv_f32_kernel<0>, grid, dim3(256), 0, stream, *p); break;
    case 1: hipLaunchKernelGGL(conv_f32_kernel<1>, grid, dim3(256), 0, stream, *p); break;
    case 2: hipLaunchKernelGGL(conv_f32_kernel<2>, grid, dim3(256), 0, stream, *p); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
