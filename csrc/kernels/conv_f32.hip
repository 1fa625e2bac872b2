// fp32 implicit-GEMM NHWC convolution on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation -- a k-ordered
// fmaf chain, no TF32/xf32 shortcut exists on gfx950) for the engine's
// precision="fp32" parity mode: every conv of the reference (jax_raft/model.py
// :101-159, :238-255, :275-290, :304-310, :347-349, :389-394) in the reference's
// own precision, and (as a 1x1 "conv" whose weight rows are fmap2's pixels) the
// all-pairs correlation GEMM (:472-481).
//
// Design: 4 waves (2 x 2) per block, 64 x 64 block tiles (output channel x
// pixel; 2 x 2 MFMA tiles per wave), 32-deep K stages double-buffered in LDS,
// global loads one stage ahead in registers; split-K with an ordered reduction
// for grids of fewer than 4 blocks per CU.  Weights are plain row-major [cout][K] with
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

constexpr int FPAD = 4;   // LDS rows of FBK + 4 floats (36 / 20): conflict-free b32 fragment reads

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

// Block tile BCO x BP = (32 WM) x (32 WN) (output channels x pixels), 2 x 2
// waves of (16 WM) x (16 WN) (WM x WN MFMA tiles: WM + WN LDS reads per WM x WN
// MFMAs), FBK-deep K stages double-buffered in LDS, loads one stage ahead.
// SPLIT: split-K over blockIdx.z (p.ksplit ranges of K stages); raw partial sums
// go to p.part [ksplit][M][coutp] and conv_f32_reduce applies the epilogue.
template <int EPI, bool SPLIT, int WM, int WN, int FBK>
__global__ __launch_bounds__(256) void conv_f32_kernel(const ConvF32Params p) {
  constexpr int BCO = 32 * WM, BP = 32 * WN;
  constexpr int CPR = FBK / 4, RPP = 256 / CPR;       // 16-B chunks per row, rows per staging pass
  constexpr int NA = BCO / RPP, NB = BP / RPP;        // staging passes of A / B
  static_assert(NA >= 1 && NB >= 1 && BCO % RPP == 0 && BP % RPP == 0, "tile");
  __shared__ float sA[2][BCO][FBK + FPAD];
  __shared__ float sB[2][BP][FBK + FPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p0 = blockIdx.x * BP, co0 = blockIdx.y * BCO;
  const int OHW = p.OH * p.OW;
  const int kc = tid % CPR, r0 = tid / CPR;
  int ihb[NB], iwb[NB];
  long xbase[NB];
  bool pok[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int m = p0 + r0 + RPP * i;
    pok[i] = m < p.M;
    const int mm = pok[i] ? m : 0;
    const int n = mm / OHW, rem = mm - n * OHW, oh = rem / p.OW, ow = rem - oh * p.OW;
    ihb[i] = oh * p.SH - p.PH;
    iwb[i] = ow * p.SW - p.PW;
    xbase[i] = (long)n * p.H * p.W * p.x_cs + p.x_coff;
  }
  const int nks_all = (p.K + FBK - 1) / FBK;
  int ks_begin = 0, nks = nks_all;
  if constexpr (SPLIT) {
    ks_begin = (int)((long)nks_all * blockIdx.z / p.ksplit);
    nks = (int)((long)nks_all * (blockIdx.z + 1) / p.ksplit) - ks_begin;
  }
  float4 ra[NA], rb[NB];
  auto load = [&](int ks) {
    const int k = (ks_begin + ks) * FBK + kc * 4;
    const bool kok = k < p.K;
    const int tap = kok ? k / p.cin4 : 0, ci = k - tap * p.cin4;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int co = co0 + r0 + RPP * i;
      ra[i] = (kok && co < p.cout) ? *(const float4*)(p.w + (long)co * p.K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int ih = ihb[i] + kh, iw = iwb[i] + kw;
      const bool ok = kok && pok[i] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      rb[i] = ok ? *(const float4*)(p.x + xbase[i] + ((long)ih * p.W + iw) * p.x_cs + ci) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) *(float4*)&sA[buf][r0 + RPP * i][kc * 4] = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) *(float4*)&sB[buf][r0 + RPP * i][kc * 4] = rb[i];
  };
  const int wco = (wave & 1) * 16 * WM, wp = (wave >> 1) * 16 * WN;
  const int li = lane & 15, lk = lane >> 4;
  f32x4 acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
#pragma unroll
    for (int kk = 0; kk < FBK / 4; ++kk) {
      float a[WM], b[WN];
#pragma unroll
      for (int t = 0; t < WM; ++t) a[t] = sA[buf][wco + 16 * t + li][4 * kk + lk];
#pragma unroll
      for (int u = 0; u < WN; ++u) b[u] = sB[buf][wp + 16 * u + li][4 * kk + lk];
#pragma unroll
      for (int t = 0; t < WM; ++t)
#pragma unroll
        for (int u = 0; u < WN; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[u], acc[t][u], 0, 0, 0);
    }
    if (ks + 1 < nks) store(buf ^ 1);
    __syncthreads();
  }
  // D: lane (col = pixel li, rows 4 lk .. 4 lk + 3) of tile (t, u)
#pragma unroll
  for (int t = 0; t < WM; ++t) {
    const int c0 = co0 + wco + 16 * t + 4 * lk;
    if (c0 >= p.cout) continue;
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int m = p0 + wp + 16 * u + li;
      if (m >= p.M) continue;
      if constexpr (SPLIT) {
        const int coutp = (p.cout + 3) & ~3;
        *(f32x4*)(p.part + ((long)blockIdx.z * p.M + m) * coutp + c0) = acc[t][u];
      } else {
        float v[4] = {acc[t][u][0], acc[t][u][1], acc[t][u][2], acc[t][u][3]};
        f32_epilogue<EPI>(p, v, m, c0);
      }
    }
  }
}

// Split-K reduction: thread = (pixel, 4-channel chunk); partials summed in split
// order (deterministic), then the conv's epilogue.
template <int EPI>
__global__ __launch_bounds__(256) void conv_f32_reduce(const ConvF32Params p) {
  const int coutp = (p.cout + 3) & ~3, nc = coutp >> 2;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)p.M * nc) return;
  const int m = (int)(idx / nc), c0 = (int)(idx - (long)m * nc) * 4;
  f32x4 s = *(const f32x4*)(p.part + (long)m * coutp + c0);
  for (int z = 1; z < p.ksplit; ++z) s += *(const f32x4*)(p.part + ((long)z * p.M + m) * coutp + c0);
  float v[4] = {s[0], s[1], s[2], s[3]};
  f32_epilogue<EPI>(p, v, m, c0);
}

template <int EPI, int WM, int WN, int FBK>
int launch_tile(const ConvF32Params* p, hipStream_t stream) {
  const unsigned gx = (p->M + 32 * WN - 1) / (32 * WN), gy = (p->cout + 32 * WM - 1) / (32 * WM);
  if (p->ksplit > 1) {
    hipLaunchKernelGGL((conv_f32_kernel<EPI, true, WM, WN, FBK>), dim3(gx, gy, p->ksplit), dim3(256), 0, stream, *p);
    const long n = (long)p->M * ((p->cout + 3) / 4);
    hipLaunchKernelGGL((conv_f32_reduce<EPI>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, *p);
  } else {
    hipLaunchKernelGGL((conv_f32_kernel<EPI, false, WM, WN, FBK>), dim3(gx, gy), dim3(256), 0, stream, *p);
  }
  return (int)hipGetLastError();
}

// 64 x 64 tiles (2 x 2 MFMA tiles per wave, 32-deep stages).  Measured at raft_large
// 440x1024, 32 iterations, batch 1 (fp32 forward): 22.6 ms; 128 x 128 tiles (4 x 4 per
// wave) with 16- / 32-deep stages 28.0 / 27.5 ms, 128 x 64 26.4 ms.
template <int EPI>
int launch_f32(const ConvF32Params* p, hipStream_t stream) {
  return launch_tile<EPI, 2, 2, 32>(p, stream);
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
  if (p->ksplit > 1 && (!p->part || p->ksplit > (p->K + 31) / 32)) return (int)hipErrorInvalidValue;
  switch (epi) {
    case 0: return launch_f32<0>(p, stream);
    case 1: return launch_f32<1>(p, stream);
    case 2: return launch_f32<2>(p, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
