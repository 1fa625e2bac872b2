// Flow-head output conv (3x3, hidden -> 2) fused with the coordinate update.
//
// Replaces FlowHead.conv2 (jax_raft/model.py:347-350) and the update
// `coords1 = coords1 + delta` (model.py:505) of the RAFT loop.  With only two
// output channels an implicit-GEMM MFMA tile wastes 7/8 of its rows, and the
// conv sits on the loop's critical path, so it gets its own kernel:
//   * a block of four waves per 64-pixel row segment; the 3 x 66 pixel halo of
//     each 64-channel chunk is staged in LDS (rows padded to 136 B:
//     conflict-free ds_read_b128 across lanes), all loads of a chunk in flight
//     at once and the next chunk prefetched during the current one's math;
//   * lane = pixel, wave = channel quarter: each lane accumulates both outputs
//     over its wave's 16 channels of every tap with v_dot2_f32_bf16; the
//     weights (2 x 9 x cin bf16) are staged into LDS once per block and read
//     as wave-uniform (broadcast) ds_read_b128;
//   * the four channel quarters meet through LDS, then the fused
//     epilogue: coords += delta, flow = coords - grid written as fp32 and as
//     bf16 into the GRU input buffers (hx, qx) and the motion encoder's flow
//     input (flow8), exactly as the conv kernels' EPI_FLOW.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int SEG = 64;          // output pixels per block (one per lane)
constexpr int TW = SEG + 2;      // halo columns
constexpr int RS = 68;           // LDS row stride in bf16 (64 channels + 4 pad = 136 B)

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

JR_DEVICE float dot2(unsigned a, unsigned b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a), __builtin_bit_cast(bf16x2, b), c, false);
}

// wt: bf16 [2][9][cin] (output-major, then tap, then channel: contiguous channel pairs for dot2)
template <int CIN>
__global__ __launch_bounds__(256) void flow_head_kernel(const bf16* __restrict__ fm, int fcs,
                                                       const unsigned* __restrict__ wt, const float* __restrict__ bias,
                                                       int h, int w, float* __restrict__ coords,
                                                       float* __restrict__ flow32, bf16* __restrict__ hx, int hx_cs,
                                                       int hx_off, bf16* __restrict__ qx, int qx_cs, int qx_off,
                                                       bf16* __restrict__ f8, int f8_cs) {
  __shared__ __attribute__((aligned(16))) bf16 tile[3 * TW * RS];
  __shared__ float2 part[3][SEG];
  __shared__ __attribute__((aligned(16))) unsigned wl[2 * 9 * CIN / 2];
  const int tid = threadIdx.x;
  for (int e = tid; e < 2 * 9 * CIN / 8; e += 256) ((u32x4*)wl)[e] = ((const u32x4*)wt)[e];
  const int lane = tid & 63;
  const int segs = (w + SEG - 1) / SEG;
  const int seg = blockIdx.x % segs;
  const int ny = blockIdx.x / segs;               // n * h + y
  const int y = ny % h;
  const long img0 = (long)(ny - y) * w;           // first pixel of image n
  const int x0 = seg * SEG;
  const int px = lane;                             // output pixel of this lane
  const int qw = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave = channel quarter (provably uniform)

  // Halo staging: 3 x TW pixels x 64 channels = NE 16-B pieces, 8 lanes per
  // pixel row.  All NL loads of a chunk are in flight at once (registers), and
  // the next chunk's loads are issued before the current chunk's dot products.
  constexpr int NE = 3 * TW * 8;
  constexpr int NL = (NE + 255) / 256;
  long goff[NL];
  int soff[NL];
  bool gok[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = tid + 256 * i;
    const int pr = e >> 3, ck = e & 7;
    const int r = pr / TW, col = pr - r * TW;
    const int yy = y - 1 + r, xx = x0 - 1 + col;
    gok[i] = e < NE && (unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w;
    goff[i] = gok[i] ? (img0 + (long)yy * w + xx) * fcs + ck * 8 : 0;
    soff[i] = e < NE ? pr * RS + ck * 8 : -1;
  }
  u32x4 st[NL];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < NL; ++i)
      st[i] = gok[i] ? *(const u32x4*)(fm + goff[i] + c0) : u32x4{0u, 0u, 0u, 0u};
  };
  load(0);
  float s0 = 0.f, s1 = 0.f;
#pragma unroll 1
  for (int c0 = 0; c0 < CIN; c0 += 64) {
#pragma unroll
    for (int i = 0; i < NL; ++i)
      if (soff[i] >= 0) *(u32x4*)(tile + soff[i]) = st[i];
    __syncthreads();
    if (c0 + 64 < CIN) load(c0 + 64);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int r = t / 3, kw = t - r * 3;
      const bf16* src = tile + (r * TW + px + kw) * RS + qw * 16;
      const u32x4* w0 = (const u32x4*)(wl + ((0 * 9 + t) * CIN + c0 + qw * 16) / 2);
      const u32x4* w1 = (const u32x4*)(wl + ((1 * 9 + t) * CIN + c0 + qw * 16) / 2);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x4 a = *(const u32x4*)(src + q * 8);
        const u32x4 b0 = w0[q], b1 = w1[q];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s0 = dot2(a[j], b0[j], s0);
          s1 = dot2(a[j], b1[j], s1);
        }
      }
    }
    __syncthreads();
  }
  if (qw > 0) part[qw - 1][px] = float2{s0, s1};
  __syncthreads();
  const int x = x0 + px;
  if (qw == 0 && x < w) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      s0 += part[k][px].x;
      s1 += part[k][px].y;
    }
    const long m = img0 + (long)y * w + x;
    const float cx = coords[2 * m] + s0 + bias[0];
    const float cy = coords[2 * m + 1] + s1 + bias[1];
    coords[2 * m] = cx;
    coords[2 * m + 1] = cy;
    const float fx = cx - (float)x;
    const float fy = cy - (float)y;
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
}

}  // namespace

extern "C" int jr_flow_head(const void* fm, int fcs, const void* wt, const float* bias, int N, int h, int w, int cin,
                            float* coords, float* flow32, void* hx, int hx_cs, int hx_off, void* qx, int qx_cs,
                            int qx_off, void* f8, int f8_cs, hipStream_t stream) {
  if (fcs % 8) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)(N * h * ((w + SEG - 1) / SEG)));
#define JR_FH(C)                                                                                                  \
  hipLaunchKernelGGL(flow_head_kernel<C>, grid, dim3(256), 0, stream, (const bf16*)fm, fcs, (const unsigned*)wt,   \
                     bias, h, w, coords, flow32, (bf16*)hx, hx_cs, hx_off, (bf16*)qx, qx_cs, qx_off, (bf16*)f8, f8_cs)
  if (cin == 256) JR_FH(256);
  else if (cin == 128) JR_FH(128);
  else return (int)hipErrorInvalidValue;
#undef JR_FH
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Flow-head output conv as "1x1 GEMM + tap sum" (the default engine path).
// A 3x3 conv with 2 outputs is linear in its input, so
//   delta(p) = b + sum_{kh,kw} W[kh][kw]^T fm(p + (kh-1, kw-1))
//            = b + sum_tap t[p + d_tap][tap],   t[q][tap] = W[tap]^T fm(q)
// t (9 taps x 2 outputs per pixel) is ONE 1x1 implicit-GEMM conv over fm
// (K = cin, N = 18: fm is read once instead of 9 times), and this kernel adds
// the 9 shifted partials (zero padding = skipping out-of-map neighbours)
// and applies the fused epilogue of EPI_FLOW: coords += delta, flow =
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
