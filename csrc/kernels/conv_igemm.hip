// NHWC implicit-GEMM convolution on gfx950 MFMA (bf16 in, fp32 accumulate).
//
// Replaces every convolution of the reference RAFT (flax.linen.Conv sites in
// jax_raft/model.py:101-159 (ConvNormActivation), :238-255 (encoders),
// :275-290 (MotionEncoder), :304-310 (ConvGRU), :347-349 (FlowHead),
// :389-394 (MaskPredictor)).  Design (MI355X-first, not a translation):
//
//  * "Swapped" GEMM orientation: the MFMA A operand is the packed weight
//    matrix W[co][k] and the B operand the implicit im2col X[pixel][k].  The
//    16x16x32 accumulator then holds, per lane, 4 consecutive output channels
//    of ONE pixel; with the A-row permutation below each lane owns 4*TM
//    contiguous channels, so the epilogue is pixel-local and vectorised
//    (16-32 B stores, residual/GRU-state loads as whole vectors).
//  * K = (kh, kw, cin8) flattened in 8-channel (16 B) chunks, so any kernel
//    shape (1x1, 3x3, 7x7, 1x5, 5x1, strided) runs through one loader.
//  * 64-deep K stages, double-buffered LDS, register-staged global loads
//    issued before the MFMA block of the previous stage (one barrier per
//    stage).  LDS rows are 128 B with XOR swizzles chosen so that the
//    ds_read_b128 fragment reads of both operands are bank-conflict free.
//  * Fused epilogues: bias, residual, activation (incl. the context-encoder
//    tanh/relu split), scaling, dual stores into concat buffers, and the
//    ConvGRU gate/blend and flow-head coordinate update of the RAFT loop.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;

JR_DEVICE int swzA(int row) { return ((row >> 1) & 1) | ((row >> 3) & 6); }
JR_DEVICE int swzB(int row) { return (row >> 1) & 7; }

template <int NV>
JR_DEVICE void store_bf16(bf16* dst, const float* v) {
  if constexpr (NV % 8 == 0) {
#pragma unroll
    for (int c = 0; c < NV / 8; ++c) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[c * 8 + j]);
      *(bf16x8*)(dst + c * 8) = o;
    }
  } else {
    static_assert(NV == 4, "NV");
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
    *(bf16x4*)dst = o;
  }
}

template <int NV>
JR_DEVICE void load_bf16(const bf16* src, float* v) {
  if constexpr (NV % 8 == 0) {
#pragma unroll
    for (int c = 0; c < NV / 8; ++c) {
      bf16x8 o = *(const bf16x8*)(src + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c * 8 + j] = bf2f(o[j]);
    }
  } else {
    bf16x4 o = *(const bf16x4*)src;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = bf2f(o[j]);
  }
}

template <int NV>
JR_DEVICE void store_f32(float* dst, const float* v) {
#pragma unroll
  for (int c = 0; c < NV / 4; ++c) *(f32x4*)(dst + 4 * c) = f32x4{v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
}

template <int NV>
JR_DEVICE void load_f32(const float* src, float* v) {
#pragma unroll
  for (int c = 0; c < NV / 4; ++c) {
    f32x4 o = *(const f32x4*)(src + 4 * c);
    v[4 * c] = o[0]; v[4 * c + 1] = o[1]; v[4 * c + 2] = o[2]; v[4 * c + 3] = o[3];
  }
}

template <int BCO, int BP, int WCO, int EPI>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const ConvParams p) {
  constexpr int WP = 4 / WCO;
  constexpr int WTCO = BCO / WCO;
  constexpr int WTP = BP / WP;
  constexpr int TM = WTCO / 16;
  constexpr int TN = WTP / 16;
  constexpr int NV = 4 * TM;              // contiguous channels per lane
  constexpr int XR = BP / 32;             // X rows loaded per thread
  constexpr int WR = BCO >= 32 ? BCO / 32 : 1;
  constexpr int A_ELEMS = BCO * BK;
  constexpr int B_ELEMS = BP * BK;
  static_assert(TM >= 1 && TN >= 1 && WCO * WP == 4, "tile");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (A_ELEMS + B_ELEMS)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wco = wave % WCO;
  const int wp = wave / WCO;
  const int p0 = blockIdx.x * BP;
  const int co0 = blockIdx.y * BCO;
  const int ch = tid & 7;

  const bf16* __restrict__ xb = (const bf16*)p.x;
  const bf16* __restrict__ wb = (const bf16*)p.w;
  const int OHW = p.OH * p.OW;

  // Per-thread im2col row descriptors (fixed across the K loop).
  int ih0[XR], iw0[XR];
  long rbase[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int m = p0 + (tid >> 3) + 32 * i;
    if (m < p.M) {
      const int n = m / OHW;
      const int rem = m - n * OHW;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      ih0[i] = oh * p.SH - p.PH;
      iw0[i] = ow * p.SW - p.PW;
      rbase[i] = (long)n * p.H * p.W * p.x_cstride + p.x_coff;
    } else {
      ih0[i] = -(1 << 28);
      iw0[i] = -(1 << 28);
      rbase[i] = 0;
    }
  }

  // K-chunk state of this thread's chunk column: kc = ks*8 + ch.
  const int cpt = p.cin8 >> 3;
  int tap = ch / cpt;
  int cc = ch - tap * cpt;
  int kh = tap / p.KW;
  int kw = tap - kh * p.KW;

  u32x4 xr[XR];
  u32x4 wr[WR];

  auto load_stage = [&](int ks) {
    const bool kvalid = kh < p.KH;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int ih = ih0[i] + kh;
      const int iw = iw0[i] + kw;
      const bool ok = kvalid && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      if (ok) {
        xr[i] = *(const u32x4*)(xb + rbase[i] + (long)(ih * p.W + iw) * p.x_cstride + cc * 8);
      } else {
        xr[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int row = (tid >> 3) + 32 * i;
      const int co = co0 + row;
      const bool act_thread = (BCO >= 32) || (tid < BCO * 8);
      if (act_thread && co < p.cout_pad) {
        wr[i] = *(const u32x4*)(wb + (long)co * p.kpad + ks * BK + ch * 8);
      } else {
        wr[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto advance = [&]() {
    cc += 8;
    while (cc >= cpt) {
      cc -= cpt;
      if (++kw == p.KW) { kw = 0; ++kh; }
    }
  };
  auto store_stage = [&](int buf) {
    bf16* sA = smem + buf * (A_ELEMS + B_ELEMS);
    bf16* sB = sA + A_ELEMS;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *(u32x4*)(sB + r * BK + ((ch ^ swzB(r)) << 3)) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int r = (tid >> 3) + 32 * i;
      if ((BCO >= 32) || (tid < BCO * 8)) *(u32x4*)(sA + r * BK + ((ch ^ swzA(r)) << 3)) = wr[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nks = p.kpad / BK;
  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int li = lane & 15;
  const int lq = lane >> 4;
  for (int ks = 0; ks < nks; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nks;
    if (more) {
      advance();
      load_stage(ks + 1);
    }
    const bf16* sA = smem + cur * (A_ELEMS + B_ELEMS);
    const bf16* sB = sA + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + lq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wco * WTCO + (li >> 2) * NV + tm * 4 + (li & 3);
        af[tm] = *(const bf16x8*)(sA + row * BK + ((chunk ^ swzA(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wp * WTP + tn * 16 + li;
        bfr[tn] = *(const bf16x8*)(sB + row * BK + ((chunk ^ swzB(row)) << 3));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  const int cbase = co0 + wco * WTCO + lq * NV;
  if (cbase >= p.cout) return;
  const bool full = cbase + NV <= p.cout;
  float bias[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) bias[j] = (cbase + j < p.cout) ? p.bias[cbase + j] : 0.f;

#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int m = p0 + wp * WTP + tn * 16 + li;
    if (m >= p.M) continue;
    float v[NV];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[tm * 4 + r] = acc[tm][tn][r] + bias[tm * 4 + r];

    if constexpr (EPI == EPI_STD) {
      if (p.res) {
        float rv[NV];
        const bf16* rp = (const bf16*)p.res + (long)m * p.res_cstride + p.res_coff + cbase;
        if (full) {
          load_bf16<NV>(rp, rv);
        } else {
#pragma unroll
          for (int j = 0; j < NV; ++j) rv[j] = (cbase + j < p.cout) ? bf2f(rp[j]) : 0.f;
        }
        if (p.res_post) {
#pragma unroll
          for (int j = 0; j < NV; ++j) v[j] = fmaxf(apply_act(v[j], p.act, cbase + j, p.split) + rv[j], 0.f);
        } else {
#pragma unroll
          for (int j = 0; j < NV; ++j) v[j] = apply_act(v[j] + rv[j], p.act, cbase + j, p.split);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = apply_act(v[j], p.act, cbase + j, p.split);
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] *= p.alpha;
      if (p.y_fp32) {
        float* yp = (float*)p.y + (long)m * p.y_cstride + p.y_coff + cbase;
        if (full) store_f32<NV>(yp, v);
        else {
#pragma unroll
          for (int j = 0; j < NV; ++j) if (cbase + j < p.cout) yp[j] = v[j];
        }
      } else {
        bf16* yp = (bf16*)p.y + (long)m * p.y_cstride + p.y_coff + cbase;
        if (full) store_bf16<NV>(yp, v);
        else {
#pragma unroll
          for (int j = 0; j < NV; ++j) if (cbase + j < p.cout) yp[j] = f2bf(v[j]);
        }
      }
      if (p.y2) {
        bf16* yp = (bf16*)p.y2 + (long)m * p.y2_cstride + p.y2_coff + cbase;
        if (full) store_bf16<NV>(yp, v);
        else {
#pragma unroll
          for (int j = 0; j < NV; ++j) if (cbase + j < p.cout) yp[j] = f2bf(v[j]);
        }
      }
      if (p.h32) {  // fp32 copy of the channels below `split` (context-encoder hidden state)
        if (cbase < p.split) {
          float* hp = p.h32 + (long)m * p.hidden + cbase;
#pragma unroll
          for (int j = 0; j < NV; ++j) if (cbase + j < p.split) hp[j] = v[j];
        }
      }
    } else if constexpr (EPI == EPI_GRU_A) {
      // [z | r] logits -> z (fp32) and r*h (bf16) into the q-input buffer.
      const int hd = p.hidden;
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] = sigmoidf_(v[j]);
      if (cbase < hd) {
        store_f32<NV>((float*)p.zbuf + (long)m * hd + cbase, v);
      } else {
        const int hc = cbase - hd;
        float h[NV];
        load_f32<NV>(p.h32 + (long)m * hd + hc, h);
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] *= h[j];
        store_bf16<NV>((bf16*)p.y + (long)m * p.y_cstride + p.y_coff + hc, v);
      }
    } else if constexpr (EPI == EPI_GRU_B) {
      const int hd = p.hidden;
      float z[NV], h[NV];
      load_f32<NV>((const float*)p.zbuf + (long)m * hd + cbase, z);
      float* hp = p.h32 + (long)m * hd + cbase;
      load_f32<NV>(hp, h);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float q = tanhf_(v[j]);
        v[j] = (1.0f - z[j]) * h[j] + z[j] * q;
      }
      store_f32<NV>(hp, v);
      store_bf16<NV>((bf16*)p.y + (long)m * p.y_cstride + p.y_coff + cbase, v);
      if (p.y2) store_bf16<NV>((bf16*)p.y2 + (long)m * p.y2_cstride + p.y2_coff + cbase, v);
    } else if constexpr (EPI == EPI_FLOW) {
      if (cbase == 0) {
        const int rem = m % OHW;
        const int py = rem / p.OW;
        const int px = rem - py * p.OW;
        const float cx = p.coords[2 * (long)m] + v[0];
        const float cy = p.coords[2 * (long)m + 1] + v[1];
        p.coords[2 * (long)m] = cx;
        p.coords[2 * (long)m + 1] = cy;
        const float fx = cx - (float)px;
        const float fy = cy - (float)py;
        p.flow32[2 * (long)m] = fx;
        p.flow32[2 * (long)m + 1] = fy;
        bf16* yp = (bf16*)p.y + (long)m * p.y_cstride + p.y_coff;
        yp[0] = f2bf(fx); yp[1] = f2bf(fy);
        if (p.y2) {
          bf16* y2p = (bf16*)p.y2 + (long)m * p.y2_cstride + p.y2_coff;
          y2p[0] = f2bf(fx); y2p[1] = f2bf(fy);
        }
        if (p.y3) {
          bf16* y3p = (bf16*)p.y3 + (long)m * p.y3_cstride + p.y3_coff;
          y3p[0] = f2bf(fx); y3p[1] = f2bf(fy);
        }
      }
    }
  }
}

template <int BCO, int BP, int WCO>
int launch_cfg(const ConvParams* p, int epi, hipStream_t s) {
  dim3 grid((p->M + BP - 1) / BP, (p->cout + BCO - 1) / BCO);
  dim3 block(256);
  switch (epi) {
    case EPI_STD: hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, EPI_STD>), grid, block, 0, s, *p); break;
    case EPI_GRU_A: hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, EPI_GRU_A>), grid, block, 0, s, *p); break;
    case EPI_GRU_B: hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, EPI_GRU_B>), grid, block, 0, s, *p); break;
    case EPI_FLOW: hipLaunchKernelGGL((conv_igemm_kernel<BCO, BP, WCO, EPI_FLOW>), grid, block, 0, s, *p); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int jr_conv_forward(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  if (p->M <= 0) return 0;
  switch (cfg) {
    case 0: return launch_cfg<128, 128, 2>(p, epi, stream);
    case 1: return launch_cfg<64, 128, 1>(p, epi, stream);
    case 2: return launch_cfg<128, 64, 2>(p, epi, stream);
    case 3: return launch_cfg<16, 256, 1>(p, epi, stream);
    case 4: return launch_cfg<64, 64, 1>(p, epi, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
