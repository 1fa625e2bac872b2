// Halo 3x3 / stride-1 convolution: every 3x3 "same" conv of the reference RAFT
// (jax_raft/model.py:120-159 ConvNormActivation inside the encoders' residual /
// bottleneck blocks :162-216, the motion encoder :275-289, flow head :347-349, mask
// predictor :389-390) as an alternative tile kernel to the implicit GEMM.
//
// The implicit GEMM (conv_igemm.h) re-derives an im2col row descriptor for every staged
// row of every K stage; on the encoder shapes that per-tile address arithmetic, not MFMA
// or memory, bounds it (~1400 VALU + 1050 SALU per wave for 72 MFMAs, profiles/
// r3_encoder_conv_study.md).  Here a workgroup owns a TR x TC block of output pixels,
// loads its (TR + 2) x (TC + 2) input footprint into LDS once (zero outside the image; (TR + 3) x
// (TC + 3) for the 4x4 stem),
// and reads the B fragment of tap (u, v) for output pixel (i, j) from footprint row
// (i + u) * (TC + 2) + j + v: a constant offset per tap, no per-stage descriptors.  The
// weights stream per wave from L2 in MFMA fragment order (ops/native.py:pack_gru_halo,
// one contiguous 1 KB load per 32 x 16 fragment) through a register ring; each fragment
// feeds TN 32-pixel blocks (A bytes per MFMA = 1 KB / TN).
//
// Waves: WCO x WPX; wave (wc, wp) computes output channels co0 + 32 wc + [0, 32) for the
// pixel blocks wp * TN + [0, TN) of the tile.  Epilogue = EPI_STD of conv_igemm (bias,
// residual pre / post, relu, bf16 store + copy), plus optional per-channel (sum, sumsq)
// partials of the stored values for a following instance norm.
#include "halo.h"

namespace {

// Footprint image: pixel row r = fy * (TC + 2) + fx holds CIN channels in P 16-B chunks
// (P = 8 / 16 / 32 for CIN <= 64 / 128 / 256).  Chunk c of pixel (fy, fx) sits in slot
// c ^ kx(key) of its row, key = (fx + TC * fy) & 15: the 16 lanes of one ds_read_b128 lane
// group read 16 pixels of consecutive keys (lane_px below), so for every tap (a constant shift
// of fx / fy) they hit 16 distinct 16-B slots of the 256-B bank window.  With P = 8 two rows
// share a window: the row parity (fx & 1, TC + 2 even) picks the half, key >> 1 the slot.
template <int P>
JR_DEVICE constexpr int key_x(int key) { return P == 8 ? (key >> 1) & 7 : key & 15; }

// position of lane rho (0..31) in its 32-pixel block: the ds_read_b128 lane groups
// {0-3, 12-15, 20-27} and {4-11, 16-19, 28-31} get pixels 0..15 and 16..31 (guide: LDS table)
JR_DEVICE int lane_px(int rho) {
  return rho < 4 ? rho : rho < 12 ? rho + 12 : rho < 16 ? rho - 8 : rho < 20 ? rho + 8 : rho < 28 ? rho - 12 : rho;
}

template <int CIN>
constexpr int pitch_of() { return CIN <= 64 ? 8 : CIN <= 128 ? 16 : 32; }

// INN: the input is normalised (+ residual) while loading (p.in_stats set); a separate
// instantiation so the plain convs keep their register budget
// occupancy floors: the 64-channel configs 4 waves / SIMD (ring 8 deep, 120 VGPRs: encoder layer 1
// 44.2 -> 41.4 us, with stats 48.3 -> 43.5, profiles/r5_halo_l1_occupancy.txt; the normalising
// loader too, with its footprint loads in batches of 3 to fit: 52.9 -> 51.3 us with norm + stats,
// 58.4 -> 55.9 with the residual); the 96-channel normalising ones 3 (ring 8 deep: layer 2 with
// norm + stats 35.6 -> 30.3 us, profiles/r5_halo_l2_occupancy.txt; the same for the 128-channel
// ones measured slower); the other normalising small-tile configs 2 (without it they took 300-420
// VGPRs, one wave per SIMD).  The workgroup counts are the ones hipcc caps at these budgets
// without spilling.
template <int CIN, int WCO, int WPX, int TN, bool INN>
constexpr int halo_min_blocks() {
  return TN > 2 ? 1 : CIN <= 64 ? 4 : CIN <= 96 ? (INN ? 3 : 1) : !INN ? 1 : WCO * WPX == 1 ? 4 : WCO * WPX <= 4 ? 2 : 1;
}

// KS: the kernel size (3: every 3x3 / pad-1 conv; 4: the encoders' 7x7 / stride-2 stem as a 4x4 conv
// over the 2x2 space-to-depth input, pads 2 / 1, ops/native.py:s2d_stem_kernel)
template <int CIN, int WCO, int WPX, int TN, int TR, int TC, bool INN, int KS = 3>
__global__ __launch_bounds__(64 * WCO * WPX, (halo_min_blocks<CIN, WCO, WPX, TN, INN>()))
void conv_halo_kernel(const ConvHaloParams p) {
  constexpr int NT = 64 * WCO * WPX;
  constexpr int P = pitch_of<CIN>();
  constexpr int CC = CIN / 8;
  constexpr int SPT = CIN / 16;           // k-steps per tap
  constexpr int S = KS * KS * SPT;
  constexpr int PAD = KS / 2;             // top / left padding (the footprint's first row / column)
  // weight ring depth: 16 fragments, 8 for the 4-block waves at 2 waves / SIMD (256 VGPRs; each
  // fragment there feeds 4 MFMAs, so 8 in flight still cover ~1000 cycles of L2 latency)
  constexpr bool WIDE = TN >= 4 && WCO * WPX > 4;
  // 12- / 16-wave workgroups (3 / 4 waves per SIMD, <= 168 / 128 VGPRs): 8-deep rings too
  constexpr bool MANY = WCO * WPX >= 12;
  constexpr int PD = S >= 16 ? (WCO * WPX >= 16 ? 4 : (WIDE || MANY || CIN <= 96) ? 8 : 16) : S;   // (64 / 96 ch: 4 waves / SIMD)
  constexpr int FW = TC + KS - 1;
  constexpr int NFP = (TR + KS - 1) * FW;
  constexpr int RB = P * 16;              // footprint row bytes
  static_assert(TR * TC <= 32 * WPX * TN && (TC == 16 || TC == 8), "tile");
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  char* const lds_b = (char*)lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rho = lane & 31, hh = lane >> 5;
  const int wc = wave % WCO, wp = wave / WCO;

  const int per_img = p.tiles_y * p.tiles_x;
  const int n = blockIdx.x / per_img;
  const int rem = blockIdx.x - n * per_img;
  const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
  const int y0 = ty * TR, x0 = tx * TC;
  const int co_blk = blockIdx.y * WCO + wc;   // this wave's 32-channel output block

  // weight ring first (its latency overlaps the footprint load)
  const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.w_bytes, 0x00020000);
  const unsigned w_base = (unsigned)(co_blk * S * 64 + lane) * 16u;
  bf16x8 ring[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) ring[d] = __builtin_bit_cast(bf16x8, bload(ws, w_base + (unsigned)d * 1024u));

  // footprint -> LDS: batches of up to 16 loads per thread in flight; the input instance norm
  // (per-channel scale / shift of image n) and the optional residual are applied on the way, the
  // tile's own pixels optionally written back (xn)
  {
    const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.in_res, (short)0, (int)p.in_res_bytes, 0x00020000);
    constexpr int TOTAL = NFP * CC;
    constexpr int NL = (TOTAL + NT - 1) / NT;
    // the normalising loader holds the residual chunks too
    constexpr int NBMAX = MANY ? 4 : INN && CIN <= 64 ? 3 : INN || WIDE ? 8 : 16;
    constexpr int NBAT = NL < NBMAX ? NL : NBMAX;
    constexpr bool norm = INN;
    const bool resid = INN && p.in_res != nullptr;
    // Normalisation constants in registers: NT is a multiple of CC, so the 16-B chunk (8 channels)
    // a thread loads is the same for every footprint pixel it handles, c = tid % CC.  Scale / shift
    // of the input and of the residual (1 / 0 when it is not normalised), and the two relus as
    // max(v, lo) with lo = 0 or -inf: branch-free arithmetic per element instead of an LDS table
    // read per chunk (3-way bank conflicts) and per-element flag tests (profiles/
    // r5_halo_norm_pmc.txt: encoder layer 2 VALU / MFMA 13.5 -> 11.3, LDS conflicts 17 -> 3.6 %,
    // 38.2 -> 34.2 us; packed v_pk_fma_f32 pairs measured slower).
    static_assert(!INN || NT % CC == 0, "normalising loader: fixed chunk per thread");
    float na[8], nb[8], ra[8], rb[8];
    float lo_pre = 0.f, lo_post = 0.f;
    if constexpr (INN) {
      const int c = tid % CC;
      const float inv = 1.0f / (float)p.in_hw;
      auto coef = [&](const float* stt, float (&A)[8], float (&Bv)[8]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float* t = stt + ((long)n * CIN + 8 * c + j) * 2;
          const float mu = t[0] * inv;
          const float var = fmaxf(t[1] * inv - mu * mu, 0.f);
          A[j] = rsqrtf(var + p.in_eps);
          Bv[j] = -mu * A[j];
        }
      };
      coef(p.in_stats, na, nb);
      if (resid && p.in_res_stats != nullptr) {
        coef(p.in_res_stats, ra, rb);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { ra[j] = 1.f; rb[j] = 0.f; }
      }
      // in_relu bit 1: the relu of the block's last ConvNormActivation, before the residual add
      // (model.py:171-180: relu(x + relu(IN(conv2)))); bit 0: the relu after it
      lo_pre = (p.in_relu & 2) ? 0.f : -__builtin_inff();
      lo_post = (p.in_relu & 1) ? 0.f : -__builtin_inff();
    }
#pragma unroll
    for (int l0 = 0; l0 < NL; l0 += NBAT) {
      u32x4 v[NBAT], vr[NBAT];
      int dst[NBAT], pix[NBAT];
#pragma unroll
      for (int k = 0; k < NBAT; ++k) {
        const int idx = (l0 + k) * NT + tid;
        const int f = idx / CC, c = idx - f * CC;
        const int fy = f / FW, fx = f - fy * FW;
        const int y = y0 - PAD + fy, x = x0 - PAD + fx;
        const bool live = l0 + k < NL && idx < TOTAL;
        const bool in = live && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
        const int m = (n * p.H + y) * p.W + x;
        const unsigned off = (unsigned)m * (unsigned)p.xcs * 2u + (unsigned)(p.xoff + 8 * c) * 2u;
        v[k] = bload(xs, in ? off : HOOB);
        // zero (out-of-range read) without a residual: it then adds 0 * 1 + 0
        if (INN) vr[k] = bload(rs, in && resid ? (unsigned)m * (unsigned)p.in_rcs * 2u + (unsigned)(16 * c) : HOOB);
        // destination byte offset; bit 30: padding (stays zero through the norm), -1: none
        dst[k] = !live ? -1 : (f * RB + ((c ^ key_x<P>(fx + TC * fy)) << 4)) | (in ? 0 : 1 << 30) | (c << 20);
        // image pixel of a tile-own footprint pixel (xn write-back), else -1
        pix[k] = in && fy >= PAD && fy < PAD + TR && fx >= PAD && fx < PAD + TC ? m : -1;
      }
#pragma unroll
      for (int k = 0; k < NBAT; ++k) {
        if (dst[k] < 0) continue;
        if (norm && !(dst[k] >> 30)) {
          const int c = (dst[k] >> 20) & 63;
          bf16x8 e = __builtin_bit_cast(bf16x8, v[k]);
          const bf16x8 er = __builtin_bit_cast(bf16x8, vr[k]);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float fv = fmaxf(fmaf(bf2f(e[j]), na[j], nb[j]), lo_pre);
            fv = fmaxf(fv + fmaf(bf2f(er[j]), ra[j], rb[j]), lo_post);
            e[j] = f2bf(fv);
          }
          v[k] = __builtin_bit_cast(u32x4, e);
          if (p.xn && pix[k] >= 0) *(u32x4*)((bf16*)p.xn + (long)pix[k] * p.xncs + 8 * c) = v[k];
        }
        *(u32x4*)(lds_b + (dst[k] & 0xfffff)) = v[k];
      }
    }
  }

  // this lane's output pixels: byte offset of footprint row of tap (0, 0), its key, image pixel
  int rb0[TN], key0[TN], om[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int q = 32 * (wp * TN + b) + lane_px(rho);
    const int i = q / TC, j = q - i * TC;
    const bool ok = i < TR && y0 + i < p.H && x0 + j < p.W;
    rb0[b] = ok ? (i * FW + j) * RB : 0;
    key0[b] = ok ? j + TC * i : 0;
    om[b] = ok ? (n * p.H + y0 + i) * p.W + x0 + j : -1;
  }
  __syncthreads();

  f32x16 acc[TN];
  pipe_gemm<TN, S, PD>(
      acc, ring,
      [&](int s) { return __builtin_bit_cast(bf16x8, bload(ws, w_base + (unsigned)s * 1024u)); },
      [&](int s, int b) {
        const int tap = s / SPT, kc = s - tap * SPT;
        const int u = tap / KS, v = tap % KS;
        // slot of chunk 2 kc + hh: (2 kc) ^ (kx ^ hh); the tap's row shift is an immediate offset
        const int kxh = (key_x<P>(key0[b] + v + TC * u) ^ hh) << 4;
        return *(const bf16x8*)(lds_b + (rb0[b] + (((2 * kc) << 4) ^ kxh)) + (u * FW + v) * RB);
      });
  // epilogue: lane holds channels c0 .. c0 + 15 of pixel om[b]
  const int c0 = 32 * co_blk + 16 * hh;
  if (c0 >= p.cout) return;
  const bool full = c0 + 16 <= p.cout;
  float bv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) bv[k] = c0 + k < p.cout ? p.bias[c0 + k] : 0.f;
  float ssum[16], ssq[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) ssum[k] = ssq[k] = 0.f;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int m = om[b];
    if (m < 0) continue;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = acc[b][k] + bv[k];
    float r[16];
    if (p.res) {
      const bf16* rp = (const bf16*)p.res + (long)m * p.rcs + p.roff + c0;
      if (full) load_bf16<16>(rp, r);
      else {
#pragma unroll
        for (int k = 0; k < 16; ++k) r[k] = c0 + k < p.cout ? bf2f(rp[k]) : 0.f;
      }
      if (!p.res_post) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] += r[k];
      }
    }
    if (p.act == ACT_RELU) {
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = fmaxf(v[k], 0.f);
    }
    if (p.res && p.res_post) {
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = fmaxf(v[k] + r[k], 0.f);
    }
    bf16* yp = (bf16*)p.y + (long)m * p.ycs + p.yoff + c0;
    bf16* y2p = p.y2 ? (bf16*)p.y2 + (long)m * p.y2cs + p.y2off + c0 : nullptr;
    if (full) {
      store_bf16<16>(yp, v);
      if (y2p) store_bf16<16>(y2p, v);
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (c0 + k < p.cout) {
          yp[k] = f2bf(v[k]);
          if (y2p) y2p[k] = f2bf(v[k]);
        }
    }
    if (p.stats_part) {   // statistics of the stored (bf16-rounded) values, as channel_stats reads them
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float s = bf2f(f2bf(v[k]));
        ssum[k] += s;
        ssq[k] += s * s;
      }
    }
  }
  if (p.stats_part) {
    // sum over the 32 pixel lanes of each lane half (channels 16 hh + k) as a transposing
    // butterfly: every exchange step hands the partner half of the channels the lane still
    // carries, so 2 x (8 + 4 + 2 + 1 + 1) exchanges replace 2 x 16 x 5 lane shuffles (the 5-step
    // all-reduce per channel cost +16 us on the encoder's 64-channel layer, profiles/
    // r5_halo_epi_costs.txt).  Only the first step crosses a 16-lane row (ds_swizzle); the
    // others are DPP row permutes whose pairing (xor 15, xor 7, xor 2, xor 1) flips the bit
    // that picks the half.  Lane rho ends with channel 8 b4 + 4 b3 + 2 b2 + b1 (b = bits of rho).
    const int b4 = (rho >> 4) & 1, b3 = (rho >> 3) & 1, b2 = (rho >> 2) & 1, b1 = (rho >> 1) & 1;
    auto swz16 = [](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401F)); };
    auto dpp = [](float v, auto ctrl) {
      return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), decltype(ctrl)::value, 0xF, 0xF, false));
    };
    using Mirror = std::integral_constant<int, 0x140>;
    using HalfMirror = std::integral_constant<int, 0x141>;
    using Xor2 = std::integral_constant<int, 0x4E>;
    using Xor1 = std::integral_constant<int, 0xB1>;
    float s8[8], q8[8], s4[4], q4[4], s2[2], q2[2];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s8[j] = (b4 ? ssum[8 + j] : ssum[j]) + swz16(b4 ? ssum[j] : ssum[8 + j]);
      q8[j] = (b4 ? ssq[8 + j] : ssq[j]) + swz16(b4 ? ssq[j] : ssq[8 + j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s4[j] = (b3 ? s8[4 + j] : s8[j]) + dpp(b3 ? s8[j] : s8[4 + j], Mirror{});
      q4[j] = (b3 ? q8[4 + j] : q8[j]) + dpp(b3 ? q8[j] : q8[4 + j], Mirror{});
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      s2[j] = (b2 ? s4[2 + j] : s4[j]) + dpp(b2 ? s4[j] : s4[2 + j], HalfMirror{});
      q2[j] = (b2 ? q4[2 + j] : q4[j]) + dpp(b2 ? q4[j] : q4[2 + j], HalfMirror{});
    }
    float s1 = (b1 ? s2[1] : s2[0]) + dpp(b1 ? s2[0] : s2[1], Xor2{});
    float q1 = (b1 ? q2[1] : q2[0]) + dpp(b1 ? q2[0] : q2[1], Xor2{});
    s1 += dpp(s1, Xor1{});
    q1 += dpp(q1, Xor1{});
    const int ch = 8 * b4 + 4 * b3 + 2 * b2 + b1;
    if ((rho & 1) == 0 && c0 + ch < p.cout) {
      const int nb = per_img * WPX;
      float* o = p.stats_part + (((long)n * nb + rem * WPX + wp) * p.cout + c0 + ch) * 2;
      *(float2*)o = make_float2(s1, q1);
    }
  }
}

struct HaloCfg {
  int cin, wco, wpx, tn, tr, tc;
  int ks = 3;
};

// tile configs (cfg id = index): encoder shapes (64 / 96 / 128 channels, large pixel tiles
// sharing each weight fragment across 2-4 pixel blocks) and the refinement loop's 128 / 256-
// channel convs at batch 1 (small tiles: 7040 pixels must still give >= 256 workgroups)
constexpr HaloCfg kCfgs[] = {
    {64, 2, 2, 4, 16, 16},  {64, 2, 2, 2, 8, 16},  {96, 3, 2, 2, 8, 16},  {96, 3, 1, 2, 4, 16},
    {128, 4, 2, 2, 8, 16},  {128, 4, 1, 2, 4, 16}, {128, 2, 2, 2, 8, 16}, {128, 2, 1, 1, 4, 8},
    {256, 2, 2, 2, 8, 16},  {256, 2, 1, 1, 4, 8},  {128, 4, 1, 1, 4, 8},  {256, 4, 1, 1, 4, 8},
    {256, 2, 1, 2, 4, 16},
    // all output channels of a loop conv in one workgroup, 128-pixel tiles (batch >= 4): the
    // footprint is loaded once for every channel and each 1 KB weight fragment feeds 4 MFMAs, so
    // the per-CU weight stream from L2 (the bound of the 64-pixel / 64-channel tiles) is 1/4 of it
    {256, 6, 1, 4, 8, 16},  {256, 4, 1, 4, 8, 16},  {128, 8, 1, 4, 8, 16},  {128, 2, 1, 4, 8, 16},
    {256, 6, 1, 2, 4, 16},  {256, 4, 1, 2, 4, 16},
    // one 32-channel block per workgroup, 128-pixel tiles (batch 1): a CU streams 1/6 - 1/8 of the
    // weights a whole-cout tile needs (the per-CU L2 stream bounds the 7040-pixel loop convs), the
    // footprint is re-read per channel block from L2 instead
    {256, 1, 2, 2, 8, 16},  {256, 1, 4, 1, 8, 16},  {128, 1, 2, 2, 8, 16},  {128, 1, 4, 1, 8, 16},
    // the space-to-depth stem (4x4 over 16 input channels, 64 outputs)
    {16, 2, 2, 2, 8, 16, 4},  {16, 2, 2, 4, 16, 16, 4},
    // round 6: 128-pixel tiles with 2-block waves split over the pixels (WPX = 2), so every SIMD
    // holds the same number of waves (the 6-wave whole-cout tiles above leave two SIMDs with
    // twice the MFMAs of the other two), and 256-pixel tiles for the 128-channel convs
    {256, 6, 2, 2, 8, 16},  {256, 4, 2, 2, 8, 16},  {128, 8, 2, 2, 8, 16},  {128, 4, 2, 4, 16, 16},
    {128, 2, 4, 2, 16, 16},
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

int lds_bytes(const HaloCfg& c) {
  const int P = c.cin <= 64 ? 8 : c.cin <= 128 ? 16 : 32;
  return (c.tr + c.ks - 1) * (c.tc + c.ks - 1) * P * 16 + c.cin * 16;   // footprint (+ slack)
}

template <int CIN, int WCO, int WPX, int TN, int TR, int TC, bool INN, int KS>
int launch_v(const ConvHaloParams& p, hipStream_t s, int lds) {
  static const bool attr = hipFuncSetAttribute((const void*)conv_halo_kernel<CIN, WCO, WPX, TN, TR, TC, INN, KS>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!attr) return (int)hipErrorInvalidValue;
  const int cpad = (p.cout + 32 * WCO - 1) / (32 * WCO);
  hipLaunchKernelGGL((conv_halo_kernel<CIN, WCO, WPX, TN, TR, TC, INN, KS>), dim3(p.ntiles, cpad), dim3(64 * WCO * WPX), lds,
                     s, p);
  return (int)hipGetLastError();
}

template <int CIN, int WCO, int WPX, int TN, int TR, int TC, int KS = 3>
int launch(const ConvHaloParams& p, hipStream_t s, int lds) {
  if (p.TR != TR || p.TC != TC) return (int)hipErrorInvalidValue;
  return p.in_stats ? launch_v<CIN, WCO, WPX, TN, TR, TC, true, KS>(p, s, lds)
                    : launch_v<CIN, WCO, WPX, TN, TR, TC, false, KS>(p, s, lds);
}

}  // namespace

extern "C" int jr_conv_halo_cfg(int cfg, int* o) {
  if (cfg < 0 || cfg >= kNumCfgs) return 0;
  const HaloCfg& c = kCfgs[cfg];
  o[0] = c.cin; o[1] = c.wco; o[2] = c.wpx; o[3] = c.tn; o[4] = c.tr; o[5] = c.tc;
  return 1;
}

extern "C" int jr_conv_halo_lds(int cfg) { return cfg < 0 || cfg >= kNumCfgs ? 0 : lds_bytes(kCfgs[cfg]); }

extern "C" int jr_conv_halo_ks(int cfg) { return cfg < 0 || cfg >= kNumCfgs ? 0 : kCfgs[cfg].ks; }

extern "C" int jr_conv_halo(const ConvHaloParams* p, int cfg, hipStream_t stream) {
  if (cfg < 0 || cfg >= kNumCfgs || p->ntiles <= 0) return (int)hipErrorInvalidValue;
  const HaloCfg& c = kCfgs[cfg];
  const int lds = lds_bytes(c);
#define JR_HALO_CONV(CIN_, WCO_, WPX_, TN_, TR_, TC_) \
  if (c.ks == 3 && c.cin == CIN_ && c.wco == WCO_ && c.wpx == WPX_ && c.tn == TN_ && c.tr == TR_ && c.tc == TC_) \
    return launch<CIN_, WCO_, WPX_, TN_, TR_, TC_>(*p, stream, lds);
#define JR_HALO_CONV4(CIN_, WCO_, WPX_, TN_, TR_, TC_) \
  if (c.ks == 4 && c.cin == CIN_ && c.wco == WCO_ && c.wpx == WPX_ && c.tn == TN_ && c.tr == TR_ && c.tc == TC_) \
    return launch<CIN_, WCO_, WPX_, TN_, TR_, TC_, 4>(*p, stream, lds);
  JR_HALO_CONV(64, 2, 2, 4, 16, 16) JR_HALO_CONV(64, 2, 2, 2, 8, 16) JR_HALO_CONV(96, 3, 2, 2, 8, 16)
  JR_HALO_CONV(96, 3, 1, 2, 4, 16) JR_HALO_CONV(128, 4, 2, 2, 8, 16) JR_HALO_CONV(128, 4, 1, 2, 4, 16)
  JR_HALO_CONV(128, 2, 2, 2, 8, 16) JR_HALO_CONV(128, 2, 1, 1, 4, 8) JR_HALO_CONV(256, 2, 2, 2, 8, 16)
  JR_HALO_CONV(256, 2, 1, 1, 4, 8) JR_HALO_CONV(128, 4, 1, 1, 4, 8) JR_HALO_CONV(256, 4, 1, 1, 4, 8)
  JR_HALO_CONV(256, 2, 1, 2, 4, 16) JR_HALO_CONV(256, 6, 1, 4, 8, 16) JR_HALO_CONV(256, 4, 1, 4, 8, 16)
  JR_HALO_CONV(128, 8, 1, 4, 8, 16) JR_HALO_CONV(128, 2, 1, 4, 8, 16) JR_HALO_CONV(256, 6, 1, 2, 4, 16)
  JR_HALO_CONV(256, 4, 1, 2, 4, 16) JR_HALO_CONV(256, 1, 2, 2, 8, 16) JR_HALO_CONV(256, 1, 4, 1, 8, 16)
  JR_HALO_CONV(128, 1, 2, 2, 8, 16) JR_HALO_CONV(128, 1, 4, 1, 8, 16)
  JR_HALO_CONV(256, 6, 2, 2, 8, 16) JR_HALO_CONV(256, 4, 2, 2, 8, 16) JR_HALO_CONV(128, 8, 2, 2, 8, 16)
  JR_HALO_CONV(128, 4, 2, 4, 16, 16) JR_HALO_CONV(128, 2, 4, 2, 16, 16)
  JR_HALO_CONV4(16, 2, 2, 2, 8, 16) JR_HALO_CONV4(16, 2, 2, 4, 16, 16)
#undef JR_HALO_CONV4
#undef JR_HALO_CONV
  return (int)hipErrorInvalidValue;
}
