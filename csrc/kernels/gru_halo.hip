// Halo-tiled fused ConvGRU stage (reference jax_raft/model.py:293-312 ConvGRU,
// :315-334 RecurrentBlock) for every map size and both RAFT recurrent blocks:
//
//   z, r = sigmoid(conv_zr([h | x]) + ctx_zr)        GEMM 1
//   q    = tanh(conv_q([r h | x]) + ctx_q)           GEMM 2
//   h'   = (1 - z) h + z q
//
// (ctx_* = the loop-invariant context share of the gates + their biases, a per-pixel
// bias map computed once in the prologue, runtime/engine.py.)
//
// Geometry.  A workgroup owns an output tile (mode 0: a run of L pixels along the
// tap axis of raft_large's 1x5 / 5x1 stages; mode 1: a TR x TC block for
// raft_small's 3x3 GRU).  GEMM 2 needs r*h on the tile's halo region (tile + the
// conv's reach: +-2 along the run / +-1 around the block), so r is recomputed there
// (GEMM 1 runs on the region, z only on the tile) and r*h is written to an LDS image
// that GEMM 2 reads shifted by the tap.  All of [h | x] the tile touches (the region
// + another reach: the "footprint", <= 132 x 256 channels) is loaded into LDS once,
// so both GEMMs read their B fragments from LDS; only the weights stream, from L2
// straight into the MFMA A registers through a ring PD k-steps deep (fragment-
// ordered packing: one contiguous 1 KB wave load per 32 x 16 A fragment).
//
// Waves: 2 hd / 32 (8 for raft_large, 6 for raft_small).  GEMM 1: wave w owns
// output-channel block w of [z | r] (the first half z: on the tile's pixels; the
// second half r: on the region's).  GEMM 2: the z waves compute q block w over the
// r*h part of K, the r waves the same q block over the x part; the r waves hand their
// fp32 partial sums over through LDS and the z waves -- which hold z for exactly those
// (channel, pixel) fragments in registers -- finish tanh + blend.  No z / r*h global
// round trip and one launch per stage at any batch (tiles sized to fill the 256 CUs:
// a batch-1 440x1024 frame gives 220-275 of them).
//
// h' is written to a buffer other than hsrc: neighbouring tiles read this tile's h.
//
// MFMA: v_mfma_f32_32x32x16_bf16 (A = weights, 32 channels; B = 32 pixels).  The
// packed weight rows are permuted so that accumulator register i of lane half hh
// is channel 16 hh + i: every epilogue lane owns 16 contiguous channels of one pixel.
#include "halo.h"

namespace {

// tile geometry of one workgroup (all wave-uniform)
struct Tile {
  int n, y0, x0, line, s0;
  int FW, RW;           // footprint / region row widths (mode 0: one row)
  int nreg, nout;       // region / output pixels
};

template <int HD, int CIN, int MODE, int NB1, int NB2>
struct Halo {
  static constexpr int NHB = HD / 32;           // channel blocks per gate
  static constexpr int NW = 2 * NHB;            // waves
  static constexpr int NT = NW * 64;
  static constexpr int TAPS = MODE == 0 ? 5 : 9;
  static constexpr int CC = CIN / 8;            // 16-B chunks per footprint pixel
  static constexpr int HC = HD / 8;             // chunks of h
  static constexpr int SPT = CIN / 16;          // GEMM 1 k-steps per tap
  static constexpr int KS = TAPS * SPT;         // k-steps of both packed weights
  static constexpr int SRH = HD / 16;           // GEMM 2 k-steps per tap: r*h part
  static constexpr int SX = (CIN - HD) / 16;    //                          x part
  // weight ring depths (k-steps = 1 KB loads in flight per wave): the stream from L2 is this
  // kernel's bound at batch 1 (Little's law: bytes in flight / L2 latency under load)
  // (4-block outputs at 2 waves / SIMD: shallower rings keep the 256-VGPR budget without spills)
  static constexpr int PD1 = NB1 + NB2 <= 3 ? 24 : NB1 >= 5 ? 6 : NB2 >= 4 ? 8 : 16;
  static constexpr int PD2 = NB2 >= 4 ? 6 : NB2 >= 2 ? (HD == 96 ? 8 : 12) : 16;
  static_assert(CIN % 16 == 0 && HD % 32 == 0 && CC <= 32 && HC <= 16 && SRH == SX, "geometry");
};

template <int HD, int CIN, int MODE, int NB1, int NB2>
__global__ __launch_bounds__(4 * HD) void gru_halo_kernel(const GruHaloParams p) {
  using C = Halo<HD, CIN, MODE, NB1, NB2>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rho = lane & 31, hh = lane >> 5;

  // ------------------------------------------------------------ tile geometry
  Tile t;
  {
    const int per_img = p.tiles_y * p.tiles_x;
    const int b = blockIdx.x;
    t.n = b / per_img;
    const int rem = b - t.n * per_img;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    if (MODE == 0) {
      t.line = ty;
      t.s0 = tx * p.TC;
      t.FW = p.TC + 8;
      t.RW = p.TC + 4;
      t.nreg = p.TC + 4;
      t.nout = p.TC;
      t.y0 = t.x0 = 0;
    } else {
      t.y0 = ty * p.TR;
      t.x0 = tx * p.TC;
      t.FW = p.TC + 4;
      t.RW = p.TC + 2;
      t.nreg = (p.TR + 2) * (p.TC + 2);
      t.nout = p.TR * p.TC;
      t.line = t.s0 = 0;
    }
  }
  const int nfp = MODE == 0 ? p.TC + 8 : (p.TR + 4) * (p.TC + 4);
  const int HW = p.H * p.W;
  // image pixel of a footprint / region / output index (-1 outside the image or the tile)
  auto pix1d = [&](int pos) -> int {
    const int len = p.axis ? p.H : p.W;
    if ((unsigned)pos >= (unsigned)len) return -1;
    return p.axis ? t.n * HW + pos * p.W + t.line : t.n * HW + t.line * p.W + pos;
  };
  auto pix2d = [&](int y, int x) -> int {
    if ((unsigned)y >= (unsigned)p.H || (unsigned)x >= (unsigned)p.W) return -1;
    return t.n * HW + y * p.W + x;
  };
  auto fpix = [&](int f) -> int {
    if (MODE == 0) return pix1d(t.s0 - 4 + f);
    const int c = f / t.FW, d = f - c * t.FW;
    return pix2d(t.y0 - 2 + c, t.x0 - 2 + d);
  };

  bf16* const F = lds;                              // footprint image [nfp][256]
  const int f_rows = MODE == 0 ? p.TC + 8 : (p.TR + 4) * (p.TC + 4);
  const int f_elems = max(f_rows * FPITCH, C::NHB * NB2 * 4 * 256 * 2);   // P (fp32 partials) aliases F
  bf16* const R = lds + ((f_elems + 7) & ~7);       // r*h image [32 NB1][128]
  float* const P = (float*)lds;

  const __amdgpu_buffer_rsrc_t hs = __builtin_amdgcn_make_buffer_rsrc((void*)p.hsrc, (short)0, (int)p.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc((void*)p.xsrc, (short)0, (int)p.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t was = __builtin_amdgcn_make_buffer_rsrc((void*)p.wa, (short)0, (int)p.wa_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wbs = __builtin_amdgcn_make_buffer_rsrc((void*)p.wb, (short)0, (int)p.wb_bytes, 0x00020000);

  // ------------------------------------------------ GEMM 1 weight ring: first loads
  const bool zwave = wave < C::NHB;
  const unsigned wa_base = (unsigned)(wave * C::KS * 64 + lane) * 16u;
  bf16x8 ring[C::PD1];
#pragma unroll
  for (int d = 0; d < C::PD1; ++d) ring[d] = __builtin_bit_cast(bf16x8, bload(was, wa_base + (unsigned)d * 1024u));

  // ------------------------------------------------ footprint -> LDS (zero outside the image)
  {
    auto fill = [&](const __amdgpu_buffer_rsrc_t& rs, int c_lo, int c_n) {
      const int total = nfp * c_n;
      for (int base = 0; base < total; base += 4 * C::NT) {
        u32x4 v[4];
        int fr[4], ch[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int idx = base + k * C::NT + tid;
          const int f = idx / c_n, c = c_lo + (idx - f * c_n);
          fr[k] = idx < total ? f : -1;
          ch[k] = c;
          const int m = idx < total ? fpix(f) : -1;
          v[k] = bload(rs, m >= 0 ? (unsigned)m * (unsigned)p.cs * 2u + (unsigned)c * 16u : HOOB);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (fr[k] >= 0) *(u32x4*)(F + f_off(fr[k], ch[k])) = v[k];
      }
    };
    fill(hs, 0, C::HC);
    fill(xs, C::HC, C::CC - C::HC);
  }

  // ------------------------------------------------ per-lane pixel rows
  // output pixels (GEMM 1 of z, GEMM 2, epilogue 2): F row of the pixel's centre, R row of
  // its tap-0 neighbour, image pixel
  int of[NB2], orr[NB2], om[NB2];
#pragma unroll
  for (int b = 0; b < NB2; ++b) {
    const int q = 32 * b + rho;
    const bool ok = q < t.nout;
    if (MODE == 0) {
      of[b] = ok ? q + 4 : 4;
      orr[b] = ok ? q : 0;
      om[b] = ok ? pix1d(t.s0 + q) : -1;
    } else {
      const int i = q / p.TC, j = q - i * p.TC;
      of[b] = ok ? (i + 2) * t.FW + (j + 2) : t.FW + 1;
      orr[b] = ok ? i * t.RW + j : 0;
      om[b] = ok ? pix2d(t.y0 + i, t.x0 + j) : -1;
    }
  }
  // region pixels (GEMM 1 of r, epilogue 1): F row of tap 0, image pixel
  int rf[NB1], rm[NB1];
#pragma unroll
  for (int b = 0; b < NB1; ++b) {
    const int g = 32 * b + rho;
    const bool ok = g < t.nreg;
    if (MODE == 0) {
      rf[b] = ok ? g : 0;
      rm[b] = ok ? pix1d(t.s0 - 2 + g) : -1;
    } else {
      const int a = g / t.RW, c = g - a * t.RW;
      rf[b] = ok ? a * t.FW + c : 0;
      rm[b] = ok ? pix2d(t.y0 - 1 + a, t.x0 - 1 + c) : -1;
    }
  }
  // tap offsets (compile-time tap): footprint rows / r*h rows
  auto tapF = [&](int tap) { return MODE == 0 ? tap : (tap / 3) * t.FW + tap % 3; };
  auto tapR = [&](int tap) { return MODE == 0 ? tap : (tap / 3) * t.RW + tap % 3; };
  // the z lanes read the footprint at their output pixel's tap-0 neighbour: centre - reach
  const int zoff = MODE == 0 ? -2 : -(t.FW + 1);

  __syncthreads();   // footprint complete

  // ------------------------------------------------------------------ GEMM 1
  // wave w: block w of [z | r] (z: the tile's NB2 pixel blocks, r: the region's NB1)
  auto loadA1 = [&](int st) { return __builtin_bit_cast(bf16x8, bload(was, wa_base + (unsigned)st * 1024u)); };
  auto gemm1 = [&](auto nbc, const int (&rows)[decltype(nbc)::value], int roff, f32x16 (&acc)[decltype(nbc)::value]) {
    constexpr int NB = decltype(nbc)::value;
    pipe_gemm<NB, C::KS, C::PD1>(acc, ring, loadA1, [&](int st, int b) {
      const int tap = st / C::SPT, kc = st - tap * C::SPT;
      return *(const bf16x8*)(F + f_off(rows[b] + roff + tapF(tap), 2 * kc + hh));
    });
  };

  const int c0 = (wave % C::NHB) * 32 + 16 * hh;   // this lane's 16 channels within its gate
  // bias-map chunks (bf16, 16 channels = 2 x 16 B) of an epilogue, loaded ahead of the GEMM that
  // precedes it; unconditional (pixel clamped): a branch around a load makes hipcc drain vmcnt
  auto map_pre = [&](int m, int coff, u32x4 (&r)[2]) {
    const u32x4* q = (const u32x4*)((const bf16*)p.bmap + (long)(m >= 0 ? m : 0) * p.bmap_cs + coff);
    r[0] = q[0];
    r[1] = q[1];
  };
  auto map_f = [](const u32x4 (&r)[2], float* v) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = bf2f(__builtin_bit_cast(bf16x8, r[0])[k]);
      v[8 + k] = bf2f(__builtin_bit_cast(bf16x8, r[1])[k]);
    }
  };
  float zreg[NB2][16];
  // epilogue 1 of the z waves: z = sigmoid(acc + map) kept in registers for the blend
  auto epi_z = [&](const f32x16 (&acc)[NB2], const u32x4 (&bm)[NB2][2]) {
#pragma unroll
    for (int b = 0; b < NB2; ++b) {
      float bv[16];
      map_f(bm[b], bv);
#pragma unroll
      for (int k = 0; k < 16; ++k) zreg[b][k] = sigmoidf_(acc[b][k] + bv[k]);
      if (p.zo && om[b] >= 0) store_bf16<16>((bf16*)p.zo + (long)om[b] * HD + c0, zreg[b]);   // training: z
    }
  };
  // epilogue 1 of the r waves: r*h (h = the bf16 loop state of the footprint) -> R, zero outside
  // the image
  auto epi_r = [&](const f32x16 (&acc)[NB1], const u32x4 (&bm)[NB1][2]) {
#pragma unroll
    for (int b = 0; b < NB1; ++b) {
      const int g = 32 * b + rho;
      float bv[16], hv[16];
      map_f(bm[b], bv);
      const int fc = rf[b] + (MODE == 0 ? 2 : t.FW + 1);   // the region pixel's own footprint row
      const bf16x8 h0 = *(const bf16x8*)(F + f_off(fc, c0 >> 3));
      const bf16x8 h1 = *(const bf16x8*)(F + f_off(fc, (c0 >> 3) + 1));
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        hv[k] = bf2f(h0[k]);
        hv[8 + k] = bf2f(h1[k]);
      }
      bf16x8 o0, o1;
      const bool in = rm[b] >= 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o0[k] = f2bf(in ? sigmoidf_(acc[b][k] + bv[k]) * hv[k] : 0.f);
        o1[k] = f2bf(in ? sigmoidf_(acc[b][8 + k] + bv[8 + k]) * hv[8 + k] : 0.f);
      }
      *(bf16x8*)(R + r_off(g, c0 >> 3)) = o0;
      *(bf16x8*)(R + r_off(g, (c0 >> 3) + 1)) = o1;
      if (p.ro && in) {   // training: r and r*h of the tile's own pixels (the region minus the halo)
        const bool own = MODE == 0 ? (g >= 2 && g - 2 < t.nout)
                                   : (g / t.RW >= 1 && g / t.RW <= p.TR && g % t.RW >= 1 && g % t.RW <= p.TC);
        if (own) {
          float rv[16];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            rv[k] = sigmoidf_(acc[b][k] + bv[k]);
            rv[8 + k] = sigmoidf_(acc[b][8 + k] + bv[8 + k]);
          }
          store_bf16<16>((bf16*)p.ro + (long)rm[b] * HD + c0, rv);
          bf16* rp = (bf16*)p.rh + (long)rm[b] * p.rh_cs + c0;
          *(bf16x8*)rp = o0;
          *(bf16x8*)(rp + 8) = o1;
        }
      }
    }
  };
  if constexpr (NB1 == NB2) {
    // one GEMM body for both wave kinds (two identical bodies in the two branches of a wave-
    // uniform `if` get merged by hipcc's CFG simplification into one that spills)
    int rows[NB1], pm[NB1];
#pragma unroll
    for (int b = 0; b < NB1; ++b) {
      rows[b] = zwave ? of[b] + zoff : rf[b];
      pm[b] = zwave ? om[b] : rm[b];
    }
    u32x4 bm[NB1][2];
#pragma unroll
    for (int b = 0; b < NB1; ++b) map_pre(pm[b], (zwave ? 0 : HD) + c0, bm[b]);
    f32x16 acc[NB1];
    gemm1(std::integral_constant<int, NB1>{}, rows, 0, acc);
    if (zwave) epi_z(acc, bm);
    else epi_r(acc, bm);
  } else if (zwave) {
    u32x4 bm[NB2][2];
#pragma unroll
    for (int b = 0; b < NB2; ++b) map_pre(om[b], c0, bm[b]);
    f32x16 acc[NB2];
    gemm1(std::integral_constant<int, NB2>{}, of, zoff, acc);
    epi_z(acc, bm);
  } else {
    u32x4 bm[NB1][2];
#pragma unroll
    for (int b = 0; b < NB1; ++b) map_pre(rm[b], HD + c0, bm[b]);
    f32x16 acc[NB1];
    gemm1(std::integral_constant<int, NB1>{}, rf, 0, acc);
    epi_r(acc, bm);
  }

  // ------------------------------------------------------------------ GEMM 2
  // q block qb = wave % NHB; z waves: the r*h k-steps (B from R), r waves: the x k-steps
  // (B from F).  Weight k-step of (tap, j): tap * SPT + j (r*h) / tap * SPT + SRH + j (x).
  const int qb = wave % C::NHB;
  const unsigned wb_base = (unsigned)(qb * C::KS * 64 + lane) * 16u;
  constexpr int S2 = C::TAPS * C::SRH;
  auto kstep2 = [&](int s) { return (s / C::SRH) * C::SPT + (zwave ? 0 : C::SRH) + s % C::SRH; };
  bf16x8 ring2[C::PD2];
#pragma unroll
  for (int d = 0; d < C::PD2; ++d)
    ring2[d] = __builtin_bit_cast(bf16x8, bload(wbs, wb_base + (unsigned)kstep2(d) * 1024u));
  f32x16 acc2[NB2];

  // epilogue 2 operands of the z waves, loaded ahead of GEMM 2: the q bias map, and (NB2 <= 2)
  // the fp32 state of the output pixels
  constexpr bool PRE_H = NB2 <= 2;
  constexpr bool PRE_Q = NB2 <= 3;   // 4-block tiles: the q bias map is read in the epilogue (VGPRs)
  u32x4 bq[PRE_Q ? NB2 : 1][2];
  f32x4 hpre[PRE_H ? NB2 : 1][4];
  if (zwave) {
#pragma unroll
    for (int b = 0; b < NB2; ++b) {
      if constexpr (PRE_Q) map_pre(om[b], 2 * HD + c0, bq[b]);
      if constexpr (PRE_H) {
        const f32x4* hq = (const f32x4*)((p.h32in ? p.h32in : p.h32) + (long)(om[b] >= 0 ? om[b] : 0) * HD + c0);
#pragma unroll
        for (int k = 0; k < 4; ++k) hpre[b][k] = hq[k];
      }
    }
  }

  __syncthreads();   // r*h image complete

  auto loadA2 = [&](int st) { return __builtin_bit_cast(bf16x8, bload(wbs, wb_base + (unsigned)kstep2(st) * 1024u)); };
  {
    // z waves: r*h rows of R; r waves: x rows of F -- one body, the image base and row per wave
    const bf16* img = zwave ? R : F;
    int rows2[NB2];
#pragma unroll
    for (int b = 0; b < NB2; ++b) rows2[b] = zwave ? orr[b] : of[b] + zoff;
    const int pitch = zwave ? RPITCH : FPITCH;
    const int cbase = zwave ? 0 : C::HC;
    const int tstride = MODE == 0 ? 0 : (zwave ? t.RW : t.FW);
    pipe_gemm<NB2, S2, C::PD2>(acc2, ring2, loadA2, [&](int st, int b) {
      const int tap = st / C::SRH, j = st - tap * C::SRH;
      const int row = rows2[b] + (MODE == 0 ? tap : (tap / 3) * tstride + tap % 3);
      const int ch = cbase + 2 * j + hh;
      return *(const bf16x8*)(img + row * pitch + (((ch & 16) | ((ch ^ row) & 15)) << 3));
    });
  }

  __syncthreads();   // every footprint read done: P may overwrite F
  if (!zwave) {
    const int w2 = wave - C::NHB;
#pragma unroll
    for (int b = 0; b < NB2; ++b)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        *(f32x4*)(P + (((w2 * NB2 + b) * 4 + q4) * 64 + lane) * 4) =
            f32x4{acc2[b][4 * q4], acc2[b][4 * q4 + 1], acc2[b][4 * q4 + 2], acc2[b][4 * q4 + 3]};
  }
  __syncthreads();
  if (!zwave) return;

  // ------------------------------------------------------------ epilogue 2
#pragma unroll
  for (int b = 0; b < NB2; ++b) {
    const int m = om[b];
    if (m < 0) continue;
    float bv[16], h[16], v[16];
    if constexpr (PRE_Q) {
      map_f(bq[b], bv);
    } else {
      u32x4 bqe[2];
      map_pre(m, 2 * HD + c0, bqe);
      map_f(bqe, bv);
    }
    float* hp = p.h32 + (long)m * HD + c0;
    if constexpr (PRE_H) {
#pragma unroll
      for (int k = 0; k < 16; ++k) h[k] = hpre[b][k >> 2][k & 3];
    } else {
      load_f32<16>(p.h32in ? p.h32in + (long)m * HD + c0 : hp, h);
    }
    float qv[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const f32x4 o = *(const f32x4*)(P + (((qb * NB2 + b) * 4 + q4) * 64 + lane) * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * q4 + e;
        const float q = tanhf_(acc2[b][k] + o[e] + bv[k]);
        const float z = zreg[b][k];
        qv[k] = q;
        v[k] = (1.0f - z) * h[k] + z * q;
      }
    }
    if (p.qo) store_bf16<16>((bf16*)p.qo + (long)m * HD + c0, qv);   // training: q
    store_f32<16>(hp, v);
    store_bf16<16>((bf16*)p.y + (long)m * p.y_cs + c0, v);
    if (p.y2) store_bf16<16>((bf16*)p.y2 + (long)m * p.y2_cs + c0, v);
  }
}

template <int HD, int MODE, int NB1, int NB2>
int lds_bytes(int TR, int TC) {
  using C = Halo<HD, HD * 2, MODE, NB1, NB2>;
  const int f_rows = MODE == 0 ? TC + 8 : (TR + 4) * (TC + 4);
  const int f_elems = std::max(f_rows * FPITCH, C::NHB * NB2 * 4 * 256 * 2);
  return (((f_elems + 7) & ~7) + 32 * NB1 * RPITCH) * 2;
}

// the kernel may take up to 160 KiB of dynamic LDS (set once, at plan build: jr_gru_halo_lds)
template <int HD, int MODE, int NB1, int NB2>
bool lds_attr() {
  static const bool ok = hipFuncSetAttribute((const void*)gru_halo_kernel<HD, 2 * HD, MODE, NB1, NB2>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  return ok;
}

template <int HD, int MODE, int NB1, int NB2>
int launch(const GruHaloParams& p, hipStream_t s) {
  constexpr int CIN = 2 * HD;
  using C = Halo<HD, CIN, MODE, NB1, NB2>;
  const int lds = lds_bytes<HD, MODE, NB1, NB2>(p.TR, p.TC);
  if (lds > 160 * 1024 || !lds_attr<HD, MODE, NB1, NB2>()) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((gru_halo_kernel<HD, CIN, MODE, NB1, NB2>), dim3(p.ntiles), dim3(C::NT), lds, s, p);
  return (int)hipGetLastError();
}

// the instantiated (hd, mode, nb1, nb2) set: raft_large's 5-tap runs and raft_small's 3x3 blocks
// (4-block outputs: whole 128-pixel rows of the 1x5 stage at batch >= 4, one workgroup per CU)
#define JR_HALO_CASES(X)                                                                     \
  X(128, 0, 1, 1) X(128, 0, 2, 1) X(128, 0, 2, 2) X(128, 0, 3, 2) X(128, 0, 3, 3) X(128, 0, 5, 4) \
  X(96, 1, 2, 1) X(96, 1, 2, 2) X(96, 1, 3, 2)

}  // namespace

extern "C" int jr_gru_halo(const GruHaloParams* p, hipStream_t stream) {
  if (p->ntiles <= 0) return 0;
  const int hd = p->cs / 2;   // the loop buffers hold [h | x], x padded to hd channels
#define X(HD_, MODE_, NB1_, NB2_) \
  if (hd == HD_ && p->mode == MODE_ && p->nb1 == NB1_ && p->nb2 == NB2_) return launch<HD_, MODE_, NB1_, NB2_>(*p, stream);
  JR_HALO_CASES(X)
#undef X
  return (int)hipErrorInvalidValue;
}

extern "C" int jr_gru_halo_lds(int hd, int mode, int TR, int TC, int nb1, int nb2) {
#define X(HD_, MODE_, NB1_, NB2_) \
  if (hd == HD_ && mode == MODE_ && nb1 == NB1_ && nb2 == NB2_)                                \
    return lds_attr<HD_, MODE_, NB1_, NB2_>() ? lds_bytes<HD_, MODE_, NB1_, NB2_>(TR, TC) : 0;
  JR_HALO_CASES(X)
#undef X
  return 0;
}
