// Fused ConvGRU stage for the raft_large refinement loop (reference
// jax_raft/model.py:301-312 ConvGRU, :315-329 RecurrentBlock: a 1x5 then a
// 5x1 ConvGRU over [h | x], hidden 128, x = [motion | flow] 128 channels):
//
//   z, r = sigmoid(conv_zr([h | x]) + ctx_zr)      GEMM 1: 256 x 128 px, K = 5 x 256
//   q    = tanh(conv_q([r h | x]) + ctx_q)         GEMM 2: 128 x 128 px, K = 5 x 256
//   h'   = (1 - z) h + z q
//
// (ctx_* = the loop-invariant context-feature share + gate biases, a per-pixel
// bias map computed once in the prologue, runtime/engine.py.)
//
// The unfused loop runs this as two implicit-GEMM launches (EPI_GRU_A /
// EPI_GRU_B in conv_igemm.h) that hand z and r*h over through global memory.
// Here one workgroup owns a tile whose pixels contain every tap neighbour of
// every pixel: for the 1x5 stage a whole image row (W <= 128), for the 5x1
// stage J whole image columns (J * H <= 128).  So r*h of the tile's pixels is
// all GEMM 2 needs: it is written once into an LDS image (zero rows at both
// ends of each run = the conv's zero padding) and GEMM 2 reads its B
// fragments straight from that image, shifted by the tap.  z stays in the
// registers of the waves that produced it: GEMM 1's 16 waves tile 4 x 64
// channels x 4 x 32 pixels; waves 0-7 own the z channels and, in GEMM 2, the
// same 64 x 32 (channel, pixel) tiles of q, so the blend is register-local.
// Waves 8-15 (the r channels) write r*h, then only stage GEMM 2's operands.
// No z / r*h global round trip, one launch instead of two, and nothing else
// reads the tile's h while it is replaced (tap neighbours never leave the
// tile), so h' is written in place.
//
// MFMA: v_mfma_f32_32x32x16_bf16, operands staged as in kernel M32
// (conv_igemm.h: 64-deep K stages, register-staged global loads two stages
// ahead, double-buffered LDS with the swzB swizzle, permuted weight rows from
// ops/native.py:pack_weight so each lane owns 16 contiguous channels).
#include <cstdlib>

#include "conv_igemm.h"

namespace {

constexpr int HD = 128;            // hidden channels
constexpr int CIN = 256;           // [h | x] channels per tap
constexpr int KPAD = 5 * CIN;      // packed K of both GEMMs
constexpr int NSTG = KPAD / BK;    // 20 stages
constexpr int AROWS = 2 * HD;      // GEMM 1 rows
constexpr int ASTAGE = AROWS * BK; // one GEMM 1 weight stage (GEMM 2: HD * BK)
constexpr int IMG_ROWS = 136;      // tile image rows: J * (L + 4) <= 136
constexpr unsigned OOB = 0x80000000u;
// GEMM 2: two HD-row weight buffers + the z image (HD pixel rows x HD channels) in GEMM 1's staging
static_assert(2 * HD * BK + 128 * HD <= 2 * ASTAGE, "G2ALL: GEMM 2 buffers + the z image fit GEMM 1's staging");

// z image: rows of 128 channels (16 chunks of 16 B), chunk c of row R at c ^ (R & 15)
JR_DEVICE int rh_off(int row, int chunk) { return row * HD + ((chunk ^ (row & 15)) << 3); }
// tile image: rows of 256 channels (32 chunks); the XOR spreads the 32-row B-fragment reads of one
// chunk (row stride 512 B = 2 x 64 banks) over 16 distinct 16-B slots: conflict-free
// ds_read_b128 lane groups ({0-3, 12-15, 20-27} / {4-11, 16-19, 28-31} -> rows mod 16 distinct)
JR_DEVICE int img_off(int row, int chunk) { return row * CIN + ((chunk ^ (row & 15)) << 3); }

template <int NV>
JR_DEVICE void load_map(const GruFusedParams& p, int m, int c, float* v) {
  const long o = (long)m * p.bmap_cs + c;
  if (p.bmap_bf16) load_bf16<NV>((const bf16*)p.bmap + o, v);
  else load_f32<NV>((const float*)p.bmap + o, v);
}

template <bool G2ALL>
__global__ __launch_bounds__(1024) void gru_fused_kernel(const GruFusedParams p) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * ASTAGE + IMG_ROWS * CIN];
  bf16* const img = smem + 2 * ASTAGE;   // the tile's [h | x] rows (+ zero pad rows); h -> r*h after GEMM 1

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave & 3, wp = wave >> 2;   // 64-channel group, 32-pixel group
  const int rho = lane & 31, hh = lane >> 5;
  const int tile = blockIdx.x;
  auto stamp = [&](int k) {
    if (p.dbg && tid == 0) p.dbg[tile * 6 + k] = (long long)wall_clock64();
  };
  stamp(0);
  const int n = tile / p.tiles_per_img, tt = tile - n * p.tiles_per_img;
  const int npx = p.J * p.L;
  auto pix = [&](int pl) -> int {   // tile pixel -> global pixel index (or -1)
    if (pl >= npx) return -1;
    const int j = pl / p.L, r = pl - j * p.L;
    const int y = p.vertical ? r : tt;
    const int x = p.vertical ? tt * p.J + j : r;
    return (n * p.H + y) * p.W + x;
  };

  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc((void*)p.hx, (short)0, (int)p.hx_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t was = __builtin_amdgcn_make_buffer_rsrc((void*)p.wa, (short)0, (int)p.wa_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wbs = __builtin_amdgcn_make_buffer_rsrc((void*)p.wb, (short)0, (int)p.wb_bytes, 0x00020000);

  // loader: thread -> weight row lrow (and lrow + 128), 16-B chunk ch of a 64-deep K stage
  const int lrow = tid >> 3, ch = tid & 7;
  const unsigned aoff = (unsigned)(lrow * KPAD * 2 + ch * 16);
  auto kofs = [&](int s) { return (unsigned)((s >> 2) * CIN + (s & 3) * 64) * 2u; };
  auto sA_of = [&](int buf) { return smem + buf * ASTAGE; };
  auto putA = [&](bf16* base, int row, const u32x4& v) { *(u32x4*)(base + row * BK + ((ch ^ swzA(row)) << 3)) = v; };

  // The tile image: run j's rows j (L + 4) .. j (L + 4) + L + 3 hold the run's L pixels between two
  // zero rows at each end (the conv's zero padding along the tap axis), all 256 channels.  Loaded
  // once: GEMM 1's B fragment of tap t is row (pixel row + t), GEMM 2's x channels are read from
  // it too and its r*h channels from the h part, which epilogue 1 overwrites with r*h.  (The
  // round-4 form staged B per K stage from global memory: 5 x the tile's bytes per GEMM.)
  constexpr int NIMG = (IMG_ROWS * 32 + 1023) / 1024;
  u32x4 iv[NIMG];
  const int nrow = p.J * (p.L + 4);
#pragma unroll
  for (int k = 0; k < NIMG; ++k) {
    const int idx = k * 1024 + tid, R = idx >> 5, c = idx & 31;
    const int j = R / (p.L + 4), r = R - j * (p.L + 4) - 2;
    const bool in = R < nrow && (unsigned)r < (unsigned)p.L;
    const int m = in ? pix(j * p.L + r) : 0;
    iv[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
        xs, in ? (unsigned)m * (unsigned)p.hx_cs * 2u + (unsigned)c * 16u : OOB, 0, 0));
  }

  // ---------------------------------------------------------------- GEMM 1
  struct Regs { u32x4 a0, a1; };
  auto issue1 = [&](Regs& r, int s) {
    const bool kin = s < NSTG;
    r.a0 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(was, kin ? aoff + kofs(s) : OOB, 0, 0));
    r.a1 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
        was, kin ? aoff + (unsigned)(128 * KPAD * 2) + kofs(s) : OOB, 0, 0));
  };
  auto store1 = [&](const Regs& r, int buf) {
    putA(sA_of(buf), lrow, r.a0);
    putA(sA_of(buf), lrow + 128, r.a1);
  };
  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[t][k] = 0.f;
  const int prow = wp * 32 + rho;   // this lane's pixel row in the tile
  const int m = pix(prow);
  const int jrun = prow / p.L;
  const int rh_row = prow < npx ? jrun * (p.L + 4) + (prow - jrun * p.L) : 0;   // + tap = shifted row
  // B fragment of stage s (tap s / 4, 64-channel block s % 4): this lane's pixel row shifted by the tap
  auto bimg = [&](int s, int chunk) {
    const int row = rh_row + (s >> 2);
    return *(const bf16x8*)(img + img_off(row, (s & 3) * 8 + chunk));
  };
  // bf16 bias-map chunks of this lane's pixel, loaded during the last K stages of a GEMM
  // (its epilogue then starts without a dependent global load)
  // Unconditional loads (pixel clamped, an fp32 map read as bf16 chunks stays in bounds): a
  // branch around them makes hipcc wait vmcnt(0) for them before the next LDS store of staged
  // operands (measured +1-2.4 us per GEMM).
  const int mld = m >= 0 ? m : 0;
  auto pre_map = [&](u32x4 (&r)[2], int c) {
    const u32x4* q = (const u32x4*)((const bf16*)p.bmap + (long)mld * p.bmap_cs + c);
    r[0] = q[0];
    r[1] = q[1];
  };
  auto map16 = [&](const u32x4 (&r)[2], int c, float* v) {   // bias map values: prefetched (bf16) or loaded
    if (p.bmap_bf16) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[k] = bf2f(__builtin_bit_cast(bf16x8, r[0])[k]);
        v[8 + k] = bf2f(__builtin_bit_cast(bf16x8, r[1])[k]);
      }
    } else {
      load_map<16>(p, m, c, v);
    }
  };
  auto mma_stage = [&](const bf16* sA, int arow0, int s) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int chunk = kk * 2 + hh;
      const bf16x8 b = bimg(s, chunk);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int row = arow0 + m32_arow(t, rho);
        const bf16x8 a = *(const bf16x8*)(sA + row * BK + ((chunk ^ swzA(row)) << 3));
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t], 0, 0, 0);
      }
    }
  };
  u32x4 bm1[2][2];
  {
    Regs ra, rb;
    issue1(ra, 0);
    issue1(rb, 1);
#pragma unroll
    for (int k = 0; k < NIMG; ++k) {
      const int idx = k * 1024 + tid, R = idx >> 5, c = idx & 31;
      if (R < IMG_ROWS) *(u32x4*)(img + img_off(R, c)) = iv[k];
    }
    store1(ra, 0);
    __syncthreads();
#pragma nounroll
    for (int s = 0; s < NSTG - 2; s += 2) {
      issue1(ra, s + 2);
      mma_stage(sA_of(0), wco * 64, s);
      store1(rb, 1);
      __syncthreads();
      issue1(rb, s + 3);
      mma_stage(sA_of(1), wco * 64, s + 1);
      store1(ra, 0);
      __syncthreads();
    }
    // last two stages: no operand loads left; the epilogue's bias-map chunks load instead
#pragma unroll
    for (int t = 0; t < 2; ++t) pre_map(bm1[t], wco * 64 + 32 * t + 16 * hh);
    mma_stage(sA_of(0), wco * 64, NSTG - 2);
    store1(rb, 1);
    __syncthreads();
    mma_stage(sA_of(1), wco * 64, NSTG - 1);
    __syncthreads();   // GEMM 1 staging and the image's h part free
  }

  stamp(1);
  // GEMM 2's first two stages' weights load during epilogue 1
  auto sA2 = [&](int buf) { return smem + buf * (HD * BK); };
  auto issue2 = [&](u32x4& r, int s) {
    r = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wbs, s < NSTG ? aoff + kofs(s) : OOB, 0, 0));
  };
  u32x4 ra2, rb2;
  issue2(ra2, 0);
  issue2(rb2, 1);

  // ------------------------------------------------------------ epilogue 1
  // lane: channels c0 + [0, 16) (c0 = 64 wco + 32 t + 16 hh) of tile pixel prow
  // G2ALL: z goes to an LDS image behind GEMM 2's two weight buffers
  bf16* const zimg = smem + 2 * HD * BK;
  [[maybe_unused]] bf16x8 z[2][2];   // z as bf16 (the unfused path's default gate storage, EPI_GRU_A z_bf16)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c0 = wco * 64 + 32 * t + 16 * hh;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = acc[t][k];
    if (m >= 0) {
      float b[16];
      map16(bm1[t], c0, b);
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = sigmoidf_(v[k] + b[k]);
    }
    if (wco < 2) {
      bf16x8 o0, o1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o0[k] = f2bf(v[k]);
        o1[k] = f2bf(v[8 + k]);
      }
      if constexpr (G2ALL) {
        *(bf16x8*)(zimg + rh_off(prow, c0 >> 3)) = o0;
        *(bf16x8*)(zimg + rh_off(prow, (c0 >> 3) + 1)) = o1;
      } else {
        z[t][0] = o0;
        z[t][1] = o1;
      }
    } else if (m >= 0) {   // r * h (h: this pixel's bf16 row of the image, as the unfused EPI_GRU_A)
      // the lane reads and then replaces the same 16 h channels of its own pixel: no other lane
      // touches them, and GEMM 1's readers are past the barrier above
      const int chunk = (c0 - HD) >> 3;
      bf16x8* const d0 = (bf16x8*)(img + img_off(rh_row + 2, chunk));
      bf16x8* const d1 = (bf16x8*)(img + img_off(rh_row + 2, chunk + 1));
      const bf16x8 h0 = *d0, h1 = *d1;
      bf16x8 o0, o1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o0[k] = f2bf(v[k] * bf2f(h0[k]));
        o1[k] = f2bf(v[8 + k] * bf2f(h1[k]));
      }
      *d0 = o0;
      *d1 = o1;
    }
  }

  // ---------------------------------------------------------------- GEMM 2
  // stages s = (tap, cb): cb 0, 1 = the r*h channels, cb 2, 3 = x -- both from the image.
  // G2ALL: all 16 waves, 32 x 32 (channel, pixel) tiles; else the 8 z waves keep GEMM 1's
  // 64 x 32 tiles (z in registers), the others only stage the weights.
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[t][k] = 0.f;
  auto putA2 = [&](int buf, const u32x4& v) { putA(sA2(buf), lrow, v); };
  const int arow2 = 64 * (wco >> 1) + m32_arow(wco & 1, rho);   // G2ALL: channels 32 wco + ..
  auto compute2 = [&](int buf, int s) {
    if constexpr (G2ALL) {
      const bf16* sA = sA2(buf);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int chunk = kk * 2 + hh;
        const bf16x8 b = bimg(s, chunk);
        const bf16x8 a = *(const bf16x8*)(sA + arow2 * BK + ((chunk ^ swzA(arow2)) << 3));
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[0], 0, 0, 0);
      }
    } else {
      if (wco >= 2) return;   // waves 8-15 only stage operands
      mma_stage(sA2(buf), wco * 64, s);
    }
  };
  __syncthreads();   // r*h (and z) images complete
  stamp(2);
  putA2(0, ra2);
  __syncthreads();
#pragma nounroll
  for (int s = 0; s < NSTG - 2; s += 2) {
    issue2(ra2, s + 2);
    compute2(0, s);
    putA2(1, rb2);
    __syncthreads();
    issue2(rb2, s + 3);
    compute2(1, s + 1);
    putA2(0, ra2);
    __syncthreads();
  }
  // last two stages: the epilogue's bias-map chunks and fp32 state load instead of operands
  constexpr int NT = G2ALL ? 1 : 2;
  u32x4 bm2[NT][2];
  [[maybe_unused]] f32x4 h2[4];   // G2ALL: the fp32 state too (the 8-wave variant has no registers to spare)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c0 = G2ALL ? 32 * wco + 16 * hh : wco * 64 + 32 * t + 16 * hh;
    // 8-wave GEMM 2: waves wco >= 2 (c0 >= HD) have no epilogue 2 -- keep their (unused) load
    // inside the map row: q channels 2 HD + c0 + 16 would pass the row's end (384)
    pre_map(bm2[t], 2 * HD + (c0 < HD ? c0 : 0));
    if constexpr (G2ALL) {
      const f32x4* hq = (const f32x4*)(p.h32 + (long)mld * HD + c0);
#pragma unroll
      for (int k = 0; k < 4; ++k) h2[k] = hq[k];
    }
  }
  compute2(0, NSTG - 2);
  putA2(1, rb2);
  __syncthreads();
  compute2(1, NSTG - 1);

  // ------------------------------------------------------------ epilogue 2
  stamp(3);
  if ((!G2ALL && wco >= 2) || m < 0) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c0 = G2ALL ? 32 * wco + 16 * hh : wco * 64 + 32 * t + 16 * hh;
    bf16x8 zz[2];
    if constexpr (G2ALL) {
      zz[0] = *(const bf16x8*)(zimg + rh_off(prow, c0 >> 3));
      zz[1] = *(const bf16x8*)(zimg + rh_off(prow, (c0 >> 3) + 1));
    } else {
      zz[0] = z[t][0];
      zz[1] = z[t][1];
    }
    float b[16], h[16], v[16];
    map16(bm2[t], 2 * HD + c0, b);
    float* hp = p.h32 + (long)m * HD + c0;
    if constexpr (G2ALL) {
#pragma unroll
      for (int k = 0; k < 16; ++k) h[k] = h2[k >> 2][k & 3];
    } else {
      load_f32<16>(hp, h);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float q = tanhf_(acc[t][k] + b[k]);
      const float zk = bf2f(zz[k >> 3][k & 7]);
      v[k] = (1.0f - zk) * h[k] + zk * q;
    }
    store_f32<16>(hp, v);
    store_bf16<16>((bf16*)p.y + (long)m * p.y_cs + c0, v);
    if (p.y2) store_bf16<16>((bf16*)p.y2 + (long)m * p.y2_cs + c0, v);
  }
  stamp(4);
}

}  // namespace

extern "C" int jr_gru_fused(const GruFusedParams* p, hipStream_t stream) {
  if (p->ntiles <= 0) return 0;
  // GEMM 2 on all 16 waves with z through LDS (the engine's choice) or on the 8 z waves with z
  // in registers (p->g2all = 0; profiles/r3_gru_fused_ab.txt)
  if (p->g2all) hipLaunchKernelGGL(gru_fused_kernel<true>, dim3(p->ntiles), dim3(1024), 0, stream, *p);
  else hipLaunchKernelGGL(gru_fused_kernel<false>, dim3(p->ntiles), dim3(1024), 0, stream, *p);
  return (int)hipGetLastError();
}
