// Channel-split ConvGRU stage (reference jax_raft/model.py:293-312 ConvGRU, :315-334
// RecurrentBlock: raft_large's 1x5 then 5x1 stage, hidden 128, loop input [h | motion | flow]
// = 256 channels; the context share of the gates is a per-pixel bias map, runtime/engine.py):
//
//   launch A:  z, r = sigmoid(conv_zr([h | x]) + ctx_zr)  ->  z (bf16), r*h into the q input buffer
//   launch B:  q = tanh(conv_q([r h | x]) + ctx_q);  h' = (1 - z) h + z q
//
// Why two launches.  The fused kernels (gru_fused.hip, gru_halo.hip) give one workgroup ALL of a
// stage's weights (5 x 256 x 384 bf16 = 983 KB) for its pixel tile, because q needs r*h of every
// hidden channel on the tile's footprint.  A CU then streams ~1 MB of weights from L2 per stage,
// which at the per-CU L2 rate (~70 GB/s, MI355X_MICROARCH.md "Indexed rows") and the latency of a
// register ring sets the stage time (r5 PMC: 20-24 % MFMA busy, 43 % issue stalls,
// profiles/r5_pmc_b4.txt).  Splitting the output channels over workgroups (NT = 64 or 128 of
// them per workgroup) and giving each workgroup a wide pixel tile (128-256 pixels) balances the
// two streams instead: weights K x NT x 2 B + the tile's footprint (P + halo) x 512 B per CU,
// 2-3x fewer bytes than the fused kernels', at the price of one more launch and a 7 MB (batch 4)
// z / r*h round trip through L2.
//
// Geometry.  A tile is J runs of up to L consecutive pixels along the tap axis (1x5: a row
// segment, 5x1: a column segment); its footprint is the runs extended by the taps' reach (+-2),
// zero outside the image (the conv's zero padding).  The K loop walks KC-channel slabs of the 256
// input channels; each slab's footprint rows and the tile's weight fragments (5 taps x KC/16
// k-steps x CB 32-channel blocks, MFMA fragment order, ops/native.py:pack_gru_split) are staged
// global -> registers -> LDS one slab ahead (double buffer), and every wave reads its A fragments
// (weights) and B fragments (pixels, the footprint row shifted by the tap) from LDS.
//
// Waves: (CB / CBW) x (PB / PBW); a wave owns CBW channel blocks x PBW pixel blocks, so each k-step
// is CBW + PBW conflict-free ds_read_b128 for CBW * PBW v_mfma_f32_32x32x16_bf16.
#include "halo.h"

namespace {

constexpr int SHD = 128;        // hidden channels
constexpr int SCIN = 256;       // loop input channels per pixel ([h | motion | flow])
constexpr int STAPS = 5;

// position of lane rho in its 32-pixel block (conv_halo.hip: the ds_read_b128 lane groups
// {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31} read 16 consecutive pixels each)
JR_DEVICE int split_lane_px(int rho) {
  return rho < 4 ? rho : rho < 12 ? rho + 12 : rho < 16 ? rho - 8 : rho < 20 ? rho + 8 : rho < 28 ? rho - 12 : rho;
}

template <int PB, int CB, int KC, int CBW, int PBW>
struct SplitCfg {
  static constexpr int NWC = CB / CBW, NWP = PB / PBW, NW = NWC * NWP, NT = 64 * NW;
  static constexpr int NSLAB = SCIN / KC;
  static constexpr int KK = KC / 16;              // k-steps per tap per slab
  static constexpr int CPR = KC / 8;              // 16-B chunks per footprint row
  static constexpr int RPW = 256 / (KC * 2);      // footprint rows per 256-B bank window
  static constexpr int FROWS = 36 * PB;           // footprint rows (host: J (L + 4) <= FROWS)
  static constexpr int A_BYTES = STAPS * KK * CB * 1024;
  static constexpr int F_BYTES = FROWS * KC * 2;
  static constexpr int BUF = A_BYTES + F_BYTES;
  static_assert(CB % CBW == 0 && PB % PBW == 0 && SCIN % KC == 0 && (KC == 32 || KC == 64), "split geometry");
  static_assert(2 * BUF <= 160 * 1024, "LDS");
};

// LDS-only workgroup barrier: __syncthreads() would also wait for every outstanding global load
// (vmcnt(0)), i.e. drain the next slabs' prefetch at every slab boundary
JR_DEVICE void split_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// byte offset of chunk c of footprint row f: the 16 consecutive rows a b128 lane group reads
// (one logical chunk) land in 16 distinct 16-B slots of the 256-B bank window
template <int KC>
JR_DEVICE int fslot(int f, int c) {
  constexpr int CPR = KC / 8, RPW = 256 / (KC * 2);
  return f * KC * 2 + ((c ^ ((f / RPW) % CPR)) << 4);
}

template <int PB, int CB, int KC, int CBW, int PBW, int MODE>
__global__ __launch_bounds__(64 * (CB / CBW) * (PB / PBW)) void gru_split_kernel(const GruSplitParams p) {
  using C = SplitCfg<PB, CB, KC, CBW, PBW>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rho = lane & 31, hh = lane >> 5;
  const int wc = wave % C::NWC, wp = wave / C::NWC;

  // XCD-aware order: the ctiles channel tiles of one pixel tile get block ids equal mod 8 (one XCD
  // under round-robin placement: they share the footprint in that XCD's L2; speed only)
  int ptile, ctile;
  {
    const int b = blockIdx.x, x = b & 7, q = b >> 3;
    ptile = (q / p.ctiles) * 8 + x;
    ctile = q - (q / p.ctiles) * p.ctiles;
    if (ptile >= p.ptiles) return;
  }
  auto stamp = [&](int k) {
    if (p.dbg && tid == 0) p.dbg[blockIdx.x * 12 + k] = (long long)wall_clock64();
  };
  stamp(0);
  const int line_len = p.axis ? p.H : p.W;
  const int HW = p.H * p.W;
  auto line_pix = [&](int j, int pos_in_line) -> int {   // image pixel of position pos of run j's line, -1 outside
    const int r = ptile * p.J + j;
    const int line = r / p.rpl;
    if (line >= p.lines || (unsigned)pos_in_line >= (unsigned)line_len) return -1;
    const int n = line / (p.axis ? p.W : p.H), l = line - n * (p.axis ? p.W : p.H);
    return p.axis ? n * HW + pos_in_line * p.W + l : n * HW + l * p.W + pos_in_line;
  };
  auto run_start = [&](int j) { return ((ptile * p.J + j) % p.rpl) * p.L; };
  auto run_len = [&](int j) {
    const int r = ptile * p.J + j;
    if (r / p.rpl >= p.lines) return 0;
    return min(p.L, line_len - (r % p.rpl) * p.L);
  };
  const int FW = p.L + 4;                 // footprint rows per run
  const int frows = p.J * FW;

  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc((void*)p.src, (short)0, (int)p.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.w_bytes, 0x00020000);

  // ---------------------------------------------------------------- staging (one slab ahead)
  // weight chunks and footprint chunks in separate, uniformly typed loops (a per-lane choice of
  // the buffer resource would make hipcc emit a waterfall loop around every load)
  constexpr int NA = C::A_BYTES / 16 / C::NT;                       // weight chunks per thread
  constexpr int NF = (C::FROWS * C::CPR + C::NT - 1) / C::NT;       // footprint chunks per thread
  static_assert(NA * C::NT * 16 == C::A_BYTES, "weight slab chunks must divide over the threads");
  int foff[NF];   // byte offset (in the source) of each staged footprint chunk's slab-0 bytes; -1: zero, -2: none
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const int e = k * C::NT + tid;
    const int f = e / C::CPR, c = e - (e / C::CPR) * C::CPR;
    int v = -2;
    if (f < frows) {
      const int j = f / FW, i = f - j * FW;
      const int m = run_len(j) > 0 ? line_pix(j, run_start(j) + i - 2) : -1;
      v = m >= 0 ? m * p.src_cs * 2 + c * 16 : -1;
    }
    foff[k] = v;
  }
  const unsigned wbase = (unsigned)((ctile * C::NSLAB) * C::A_BYTES) + (unsigned)tid * 16u;
  // the loads of slab s are issued DEPTH slabs before it is computed: two register sets when the
  // per-thread staging is small (8-wave tiles), so ~2 slabs of compute cover the L2 / HBM latency
  constexpr int DEPTH = NA + NF <= 12 ? 2 : 1;
  u32x4 sa[DEPTH][NA], sf[DEPTH][NF];
  auto issue = [&](int s, int r) {
#pragma unroll
    for (int k = 0; k < NA; ++k) sa[r][k] = bload(wrs, wbase + (unsigned)(s * C::A_BYTES + k * C::NT * 16));
#pragma unroll
    for (int k = 0; k < NF; ++k)
      sf[r][k] = bload(srs, foff[k] >= 0 ? (unsigned)foff[k] + (unsigned)(s * KC * 2) : HOOB);
  };
  auto commit = [&](int buf, int r) {
    char* const base = lds + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < NA; ++k) *(u32x4*)(base + (k * C::NT + tid) * 16) = sa[r][k];
#pragma unroll
    for (int k = 0; k < NF; ++k) {
      const int e = k * C::NT + tid;
      if (foff[k] != -2) *(u32x4*)(base + C::A_BYTES + fslot<KC>(e / C::CPR, e % C::CPR)) = sf[r][k];
    }
  };

  // ---------------------------------------------------------------- per-lane pixel rows
  const int npx = p.J * p.L;
  int frow[PBW], opix[PBW];
#pragma unroll
  for (int b = 0; b < PBW; ++b) {
    const int q = 32 * (wp * PBW + b) + split_lane_px(rho);
    const int j = q / p.L, i = q - j * p.L;
    const bool ok = q < npx && i < run_len(j);
    frow[b] = ok ? j * FW + i : 0;    // footprint row of tap 0 (the pixel's centre is row + 2)
    opix[b] = ok ? line_pix(j, run_start(j) + i) : -1;
  }

  f32x16 acc[CBW][PBW];
#pragma unroll
  for (int a = 0; a < CBW; ++a)
#pragma unroll
    for (int b = 0; b < PBW; ++b)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[a][b][k] = 0.f;

  // epilogue operands (independent of the GEMM): loaded during the last slab's MFMAs
  constexpr bool EPRE = CBW * PBW <= 2;
  u32x4 ep0[EPRE ? CBW * PBW : 1][2], ep1[EPRE ? CBW * PBW : 1][2];
  f32x4 ep2[EPRE ? CBW * PBW : 1][4];
  auto epi_pre = [&]() {
#pragma unroll
    for (int a = 0; a < CBW; ++a) {
      const int co = 32 * (ctile * CB + wc * CBW + a) + 16 * hh;
#pragma unroll
      for (int b = 0; b < PBW; ++b) {
        const long m = opix[b] >= 0 ? opix[b] : 0;   // unconditional (clamped): no branch around the loads
        const int e = a * PBW + b;
        const u32x4* q = (const u32x4*)((const bf16*)p.bmap + m * p.bmap_cs + (MODE == 0 ? co : 2 * SHD + co));
        ep0[e][0] = q[0];
        ep0[e][1] = q[1];
        if (MODE == 0) {
          const u32x4* hq = (const u32x4*)((const bf16*)p.src + m * p.src_cs + (co >= SHD ? co - SHD : 0));
          ep1[e][0] = hq[0];
          ep1[e][1] = hq[1];
        } else {
          const u32x4* zq = (const u32x4*)((const bf16*)p.zb + m * SHD + co);
          ep1[e][0] = zq[0];
          ep1[e][1] = zq[1];
          const f32x4* hq = (const f32x4*)(p.h32 + m * SHD + co);
#pragma unroll
          for (int k = 0; k < 4; ++k) ep2[e][k] = hq[k];
        }
      }
    }
  };

  issue(0, 0);
  if (DEPTH == 2 && C::NSLAB > 1) issue(1, 1);
  commit(0, 0);
  split_lds_sync();
  stamp(1);
  for (int s = 0; s < C::NSLAB; ++s) {
    if (DEPTH == 1 && s + 1 < C::NSLAB) issue(s + 1, 0);
    if (DEPTH == 2 && s + 2 < C::NSLAB) issue(s + 2, s & 1);   // set s & 1 was committed (slab s)
    if (EPRE && s == C::NSLAB - 1) epi_pre();
    const char* const A = lds + (s & 1) * C::BUF;
    const char* const F = A + C::A_BYTES;
    // k-step st = (tap, kk); the fragments of step st + 1 are read from LDS while step st's MFMAs
    // run (one wave per SIMD: nothing else would hide the LDS latency)
    constexpr int S = STAPS * C::KK;
    auto rd = [&](int st, bf16x8 (&af)[CBW], bf16x8 (&bfr)[PBW]) {
      const int tap = st / C::KK, kk = st - tap * C::KK;
#pragma unroll
      for (int a = 0; a < CBW; ++a)
        af[a] = *(const bf16x8*)(A + ((tap * C::KK + kk) * CB + wc * CBW + a) * 1024 + lane * 16);
#pragma unroll
      for (int b = 0; b < PBW; ++b) bfr[b] = *(const bf16x8*)(F + fslot<KC>(frow[b] + tap, 2 * kk + hh));
    };
    bf16x8 af0[CBW], bf0[PBW], af1[CBW], bf1[PBW];
    rd(0, af0, bf0);
#pragma unroll
    for (int st = 0; st < S; ++st) {
      bf16x8 (&ac)[CBW] = (st & 1) ? af1 : af0;
      bf16x8 (&bc)[PBW] = (st & 1) ? bf1 : bf0;
      bf16x8 (&an)[CBW] = (st & 1) ? af0 : af1;
      bf16x8 (&bn)[PBW] = (st & 1) ? bf0 : bf1;
      if (st + 1 < S) rd(st + 1, an, bn);
#pragma unroll
      for (int a = 0; a < CBW; ++a)
#pragma unroll
        for (int b = 0; b < PBW; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[a], bc[b], acc[a][b], 0, 0, 0);
      if (st + 1 < S) __builtin_amdgcn_sched_group_barrier(0x100, CBW + PBW, 0);   // next step's DS reads first
      __builtin_amdgcn_sched_group_barrier(0x008, CBW * PBW, 0);                    // then this step's MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
    if (s + 1 < C::NSLAB) commit((s + 1) & 1, DEPTH == 2 ? (s + 1) & 1 : 0);
    split_lds_sync();
    if (s < 8) stamp(2 + s);
  }

  // ---------------------------------------------------------------- epilogues
  // lane (rho, hh) of acc[a][b] holds channels 16 hh + [0, 16) of block (ctile CB + wc CBW + a) for
  // the pixel opix[b] (pack_gru_split permutes the weight rows so, as pack_gru_halo does)
#pragma unroll
  for (int a = 0; a < CBW; ++a) {
    const int co = 32 * (ctile * CB + wc * CBW + a) + 16 * hh;
#pragma unroll
    for (int b = 0; b < PBW; ++b) {
      const int m = opix[b];
      if (m < 0) continue;
      float bv[16], v[16];
      const int e = a * PBW + b;
      auto unpack = [](const u32x4 (&r)[2], float* o) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o[k] = bf2f(__builtin_bit_cast(bf16x8, r[0])[k]);
          o[8 + k] = bf2f(__builtin_bit_cast(bf16x8, r[1])[k]);
        }
      };
      if constexpr (EPRE) unpack(ep0[e], bv);
      else load_bf16<16>((const bf16*)p.bmap + (long)m * p.bmap_cs + (MODE == 0 ? co : 2 * SHD + co), bv);
      if (MODE == 0) {
        if (co < SHD) {   // z
#pragma unroll
          for (int k = 0; k < 16; ++k) v[k] = sigmoidf_(acc[a][b][k] + bv[k]);
          store_bf16<16>((bf16*)p.zb + (long)m * SHD + co, v);
        } else {          // r * h (h: the bf16 loop state the conv read)
          const int c = co - SHD;
          float h[16];
          if constexpr (EPRE) unpack(ep1[e], h);
          else load_bf16<16>((const bf16*)p.src + (long)m * p.src_cs + c, h);
#pragma unroll
          for (int k = 0; k < 16; ++k) v[k] = sigmoidf_(acc[a][b][k] + bv[k]) * h[k];
          store_bf16<16>((bf16*)p.rh + (long)m * p.rh_cs + c, v);
        }
      } else {            // q, blend: h' = (1 - z) h + z q (fp32 state)
        float z[16], h[16];
        float* hp = p.h32 + (long)m * SHD + co;
        if constexpr (EPRE) {
          unpack(ep1[e], z);
#pragma unroll
          for (int k = 0; k < 16; ++k) h[k] = ep2[e][k >> 2][k & 3];
        } else {
          load_bf16<16>((const bf16*)p.zb + (long)m * SHD + co, z);
          load_f32<16>(hp, h);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = (1.0f - z[k]) * h[k] + z[k] * tanhf_(acc[a][b][k] + bv[k]);
        store_f32<16>(hp, v);
        store_bf16<16>((bf16*)p.y + (long)m * p.y_cs + co, v);
        if (p.y2) store_bf16<16>((bf16*)p.y2 + (long)m * p.y2_cs + co, v);
      }
    }
  }
  stamp(10);
}

struct SplitCfgId {
  int pb, cb, kc, cbw, pbw;
};
// tile configs (cfg id = index): batch >= 4 (8 pixel blocks) and batch-1 (4 / 2 pixel blocks) tiles
constexpr SplitCfgId kSplitCfgs[] = {
    {8, 2, 64, 2, 2},   // 0: 256 px x 64 ch, 4 waves
    {8, 4, 32, 2, 2},   // 1: 256 px x 128 ch, 8 waves
    {4, 2, 64, 2, 1},   // 2: 128 px x 64 ch, 4 waves
    {4, 1, 64, 1, 1},   // 3: 128 px x 32 ch, 4 waves
    {2, 2, 64, 1, 1},   // 4: 64 px x 64 ch, 4 waves
    {8, 1, 64, 1, 2},   // 5: 256 px x 32 ch, 4 waves
    {8, 2, 64, 1, 2},   // 6: 256 px x 64 ch, 8 waves (two per SIMD: each hides the other's latencies)
    {4, 2, 64, 1, 1},   // 7: 128 px x 64 ch, 8 waves
};
constexpr int kNumSplitCfgs = sizeof(kSplitCfgs) / sizeof(kSplitCfgs[0]);

template <int PB, int CB, int KC, int CBW, int PBW, int MODE>
int launch_split(const GruSplitParams& p, hipStream_t s) {
  using C = SplitCfg<PB, CB, KC, CBW, PBW>;
  static const bool attr = hipFuncSetAttribute((const void*)gru_split_kernel<PB, CB, KC, CBW, PBW, MODE>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!attr) return (int)hipErrorInvalidValue;
  if (p.J * (p.L + 4) > C::FROWS || p.J * p.L > 32 * PB) return (int)hipErrorInvalidValue;
  const int groups = (p.ptiles + 7) / 8;
  hipLaunchKernelGGL((gru_split_kernel<PB, CB, KC, CBW, PBW, MODE>), dim3(groups * 8 * p.ctiles), dim3(C::NT),
                     2 * C::BUF, s, p);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int jr_gru_split_cfg(int cfg, int* o) {
  if (cfg < 0 || cfg >= kNumSplitCfgs) return 0;
  const SplitCfgId& c = kSplitCfgs[cfg];
  o[0] = c.pb; o[1] = c.cb; o[2] = c.kc; o[3] = c.cbw; o[4] = c.pbw;
  return 1;
}

extern "C" int jr_gru_split(const GruSplitParams* p, int cfg, hipStream_t stream) {
  if (cfg < 0 || cfg >= kNumSplitCfgs || p->ptiles <= 0) return (int)hipErrorInvalidValue;
  const SplitCfgId& c = kSplitCfgs[cfg];
#define JR_SPLIT(PB_, CB_, KC_, CBW_, PBW_)                                                          \
  if (c.pb == PB_ && c.cb == CB_ && c.kc == KC_ && c.cbw == CBW_ && c.pbw == PBW_)                    \
    return p->mode ? launch_split<PB_, CB_, KC_, CBW_, PBW_, 1>(*p, stream)                            \
                   : launch_split<PB_, CB_, KC_, CBW_, PBW_, 0>(*p, stream);
  JR_SPLIT(8, 2, 64, 2, 2) JR_SPLIT(8, 4, 32, 2, 2) JR_SPLIT(4, 2, 64, 2, 1) JR_SPLIT(4, 1, 64, 1, 1)
  JR_SPLIT(2, 2, 64, 1, 1) JR_SPLIT(8, 1, 64, 1, 2) JR_SPLIT(8, 2, 64, 1, 2) JR_SPLIT(4, 2, 64, 1, 1)
#undef JR_SPLIT
  return (int)hipErrorInvalidValue;
}
