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
  u32x4 sa[NA], sf[NF];
  auto issue = [&](int s) {
#pragma unroll
    for (int k = 0; k < NA; ++k) sa[k] = bload(wrs, wbase + (unsigned)(s * C::A_BYTES + k * C::NT * 16));
#pragma unroll
    for (int k = 0; k < NF; ++k) sf[k] = bload(srs, foff[k] >= 0 ? (unsigned)foff[k] + (unsigned)(s * KC * 2) : HOOB);
  };
  auto commit = [&](int buf) {
    char* const base = lds + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < NA; ++k) *(u32x4*)(base + (k * C::NT + tid) * 16) = sa[k];
#pragma unroll
    for (int k = 0; k < NF; ++k) {
      const int e = k * C::NT + tid;
      if (foff[k] != -2) *(u32x4*)(base + C::A_BYTES + fslot<KC>(e / C::CPR, e % C::CPR)) = sf[k];
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

  issue(0);
  commit(0);
  __syncthreads();
  for (int s = 0; s < C::NSLAB; ++s) {
    if (s + 1 < C::NSLAB) issue(s + 1);
    const char* const A = lds + (s & 1) * C::BUF;
    const char* const F = A + C::A_BYTES;
#pragma unroll
    for (int tap = 0; tap < STAPS; ++tap) {
#pragma unroll
      for (int kk = 0; kk < C::KK; ++kk) {
        bf16x8 af[CBW], bfr[PBW];
#pragma unroll
        for (int a = 0; a < CBW; ++a)
          af[a] = *(const bf16x8*)(A + ((tap * C::KK + kk) * CB + wc * CBW + a) * 1024 + lane * 16);
#pragma unroll
        for (int b = 0; b < PBW; ++b) {
          const int f = frow[b] + tap;
          bfr[b] = *(const bf16x8*)(F + fslot<KC>(f, 2 * kk + hh));
        }
#pragma unroll
        for (int a = 0; a < CBW; ++a)
#pragma unroll
          for (int b = 0; b < PBW; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
      }
    }
    if (s + 1 < C::NSLAB) commit((s + 1) & 1);
    __syncthreads();
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
      load_bf16<16>((const bf16*)p.bmap + (long)m * p.bmap_cs + (MODE == 0 ? co : 2 * SHD + co), bv);
      if (MODE == 0) {
        if (co < SHD) {   // z
#pragma unroll
          for (int k = 0; k < 16; ++k) v[k] = sigmoidf_(acc[a][b][k] + bv[k]);
          store_bf16<16>((bf16*)p.zb + (long)m * SHD + co, v);
        } else {          // r * h (h: the bf16 loop state the conv read)
          const int c = co - SHD;
          float h[16];
          load_bf16<16>((const bf16*)p.src + (long)m * p.src_cs + c, h);
#pragma unroll
          for (int k = 0; k < 16; ++k) v[k] = sigmoidf_(acc[a][b][k] + bv[k]) * h[k];
          store_bf16<16>((bf16*)p.rh + (long)m * p.rh_cs + c, v);
        }
      } else {            // q, blend: h' = (1 - z) h + z q (fp32 state)
        float z[16], h[16];
        load_bf16<16>((const bf16*)p.zb + (long)m * SHD + co, z);
        float* hp = p.h32 + (long)m * SHD + co;
        load_f32<16>(hp, h);
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = (1.0f - z[k]) * h[k] + z[k] * tanhf_(acc[a][b][k] + bv[k]);
        store_f32<16>(hp, v);
        store_bf16<16>((bf16*)p.y + (long)m * p.y_cs + co, v);
        if (p.y2) store_bf16<16>((bf16*)p.y2 + (long)m * p.y2_cs + co, v);
      }
    }
  }
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
  JR_SPLIT(2, 2, 64, 1, 1) JR_SPLIT(8, 1, 64, 1, 2)
#undef JR_SPLIT
  return (int)hipErrorInvalidValue;
}
