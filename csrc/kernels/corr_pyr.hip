// Correlation pyramid, blocked bf16 layout (the engine's): a persistent, write-streaming
// build of all L levels (reference CorrBlock, jax_raft/model.py:418-446 + 472-481: the
// all-pairs volume f1 . f2^T / sqrt(C), then 2x2 average pools with floor semantics).
//
// The volume (533 MB at raft_large batch 4) is the only traffic that has to reach HBM; the
// tile kernel of corr.hip re-read both feature maps per 128 x 128 tile (1.6 GB of L2 reads,
// 382 MB past L2: profiles/r4_corr_study.md).  Here:
//   * one workgroup per CU walks a contiguous run of (image, query tile, target tile) items,
//     target tile fastest; runs are XCD-contiguous, so an XCD's CUs read one image's f2;
//   * a wave keeps its 32 queries' features in registers (the MFMA B operand) for the whole
//     run; only the 128-target tile (8 x 16 pixels, the MFMA A operand) is staged in LDS,
//     its loads for item k + 1 in flight during item k's MFMAs;
//   * D[target][query]: a lane holds 16 targets of ONE query (rows 2n, 2n+1 of the tile,
//     4 consecutive x twice), so the 2x2 / 4x4 pools are in-lane sums and the 8x8 one needs
//     one lane^32 exchange;
//   * levels 0 / 1 are transposed through an LDS staging area into whole 256 / 64-byte
//     per-query blocks and written with coalesced 16-B stores; levels 2 / 3 are gathered per
//     tile row in LDS and written as whole lines;
//   * barriers wait for LDS only: an item's stores drain during the next item's MFMAs (the
//     next B tile's loads are issued after them, so waiting for those loads is the only
//     point that waits for the stores).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

JR_DEVICE unsigned pack_bf16x2(float a, float b) {
  return (unsigned)__builtin_bit_cast(unsigned short, f2bf(a)) | ((unsigned)__builtin_bit_cast(unsigned short, f2bf(b)) << 16);
}

// KS = C / 16 feature-channel k-steps; OCC workgroups per CU (the 256-channel variant needs
// 64 query + 64 accumulator + 64 staging registers per lane: one workgroup per CU)
// LDS-only barrier: the global stores and the next tile's loads stay in flight
// (__syncthreads() would drain vmcnt, i.e. wait for every store of the item: measured
// 270 us at batch 4 with it)
JR_DEVICE void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int KS, int OCC>
__global__ __launch_bounds__(256, OCC) void corr_pyr_blocked_kernel(const bf16* __restrict__ f1,
                                                                  const bf16* __restrict__ f2, int h, int w, int cs,
                                                                  bf16* __restrict__ l0, bf16* __restrict__ l1,
                                                                  bf16* __restrict__ l2, bf16* __restrict__ l3,
                                                                  int nlev, float scale, int items, int nwg,
                                                                  int acc23, int qtmajor, int dbg) {
  constexpr int C = 16 * KS;
  constexpr int RB = 2 * C;               // bytes of one target row in the B tile
  constexpr int CPR = C / 8;              // 16-B chunks per target row
  constexpr int NLD = 128 * CPR / 256;    // B-tile chunks per thread
  constexpr int BT = 128 * RB;            // LDS: [B tile | level 0 / 1 staging (40 KB) | level 2 / 3 rows]
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rho = lane & 31, hh = lane >> 5;
  const int P = h * w, ntx = w >> 4, nty = (h + 7) >> 3, ntt = ntx * nty, nqt = (P + 127) >> 7;
  const int h1 = h >> 1, h2 = h1 >> 1, w2 = (w >> 1) >> 1, h3 = h2 >> 1, w3 = w2 >> 1;
  const long qs0 = (long)ntt * 128, qs1 = (long)ntt * 32;   // per-query blocked level sizes
  // XCD-contiguous logical id: block g runs on XCD g % 8
  const int g = blockIdx.x, lid = (g & 7) * (nwg >> 3) + (g >> 3);
  const int i0 = (int)((long)items * lid / nwg), i1 = (int)((long)items * (lid + 1) / nwg);
  if (i0 >= i1) return;

  u32x4 bst[NLD];
  auto load_b = [&](int b, int ty_t, int tx_t) {   // B tile of an item -> registers
    const int ty0 = ty_t * 8, tx0 = tx_t * 16;
    const bf16* base = f2 + (long)b * P * cs;
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = k * 256 + tid, tr = idx / CPR, c = idx % CPR;
      const int ty = min(ty0 + (tr >> 4), h - 1), tx = tx0 + (tr & 15);
      bst[k] = *(const u32x4*)(base + (long)(ty * w + tx) * cs + 8 * c);
    }
  };
  auto store_b = [&]() {          // registers -> LDS, chunk c of target row tr in slot c ^ (tr & 15)
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = k * 256 + tid, tr = idx / CPR, c = idx % CPR;
      *(u32x4*)(sm + tr * RB + ((c ^ (tr & 15)) << 4)) = bst[k];
    }
  };

  bf16x8 qf[KS];   // this lane's query features (MFMA B operand): channels 16 ks + 8 hh ..
  int cur_q = -1;
  // item coordinates, advanced incrementally (image b, query tile qt, target tile row / column)
  int b = i0 / (ntt * nqt), qt = (i0 / ntt) % nqt, ty_t = (i0 % ntt) / ntx, tx_t = i0 % ntx;
  load_b(b, ty_t, tx_t);
  store_b();
  __syncthreads();
  for (int it = i0; it < i1; ++it) {
    int nb = b, nq_t = qt, nty_t = ty_t, ntx_t = tx_t + 1;
    if (ntx_t == ntx) {
      ntx_t = 0;
      if (++nty_t == nty) {
        nty_t = 0;
        if (++nq_t == nqt) { nq_t = 0; ++nb; }
      }
    }
    const int tt = ty_t * ntx + tx_t;
    const int qtile = b * nqt + qt;
    if (qtile != cur_q) {
      cur_q = qtile;
      const int q = min(qt * 128 + wave * 32 + rho, P - 1);
      const bf16* qp = f1 + ((long)b * P + q) * cs + 8 * hh;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) qf[ks] = *(const bf16x8*)(qp + 16 * ks);
    }
    if (it + 1 < i1) load_b(nb, nty_t, ntx_t);   // in flight during the MFMAs

    // D[target 32 n + m][query] over 4 target blocks
    f32x16 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[n][k] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 a[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int tr = 32 * n + rho, c = 2 * ks + hh;
        a[n] = *(const bf16x8*)(sm + tr * RB + ((c ^ (tr & 15)) << 4));
      }
#pragma unroll
      for (int n = 0; n < 4; ++n)
        if (!(dbg & 2)) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[n], qf[ks], acc[n], 0, 0, 0);
    }

    const int qi = wave * 32 + rho;          // query within the tile
    const int q = qt * 128 + qi;
    const bool qok = q < P;
    const int sw0 = qi & 15, sw1 = (qi >> 1) & 15;
    char* st0 = sm + BT;                     // level 0: [128 q][32 units of 8 B]
    char* st1 = st0 + 128 * 256;             // level 1: [128 q][16 units of 4 B]
    float s2[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, s3[2] = {0.f, 0.f};
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int xg = 0; xg < 2; ++xg) {
        float v[2][4];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
          for (int i = 0; i < 4; ++i) v[rr][i] = acc[n][rr * 8 + xg * 4 + i] * scale;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {   // level 0: row 2n + rr, x = 8 xg + 4 hh .. + 3
          const int u = (2 * n + rr) * 4 + 2 * xg + hh;
          const unsigned lo = pack_bf16x2(v[rr][0], v[rr][1]), hi = pack_bf16x2(v[rr][2], v[rr][3]);
          *(u32x2*)(st0 + qi * 256 + ((u ^ sw0) << 3)) = u32x2{lo, hi};
        }
        const float p0 = 0.25f * (v[0][0] + v[0][1] + v[1][0] + v[1][1]);
        const float p1 = 0.25f * (v[0][2] + v[0][3] + v[1][2] + v[1][3]);
        {   // level 1: row n, x1 = 4 xg + 2 hh, + 1
          const int u = n * 4 + 2 * xg + hh;
          *(unsigned*)(st1 + qi * 64 + ((u ^ sw1) << 2)) = pack_bf16x2(p0, p1);
        }
        s2[n >> 1][xg] += p0 + p1;
        s3[xg] += p0 + p1;
      }
    }
    // level 2 (rows 2 ty_t + m, x2 = 4 tx_t + 2 xg + hh): lane hh = m writes row m
    // levels 2 / 3 of a target tile are 4 / 2 cells of a query row: gathered in LDS (acc23,
    // 128 q x 2 rows x w2 + 128 q x w3 cells) and written once the WG's run of the tile row ends,
    // as whole lines (8 tiles x 8 B per query row); else straight out
    char* a2 = st1 + 128 * 64;
    char* a3 = a2 + 128 * 2 * w2 * 2;
    if (nlev >= 3) {   // level 2 (rows 2 ty_t + m, x2 = 4 tx_t + 2 xg + hh): lane hh = m takes row m
      const float snd0 = hh ? s2[0][0] : s2[1][0], snd1 = hh ? s2[0][1] : s2[1][1];
      const float r0 = __shfl_xor(snd0, 32), r1 = __shfl_xor(snd1, 32);
      const float own0 = hh ? s2[1][0] : s2[0][0], own1 = hh ? s2[1][1] : s2[0][1];
      // x2 order: (hh 0, xg 0), (hh 1, xg 0), (hh 0, xg 1), (hh 1, xg 1); s2 holds 4 level-1 cells
      const float c0 = 0.25f * (hh ? r0 : own0), c1 = 0.25f * (hh ? own0 : r0);
      const float c2 = 0.25f * (hh ? r1 : own1), c3 = 0.25f * (hh ? own1 : r1);
      const u32x2 v2 = u32x2{pack_bf16x2(c0, c1), pack_bf16x2(c2, c3)};
      const int Y2 = 2 * ty_t + hh;
      if (acc23)
        *(u32x2*)(a2 + ((qi * 2 + hh) * w2 + 4 * tx_t) * 2) = v2;
      else if (qok && Y2 < h2)
        *(u32x2*)(l2 + (((long)b * P + q) * h2 + Y2) * w2 + 4 * tx_t) = v2;
    }
    if (nlev >= 4) {   // level 3: one cell pair per query, x3 = 2 tx_t + xg
      const float t0 = s3[0] + __shfl_xor(s3[0], 32), t1 = s3[1] + __shfl_xor(s3[1], 32);
      const unsigned v3 = pack_bf16x2(t0 * 0.0625f, t1 * 0.0625f);
      if (acc23) {
        if (hh == 0) *(unsigned*)(a3 + (qi * w3 + 2 * tx_t) * 2) = v3;
      } else if (qok && hh == 0 && ty_t < h3) {
        *(unsigned*)(l3 + (((long)b * P + q) * h3 + ty_t) * w3 + 2 * tx_t) = v3;
      }
    }
    lds_sync();   // the B tile is consumed, the outputs staged
    if (it + 1 < i1) store_b();   // (waits for its loads: issued after the previous item's stores)
    // levels 0 / 1: whole per-query blocks, 16 threads per query row of 256 B
    {
      const long qrow = (long)b * P + qt * 128;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx = k * 256 + tid, qj = idx >> 4, c = idx & 15, s = qj & 15;
        u32x4 v = *(const u32x4*)(st0 + qj * 256 + ((c ^ (s >> 1)) << 4));
        if (s & 1) v = u32x4{v[2], v[3], v[0], v[1]};
        const long o0 = qtmajor ? ((((long)b * nqt + qt) * ntt + tt) * 128 + qj) * 128 : (qrow + qj) * qs0 + (long)tt * 128;
        if (qt * 128 + qj < P && !(dbg & 1)) *(u32x4*)(l0 + o0 + 8 * c) = v;
      }
      if (nlev >= 2) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int idx = k * 256 + tid, qj = idx >> 2, c = idx & 3, s = (qj >> 1) & 15;
          // 16-B chunk c = 4-B units 4c .. 4c + 3, stored at slots (4c + i) ^ s
          unsigned e[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) e[i] = *(const unsigned*)(st1 + qj * 64 + (((4 * c + i) ^ s) << 2));
          const long o1 = qtmajor ? ((((long)b * nqt + qt) * ntt + tt) * 128 + qj) * 32 : (qrow + qj) * qs1 + (long)tt * 32;
          if (qt * 128 + qj < P && !(dbg & 1)) *(u32x4*)(l1 + o1 + 8 * c) = u32x4{e[0], e[1], e[2], e[3]};
        }
      }
      if (acc23 && nlev >= 3 && (tx_t == ntx - 1 || it + 1 == i1)) {
        // this WG's run of tile row ty_t ends: tiles tx_lo .. tx_t of it are in LDS
        const int tx_lo = tx_t - (it - (it - tx_t > i0 ? it - tx_t : i0));
        const int nt = tx_t - tx_lo + 1;
        for (int idx = tid; idx < 128 * 2 * nt; idx += 256) {
          const int qj = idx / (2 * nt), r = idx - qj * 2 * nt, m = r / nt, t = tx_lo + r - m * nt;
          const int Y2 = 2 * ty_t + m;
          if (qt * 128 + qj < P && Y2 < h2)
            *(u32x2*)(l2 + ((qrow + qj) * h2 + Y2) * w2 + 4 * t) = *(const u32x2*)(a2 + ((qj * 2 + m) * w2 + 4 * t) * 2);
        }
        if (nlev >= 4 && ty_t < h3) {
          for (int idx = tid; idx < 128 * nt; idx += 256) {
            const int qj = idx / nt, t = tx_lo + idx - qj * nt;
            if (qt * 128 + qj < P)
              *(unsigned*)(l3 + ((qrow + qj) * h3 + ty_t) * w3 + 2 * t) = *(const unsigned*)(a3 + (qj * w3 + 2 * t) * 2);
          }
        }
      }
    }
    lds_sync();   // B(it + 1) in place; staging reads done
    b = nb; qt = nq_t; ty_t = nty_t; tx_t = ntx_t;
  }
}

}  // namespace

// Returns hipErrorNotSupported when the shape is not one this kernel handles (the caller
// falls back to the tile kernel of corr.hip).
extern "C" int jr_corr_pyramid_blocked(const void* f1, const void* f2, int B, int h, int w, int C, int cs, void* l0,
                                       void* l1, void* l2, void* l3, int nlev, float scale, hipStream_t stream) {
  if ((C != 128 && C != 256) || w % 16 || cs % 8 || nlev < 1 || nlev > 4 || h < 8) return (int)hipErrorNotSupported;
  for (void* p : {l0, l1, l2, l3})
    if (reinterpret_cast<uintptr_t>(p) % 16) return (int)hipErrorNotSupported;
  const long P = (long)h * w, nqt = (P + 127) / 128, ntt = (long)(w / 16) * ((h + 7) / 8);
  const long items_l = (long)B * nqt * ntt;
  if (items_l >= (1L << 31)) return (int)hipErrorNotSupported;
  const int items = (int)items_l;
  const int occ = 1;
  static const int qtm = getenv("JR_PYR_QT") != nullptr;   // experiment: query-tile-major levels 0 / 1
  static const int dbg = getenv("JR_PYR_DBG") ? atoi(getenv("JR_PYR_DBG")) : 0;   // 1: no L0/L1 stores, 2: no MFMA
  int nwg = occ * 256;
  if (items < nwg) nwg = (int)((items + 7) / 8 * 8);
  // the B tile, the level 0 / 1 staging (40 KB), the level 2 / 3 rows (w <= 256)
  const int w2 = w / 4, w3 = w / 8;
  const int acc23 = w <= 256 && nlev >= 3;
  const int lds = 128 * 2 * C + 128 * (256 + 64) + (acc23 ? 128 * (2 * w2 + w3) * 2 : 0);
  if (lds > 160 * 1024 / occ) return (int)hipErrorNotSupported;
#define JR_PYR(KS_, OCC_)                                                                                        \
  {                                                                                                              \
    static const bool attr = hipFuncSetAttribute((const void*)corr_pyr_blocked_kernel<KS_, OCC_>,               \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 / OCC_) == hipSuccess; \
    if (!attr) return (int)hipErrorInvalidValue;                                                                 \
    hipLaunchKernelGGL((corr_pyr_blocked_kernel<KS_, OCC_>), dim3(nwg), dim3(256), lds, stream, (const bf16*)f1,        \
                       (const bf16*)f2, h, w, cs, (bf16*)l0, (bf16*)l1, (bf16*)l2, (bf16*)l3, nlev, scale, items,  \
                       nwg, acc23, qtm, dbg);                                                                            \
  }
  if (C == 256) JR_PYR(16, 1) else JR_PYR(8, 1)
#undef JR_PYR
  return (int)hipGetLastError();
}
