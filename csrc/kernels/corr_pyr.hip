// Correlation pyramid, blocked bf16 layout (the engine's): a persistent, write-streaming
// build of all L levels (reference CorrBlock, jax_raft/model.py:418-446 + 472-481: the
// all-pairs volume f1 . f2^T / sqrt(C), then 2x2 average pools with floor semantics).
//
// The volume (533 MB at raft_large batch 4) is the only traffic that has to reach HBM; the
// tile kernel of corr.hip re-read both feature maps per 128 x 128 tile (1.6 GB of L2 reads,
// 382 MB past L2 in round 4; the current kernels' traffic: profiles/r5_corr_study.md).  Here:
//   * one workgroup (8 waves) per CU walks a contiguous run of (image, query tile, target tile) items,
//     target tile fastest; runs are XCD-contiguous, so an XCD's CUs read one image's f2;
//   * a wave keeps its 32 queries' features in registers (the MFMA B operand) for the whole
//     run (two waves per query group, each for half the target tile); only the 128-target tile (8 x 16 pixels, the MFMA A operand) is staged in LDS,
//     its loads for item k + 1 in flight during item k's MFMAs;
//   * D[target][query]: a lane holds 16 targets of ONE query (rows 2n, 2n+1 of the tile,
//     4 consecutive x twice), so the 2x2 pools are in-lane sums, the 4x4 ones need one
//     lane^32 exchange and the 8x8 ones combine the two waves' exact level-2 cells in LDS;
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

// LDS-only barrier: the global stores and the next tile's loads stay in flight
// (__syncthreads() would drain vmcnt, i.e. wait for every store of the item)
JR_DEVICE void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// KS = C / 16 feature-channel k-steps.  8 waves, one workgroup per CU: wave (qg, th) holds
// queries 32 qg .. of the tile (64 registers of features) and computes target blocks 2 th,
// 2 th + 1 (tile rows 4 th .. 4 th + 3): two waves per SIMD hide each other's LDS / epilogue
// latency (the 4-wave form measured 255 us at batch 4, one wave per SIMD).
template <int KS>
__global__ __launch_bounds__(512, 1) void corr_pyr_blocked_kernel(const bf16* __restrict__ f1,
                                                                 const bf16* __restrict__ f2, int h, int w, int cs,
                                                                 bf16* __restrict__ l0, bf16* __restrict__ l1,
                                                                 bf16* __restrict__ l2, bf16* __restrict__ l3,
                                                                 int nlev, float scale, int items, int nwg,
                                                                 int acc23) {
  constexpr int C = 16 * KS;
  constexpr int NT = 512;
  constexpr int RB = 2 * C;               // bytes of one target row in the B tile
  constexpr int CPR = C / 8;              // 16-B chunks per target row
  constexpr int NLD = 128 * CPR / NT;     // B-tile chunks per thread
  constexpr int BT = 128 * RB;
  // LDS: [B tile | level 0 staging 32 KB | level 1 staging 8 KB | level 2 cells of the item
  //       (fp32, 4 KB) | level 2 rows (bf16, 128 q x 2 x w2) | level 3 row (bf16, 128 q x w3)]
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rho = lane & 31, hh = lane >> 5;
  const int qg = wave & 3, th = wave >> 2;
  const int P = h * w, ntx = w >> 4, nty = (h + 7) >> 3, ntt = ntx * nty, nqt = (P + 127) >> 7;
  const int h1 = h >> 1, h2 = h1 >> 1, w2 = (w >> 1) >> 1, h3 = h2 >> 1, w3 = w2 >> 1;
  const long qs0 = (long)ntt * 128, qs1 = (long)ntt * 32;   // per-query blocked level sizes
  // XCD-contiguous logical id: block g runs on XCD g % 8
  const int g = blockIdx.x, lid = (g & 7) * (nwg >> 3) + (g >> 3);
  const int i0 = (int)((long)items * lid / nwg), i1 = (int)((long)items * (lid + 1) / nwg);
  if (i0 >= i1) return;
  char* st0 = sm + BT;
  char* st1 = st0 + 128 * 256;
  float* l2c = (float*)(st1 + 128 * 64);   // [128 q][2 rows][4 cells]
  char* a2 = (char*)(l2c + 128 * 8);
  char* a3 = a2 + 128 * 2 * w2 * 2;

  u32x4 bst[NLD];
  auto load_b = [&](int b, int ty_t, int tx_t) {   // B tile of an item -> registers
    const int ty0 = ty_t * 8, tx0 = tx_t * 16;
    const bf16* base = f2 + (long)b * P * cs;
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = k * NT + tid, tr = idx / CPR, c = idx % CPR;
      const int ty = min(ty0 + (tr >> 4), h - 1), tx = tx0 + (tr & 15);
      bst[k] = *(const u32x4*)(base + (long)(ty * w + tx) * cs + 8 * c);
    }
  };
  auto store_b = [&]() {          // registers -> LDS, chunk c of target row tr in slot c ^ (tr & 15)
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = k * NT + tid, tr = idx / CPR, c = idx % CPR;
      *(u32x4*)(sm + tr * RB + ((c ^ (tr & 15)) << 4)) = bst[k];
    }
  };
  // level-3 cell pair (x3 = 2 tx + 0 / 1) of tile query qj from its exact level-2 cells
  auto l3_of = [&](int qj) {
    const float* c = l2c + qj * 8;
    return pack_bf16x2(0.25f * (c[0] + c[1] + c[4] + c[5]), 0.25f * (c[2] + c[3] + c[6] + c[7]));
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
      const int q = min(qt * 128 + qg * 32 + rho, P - 1);
      const bf16* qp = f1 + ((long)b * P + q) * cs + 8 * hh;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) qf[ks] = *(const bf16x8*)(qp + 16 * ks);
    }
    if (it + 1 < i1) load_b(nb, nty_t, ntx_t);   // in flight during the MFMAs

    // D[target 32 n + m][query], n = 2 th + nn
    f32x16 acc[2];
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[nn][k] = 0.f;
    {   // A fragments one k-step ahead (all of them in flight at once would spill)
      auto read_a = [&](int ks, bf16x8 (&a)[2]) {
#pragma unroll
        for (int nn = 0; nn < 2; ++nn) {
          const int tr = 32 * (2 * th + nn) + rho, c = 2 * ks + hh;
          a[nn] = *(const bf16x8*)(sm + tr * RB + ((c ^ (tr & 15)) << 4));
        }
      };
      bf16x8 acur[2], anxt[2];
      read_a(0, acur);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) read_a(ks + 1, anxt);
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
          acc[nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[nn], qf[ks], acc[nn], 0, 0, 0);
#pragma unroll
        for (int nn = 0; nn < 2; ++nn) acur[nn] = anxt[nn];
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    const int qi = qg * 32 + rho;            // query within the tile
    const int sw0 = qi & 15, sw1 = (qi >> 1) & 15;
    float s2[2] = {0.f, 0.f};
#pragma unroll
    for (int nn = 0; nn < 2; ++nn) {
      const int n = 2 * th + nn;
#pragma unroll
      for (int xg = 0; xg < 2; ++xg) {
        float v[2][4];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
          for (int i = 0; i < 4; ++i) v[rr][i] = acc[nn][rr * 8 + xg * 4 + i] * scale;
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
        s2[xg] += p0 + p1;
      }
    }
    if (nlev >= 3) {   // level 2: row th of the tile's two, x2 = 2 xg + hh
      const float r0 = __shfl_xor(s2[0], 32), r1 = __shfl_xor(s2[1], 32);
      if (hh == 0) {
        const float c0 = 0.25f * s2[0], c1 = 0.25f * r0, c2 = 0.25f * s2[1], c3 = 0.25f * r1;
        *(f32x4*)(l2c + qi * 8 + th * 4) = f32x4{c0, c1, c2, c3};
        const u32x2 v2 = u32x2{pack_bf16x2(c0, c1), pack_bf16x2(c2, c3)};
        const int q = qt * 128 + qi, Y2 = 2 * ty_t + th;
        if (acc23)
          *(u32x2*)(a2 + ((qi * 2 + th) * w2 + 4 * tx_t) * 2) = v2;
        else if (q < P && Y2 < h2)
          *(u32x2*)(l2 + (((long)b * P + q) * h2 + Y2) * w2 + 4 * tx_t) = v2;
      }
    }
    lds_sync();   // the B tile is consumed, the outputs staged
    if (it + 1 < i1) store_b();   // (waits for its loads: issued after the previous item's stores)
    const long qrow = (long)b * P + qt * 128;
    // levels 0 / 1: whole per-query blocks, 16 threads per query row of 256 B
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = k * NT + tid, qj = idx >> 4, c = idx & 15, s = qj & 15;
      u32x4 v = *(const u32x4*)(st0 + qj * 256 + ((c ^ (s >> 1)) << 4));
      if (s & 1) v = u32x4{v[2], v[3], v[0], v[1]};
      if (qt * 128 + qj < P) *(u32x4*)(l0 + (qrow + qj) * qs0 + (long)tt * 128 + 8 * c) = v;
    }
    if (nlev >= 2) {
      const int qj = tid >> 2, c = tid & 3, s = (qj >> 1) & 15;
      // 16-B chunk c = 4-B units 4c .. 4c + 3, stored at slots (4c + i) ^ s
      unsigned e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) e[i] = *(const unsigned*)(st1 + qj * 64 + (((4 * c + i) ^ s) << 2));
      if (qt * 128 + qj < P) *(u32x4*)(l1 + (qrow + qj) * qs1 + (long)tt * 32 + 8 * c) = u32x4{e[0], e[1], e[2], e[3]};
    }
    const bool row_end = tx_t == ntx - 1 || it + 1 == i1;
    if (nlev >= 4 && tid < 128) {   // level 3 of this tile: into the row buffer, or straight out
      const int q = qt * 128 + tid;
      if (acc23) {
        if (!row_end) *(unsigned*)(a3 + (tid * w3 + 2 * tx_t) * 2) = l3_of(tid);
      } else if (q < P && ty_t < h3) {
        *(unsigned*)(l3 + ((qrow + tid) * h3 + ty_t) * w3 + 2 * tx_t) = l3_of(tid);
      }
    }
    if (acc23 && nlev >= 3 && row_end) {
      // this WG's run of tile row ty_t ends: tiles tx_lo .. tx_t of it are in LDS (the level-3
      // cells of tile tx_t straight from the level-2 cells of this item)
      const int tx_lo = tx_t - (it - (it - tx_t > i0 ? it - tx_t : i0));
      const int nt = tx_t - tx_lo + 1;
      for (int idx = tid; idx < 128 * 2 * nt; idx += NT) {
        const int qj = idx / (2 * nt), r = idx - qj * 2 * nt, m = r / nt, t = tx_lo + r - m * nt;
        const int Y2 = 2 * ty_t + m;
        if (qt * 128 + qj < P && Y2 < h2)
          *(u32x2*)(l2 + ((qrow + qj) * h2 + Y2) * w2 + 4 * t) = *(const u32x2*)(a2 + ((qj * 2 + m) * w2 + 4 * t) * 2);
      }
      if (nlev >= 4 && ty_t < h3) {
        for (int idx = tid; idx < 128 * nt; idx += NT) {
          const int qj = idx / nt, t = tx_lo + idx - qj * nt;
          if (qt * 128 + qj < P)
            *(unsigned*)(l3 + ((qrow + qj) * h3 + ty_t) * w3 + 2 * t) =
                t == tx_t ? l3_of(qj) : *(const unsigned*)(a3 + (qj * w3 + 2 * t) * 2);
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
  int nwg = 256;
  if (items < nwg) nwg = (int)((items + 7) / 8 * 8);
  // B tile, level 0 / 1 staging (40 KB), the item's level-2 cells (4 KB), the level 2 / 3 rows (w <= 256)
  const int w2 = w / 4, w3 = w / 8;
  const int acc23 = w <= 256 && nlev >= 3;
  const int lds = 128 * 2 * C + 128 * (256 + 64 + 32) + (acc23 ? 128 * (2 * w2 + w3) * 2 : 0);
  if (lds > 160 * 1024) return (int)hipErrorNotSupported;
#define JR_PYR(KS_)                                                                                              \
  {                                                                                                              \
    static const bool attr = hipFuncSetAttribute((const void*)corr_pyr_blocked_kernel<KS_>,                     \
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess; \
    if (!attr) return (int)hipErrorInvalidValue;                                                                 \
    hipLaunchKernelGGL((corr_pyr_blocked_kernel<KS_>), dim3(nwg), dim3(512), lds, stream, (const bf16*)f1,       \
                       (const bf16*)f2, h, w, cs, (bf16*)l0, (bf16*)l1, (bf16*)l2, (bf16*)l3, nlev, scale, items,  \
                       nwg, acc23);                                                                              \
  }
  if (C == 256) JR_PYR(16) else JR_PYR(8)
#undef JR_PYR
  return (int)hipGetLastError();
}
