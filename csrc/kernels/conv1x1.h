// Pointwise conv with LDS-resident weights, for the 1x1 convs of the
// refinement loop whose K is awkward for the implicit-GEMM tiles: the
// correlation features' first conv (MotionEncoder.convcorr1, model.py:275:
// 324 -> 256 + ReLU at raft_large).  The generic conv runs it as 220
// one-round 256x128 tiles with K = 328 padded to six 64-deep stages (17 us at
// batch 4); here (as in convex_head.hip):
//   * block (pixel block, output group g of 64 channels): the group's weights
//     (64 rows x K, e.g. 44 KB at K = 352) are copied once into LDS with
//     global_load_lds and read as conflict-free ds_read_b128 A fragments;
//   * each wave owns NC x 16 pixels and loads every k-step of their features
//     up front (16 B per lane and step, straight from the NHWC rows; chunks at
//     or past `kvalid` read as zero) -- one memory round trip per wave;
//   * XCD-aware block order: the groups of one pixel block run on one XCD and
//     share its L2 copy of the features;
//   * rows are permuted at pack time (ops/native.py:pack_conv1x1) so a lane
//     ends with 16 contiguous output channels of its pixel: bias + activation
//     and two 16-byte stores.
#pragma once
#include "common.h"
#include "kernels.h"

namespace {

// one block (id); sA: KS * 4 * 64 LDS entries for this group's A fragments ([k-step][row tile 4][lane])
// -- body shared with the merged launch of merged.hip
template <int KS, int NC>  // KS = padded K / 32, NC = 16-pixel tiles per wave
JR_DEVICE void conv1x1_block(const bf16* __restrict__ x, int xcs, int kvalid, const u32x4* __restrict__ wpk,
                             const float* __restrict__ bias, int act, bf16* __restrict__ y, int ycs, int ycoff, int M,
                             int ngroups, int nblk, int id, u32x4* __restrict__ sA) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = (id >> 3) % ngroups;
  const int pb = (id / (8 * ngroups)) * 8 + (id & 7);
  if (pb >= nblk) return;  // whole block, before any barrier
  const u32x4* src = wpk + (long)g * KS * 4 * 64;
  for (int f = wave; f < KS * 4; f += 4)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + f * 64 + lane),
                                     (__attribute__((address_space(3))) void*)(sA + f * 64), 16, 0, 0);
  const int col = lane & 15, q = lane >> 4;
  const int p0 = (pb * 4 + wave) * 16 * NC;
  u32x4 b[NC][KS];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const bf16* bp = x + (long)min(p0 + 16 * c + col, M - 1) * xcs + 8 * q;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      b[c][ks] = (32 * ks + 8 * q < kvalid) ? *(const u32x4*)(bp + 32 * ks) : u32x4{0u, 0u, 0u, 0u};
  }
  f32x4 acc[4][NC];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // the LDS weight copies (and the feature loads) of every wave
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, sA[(ks * 4 + t) * 64 + lane]);
#pragma unroll
      for (int c = 0; c < NC; ++c)
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, b[c][ks]), acc[t][c], 0, 0, 0);
    }
  }
  // lane (col, q): channels g*64 + 16q + (4t + j) <- acc[t][c][j] (pack-time row permutation)
  const int c0 = g * 64 + 16 * q;
  float bv[16];
#pragma unroll
  for (int i = 0; i < 16; i += 4) {
    const float4 t4 = *(const float4*)(bias + c0 + i);
    bv[i] = t4.x; bv[i + 1] = t4.y; bv[i + 2] = t4.z; bv[i + 3] = t4.w;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int m = p0 + 16 * c + col;
    if (m >= M) continue;
    bf16x8 o0, o1;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[t][c][j] + bv[4 * t + j];
        v = apply_act(v, act, c0 + 4 * t + j, 0);
        if (t < 2) o0[4 * t + j] = f2bf(v);
        else o1[4 * (t - 2) + j] = f2bf(v);
      }
    bf16* yp = y + (long)m * ycs + ycoff + c0;
    *(bf16x8*)yp = o0;
    *(bf16x8*)(yp + 8) = o1;
  }
}


template <int KS, int NC>
__global__ __launch_bounds__(256, 2) void conv1x1_lds_kernel(const bf16* __restrict__ x, int xcs, int kvalid,
                                                             const u32x4* __restrict__ wpk,
                                                             const float* __restrict__ bias, int act,
                                                             bf16* __restrict__ y, int ycs, int ycoff, int M,
                                                             int ngroups, int nblk) {
  __shared__ u32x4 sA[KS * 4 * 64];
  conv1x1_block<KS, NC>(x, xcs, kvalid, wpk, bias, act, y, ycs, ycoff, M, ngroups, nblk, blockIdx.x, sA);
}

}  // namespace
