// Shared pieces of the LDS-footprint ("halo") kernels gru_halo.hip and conv_halo.hip:
// the input a tile touches lives in LDS as an image of pixel rows, B fragments are read
// from it shifted by the tap, and the weights stream from L2 straight into the MFMA A
// registers in fragment order (ops/native.py:pack_gru_halo).
#pragma once
#include "conv_igemm.h"

namespace {

constexpr unsigned HOOB = 0x80000000u;   // buffer offset past every range: the load returns zeros
constexpr int FPITCH = 256;               // F image row: 256 bf16 (32 16-B chunks, 512 B)
constexpr int RPITCH = 128;               // r*h image row: 128 bf16 (16 chunks, 256 B)

JR_DEVICE int f_off(int row, int chunk) { return row * FPITCH + (((chunk & 16) | ((chunk ^ row) & 15)) << 3); }
JR_DEVICE int r_off(int row, int chunk) { return row * RPITCH + (((chunk ^ row) & 15) << 3); }

JR_DEVICE u32x4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// One wave's K loop: acc[b] += A(s) . B(s, b) over S k-steps.  A (the weights) streams from
// global memory through a register ring PD k-steps deep, B (pixels) comes from LDS one k-step
// ahead.  A scheduling barrier closes every k-step: without it hipcc sinks the ring refills
// towards their use (measured: 8 loads in flight instead of PD), i.e. the weight stream -- the
// bound of this kernel at batch 1 -- would run at half the depth.
template <int NB, int S, int PD, typename LA, typename RB>
JR_DEVICE void pipe_gemm(f32x16 (&acc)[NB], bf16x8 (&ring)[PD], LA&& loadA, RB&& readB) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[b][k] = 0.f;
  bf16x8 bcur[NB], bnxt[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) bcur[b] = readB(0, b);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const bf16x8 a = ring[s % PD];
    if (s + PD < S) ring[s % PD] = loadA(s + PD);
    if (s + 1 < S) {
#pragma unroll
      for (int b = 0; b < NB; ++b) bnxt[b] = readB(s + 1, b);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bcur[b], acc[b], 0, 0, 0);
#pragma unroll
    for (int b = 0; b < NB; ++b) bcur[b] = bnxt[b];
    // order inside the k-step: next B fragments (DS read), the ring refill (VMEM read), then
    // this step's MFMAs -- so the LDS latency of B(s + 1) hides behind MFMA(s)
    __builtin_amdgcn_sched_group_barrier(0x100, NB, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, NB, 0);
    asm volatile("" ::: "memory");   // no memory op crosses a k-step (IR passes ignore sched_barrier)
    __builtin_amdgcn_sched_barrier(0);
  }
}

}  // namespace
