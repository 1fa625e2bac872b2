// Inference mask head: the MaskPredictor's final 1x1 conv (256 -> 576,
// jax_raft/model.py:394-400) fused with the convex x8 upsampling of the flow
// (model.py:85-98) on gfx950 MFMA.  The 576 mask logits of a pixel never leave
// the registers.
//
// GEMM: logits[576][P] = W[576][256] . feat[256][P] on mfma_f32_16x16x32_bf16
// with tap-major rows (channel k*64 + s, the reference's own order).  Block
// (x, g) owns sub-pixel group g (sub-pixels 16g .. 16g+15 of all 9 taps = 9
// row tiles of 16 = 144 rows) for 4 waves x NC pixel column tiles of 16.  By
// the MFMA C layout (row = 4*(lane>>4) + j, column = lane & 15) each lane ends
// with the 9 logits of 4 adjacent sub-pixels of one pixel: softmax over the
// taps + the convex combination of the 3x3 flow neighbourhood in registers,
// and the 4 sub-pixels are 4 adjacent columns of one output row -> one
// 32-byte store per lane and pixel.  Unlike the generic conv epilogue
// (EPI_CONVEX, 9 taps padded to 16 per sub-pixel) no MFMA row is wasted: 576
// rows of work instead of 1024.
//
// Operands:
//   A (weights) is packed host-side (ops/native.py:pack_convex_head) as
//   [kstep 8][tap 9][group 4][lane 64][8 bf16]; a block copies its group's
//   72 KB once into LDS with global_load_lds (no VGPR staging), and each
//   lane's fragment is one conflict-free ds_read_b128 (64 lanes x 16
//   contiguous bytes).  Splitting the 576 rows over blocks (instead of all
//   rows per block) keeps the weight traffic per pixel low.
//   B (features) fragments are 16-byte global loads straight from the NHWC
//   rows (pixel = column, 8 consecutive channels = the lane's k slice).  All
//   8 k-steps of a wave's tiles are loaded at once (64 VGPRs at 2 tiles): one
//   memory round trip per block instead of one per k-step, which is what
//   bounded the k-step-pipelined variants (~25 us at raft_large batch 4:
//   waves lived the whole kernel waiting on loads; measured in round 2, the study file was never
//   committed -- the current kernel's numbers: profiles/r4_convex_persist_ab.txt).
//   Block order is XCD-aware: the 4 groups of one pixel block get block ids
//   equal mod 8, so they run on one XCD and share its L2 copy of the features.
#pragma once
#include "common.h"
#include "kernels.h"

namespace {


// group g's A fragments -> LDS (global_load_lds, no VGPR staging; completion: the caller's barrier)
JR_DEVICE void convex_head_load_a(const u32x4* __restrict__ wpk, int g, u32x4* __restrict__ sA) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int f = wave; f < 72; f += 4)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wpk + (f * 4 + g) * 64 + lane),
                                     (__attribute__((address_space(3))) void*)(sA + f * 64), 16, 0, 0);
}

// pixel block pb of group g (A fragments already in sA, or in flight when `sync`: then the block
// barrier after the B loads completes them)
template <int NC>
JR_DEVICE void convex_head_tile(const bf16* __restrict__ feat, int fcs, int fcoff, const float* __restrict__ bias,
                                float alpha, const float* __restrict__ flow, int B, int h, int w,
                                float* __restrict__ out, int g, int pb, bool sync, const u32x4* __restrict__ sA);

// one block (id) -- kernel body shared with the merged launches of merged.hip; sA: the caller's LDS
template <int NC>  // pixel column tiles of 16 per wave (1 or 2)
JR_DEVICE void convex_head_block(const bf16* __restrict__ feat, int fcs, int fcoff, const u32x4* __restrict__ wpk,
                                 const float* __restrict__ bias, float alpha, const float* __restrict__ flow, int B,
                                 int h, int w, float* __restrict__ out, const long long* __restrict__ out_slot,
                                 long out_off, int nblk, int id, u32x4* __restrict__ sA) {
  // sA: 8 * 9 * 64 LDS entries for this group's A fragments ([ks][tap][lane])
  const int g = (id >> 3) & 3, pb = (id >> 5) * 8 + (id & 7);
  if (pb >= nblk) return;  // whole block, before any barrier
  if (out_slot) out = (float*)(*out_slot) + out_off;  // output address supplied at run time (fresh tensor per call)
  convex_head_load_a(wpk, g, sA);
  convex_head_tile<NC>(feat, fcs, fcoff, bias, alpha, flow, B, h, w, out, g, pb, true, sA);
}

template <int NC>
JR_DEVICE void convex_head_tile(const bf16* __restrict__ feat, int fcs, int fcoff, const float* __restrict__ bias,
                                float alpha, const float* __restrict__ flow, int B, int h, int w,
                                float* __restrict__ out, int g, int pb, bool sync, const u32x4* __restrict__ sA) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int HW = h * w, M = B * HW;
  const int col = lane & 15, q = lane >> 4;
  const int p0 = (pb * 4 + wave) * 16 * NC;  // first pixel of this wave
  u32x4 b[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    // clamped in-bounds; the tail's columns are never stored
    const bf16* bp = feat + (long)min(p0 + 16 * c + col, M - 1) * fcs + fcoff + 8 * q;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) b[c][ks] = *(const u32x4*)(bp + 32 * ks);
  }
  f32x4 acc[9][NC];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[k][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (sync) __syncthreads();  // waits for the LDS copies (and the B loads) of every wave
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, sA[(ks * 9 + k) * 64 + lane]);
#pragma unroll
      for (int c = 0; c < NC; ++c)
        acc[k][c] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, b[c][ks]), acc[k][c], 0, 0, 0);
    }
  }

  // epilogue: lane holds sub-pixels s = 16g + 4q + j (j < 4) = output row
  // 2g + (q >> 1), columns 4*(q & 1) + j, for pixel column `col` of each tile.
  // Softmax in base 2: log2(e) folded into the scale, v_exp_f32 directly.
  const float a2 = alpha * 1.4426950408889634f;
  float bv[9][4];
  const float* bias_ = bias;
  asm volatile("" : "+s"(bias_));   // the persistent kernel's tile loop must not hoist these 36 VGPRs
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float4 t = *(const float4*)(bias_ + k * 64 + 16 * g + 4 * q);
    bv[k][0] = t.x * a2; bv[k][1] = t.y * a2; bv[k][2] = t.z * a2; bv[k][3] = t.w * a2;
  }
  const int sy = 2 * g + (q >> 1), sx0 = 4 * (q & 1);
  const long W8 = 8L * w;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int m = p0 + 16 * c + col;
    if (m >= M) continue;
    const int b_ = m / HW, rem = m - b_ * HW;
    const int y = rem / w, x = rem - y * w;
    float fx[9], fy[9];
    const float* fb = flow + 2L * b_ * HW;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
      float2 f = make_float2(0.f, 0.f);
      if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) f = *(const float2*)(fb + 2 * (yy * w + xx));
      fx[k] = f.x;
      fy[k] = f.y;
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float lg[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) lg[k] = fmaf(acc[k][c][j], a2, bv[k][j]);
      const float mx = fmaxf(fmaxf(fmaxf(lg[0], lg[1]), fmaxf(lg[2], lg[3])),
                             fmaxf(fmaxf(lg[4], lg[5]), fmaxf(fmaxf(lg[6], lg[7]), lg[8])));
      float s = 0.f, ux = 0.f, uy = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const float e = __builtin_amdgcn_exp2f(lg[k] - mx);
        s += e;
        ux = fmaf(e, fx[k], ux);
        uy = fmaf(e, fy[k], uy);
      }
      const float inv = 8.0f * rcpf_(s);
      o[2 * j] = ux * inv;
      o[2 * j + 1] = uy * inv;
    }
    float4* op = (float4*)(out + 2 * (((long)b_ * 8 * h + 8 * y + sy) * W8 + 8 * x + sx0));
    op[0] = make_float4(o[0], o[1], o[2], o[3]);
    op[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}


// Persistent form: 4 x nslot blocks (2 per CU); block (group g, slot) loads its group's 72 KB of A
// fragments ONCE and walks pixel blocks slot, slot + nslot, ... (the per-block weight copy, ~1/3 of
// the bytes the short-lived blocks move, is paid once per block instead of once per pixel block).
template <int NC>
__global__ __launch_bounds__(256, 2) void convex_head_persist_kernel(const bf16* __restrict__ feat, int fcs, int fcoff,
                                                                     const u32x4* __restrict__ wpk,
                                                                     const float* __restrict__ bias, float alpha,
                                                                     const float* __restrict__ flow, int B, int h,
                                                                     int w, float* __restrict__ out,
                                                                     const long long* __restrict__ out_slot,
                                                                     long out_off, int nblk, int nslot) {
  __shared__ u32x4 sA[8 * 9 * 64];
  const int id = blockIdx.x;
  const int g = (id >> 3) & 3, slot = (id >> 5) * 8 + (id & 7);
  if (slot >= nslot || slot >= nblk) return;
  if (out_slot) out = (float*)(*out_slot) + out_off;
  convex_head_load_a(wpk, g, sA);
  bool first = true;
  for (int pb = slot; pb < nblk; pb += nslot) {
    convex_head_tile<NC>(feat, fcs, fcoff, bias, alpha, flow, B, h, w, out, g, pb, first, sA);
    first = false;
  }
}

template <int NC>
__global__ __launch_bounds__(256, 2) void convex_head_kernel(const bf16* __restrict__ feat, int fcs, int fcoff,
                                                             const u32x4* __restrict__ wpk,
                                                             const float* __restrict__ bias, float alpha,
                                                             const float* __restrict__ flow, int B, int h, int w,
                                                             float* __restrict__ out, const long long* __restrict__ out_slot,
                                                             long out_off, int nblk) {
  __shared__ u32x4 sA[8 * 9 * 64];
  convex_head_block<NC>(feat, fcs, fcoff, wpk, bias, alpha, flow, B, h, w, out, out_slot, out_off, nblk, blockIdx.x,
                        sA);
}
}  // namespace
