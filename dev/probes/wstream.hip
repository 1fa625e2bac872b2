// Is the per-CU weight stream of the halo / GRU kernels (~30 GB/s per CU measured in situ) bound by
// every workgroup reading the SAME weight fragment at the same time (one L2 channel serving the
// whole XCD), or by the per-CU load path?  A stand-in for the K loop of conv_halo_kernel /
// pipe_gemm (halo.h): each wave streams S 1-KB A fragments of its 32-channel block through a ring
// PD deep and feeds each to TN MFMAs against a register B operand.
//   order 0: every workgroup walks k-steps 0 .. S-1 (the kernels' order)
//   order 1: workgroup g starts at k-step (g * 11) % S and wraps (same bytes, staggered in time)
//   order 2: as 0 with a private weight copy per XCD-slot (g % 64): 64 distinct streams
//   mfma 0: no MFMA, the fragment is only folded into a register (pure load stream)
// hipcc --offload-arch=gfx950 -O3 dev/probes/wstream.hip -o /tmp/ws && /tmp/ws
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

template <int S, int PD, int TN, int WCO, int WPX, int order, int mfma>
__global__ __launch_bounds__(64 * WCO * WPX, 1) void stream(const u32x4* __restrict__ w, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wc = wave % WCO;
  const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, 0x7fffffff, 0x00020000);
  const int rot = order == 1 ? (int)(blockIdx.x * 11u) % S : 0;
  const unsigned copy = order == 2 ? (blockIdx.x & 63u) * (unsigned)(WCO * S * 1024) : 0u;
  const unsigned base = copy + (unsigned)(wc * S * 64 + lane) * 16u;
  auto ld = [&](int s) {
    int k = s + rot;
    k = k >= S ? k - S : k;
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ws, base + (unsigned)k * 1024u, 0, 0));
  };
  bf16x8 ring[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) ring[d] = ld(d);
  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[b][k] = 0.f;
  bf16x8 bop;
#pragma unroll
  for (int k = 0; k < 8; ++k) bop[k] = (__bf16)(float)(lane + k);
  u32x4 x = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const bf16x8 a = ring[s % PD];
    if (s + PD < S) ring[s % PD] = ld(s + PD);
    if constexpr (mfma) {
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bop, acc[b], 0, 0, 0);
    } else {
      x ^= __builtin_bit_cast(u32x4, a);
    }
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  float r = (float)(x[0] ^ x[1] ^ x[2] ^ x[3]);
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int k = 0; k < 16; ++k) r += acc[b][k];
  if (r == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = r;   // keep the work alive
}

template <int S, int PD, int TN, int WCO, int WPX, int order, int mfma>
int run1(const char* name, const u32x4* w, float* out, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 20;
  hipLaunchKernelGGL((stream<S, PD, TN, WCO, WPX, order, mfma>), dim3(grid), dim3(64 * WCO * WPX), 0, 0, w, out);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int t = 0; t < 3; ++t) {
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL((stream<S, PD, TN, WCO, WPX, order, mfma>), dim3(grid), dim3(64 * WCO * WPX), 0, 0, w, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const double us = best * 1e3 / reps;
  const double bytes = (double)grid * WCO * WPX * S * 1024.0;
  const double mf = (double)grid * WCO * WPX * S * TN * 32.0 * 32 * 16 * 2;
  printf("%-24s grid %5d  mfma %d order %d: %8.2f us  weight stream %6.1f GB/s per CU  (%5.1f %% of MFMA peak)\n",
         name, grid, mfma, order, us, bytes / (us * 1e-6) / 256 / 1e9, mfma ? mf / (us * 1e-6) / 2.5e15 * 100 : 0.0);
  return 0;
}

template <int S, int PD, int TN, int WCO, int WPX>
int run(const char* name, const u32x4* w, float* out, int grid) {
  run1<S, PD, TN, WCO, WPX, 0, 1>(name, w, out, grid);
  run1<S, PD, TN, WCO, WPX, 1, 1>(name, w, out, grid);
  run1<S, PD, TN, WCO, WPX, 2, 1>(name, w, out, grid);
  run1<S, PD, TN, WCO, WPX, 0, 0>(name, w, out, grid);
  return 0;
}

int main() {
  u32x4* w;
  float* out;
  CK(hipMalloc(&w, 64L * 8 * 144 * 1024));
  CK(hipMemset(w, 0, 64L * 8 * 144 * 1024));
  CK(hipMalloc(&out, 1 << 24));
  // layer-3 encoder conv (128 -> 128, cfg {128, 4, 2, 2, 8, 16}): 224 workgroups at batch 4
  run<72, 16, 2, 4, 2>("cin128 wco4 wpx2 tn2", w, out, 224);
  run<72, 16, 2, 4, 2>("cin128 wco4 wpx2 tn2", w, out, 2048);
  // layer-1 (64 -> 64, cfg {64, 2, 2, 2, 8, 16}): 3584 workgroups per image half
  run<36, 8, 2, 2, 2>("cin64 wco2 wpx2 tn2", w, out, 3584);
  // loop conv (256 -> 256 class, cfg {256, 6, 1, 4, 8, 16}): 224 workgroups at batch 4
  run<144, 8, 4, 6, 1>("cin256 wco6 wpx1 tn4", w, out, 224);
  return 0;
}
