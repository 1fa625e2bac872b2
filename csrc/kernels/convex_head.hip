// Launcher of the inference mask head (kernel: convex_head.h).
#include <cstdlib>

#include "convex_head.h"


extern "C" int jr_convex_head(const void* feat, int feat_cstride, int feat_coff, const void* wpk, const float* bias,
                              float alpha, const float* flow, int B, int h, int w, float* out, const void* out_slot,
                              long out_off, int tiles, hipStream_t stream) {
  const int M = B * h * w;
  // pixel tiles per wave (`tiles` 1 / 2, or 0 = auto): 2 when that still gives
  // >= 384 blocks (2 per CU fit: 72 KB of LDS each), else 1
  auto blocks = [M](int nc) { return (M + 64 * nc - 1) / (64 * nc); };
  const int nc = tiles == 1 || tiles == 2 ? tiles : blocks(2) * 4 >= 384 ? 2 : 1;
  const int nblk = blocks(nc);
  // the persistent form when the grid would take more than one round (128 slots x 4 groups = 2 blocks
  // per CU): 23.3 -> 20.3 us at raft_large batch 4 (profiles/r4_convex_persist_ab.txt)
  if (nblk > 128) {
    const int nslot = 128;
    const dim3 pg(nslot / 8 * 32);
    if (nc == 2)
      hipLaunchKernelGGL(convex_head_persist_kernel<2>, pg, dim3(256), 0, stream, (const bf16*)feat, feat_cstride,
                         feat_coff, (const u32x4*)wpk, bias, alpha, flow, B, h, w, out, (const long long*)out_slot,
                         out_off, nblk, nslot);
    else
      hipLaunchKernelGGL(convex_head_persist_kernel<1>, pg, dim3(256), 0, stream, (const bf16*)feat, feat_cstride,
                         feat_coff, (const u32x4*)wpk, bias, alpha, flow, B, h, w, out, (const long long*)out_slot,
                         out_off, nblk, nslot);
    return (int)hipGetLastError();
  }
  const dim3 grid((nblk + 7) / 8 * 32);
  if (nc == 2)
    hipLaunchKernelGGL(convex_head_kernel<2>, grid, dim3(256), 0, stream, (const bf16*)feat, feat_cstride, feat_coff,
                       (const u32x4*)wpk, bias, alpha, flow, B, h, w, out, (const long long*)out_slot, out_off, nblk);
  else
    hipLaunchKernelGGL(convex_head_kernel<1>, grid, dim3(256), 0, stream, (const bf16*)feat, feat_cstride, feat_coff,
                       (const u32x4*)wpk, bias, alpha, flow, B, h, w, out, (const long long*)out_slot, out_off, nblk);
  return (int)hipGetLastError();
}
