// Merged launches for the one-lane refinement loop (batch 1 / raft_small): the
// flow branch's first conv (convflow1 of iteration i, jax_raft/model.py:282)
// and the deferred x8 upsampling of iteration i-1 (model.py:508: the convex
// mask head, or bilinear for raft_small) read the same just-updated flow and
// are independent, but in one in-order lane they ran back to back, each
// leaving most CUs idle at batch 1 (110 + 110..440 workgroups).  Here they are
// one grid: blocks [0, nfl) run the flow conv (conv_direct.h), the rest the
// upsampling (convex_head.h / upsample.h) -- concurrency without the ~6-12 us
// of a cross-stream graph edge.  nfl is padded to a multiple of 8, so the
// convex head keeps its XCD-aware block order (its block ids mod 8 unchanged).
#include "conv_direct.h"
#include "convex_head.h"
#include "upsample.h"

namespace {

struct FlowinArgs {
  const bf16* x; int xcs, N, H, W, PH, PW;
  const bf16x8* wp; const float* bias; int cout, relu;
  bf16* y; int ycs, ycoff;
  int gx, nfl;   // flow-conv blocks: gx x gy, padded to nfl (multiple of 8)
};

JR_DEVICE bool flowin_part(const FlowinArgs& f, int id) {
  if (id >= f.nfl) return false;
  const int by = id / f.gx, bx = id - by * f.gx;
  if (by * 128 < f.cout) conv_flowin_block<7, 7>(f.x, f.xcs, f.N, f.H, f.W, f.PH, f.PW, f.wp, f.bias, f.cout, f.relu,
                                                  f.y, f.ycs, f.ycoff, bx, by);
  return true;
}

template <int NC>
__global__ __launch_bounds__(256, 2) void flowin_convex_kernel(const FlowinArgs f, const bf16* __restrict__ feat,
                                                               int fcs, int fcoff, const u32x4* __restrict__ wpk,
                                                               const float* __restrict__ bias, float alpha,
                                                               const float* __restrict__ flow, int B, int h, int w,
                                                               float* __restrict__ out,
                                                               const long long* __restrict__ out_slot, long out_off,
                                                               int nblk) {
  if (flowin_part(f, blockIdx.x)) return;
  convex_head_block<NC>(feat, fcs, fcoff, wpk, bias, alpha, flow, B, h, w, out, out_slot, out_off, nblk,
                        blockIdx.x - f.nfl);
}

__global__ __launch_bounds__(256) void flowin_bilinear_kernel(const FlowinArgs f, const float* __restrict__ flow, int B,
                                                              int h, int w, float* __restrict__ out,
                                                              const long long* __restrict__ out_slot, long out_off) {
  if (flowin_part(f, blockIdx.x)) return;
  upsample_bilinear_elem(flow, B, h, w, out, out_slot, out_off, (long)(blockIdx.x - f.nfl) * 256 + threadIdx.x);
}

}  // namespace

extern "C" int jr_flowin_dual(const void* x, int x_cstride, int N, int H, int W, int PH, int PW, const void* w_,
                              const float* fbias, int cout, int relu, void* y, int y_cstride, int y_coff, int mode,
                              const void* feat, int feat_cstride, int feat_coff, const void* wpk, const float* cbias,
                              float alpha, const float* flow, float* out, const void* out_slot, long out_off,
                              hipStream_t stream) {
  if (cout % 32 != 0 || y_cstride % 4 != 0 || y_coff % 4 != 0 || y_coff + cout > y_cstride || x_cstride < 2 ||
      x_cstride % 2 != 0)
    return (int)hipErrorInvalidValue;
  const int M = N * H * W;
  FlowinArgs f{(const bf16*)x, x_cstride, N, H, W, PH, PW, (const bf16x8*)w_, fbias, cout, relu, (bf16*)y, y_cstride,
               y_coff, (M + 63) / 64, 0};
  f.nfl = (f.gx * ((cout / 32 + 3) / 4) + 7) / 8 * 8;
  if (mode == 1) {   // bilinear x8 of the flow [N][H][W][2] (the loop grid)
    const long total = (long)N * 64 * H * W;
    const unsigned nb = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL(flowin_bilinear_kernel, dim3(f.nfl + nb), dim3(256), 0, stream, f, flow, N, H, W, out,
                       (const long long*)out_slot, out_off);
  } else if (mode == 2) {   // convex mask head (jr_convex_head's tiling: 1 pixel tile per wave at small M)
    auto blocks = [M](int nc) { return (M + 64 * nc - 1) / (64 * nc); };
    const int nc = blocks(2) * 4 >= 384 ? 2 : 1;
    const int nblk = blocks(nc);
    const unsigned ng = (unsigned)((nblk + 7) / 8 * 32);
    if (nc == 2)
      hipLaunchKernelGGL(flowin_convex_kernel<2>, dim3(f.nfl + ng), dim3(256), 0, stream, f, (const bf16*)feat,
                         feat_cstride, feat_coff, (const u32x4*)wpk, cbias, alpha, flow, N, H, W, out,
                         (const long long*)out_slot, out_off, nblk);
    else
      hipLaunchKernelGGL(flowin_convex_kernel<1>, dim3(f.nfl + ng), dim3(256), 0, stream, f, (const bf16*)feat,
                         feat_cstride, feat_coff, (const u32x4*)wpk, cbias, alpha, flow, N, H, W, out,
                         (const long long*)out_slot, out_off, nblk);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
