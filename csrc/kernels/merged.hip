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
// With `c1` (raft_large, batch 1) the grid also runs the correlation features' 1x1
// conv (convcorr1, conv1x1.h) of the same iteration: it reads the lookup's output,
// the other two parts its flow update, so all three are independent.  Its blocks
// come between the flow conv's and the convex head's (both counts multiples of 8,
// so every part keeps its XCD-aware order), and the convex head and the 1x1 conv
// share one LDS array (either part's weight fragments).
#include "conv1x1.h"
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

struct C1Args {   // the 1x1 conv part (conv1x1.h): n1 blocks (0: none)
  const bf16* x; int xcs, kvalid; const u32x4* wpk; const float* bias; int act;
  bf16* y; int ycs, ycoff, M, ngroups, nblk, n1;
};
constexpr int C1_KS = 11;   // raft_large convcorr1: K = 324 -> 352

template <int NC>
__global__ __launch_bounds__(256, 2) void flowin_convex_kernel(const FlowinArgs f, const C1Args c1,
                                                               const bf16* __restrict__ feat,
                                                               int fcs, int fcoff, const u32x4* __restrict__ wpk,
                                                               const float* __restrict__ bias, float alpha,
                                                               const float* __restrict__ flow, int B, int h, int w,
                                                               float* __restrict__ out,
                                                               const long long* __restrict__ out_slot, long out_off,
                                                               int nblk) {
  __shared__ u32x4 sA[(8 * 9 > C1_KS * 4 ? 8 * 9 : C1_KS * 4) * 64];
  if (flowin_part(f, blockIdx.x)) return;
  const int id = blockIdx.x - f.nfl;
  if (id < c1.n1) {
    conv1x1_block<C1_KS, 2>(c1.x, c1.xcs, c1.kvalid, c1.wpk, c1.bias, c1.act, c1.y, c1.ycs, c1.ycoff, c1.M, c1.ngroups,
                            c1.nblk, id, sA);
    return;
  }
  convex_head_block<NC>(feat, fcs, fcoff, wpk, bias, alpha, flow, B, h, w, out, out_slot, out_off, nblk, id - c1.n1, sA);
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
                              const Conv1x1Args* c1a, hipStream_t stream) {
  if (cout % 32 != 0 || y_cstride % 4 != 0 || y_coff % 4 != 0 || y_coff + cout > y_cstride || x_cstride < 2 ||
      x_cstride % 2 != 0)
    return (int)hipErrorInvalidValue;
  const int M = N * H * W;
  FlowinArgs f{(const bf16*)x, x_cstride, N, H, W, PH, PW, (const bf16x8*)w_, fbias, cout, relu, (bf16*)y, y_cstride,
               y_coff, (M + 63) / 64, 0};
  f.nfl = (f.gx * ((cout / 32 + 3) / 4) + 7) / 8 * 8;
  C1Args c1{};
  if (c1a) {   // mode 2 only; up = 0 (iteration 0): the flow conv + the 1x1 conv alone
    if (mode != 2 || c1a->kpad != 32 * C1_KS || c1a->cout % 64 || c1a->kvalid > c1a->kpad || c1a->xcs % 8 ||
        c1a->ycs % 8 || c1a->ycoff % 8)
      return (int)hipErrorInvalidValue;
    c1 = C1Args{(const bf16*)c1a->x, c1a->xcs, c1a->kvalid, (const u32x4*)c1a->wpk, c1a->bias, c1a->act,
                (bf16*)c1a->y, c1a->ycs, c1a->ycoff, c1a->M, c1a->cout / 64, (c1a->M + 127) / 128, 0};
    c1.n1 = (c1.nblk + 7) / 8 * 8 * c1.ngroups;
  }
  if (mode == 1) {   // bilinear x8 of the flow [N][H][W][2] (the loop grid)
    const long total = (long)N * 64 * H * W;
    const unsigned nb = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL(flowin_bilinear_kernel, dim3(f.nfl + nb), dim3(256), 0, stream, f, flow, N, H, W, out,
                       (const long long*)out_slot, out_off);
  } else if (mode == 2) {   // convex mask head (jr_convex_head's tiling: 1 pixel tile per wave at small M)
    auto blocks = [M](int nc) { return (M + 64 * nc - 1) / (64 * nc); };
    const int nc = blocks(2) * 4 >= 384 ? 2 : 1;
    const int nblk = blocks(nc);
    const unsigned ng = out ? (unsigned)((nblk + 7) / 8 * 32) : 0u;   // out == nullptr: no upsampling part
    const dim3 grid(f.nfl + c1.n1 + ng);
    if (nc == 2)
      hipLaunchKernelGGL(flowin_convex_kernel<2>, grid, dim3(256), 0, stream, f, c1, (const bf16*)feat,
                         feat_cstride, feat_coff, (const u32x4*)wpk, cbias, alpha, flow, N, H, W, out,
                         (const long long*)out_slot, out_off, nblk);
    else
      hipLaunchKernelGGL(flowin_convex_kernel<1>, grid, dim3(256), 0, stream, f, c1, (const bf16*)feat,
                         feat_cstride, feat_coff, (const u32x4*)wpk, cbias, alpha, flow, N, H, W, out,
                         (const long long*)out_slot, out_off, nblk);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
