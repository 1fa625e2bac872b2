// Launcher of the LDS-resident-weight pointwise conv (kernel body: conv1x1.h).
#include "conv1x1.h"


extern "C" int jr_conv1x1_lds(const void* x, int x_cstride, int kvalid, int kpad, const void* wpk, const float* bias,
                              int act, void* y, int y_cstride, int y_coff, int cout, int M, hipStream_t stream) {
  if (cout % 64 || kpad % 32 || kvalid > kpad || x_cstride % 8 || y_cstride % 8 || y_coff % 8)
    return (int)hipErrorInvalidValue;
  constexpr int NC = 2;
  const int ngroups = cout / 64;
  const int nblk = (M + 64 * NC - 1) / (64 * NC);
  const dim3 grid((nblk + 7) / 8 * 8 * ngroups);
#define JR_C1(KS)                                                                                                   \
  case KS:                                                                                                          \
    hipLaunchKernelGGL((conv1x1_lds_kernel<KS, NC>), grid, dim3(256), 0, stream, (const bf16*)x, x_cstride, kvalid, \
                       (const u32x4*)wpk, bias, act, (bf16*)y, y_cstride, y_coff, M, ngroups, nblk);                 \
    break;
  switch (kpad / 32) {
    JR_C1(4) JR_C1(8) JR_C1(11) JR_C1(12)
    default: return (int)hipErrorInvalidValue;
  }
#undef JR_C1
  return (int)hipGetLastError();
}
