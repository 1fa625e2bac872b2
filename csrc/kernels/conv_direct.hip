// Launcher of the 2-channel flow conv (kernel: conv_direct.h).
#include "conv_direct.h"


extern "C" int jr_conv_direct(const void* x, int x_cstride, int N, int H, int W, int cin, int KH, int KW, int PH,
                              int PW, const void* w, const float* bias, int cout, int relu, void* y, int y_cstride,
                              int y_coff, hipStream_t stream) {
  if (cin != 2 || cout % 32 != 0 || y_cstride % 4 != 0 || y_coff % 4 != 0 || y_coff + cout > y_cstride ||
      x_cstride < 2 || x_cstride % 2 != 0)
    return (int)hipErrorInvalidValue;
  const int M = N * H * W;
  dim3 grid((M + 63) / 64, (cout / 32 + 3) / 4);
  if (KH == 7 && KW == 7)
    hipLaunchKernelGGL((conv_flowin_kernel<7, 7>), grid, dim3(256), 0, stream, (const bf16*)x, x_cstride, N, H, W, PH,
                       PW, (const bf16x8*)w, bias, cout, relu, (bf16*)y, y_cstride, y_coff);
  else if (KH == 3 && KW == 3)
    hipLaunchKernelGGL((conv_flowin_kernel<3, 3>), grid, dim3(256), 0, stream, (const bf16*)x, x_cstride, N, H, W, PH,
                       PW, (const bf16x8*)w, bias, cout, relu, (bf16*)y, y_cstride, y_coff);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
