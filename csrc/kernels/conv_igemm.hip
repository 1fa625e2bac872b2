// NHWC implicit-GEMM convolution on gfx950 MFMA: launcher dispatch over the
// tile-config families (kernel templates and design notes: conv_igemm.h).
#include "kernels.h"

extern "C" int jr_conv_family_r(const ConvParams* p, int cfg, int epi, hipStream_t stream);
extern "C" int jr_conv_family_rw(const ConvParams* p, int cfg, int epi, hipStream_t stream);
extern "C" int jr_conv_family_p(const ConvParams* p, int cfg, int epi, hipStream_t stream);
extern "C" int jr_conv_family_m32(const ConvParams* p, int cfg, int epi, hipStream_t stream);
extern "C" int jr_conv_family_d2(const ConvParams* p, int cfg, int epi, hipStream_t stream);
extern "C" int jr_conv_family_g(const ConvParams* p, int cfg, int epi, hipStream_t stream);

extern "C" int jr_conv_forward(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  if (p->M <= 0) return 0;
  int r = jr_conv_family_r(p, cfg, epi, stream);
  if (r == -1) r = jr_conv_family_rw(p, cfg, epi, stream);
  if (r == -1) r = jr_conv_family_p(p, cfg, epi, stream);
  if (r == -1) r = jr_conv_family_m32(p, cfg, epi, stream);
  if (r == -1) r = jr_conv_family_d2(p, cfg, epi, stream);
  if (r == -1) r = jr_conv_family_g(p, cfg, epi, stream);
  return r == -1 ? (int)hipErrorInvalidValue : r;
}
