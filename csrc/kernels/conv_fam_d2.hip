// Tile-config instantiations of the implicit-GEMM conv, family "d2"
// (templates in conv_igemm.h; dispatch in conv_igemm.hip).
#include "conv_igemm.h"

extern "C" int jr_conv_family_d2(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 6: return launch_cfg<128, 128, 2, 3>(p, epi, stream);
    case 7: return launch_cfg<64, 128, 1, 4>(p, epi, stream);
    case 8: return launch_cfg<128, 64, 2, 4>(p, epi, stream);
    case 9: return launch_cfg<128, 256, 2, 3>(p, epi, stream);
    case 10: return launch_cfg<64, 64, 1, 4>(p, epi, stream);
    case 11: return launch_cfg<256, 128, 2, 3>(p, epi, stream);
    default: return -1;
  }
}
