// Tile-config instantiations of the implicit-GEMM conv, family "m32"
// (templates in conv_igemm.h; dispatch in conv_igemm.hip).
#include "conv_igemm.h"

extern "C" int jr_conv_family_m32(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 12: return launch_cfg<128, 128, 2, 2>(p, epi, stream);
    case 13: return launch_cfg<64, 128, 1, 2>(p, epi, stream);
    case 14: return launch_cfg<128, 64, 2, 2>(p, epi, stream);
    case 15: return launch_cfg<64, 64, 2, 2>(p, epi, stream);
    case 25: return launch_cfg<256, 128, 4, 8>(p, epi, stream);   // 8 waves, 64x64
    case 26: return launch_cfg<128, 256, 2, 8>(p, epi, stream);   // 8 waves, 64x64
    case 27: return launch_cfg<128, 128, 2, 8>(p, epi, stream);   // 8 waves, 64x32
    case 28: return launch_cfg<64, 256, 1, 8>(p, epi, stream);    // 8 waves, 64x32
    default: return -1;
  }
}
