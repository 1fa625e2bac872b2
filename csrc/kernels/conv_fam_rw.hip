// Tile-config instantiations of the implicit-GEMM conv, family "rw":
// kernel R, 8- and 16-wave blocks (templates in conv_igemm.h; dispatch in conv_igemm.hip).
#include "conv_igemm.h"

extern "C" int jr_conv_family_rw(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 18: return launch_cfg<128, 128, 2, 6>(p, epi, stream);
    case 19: return launch_cfg<128, 128, 4, 6>(p, epi, stream);
    case 20: return launch_cfg<256, 128, 4, 6>(p, epi, stream);
    case 21: return launch_cfg<128, 128, 4, 7>(p, epi, stream);   // 16 waves, 32x32 wave tiles
    case 22: return launch_cfg<256, 128, 4, 7>(p, epi, stream);   // 16 waves, 64x32
    case 23: return launch_cfg<128, 64, 2, 6>(p, epi, stream);    // 8 waves, 64x16
    case 24: return launch_cfg<64, 128, 1, 6>(p, epi, stream);    // 8 waves, 64x16
    default: return -1;
  }
}
