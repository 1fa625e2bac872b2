// Tile-config instantiations of the implicit-GEMM conv, family "r":
// kernel R, 4-wave blocks (templates in conv_igemm.h; dispatch in conv_igemm.hip).
#include "conv_igemm.h"

extern "C" int jr_conv_family_r(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 0: return launch_cfg<128, 128, 2, 0>(p, epi, stream);
    case 1: return launch_cfg<64, 128, 1, 0>(p, epi, stream);
    case 2: return launch_cfg<128, 64, 2, 0>(p, epi, stream);
    case 3: return launch_cfg<16, 256, 1, 0>(p, epi, stream);
    case 4: return launch_cfg<64, 64, 1, 0>(p, epi, stream);
    case 5: return launch_cfg<16, 64, 1, 0>(p, epi, stream);
    case 16: return launch_cfg<256, 128, 2, 0>(p, epi, stream);
    case 17: return launch_cfg<128, 256, 2, 0>(p, epi, stream);
    default: return -1;
  }
}
