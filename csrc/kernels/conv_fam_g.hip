// Tile-config instantiations of the implicit-GEMM conv, family "g": kernel D2
// (LDS-DMA ring, counted vmcnt + raw barriers) at 8 / 16 waves per block with
// the FAST im2col loader (templates in conv_igemm.h; dispatch in conv_igemm.hip).
#include "conv_igemm.h"

extern "C" int jr_conv_family_g(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 35: return launch_cfg<256, 128, 4, 12>(p, epi, stream);   // 16 waves, 64x32, 3-stage ring
    case 36: return launch_cfg<128, 128, 4, 12>(p, epi, stream);   // 16 waves, 32x32
    case 37: return launch_cfg<128, 128, 2, 13>(p, epi, stream);   // 8 waves, 64x32
    case 38: return launch_cfg<256, 128, 4, 14>(p, epi, stream);   // 16 waves, 64x32, 2-stage ring
    case 39: return launch_cfg<256, 128, 2, 13>(p, epi, stream);   // 8 waves, 128x32
    case 40: return launch_cfg<128, 256, 2, 12>(p, epi, stream);   // 16 waves, 64x32
    case 41: return launch_cfg<64, 128, 1, 13>(p, epi, stream);    // 8 waves, 64x16
    case 42: return launch_cfg<256, 128, 4, 13>(p, epi, stream);   // 8 waves, 64x64
    case 43: return launch_cfg<256, 128, 2, 4>(p, epi, stream);    // 4 waves, 128x64 (one wave per SIMD)
    default: return -1;
  }
}
