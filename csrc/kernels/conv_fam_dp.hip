// Tile-config family DP (conv_igemm.h: conv_d2_kernel<.., PIPE = 1>): the
// LDS-DMA ring with register double-buffered MFMA fragments, at wide wave
// tiles (few LDS bytes per MFMA: 128x64 / 64x64 / 128x32 per wave).
#include "conv_igemm.h"

extern "C" int jr_conv_family_dp(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 44: return launch_cfg<256, 128, 2, 15>(p, epi, stream);   // 4 waves, 128x64, 3-stage ring
    case 45: return launch_cfg<256, 128, 4, 16>(p, epi, stream);   // 8 waves, 64x64
    case 46: return launch_cfg<256, 128, 2, 16>(p, epi, stream);   // 8 waves, 128x32
    case 47: return launch_cfg<256, 128, 4, 17>(p, epi, stream);   // 16 waves, 64x32
    case 48: return launch_cfg<128, 128, 2, 15>(p, epi, stream);   // 4 waves, 64x64
    case 49: return launch_cfg<128, 128, 2, 16>(p, epi, stream);   // 8 waves, 64x32
    case 50: return launch_cfg<256, 128, 4, 18>(p, epi, stream);   // 8 waves, 64x64, 2-stage ring
    default: return -1;
  }
}
