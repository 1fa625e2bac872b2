// Grouped-launch instantiations (conv_igemm.h: conv_grouped_kernel): the tile configs the
// autotuner picks for the one-lane loop's small convs at batch 1 (kernel R 4 / 8 waves, kernel M32).
#include "conv_igemm.h"

extern "C" int jr_conv_grouped_ok(int cfg) {
  switch (cfg) {
    case 2: case 4: case 5: case 23: case 24: case 12: case 14: case 15: return 1;
    default: return 0;
  }
}

extern "C" int jr_conv_grouped(const ConvParams* p1, const ConvParams* p2, int cfg, hipStream_t stream) {
  if (p1->M <= 0 || p2->M <= 0) return (int)hipErrorInvalidValue;
  switch (cfg) {
    case 2: return launch_grouped<128, 64, 2, 4, false>(p1, p2, stream);
    case 4: return launch_grouped<64, 64, 1, 4, false>(p1, p2, stream);
    case 5: return launch_grouped<16, 64, 1, 4, false>(p1, p2, stream);
    case 23: return launch_grouped<128, 64, 2, 8, false>(p1, p2, stream);
    case 24: return launch_grouped<64, 128, 1, 8, false>(p1, p2, stream);
    case 12: return launch_grouped<128, 128, 2, 4, true>(p1, p2, stream);
    case 14: return launch_grouped<128, 64, 2, 4, true>(p1, p2, stream);
    case 15: return launch_grouped<64, 64, 2, 4, true>(p1, p2, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
