// Tile-config instantiations of the implicit-GEMM conv, family "p": kernel P
// (kernel R's staging with register double-buffered MFMA fragments; templates
// in conv_igemm.h; dispatch in conv_igemm.hip).  Of the P tilings measured
// (4/8/16 waves, 64x64 / 64x32 wave tiles; profiles/r1_microbench_conv_cfgs.txt)
// only these two win or tie a RAFT conv: 3-5 % over kernel R on the GRU gates,
// the flow head and the correlation convs.
#include "conv_igemm.h"

extern "C" int jr_conv_family_p(const ConvParams* p, int cfg, int epi, hipStream_t stream) {
  switch (cfg) {
    case 33: return launch_cfg<128, 128, 2, 9>(p, epi, stream);    // 8 waves, 64x32
    case 34: return launch_cfg<256, 128, 4, 11>(p, epi, stream);   // 16 waves, 64x32
    default: return -1;
  }
}
