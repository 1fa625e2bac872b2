// 3x3 / stride 1 / pad 1 convolution with an LDS-resident input halo, for the
// feature / context encoders' residual convs (model.py:170-184: the
// ConvNormActivation 3x3 pairs of layer1 (64 -> 64 at H/2 x W/2) and layer3
// (128 -> 128 at H/8 x W/8)).
//
// The implicit GEMM (conv_igemm.h) streams im2col rows through LDS stage by
// stage, so every input pixel is fetched once per tap: nine times.  At 64
// output channels that is 64 MACs per fetched bf16 -- the 1/2-resolution
// layer1 convs ran at ~340 TF/s, bound by the L2 -> CU path.  Here a block
// owns a 4 x 64 output tile with all (<= 128) output channels:
//   * the (4+2) x (64+2) x cin input halo is loaded ONCE into LDS (zero
//     padded), XOR-swizzled per pixel so the fragment reads below are
//     bank-conflict free;
//   * wave w computes output row w (64 pixels = 4 MFMA column tiles) for all
//     output channels (4 or 8 MFMA row tiles); the B fragments of tap (dy, dx)
//     are the halo pixels shifted by (dy, dx) -- read straight from LDS, no
//     im2col copy; the A fragments (the packed weights, L1/L2 resident) are
//     register double-buffered one 32-deep k-step ahead;
//   * the epilogue is the implicit GEMM's (bias, activation, residual, dual
//     stores: conv_epilogue), the weights the same packed [cout_pad][kpad].
// Needs OW % 64 == 0 (a wave's 64 pixels inside one image row), cin in
// {64, 128} (= kpad / 9), cout_pad in {64, 128} (ops/native.py:halo_ok).
// Measured (tools/conv_halo_bench.py, MI355X): 109 vs 76 us (4 x 220 x 512,
// 64 -> 64) and 51 vs 18 us (4 x 55 x 128, 128 -> 128) against the best
// autotuned implicit-GEMM config -- the per-block halo load is not overlapped
// (2 blocks per CU) and the weight fragments come from L2 one k-step ahead --
// so config 44 is not an autotune candidate; it stays as a tested reference
// for a deeper-pipelined rewrite.
#include "conv_igemm.h"

namespace {

// LDS slot of 16-B chunk k8 of halo pixel pix (cin*2-byte rows): the XOR
// spreads the 16 pixels x 4 chunks of one ds_read_b128 over all 64 banks.
template <int CIN>
JR_DEVICE int halo_slot(int pix, int k8) {
  if constexpr (CIN == 64) return k8 ^ ((pix >> 1) & 7);
  else return k8 ^ (pix & 15);
}

template <int TMC, int CIN, int EPI>
__global__ __launch_bounds__(256) void conv3x3_halo_kernel(const ConvParams p, int tiles_x, int tiles_y) {
  constexpr int TH = 4, TW = 64, PWD = TW + 2, PHT = TH + 2, NPIX = PHT * PWD;
  constexpr int K8 = CIN / 8;      // 16-B chunks per pixel
  constexpr int CK = CIN / 32;     // 32-deep k-steps per tap
  constexpr int NSTEP = 9 * CK;
  constexpr int NCH = NPIX * K8;
  constexpr int PER = (NCH + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16 tile[NPIX * CIN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  int id = blockIdx.x;
  const int tx = id % tiles_x;
  id /= tiles_x;
  const int ty = id % tiles_y;
  const int n = id / tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;

  // ---- input halo -> LDS (zero outside the image), 8 loads in flight per thread
  const bf16* xb = (const bf16*)p.x + (long)n * p.H * p.W * p.x_cstride + p.x_coff;
#pragma unroll
  for (int b0 = 0; b0 < PER; b0 += 8) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = (b0 + j) * 256 + tid;
      v[j] = u32x4{0u, 0u, 0u, 0u};
      if (b0 + j < PER && c < NCH) {
        const int pix = c / K8, k8 = c - pix * K8;
        const int r = pix / PWD, col = pix - r * PWD;
        const int gy = y0 - 1 + r, gx = x0 - 1 + col;
        if ((unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W)
          v[j] = *(const u32x4*)(xb + ((long)gy * p.W + gx) * p.x_cstride + k8 * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = (b0 + j) * 256 + tid;
      if (b0 + j < PER && c < NCH) {
        const int pix = c / K8, k8 = c - pix * K8;
        *(u32x4*)(tile + pix * CIN + halo_slot<CIN>(pix, k8) * 8) = v[j];
      }
    }
  }

  // ---- A fragments: storage rows 16 tm + li, K = step * 32 + 8 lq (K order (kh, kw, cin))
  const bf16* wrow = (const bf16*)p.w + (long)li * p.kpad + 8 * lq;
  const long tstride = 16L * p.kpad;
  u32x4 a0[TMC], a1[TMC];
  auto load_a = [&](int step, u32x4 (&dst)[TMC]) {
#pragma unroll
    for (int tm = 0; tm < TMC; ++tm) dst[tm] = *(const u32x4*)(wrow + tm * tstride + step * 32);
  };
  load_a(0, a0);

  f32x4 acc[TMC][4];
#pragma unroll
  for (int tm = 0; tm < TMC; ++tm)
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // halo staged

  auto step_mma = [&](int step, const u32x4 (&a)[TMC]) {
    const int tap = step / CK, ks = step - tap * CK;
    const int dy = tap / 3, dx = tap - dy * 3;
    const int k8 = ks * 4 + lq;
    bf16x8 b[4];
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      const int pix = (wave + dy) * PWD + 16 * tn + li + dx;
      b[tn] = *(const bf16x8*)(tile + pix * CIN + halo_slot<CIN>(pix, k8) * 8);
    }
#pragma unroll
    for (int tm = 0; tm < TMC; ++tm)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[tm]), b[tn], acc[tm][tn],
                                                              0, 0, 0);
  };
#pragma unroll
  for (int step = 0; step < NSTEP; step += 2) {
    if (step + 1 < NSTEP) load_a(step + 1, a1);
    step_mma(step, a0);
    if (step + 1 < NSTEP) {
      if (step + 2 < NSTEP) load_a(step + 2, a0);
      step_mma(step + 1, a1);
    }
  }

  const int y = y0 + wave;
  if (y < p.OH) conv_epilogue<TMC, 4, EPI>(p, acc, (n * p.OH + y) * p.OW + x0, 0, lq, li);
}

}  // namespace

extern "C" int jr_conv_halo(const ConvParams* p, int epi, hipStream_t stream) {
  if (p->KH != 3 || p->KW != 3 || p->SH != 1 || p->SW != 1 || p->PH != 1 || p->PW != 1 || p->dsh || p->dsw ||
      p->OH != p->H || p->OW != p->W || p->OW % 64 || (p->cin8 != 64 && p->cin8 != 128) || p->kpad != 9 * p->cin8 ||
      (p->cout_pad != 64 && p->cout_pad != 128) || p->x_cstride % 8 || p->x_coff % 8 || epi != EPI_STD)
    return (int)hipErrorInvalidValue;
  const int tiles_x = p->OW / 64, tiles_y = (p->OH + 3) / 4;
  const dim3 grid((unsigned)(p->N * tiles_y * tiles_x));
#define JR_HALO(TMC, CIN)                                                                                     \
  hipLaunchKernelGGL((conv3x3_halo_kernel<TMC, CIN, EPI_STD>), grid, dim3(256), 0, stream, *p, tiles_x, tiles_y); \
  break;
  switch (p->cout_pad / 16 * 1000 + p->cin8) {
    case 4064: JR_HALO(4, 64)
    case 4128: JR_HALO(4, 128)
    case 8064: JR_HALO(8, 64)
    case 8128: JR_HALO(8, 128)
    default: return (int)hipErrorInvalidValue;
  }
#undef JR_HALO
  return (int)hipGetLastError();
}
