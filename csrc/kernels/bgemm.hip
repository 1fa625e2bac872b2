// Batched bf16 GEMM with fp32 accumulation for the correlation-pyramid backward
// (reference jax_raft/model.py:472-481: corr = fmap1 . fmap2^T / sqrt(C), so
// dfmap1 = dC . fmap2 and dfmap2 = dC^T . fmap1, dC the volume gradient of
// train.hip:pyr_bwd_dc):
//
//   C[b][m][n] = alpha * sum_k A[b](m, k) * B[b][k][n]
//
// B is k-major ([K][N], the feature map [pixels][channels]); A is either
// row-major [M][K] (dC for dfmap1) or k-major [K][M] (dC read as dC^T for
// dfmap2) -- so neither product needs a transposed copy of the 113 MB volume.
// 128 x 128 output tiles, 4 waves of 64 x 64 (4 x 4 v_mfma_f32_16x16x32_bf16
// tiles), 64-deep K stages staged through double-buffered LDS (register-staged
// global loads one stage ahead, one barrier per stage).  k-major operands are
// read as MFMA fragments with ds_read_b64_tr_b16 from an XOR-swizzled [k][128]
// image (the wgrad.hip scheme); the row-major A with ds_read_b128 from a
// [128][64] image (the conv_igemm.h swizzle).  grid = (M / 128, N / 128, batch).
#include "common.h"
#include "kernels.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int BK = 64, BT = 128;
constexpr int IMG = BK * BT;          // elements of one operand image
constexpr unsigned OOB = 0x80000000u;

// [k][128] image: row r holds 32 8-B units; unit u of row r at u ^ swz(r) (wgrad.hip swz<32>)
JR_DEVICE int swz32(int r) { return 4 * ((r & 3) | (((r >> 3) & 1) << 2)); }
JR_DEVICE int swzB(int row) { return (row >> 1) & 7; }

template <bool AK>
__global__ __launch_bounds__(256) void bgemm_kernel(const bf16* __restrict__ A, long a_bs, int lda,
                                                    const bf16* __restrict__ Bm, long b_bs, int ldb, int M, int N,
                                                    int K, float alpha, float* __restrict__ C32,
                                                    bf16* __restrict__ C16, long c_bs, int ldc) {
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;   // 64 x 64 wave tile (rows m, cols n)
  const int m0 = blockIdx.x * BT, n0 = blockIdx.y * BT, b = blockIdx.z;
  const bf16* Ab = A + b * a_bs;
  const bf16* Bb = Bm + b * b_bs;
  const __amdgpu_buffer_rsrc_t as = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t bs = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);

  // k-major tiles [64 k][128]: thread -> 16-B chunk kc of rows kr + 16 i;  row-major A tile [128 m][64 k]:
  // thread -> chunk ac of rows ar + 32 i
  const int kr = tid >> 4, kc = tid & 15;
  const int ar = tid >> 3, ac = tid & 7;
  struct Regs { u32x4 a[4]; u32x4 b[4]; };
  auto issue = [&](Regs& r, int k0) {
    const bool kin = k0 < K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned off;
      if constexpr (AK) off = (unsigned)(((long)(k0 + kr + 16 * i) * lda + m0 + 8 * kc) * 2);
      else off = (unsigned)(((long)(m0 + ar + 32 * i) * lda + k0 + 8 * ac) * 2);
      r.a[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(as, kin ? off : OOB, 0, 0));
      const unsigned bo = (unsigned)(((long)(k0 + kr + 16 * i) * ldb + n0 + 8 * kc) * 2);
      r.b[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(bs, kin ? bo : OOB, 0, 0));
    }
  };
  auto store = [&](const Regs& r, int buf) {
    bf16* sA = smem + buf * 2 * IMG;
    bf16* sB = sA + IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = kr + 16 * i;
      if constexpr (AK) *(u32x4*)(sA + row * BT + 4 * ((2 * kc) ^ swz32(row))) = r.a[i];
      else {
        const int arow = ar + 32 * i;
        *(u32x4*)(sA + arow * BK + ((ac ^ swzB(arow)) << 3)) = r.a[i];
      }
      *(u32x4*)(sB + row * BT + 4 * ((2 * kc) ^ swz32(row))) = r.b[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto tr = [&](const bf16* img, int r, int cb) -> s16x4 {   // rows r.., the lane's 4 columns of block cb
    const int u = cb / 4 + pp;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r * BT + 4 * (u ^ swz32(r))));
  };
  auto kfrag = [&](const bf16* img, int ks, int cb) {   // 8 consecutive k of the lane's column (k-major image)
    const int r0 = 32 * ks + 8 * g + q;
    const s16x4 lo = tr(img, r0, cb), hi = tr(img, r0 + 4, cb);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto compute = [&](int buf) {
    const bf16* sA = smem + buf * 2 * IMG;
    const bf16* sB = sA + IMG;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if constexpr (AK) af[t] = kfrag(sA, ks, wr * 64 + 16 * t);
        else {
          const int row = wr * 64 + 16 * t + (lane & 15), chunk = ks * 4 + g;
          af[t] = *(const bf16x8*)(sA + row * BK + ((chunk ^ swzB(row)) << 3));
        }
        bfr[t] = kfrag(sB, ks, wc * 64 + 16 * t);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[x], bfr[y], acc[x][y], 0, 0, 0);
    }
  };

  const int nst = K / BK;
  Regs ra;
  issue(ra, 0);
  store(ra, 0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) issue(ra, (st + 1) * BK);
    compute(buf);
    if (st + 1 < nst) store(ra, buf ^ 1);
    __syncthreads();
  }

  // lane: rows m0 + 64 wr + 16 x + 4 g + j, column n0 + 64 wc + 16 y + (lane & 15)
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long o = b * c_bs + (long)(m0 + wr * 64 + 16 * x + 4 * g + j) * ldc + n0 + wc * 64 + 16 * y + (lane & 15);
        const float v = alpha * acc[x][y][j];
        if (C32) C32[o] = v;
        else C16[o] = f2bf(v);
      }
}

}  // namespace

extern "C" int jr_bgemm(const void* A, long a_bs, int lda, int a_kmajor, const void* B, long b_bs, int ldb, int batch,
                        int M, int N, int K, float alpha, float* C32, void* C16, long c_bs, int ldc,
                        hipStream_t stream) {
  if (M % BT || N % BT || K % BK || batch <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid(M / BT, N / BT, batch);
  if (a_kmajor)
    hipLaunchKernelGGL(bgemm_kernel<true>, grid, dim3(256), 0, stream, (const bf16*)A, a_bs, lda, (const bf16*)B,
                       b_bs, ldb, M, N, K, alpha, C32, (bf16*)C16, c_bs, ldc);
  else
    hipLaunchKernelGGL(bgemm_kernel<false>, grid, dim3(256), 0, stream, (const bf16*)A, a_bs, lda, (const bf16*)B,
                       b_bs, ldb, M, N, K, alpha, C32, (bf16*)C16, c_bs, ldc);
  return (int)hipGetLastError();
}
