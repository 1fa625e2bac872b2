// Host-visible launcher API of the jax_raft_amd HIP kernels (gfx950 only).
// Every launcher is capture-safe: no allocation, no synchronisation, only
// kernel launches on the given stream.  Returns a hipError_t as int.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

// ---------------------------------------------------------------------------
// Implicit-GEMM NHWC convolution (MFMA bf16, fp32 accumulate) with fused
// epilogues.  GEMM view: D[co][pixel] = W[co][k] * im2col(X)[pixel][k],
// k = (kh, kw, cin8-chunk) flattened, cin padded to a multiple of 8.
// ---------------------------------------------------------------------------
enum ConvEpi : int {
  EPI_STD = 0,    // bias (+residual) -> act -> *alpha -> store (bf16|fp32) (+copy)
  EPI_GRU_A = 1,  // channels [0,Hd): z = sigmoid -> zbuf ; [Hd,2Hd): r = sigmoid -> rh = r*h32 -> y
  EPI_GRU_B = 2,  // q = tanh ; h = (1-z) h + z q -> h32, y (bf16 copy of h), y2 (second copy)
  // 3, 4: retired (the 3x3 flow-head conv epilogue and the EPI_CONVEX mask-head epilogue,
  //       superseded by EPI_TAPS + the update fused into the lookup, and convex_head.hip)
  EPI_BWD = 5,    // data-gradient conv of the training loop's backward (no bias): channels
                  // [0, hidden) -> seg[0], [hidden, cout) -> seg[1] (see BwdSeg)
  EPI_TAPS = 6,   // FlowHead conv1 (256 channels, bias + act) -> its features never leave the CU:
                  // times the 18 per-pixel taps of conv2 (tapw) on MFMA -> fp32 taps [M][y_cstride]
};

// One channel segment of the EPI_BWD epilogue.  Local channel lc = c - base.
//   mode 0: g = acc (+ gin) ; g = 0 where mask <= 0 or lc >= valid ; out = g (bf16 | fp32)
//   mode 1: ConvGRU blend backward (h' = (1-z) h + z q, model.py:311): g = acc (+ gin) = dL/dh'
//           gdq[lc] = g z (1-q^2) ; gdzr[lc] = g (q-h) z (1-z) ; out (fp32) = g (1-z)   (dL/dh partial)
//   mode 2: ConvGRU reset-gate backward (acc = dL/d(r h), model.py:308):
//           gdzr[hidden + lc] = acc h r (1-r) ; out (fp32) += acc r
struct BwdSeg {
  int mode;
  const void* gin; int gin_cs, gin_coff, gin_bf16;   // gradient input: fp32, or bf16 (gin_bf16)
  const void* mask; int mask_cs, mask_coff;
  int valid;
  void* out; int out_cs, out_coff, out_f32;
};

struct ConvParams {
  // input activation (bf16 NHWC with channel stride/offset)
  const void* x;
  int N, H, W;
  int x_cstride, x_coff;
  int cin8;         // input channels used for K, multiple of 8
  int KH, KW, SH, SW, PH, PW;
  int dsh, dsw;     // log2 input dilation (transposed-conv / data-gradient mode): tap reads
                    // dilated coordinate y, valid iff y % 2^dsh == 0, source row y >> dsh
  int OH, OW;
  int M;            // N*OH*OW
  long x_bytes;     // bytes addressable through x (buffer range check, <= 2 GiB)
  long w_bytes;     // bytes of w
  // packed weights [cout_pad][kpad] bf16 and fp32 bias [cout]
  const void* w;
  int kpad;         // multiple of 64
  int nkc;          // KH*KW*cin8/8 valid 8-chunks
  int cout;         // real output channels
  int cout_pad;     // rows present in w (multiple of 16)
  const float* bias;
  float alpha;
  int act;
  int split;        // ACT_SPLIT_TANH_RELU threshold channel
  // primary output
  void* y; int y_cstride, y_coff; int y_fp32;
  // optional second bf16 output copy (same channels)
  void* y2; int y2_cstride, y2_coff;
  // optional residual (bf16), added before the activation
  const void* res; int res_cstride, res_coff;
  int res_post;     // 0: act(v + res) ; 1: relu(act(v) + res)  (ResidualBlock tail, model.py:184)
  // fused-epilogue extras
  float* h32;       // GRU: fp32 hidden state [M][hidden]
  void* zbuf;       // GRU: z gate (bf16) [M][hidden]
  int hidden;
  float* coords;    // FLOW: fp32 [M][2]
  float* flow32;    // FLOW: fp32 [M][2]
  void* y3; int y3_cstride, y3_coff;  // FLOW: third bf16 flow copy
  // optional fp32 / bf16 per-pixel bias map [M][bmap_cstride], channels [bmap_coff, bmap_coff + cout),
  // added with the bias (e.g. the loop-invariant context-feature part of the ConvGRU gates)
  const void* bmap; int bmap_cstride, bmap_coff;
  int bmap_bf16;    // bias map stored as bf16 (else fp32)
  int z_bf16;       // GRU: z gate buffer stored as bf16 (else fp32)
  // 1 when every 64-deep K stage lies inside one tap (a 1x1 conv, or cin8 % 64 == 0 with at most
  // 32 taps) and there is no input dilation: the register-staged kernels then use wave-uniform
  // tap state and per-row tap bitmasks instead of per-lane im2col arithmetic
  int fast;
  // 1: XCD-aware workgroup -> tile order (conv_igemm.h:xcd_tile); 0: dispatch order
  int xcd_remap;
  // training forward extras: GRU-A also stores r (bf16 [M][hidden]); GRU-B stores q (bf16) and
  // writes the new fp32 state to h32o (else in place into h32)
  void* rbuf;
  void* qbuf;
  float* h32o;
  // EPI_BWD: channel segments and the ConvGRU backward operands ([M][hidden]; gdzr [M][2 hidden])
  BwdSeg seg[2];
  const void* gz; const void* gr; const void* gq; const float* ghp;
  void* gdq; void* gdzr;
  // EPI_TAPS: conv2 tap weights as MFMA A fragments [64-channel group 4][k-step 2][row tile 2][lane 64][8] bf16
  const void* tapw;
};

// cfg (co x px block tile): kernel R (register-staged, 16x16x32 MFMA) 0 = 128x128, 1 = 64x128,
// 2 = 128x64, 3 = 16x256, 4 = 64x64, 5 = 16x64 (narrow outputs, e.g. the 2-channel flow head),
// 16 = 256x128, 17 = 128x256 (4 waves); 18 = 128x128, 19 = 128x128, 20 = 256x128, 23 = 128x64,
// 24 = 64x128 (8 waves); 21 = 128x128, 22 = 256x128 (16 waves); kernel D2 (LDS-DMA) 6 = 128x128,
// 7 = 64x128, 8 = 128x64, 9 = 128x256, 10 = 64x64, 11 = 256x128; kernel M32 (32x32x16 MFMA)
// 12 = 128x128, 13 = 64x128, 14 = 128x64, 15 = 64x64.  The engine autotunes the choice per conv.
int jr_conv_forward(const ConvParams* p, int cfg, int epi, hipStream_t stream);

// ---------------------------------------------------------------------------
// Instance/batch-norm statistics and normalisation.
// ---------------------------------------------------------------------------
// stats[n][c][2] = (sum, sumsq) over pixels of x (bf16 NHWC, C channels, contiguous), deterministic
// two-pass reduction; `partial` must hold jr_channel_stats_partials(N, HW, C) * C * 2 floats.
int jr_channel_stats(const void* x, int N, int HW, int C, float* stats, float* partial, hipStream_t stream);
int jr_channel_stats_partials(int N, int HW, int C);
// y = post( pre(xn) + rn ), xn = (x - mean_x) * rstd_x * gamma + beta (mode_x), rn likewise for res.
// mode: 0 = identity, 1 = instance (stats per n), 2 = batch (stats summed over n).
// relu bit 0: relu on xn before the residual add; bit 1: relu on the sum.
int jr_norm_act(const void* x, const float* sx, int mode_x, const float* gamma, const float* beta,
                const void* res, const float* sr, int mode_r, const float* gamma_r, const float* beta_r,
                void* y, int N, int HW, int C, float eps, int relu, hipStream_t stream);

// ---------------------------------------------------------------------------
// Correlation pyramid (MFMA all-pairs GEMM, pooling fused) and lookup.
// ---------------------------------------------------------------------------
// f1: bf16 [B][nq][C] query pixels (nq = h*w, or a slab of query rows for
// context parallelism), f2: bf16 [B][h*w][C] (channel stride cs of both).
// levels[l]: fp32 or bf16 [B][nq][h_l][w_l]; blocked (bf16, w % 16 == 0):
// levels 0 and 1 as [B][nq][ceil(h/8)][ceil(w/16)] blocks of (8>>l) x (16>>l)
// (the pyramid kernel's tiles; corr.hip LvGeom), levels 2 and 3 row-major.
// persistent blocked-layout (bf16) pyramid build, corr_pyr.hip; hipErrorNotSupported = shape not handled
int jr_corr_pyramid_blocked(const void* f1, const void* f2, int B, int h, int w, int C, int cs, void* l0, void* l1,
                            void* l2, void* l3, int nlev, float scale, hipStream_t stream);
int jr_corr_pyramid(const void* f1, const void* f2, int B, int h, int w, int nq, int C, int cs,
                    void* lvl0, void* lvl1, void* lvl2, void* lvl3, int num_levels, float scale, int out_bf16,
                    int blocked, hipStream_t stream);
// coords fp32 [B][nq][2]; out bf16 [B*nq][out_cstride] channels l*(2r+1)^2 + i*(2r+1) + j,
// zero-filled up to out_cstride.  h, w: level-0 map size.  radius 1..6.
// Optional flow update fused ahead of the lookup (upd != nullptr, upd->on): coords
// += bias + the 3x3 sum of the FlowHead conv2 taps (jr_flow_taps' semantics, same
// summation order), then the new flow is written as jr_flow_taps writes it and
// the lookup samples around the updated coords.  Needs nq == h * w.
struct TapsUpd {
  const float* taps; int tcs; const float* bias;
  float* coords; float* flow32;
  void* hx; int hx_cs, hx_off;
  void* qx; int qx_cs, qx_off;
  void* f8; int f8_cs;
  int on;
};
int jr_corr_lookup(const void* const* levels, int num_levels, int B, int h, int w, int nq, int radius,
                   const float* coords, void* out, int out_cstride, int lv_bf16, int blocked, hipStream_t stream,
                   const TapsUpd* upd = nullptr);

// Backward of jr_corr_lookup w.r.t. the levels: accumulates into fp32 dlevels
// (same shapes as the levels).  gout: bf16 (g_bf16=1) or fp32 [B*nq][gcs].
int jr_corr_lookup_bwd(void* const* dlevels, int num_levels, int B, int h, int w, int nq, int radius,
                       const float* coords, const void* gout, int gcs, int g_bf16, hipStream_t stream);

// ---------------------------------------------------------------------------
// Flow upsampling x8.
// ---------------------------------------------------------------------------
// mask bf16 [B*h*w][576] (already scaled), flow fp32 [B*h*w][2] -> out fp32 [B][8h][8w][2]
// Fused inference mask head (convex_head.hip): 1x1 conv 256 -> 576 of the mask
// features feat bf16 [M][feat_cstride] (channels feat_coff ..+256, 16-byte
// aligned), weights packed by ops/native.py:pack_convex_head, bias fp32 [576]
// (reference channel order k*64 + s), logits * alpha -> softmax over the 9
// taps -> convex combination of 8 * flow (fp32 [M][2]) -> out (B, 8h, 8w, 2).
// tiles: 16-pixel tiles per wave (1 / 2; 0 = by problem size).
// out_slot (optional): as jr_upsample_bilinear.
int jr_convex_head(const void* feat, int feat_cstride, int feat_coff, const void* wpk, const float* bias,
                   float alpha, const float* flow, int B, int h, int w, float* out, const void* out_slot, long out_off,
                   int tiles, hipStream_t stream);
int jr_upsample_convex(const void* mask, int mask_cstride, const float* flow, int B, int h, int w,
                       float* out, hipStream_t stream);
// out_slot (optional, device int64): the output base address, read at run time
// (+ out_off floats) instead of `out` -- a captured graph can write a fresh
// output tensor per replay.
int jr_upsample_bilinear(const float* flow, int B, int h, int w, float* out, const void* out_slot, long out_off,
                         hipStream_t stream);
// Backward of jr_upsample_convex (training): mask bf16 [M][mask_cs] (the 576 logits, already
// scaled by alpha), flow fp32 [M][2], gout fp32 [B][8h][8w][2] ->
//   dmask bf16 [M][dmask_cs]: alpha * dL/dlogit (the gradient of the un-scaled mask conv output)
//   taps fp32 [M][18]: taps[q][2k + c] = dL/d flow_c at the k-th 3x3 neighbour of q
int jr_upsample_convex_bwd(const void* mask, int mask_cs, const float* flow, const float* gout, int B, int h, int w,
                           float alpha, void* dmask, int dmask_cs, float* taps, hipStream_t stream);
// Backward of jr_upsample_bilinear w.r.t. the low-res flow (deterministic gather):
// gout fp32 [B][8h][8w][2] -> dflow bf16 [M][dcs] (channels 0, 1; 2..dcs-1 zeroed)
int jr_upsample_bilinear_bwd(const float* gout, int B, int h, int w, void* dflow, int dcs, hipStream_t stream);
// dflow(p) = sum_k taps[p - d_k][2k + c] over the in-map 3x3 neighbours (d_k = (k/3-1, k%3-1)),
// written as bf16 [M][dcs] (channels 0, 1; 2..dcs-1 zeroed)
int jr_flow_gather_bwd(const float* taps, int tcs, int N, int h, int w, void* dflow, int dcs, hipStream_t stream);
// Backward of an encoder unit "y -> norm (mode 0 none / 1 instance / 2 batch, gamma/beta
// optional) -> relu (relu & 1)" whose output gradient is gout * [om > 0] (om optional: the
// ReLU'd residual-block output): dy bf16, gres fp32 (optional) = gout * [om > 0]; red fp32
// [N][C][2] = per-(n, c) (sum g, sum g*xhat) (the BN affine gradients), partial: workspace of
// jr_norm_bwd_partials(N, HW, C) * C * 2 floats.  y / gout / om / dy / gres are [N][HW][C] dense.
int jr_norm_bwd_partials(int N, int HW, int C);
int jr_norm_bwd(const void* gout, const void* om, const void* y, const float* stats, int mode, const float* gamma,
                const float* beta, int relu, int N, int HW, int C, float eps, float* red, float* partial, void* dy,
                void* gres, int gres_bf16, hipStream_t stream);
// Batched weight packing (training): one rectangular piece of one packed conv weight
// (bf16 [cout_pad][kpad], rows permuted, ops/native.py:pack_weight) from an fp32 HWIO source
// [kh][kw][cin_s][cout_s].  For dst output channel co in [co0, co1), tap, input channel ci
// in [ci0, ci1) (source indices co - co0 + so_co, ci - ci0 + so_ci):
//   mode 0 forward:       src[tap][ci'][co']
//   mode 1 data gradient: src[flip(tap)][co'][ci']   (the dst conv's in/out are the source's out/in)
//   mode 2 flow-head taps: dst (1,1,cin,18), co = 2*tap' + c: src[tap'][ci'][c]
//   mode 3 bias:          fp32 dst[co] = src[co']
// All fields 64-bit (the table is built by the host as an int64 array).
struct PackPiece {
  int64_t src, dst, kh, kw, cin_s, cout_s, cin8, kpad, co0, co1, ci0, ci1, so_co, so_ci, mode, pad;
};
int jr_pack_pieces(const void* table, int n, long max_elems, hipStream_t stream);
// Implicit-GEMM weight gradient (wgrad.hip): dW (fp32 HWIO [KH][KW][cin][cout]) and db (fp32
// [cout], optional) of the conv X (bf16 NHWC [N][H][W][xcs], channels xoff.. xoff+cin8) ->
// dY (bf16 [N][OH][OW][ycs], channels yoff.. yoff+cout).  part / bpart: split-K workspaces of
// S * cout_pad * kpad and S * cout_pad floats from jr_wgrad_plan (S <= 0: the planned S).
int jr_wgrad_plan(int M, int K, int cout, int* S, int* cout_pad, int* kpad);
// out[m] = [sum_t a[t][m] | sum_t b[t][m]] (bf16 in / out, fp32 sums; train/fused.py gate context share)
int jr_sum_iters(const void* a, const void* b, int T, long M, int Ca, int Cb, void* out, hipStream_t stream);
// the workspace plan of one conv's weight gradient (the 3x3 / stride-1 halo path or the im2col tiles)
int jr_wgrad_plan_geom(int N, int H, int W, int cin8, int KH, int KW, int SH, int SW, int PH, int PW, int OH, int OW,
                       int cout, int* S, int* cout_pad, int* kpad);
int jr_wgrad(const void* x, int xcs, int xoff, int N, int H, int W, int cin8, int KH, int KW, int SH, int SW, int PH,
             int PW, const void* dy, int ycs, int yoff, int OH, int OW, int cout, int cin, float* part, float* bpart,
             int S, float* dw, float* db, long x_bytes, long y_bytes, hipStream_t stream);
// Correlation pyramid backward: dc bf16 [M][h][w] = scale * sum_l (2x2 floor-pool adjoint)^l of the
// fp32 level gradients g_l [M][h_l][w_l] (g1..g3 may be null past L levels).
int jr_pyr_bwd_dc(const float* g0, const float* g1, const float* g2, const float* g3, int L, long M, int h, int w,
                  float scale, void* dc, hipStream_t stream);
// BatchNorm bookkeeping table (train.hip): mode 0 running-stat update from per-(n, c)
// (sum, sumsq) `src` [N][C][2] into dst0 = running mean, dst1 = running var (momentum as float
// bits, count = N*HW); mode 1 affine gradients from the norm backward's [N][C][2] reduction:
// dst0 = d scale, dst1 = d bias.  All fields 64-bit (host-built int64 table).
struct BnRow {
  int64_t src, dst0, dst1, N, C, count, momentum_bits, mode;
};
int jr_bn_table(const void* rows, int n, int max_c, hipStream_t stream);
// Sequence loss over N <= 32 predictions pred fp32 [N][P][2] vs gt fp32 [P][2]
// (valid: optional fp32 [P]): part fp32 [jr_seq_loss_blocks(P)][37] per-block
// partial sums (0..N-1: sum over valid pixels of |pred_i - gt|_1; 32: EPE sum of
// the last prediction, 33..35: its <1/<3/<5 px counts, 36: valid count).
int jr_seq_loss_blocks(long P);
int jr_seq_loss(const float* pred, const float* gt, const float* valid, long P, int N, float max_flow, float* part,
                hipStream_t stream);
// grad fp32 [N][P][2] = scale[i] * valid * sign(pred_i - gt)
int jr_seq_loss_bwd(const float* pred, const float* gt, const float* valid, long P, int N, float max_flow,
                    const float* scale, float* grad, hipStream_t stream);

// ---------------------------------------------------------------------------
// Misc.
// ---------------------------------------------------------------------------
// img1,img2 fp32 NHWC [B][H][W][3] -> bf16 [2B][H][W][8] (img1 batch first), channels 3..7 = 0.
int jr_prep_images(const float* img1, const float* img2, int B, int H, int W, void* out, hipStream_t stream);
// 2x2 space-to-depth prep: out bf16 [2B][H/2][W/2][16] (see elementwise.hip:prep_images_s2d_kernel)
int jr_prep_images_s2d(const float* img1, const float* img2, int B, int H, int W, void* out, hipStream_t stream);
// uint8 NHWC frames (any size) -> normalised, replicate-padded bf16 encoder input (elementwise.hip)
int jr_prep_u8(const void* img1, const void* img2, const float* lut, int B, int H0, int W0, int H, int W, int pt,
               int pl, int s2d, void* out, hipStream_t stream);
// coords[b][y][x] = (x, y); flow32 = 0
int jr_init_coords(float* coords, int B, int h, int w, hipStream_t stream);
// im2col of x (bf16 NHWC, channel slice) into col [N*OH*OW][kpad] in the packed-weight K order
int jr_im2col(const void* x, int N, int H, int W, int x_cstride, int x_coff, int cin8, int KH, int KW,
              int SH, int SW, int PH, int PW, int OH, int OW, int kpad, void* col, hipStream_t stream);
// copy bf16 channel slice: dst[m][doff + c] = src[m][soff + c], c < C
int jr_zero_fill(void* p, long bytes, hipStream_t stream);
// delta(p) = bias + sum of the 9 shifted per-tap partials t[p + d][tap] ([M][tcs] fp32,
// tap-major pairs), then the coordinate / flow update (flowhead.hip): coords += delta,
// flow = coords - coords0 -> flow32 (fp32) and bf16 copies into hx / qx / f8
// Pointwise conv with LDS-resident weights (conv1x1.hip): y[m][y_coff + co] =
// act(x[m][0 .. kvalid) . W + bias) for co < cout (cout % 64 == 0), weights
// packed by ops/native.py:pack_conv1x1 with K padded to kpad (128 / 256 / 352 / 384).
int jr_conv1x1_lds(const void* x, int x_cstride, int kvalid, int kpad, const void* wpk, const float* bias, int act,
                   void* y, int y_cstride, int y_coff, int cout, int M, hipStream_t stream);
// taps[m][0..24) = fm[m][fcoff .. fcoff+K) . W (K = 128 / 256, 18 real columns);
// weights packed by ops/native.py:pack_taps.  taps fp32 [M][tcs >= 24].
int jr_taps_gemm(const void* fm, int fcs, int fcoff, int K, const void* wpk, float* taps, int tcs, int M,
                 hipStream_t stream);
int jr_flow_taps(const float* t, int tcs, const float* bias, int N, int h, int w, float* coords, float* flow32,
                 void* hx, int hx_cs, int hx_off, void* qx, int qx_cs, int qx_off, void* f8, int f8_cs,
                 hipStream_t stream);
// Conv of a 2-channel input (the flow branch's 7x7 / 3x3): x bf16 NHWC
// [N][H][W][x_cstride] (channels 0, 1 used), stride 1, output H x W; w bf16
// MFMA A fragments [cout/16][NKC][64 lanes][8] (jax_raft_amd/ops/native.py:
// pack_direct_weight); bias fp32 [cout]; y bf16 channels [y_coff, y_coff +
// cout) of [N*H*W][y_cstride].  (KH, KW) in {(7, 7), (3, 3)}, cout % 32 == 0.
// Operands of jr_conv1x1_lds as one struct (the optional third part of jr_flowin_dual).
struct Conv1x1Args {
  const void* x; int xcs, kvalid, kpad; const void* wpk; const float* bias; int act;
  void* y; int ycs, ycoff, cout, M;
};
// The 7x7 flow conv of jr_conv_direct merged with the x8 upsampling of the previous iteration in one grid
// (merged.hip): mode 1 = bilinear (flow -> out), mode 2 = the convex mask head (jr_convex_head operands;
// out == nullptr: no upsampling part).  c1 (mode 2, kpad 352): jr_conv1x1_lds in the same grid.
int jr_flowin_dual(const void* x, int x_cstride, int N, int H, int W, int PH, int PW, const void* w,
                   const float* fbias, int cout, int relu, void* y, int y_cstride, int y_coff, int mode,
                   const void* feat, int feat_cstride, int feat_coff, const void* wpk, const float* cbias, float alpha,
                   const float* flow, float* out, const void* out_slot, long out_off, const Conv1x1Args* c1,
                   hipStream_t stream);
int jr_conv_direct(const void* x, int x_cstride, int N, int H, int W, int cin, int KH, int KW, int PH, int PW,
                   const void* w, const float* bias, int cout, int relu, void* y, int y_cstride, int y_coff,
                   hipStream_t stream);
int jr_copy_channels(const void* src, int s_cstride, int s_coff, void* dst, int d_cstride, int d_coff,
                     int M, int C, hipStream_t stream);

// ---------------------------------------------------------------------------
// fp32 parity mode (engine precision="fp32"; conv_f32.hip, f32.hip): the
// reference's own precision end to end -- fp32 operands on the f32 MFMA
// (v_mfma_f32_16x16x4_f32), fp32 activations, correlation and hidden state.
// ---------------------------------------------------------------------------
// Implicit-GEMM conv, fp32 NHWC: x [N][H][W][x_cs] (channels x_coff .. + cin4),
// w fp32 [cout][K], K = (kh, kw, cin4) (cin4 % 4 == 0, zero-padded), bias [cout].
// epi 0: bias (+bmap) (+res: pre-act add, or post-act add + relu when res_post)
//        -> act -> *alpha -> y (+y2) (+h32 [M][hidden] for channels < split)
// epi 1: ConvGRU z / r (cout = 2 hidden): z -> zbuf [M][hidden], r * h32 -> y
// epi 2: ConvGRU q (cout = hidden): h = (1 - z) h + z tanh(q) -> h32, y (+y2)
struct ConvF32Params {
  const float* x; int N, H, W, x_cs, x_coff, cin4;
  int KH, KW, SH, SW, PH, PW, OH, OW, M;
  const float* w; int K, cout;
  const float* bias; float alpha; int act, split;
  float* y; int y_cs, y_coff;
  float* y2; int y2_cs, y2_coff;
  const float* res; int res_cs, res_coff, res_post;
  float* h32; float* zbuf; int hidden;
  const float* bmap; int bmap_cs, bmap_coff;
  // split-K (ksplit > 1): blockIdx.z takes 1/ksplit of the K stages and writes raw
  // partial sums to part [ksplit][M][round_up(cout, 4)]; a second kernel adds them in
  // order and applies the epilogue (the loop convs at batch 1 have 110-440 blocks)
  int ksplit; float* part;
};
int jr_conv_f32(const ConvF32Params* p, int epi, hipStream_t stream);
// jr_channel_stats / jr_norm_act / jr_prep_images / jr_copy_channels /
// jr_upsample_convex on fp32 tensors (prep: [2B][H][W][4], channel 3 = 0)
int jr_channel_stats_f32(const float* x, int N, int HW, int C, float* stats, float* partial, hipStream_t stream);
int jr_norm_act_f32(const float* x, const float* sx, int mode_x, const float* res, const float* sr, int mode_r,
                    float* y, int N, int HW, int C, float eps, int relu, hipStream_t stream);
int jr_prep_images_f32(const float* img1, const float* img2, int B, int H, int W, float* out, hipStream_t stream);
int jr_copy_channels_f32(const float* src, int s_cstride, int s_coff, float* dst, int d_cstride, int d_coff, int M,
                         int C, hipStream_t stream);
int jr_upsample_convex_f32(const float* mask, int mask_cstride, const float* flow, int B, int h, int w, float* out,
                           const void* out_slot, long out_off, hipStream_t stream);
// 2x2 average pooling (floor) of per-query correlation maps: src [M][hl][wl] -> dst [M][hl/2][wl/2]
int jr_corr_pool_f32(const float* src, long M, int hl, int wl, float* dst, hipStream_t stream);
// Pyramid lookup with fp32 output (jr_corr_lookup's semantics and channel order;
// row-major fp32 levels [B*nq][h_l][w_l], no fused update): out [B*nq][out_cstride]
int jr_corr_lookup_f32(const float* const* levels, int num_levels, int B, int h, int w, int nq, int radius,
                       const float* coords, float* out, int out_cstride, hipStream_t stream);
// coords += delta (delta [M][dcs], channels 0, 1: the FlowHead output incl. its bias);
// flow = coords - coords0 -> flow32 [M][2], hx / qx (channel offsets) and flow4 [M][4] (channels 0, 1)
int jr_flow_update_f32(const float* delta, int dcs, int N, int h, int w, float* coords, float* flow32, float* hx,
                       int hx_cs, int hx_off, float* qx, int qx_cs, int qx_off, float* flow4, hipStream_t stream);

// Fused ConvGRU stage of raft_large (gru_fused.hip): z, r = sigmoid(conv_zr([h | x]) + bmap[z | r]),
// q = tanh(conv_q([r h | x]) + bmap[q]), h' = (1 - z) h + z q, for one 1x5 (row tiles) or
// 5x1 (column tiles) stage in ONE launch; r*h and z never leave the CU.
struct GruFusedParams {
  const void* hx; int hx_cs;          // bf16 [M][hx_cs]: [h (128) | x (128)]; hx_cs == 256
  const void* wa; const void* wb;     // pack_weight of [z | r] ([256][1280]) and q ([128][1280])
  const void* bmap; int bmap_cs; int bmap_bf16;   // [M][bmap_cs]: [z | r | q] context share + gate biases
  float* h32;                         // fp32 hidden state [M][128], updated in place
  void* y; int y_cs;                  // bf16 h' -> channels [0, 128) (the loop buffer hx)
  void* y2; int y2_cs;                // optional second bf16 copy of h' (channels [0, 128))
  int N, H, W;
  int vertical;                       // 0: 1x5 taps along W, tiles = image rows; 1: 5x1, tiles = J columns
  int L, J, tiles_per_img, ntiles;    // run length (W or H), runs per tile (J * L <= 128)
  int g2all;                          // 1: GEMM 2 on all 16 waves (z through LDS); 0: on the 8 z waves
  long hx_bytes, wa_bytes, wb_bytes;
  long long* dbg;                     // optional [ntiles][6] phase timestamps (s_memrealtime, tools/gru_phases.py)
};
int jr_gru_fused(const GruFusedParams* p, hipStream_t stream);

// Halo-tiled fused ConvGRU stage (gru_halo.hip) for ANY /8 map size and both RAFT
// recurrent blocks: raft_large's 1x5 / 5x1 stages (mode 0: a run of L pixels along the
// tap axis, hd 128, cin 256) and raft_small's 3x3 GRU (mode 1: a TR x TC block, hd 96,
// cin 192).  Each workgroup recomputes z / r on its tile's halo (+-2 / +-1 pixels) so
// r*h never leaves the CU; the weights stream from L2 straight into MFMA A registers.
// Reads [h | x] from hsrc (channels [0, hd)) and xsrc (channels [hd, cin)) and writes h'
// to y (a DIFFERENT buffer than hsrc: neighbouring tiles read h of this tile's pixels).
struct GruHaloParams {
  const void* hsrc; const void* xsrc; int cs;   // bf16 [M][cs] loop buffers ([h | motion | flow | pad])
  const void* wa; const void* wb;     // ops/native.py:pack_gru_halo of [z | r] and q: [cout/32][taps*cin/16][64][8]
  const void* bmap; int bmap_cs;      // bf16 [M][bmap_cs]: [z | r | q] context share + gate biases
  float* h32;                         // fp32 hidden state [M][hd], updated in place (own pixels only)
  void* y; int y_cs;                  // bf16 h' -> channels [0, hd)
  void* y2; int y2_cs;                // optional second bf16 copy of h'
  int N, H, W;
  int mode;                           // 0: 5-tap run (1x5 / 5x1), 1: 3x3 block
  int axis;                           // mode 0: 0 = taps along W (1x5), 1 = along H (5x1)
  int TR, TC;                         // output tile: mode 0 TR = 1, TC = run length L; mode 1 TR x TC
  int tiles_y, tiles_x, ntiles;       // tiles per image = tiles_y * tiles_x (mode 0: lines x segments)
  int nb1, nb2;                       // 32-pixel blocks of the halo region (GEMM 1) / the output tile
  long src_bytes, wa_bytes, wb_bytes;
  // training forward (train/fused.py): h read from h32in (null: h32, in place) and h' written to h32;
  // the gates saved for the backward, bf16 [M][hd] each (null: not stored): z, r, q, and r*h into
  // rh (channel stride rh_cs, the q conv's input buffer)
  const float* h32in;
  void* zo; void* ro; void* qo; void* rh; int rh_cs;
};
int jr_gru_halo(const GruHaloParams* p, hipStream_t stream);

// LDS bytes of one workgroup (0: the configuration is not supported)
int jr_gru_halo_lds(int hd, int mode, int TR, int TC, int nb1, int nb2);
// Halo 3x3 / stride-1 conv (conv_halo.hip): a TR x TC tile of output pixels per workgroup,
// its (TR + 2) x (TC + 2) input footprint loaded into LDS once, B fragments read from it
// shifted by the tap (no im2col address arithmetic), weights streamed in MFMA fragment order
// (ops/native.py:pack_gru_halo).  EPI_STD semantics of conv_igemm (bias, residual pre / post,
// relu, bf16 output + copy) plus an optional per-channel statistics output.
struct ConvHaloParams {
  const void* x; int xcs, xoff;        // bf16 NHWC input [N][H][W][xcs], channels xoff .. xoff + cin
  int N, H, W, cin;
  const void* w; long w_bytes;         // pack_gru_halo(kernel (3, 3, cin, cout_pad), cin)
  const float* bias; int cout;         // real output channels
  int act;                             // ACT_NONE / ACT_RELU
  void* y; int ycs, yoff;              // bf16 output
  void* y2; int y2cs, y2off;           // optional bf16 copy
  const void* res; int rcs, roff, res_post;   // optional bf16 residual (0: act(v + r), 1: relu(act(v) + r))
  float* stats_part;                   // optional [N][tiles_per_img * WPX][cout][2] (sum, sumsq) partials
  // optional instance norm (+ relu) of the INPUT, applied while the footprint is loaded:
  // x' = act((x - mean[n][c]) * rsqrt(var[n][c] + eps)) from in_stats [N][cin][2] (sum, sumsq
  // over in_hw pixels; jr_norm_act mode 1 semantics), zero padding stays zero
  const float* in_stats; int in_hw; float in_eps; int in_relu;
  // optional residual of that input (a residual block's output, built while loading):
  // x' = act(norm(x) + r) with r = in_res (bf16, channel stride in_rcs), itself instance-
  // normalised by in_res_stats if given; xn (channel stride xncs) receives x' of the tile's
  // own pixels (the block output, needed again as the next block's residual)
  const void* in_res; int in_rcs; const float* in_res_stats;
  void* xn; int xncs;
  int TR, TC, tiles_y, tiles_x, ntiles;
  long x_bytes;
  long in_res_bytes;                   // the input residual's own range (its buffer resource)
};
// cfg: index into the halo tile-config table (conv_halo.hip); 0 on success
int jr_conv_halo(const ConvHaloParams* p, int cfg, hipStream_t stream);
// table entry: {cin, WCO, WPX, TN, TR, TC} (returns 0 for an unknown cfg); LDS bytes
int jr_conv_halo_cfg(int cfg, int* out6);
int jr_conv_halo_lds(int cfg);
// kernel size of a table entry (3, or 4 for the space-to-depth stem configs; 0 for an unknown cfg)
int jr_conv_halo_ks(int cfg);
// per-channel stats [N][C][2] from partials [N][nb][C][2] (channel_stats_final_kernel)
int jr_channel_stats_final(const float* part, int N, int nb, int C, float* stats, hipStream_t stream);

// Grouped launch of two EPI_STD convs with one tile config (conv_fam_grp.hip); ok: the configs it serves.
int jr_conv_grouped(const ConvParams* p1, const ConvParams* p2, int cfg, hipStream_t stream);
int jr_conv_grouped_ok(int cfg);
// Batched bf16 GEMM, fp32 accumulation (bgemm.hip): C[b] = alpha * op(A[b]) . B[b], B k-major [K][N],
// A row-major [M][K] (a_kmajor 0) or k-major [K][M] (1); fp32 (C32) or bf16 (C16) output [M][ldc].
// M, N multiples of 128, K of 64.
int jr_bgemm(const void* A, long a_bs, int lda, int a_kmajor, const void* B, long b_bs, int ldb, int batch, int M,
             int N, int K, float alpha, float* C32, void* C16, long c_bs, int ldc, hipStream_t stream);

}  // extern "C"
