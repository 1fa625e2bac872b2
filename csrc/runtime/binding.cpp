// jax_raft_amd native runtime: TORCH_LIBRARY ops over the gfx950 kernels and
// a plan executor with hipGraph capture.
//
// The reference has no native code; XLA emits its kernels
// and runs the refinement loop as a device while-loop (jax_raft/model.py:589-603,
// nn.scan).  Here the equivalent runtime is explicit:
//   * every kernel is reachable as an eager op (torch.ops.jax_raft_amd.*),
//     used by the autograd/unfused path and by the tests;
//   * a `Plan` records launch closures (prologue / loop body / epilogue) once,
//     with all pointers, shapes and tile configs resolved, and either launches
//     them straight from C++ (no per-op Python overhead) or captures the whole
//     N-iteration forward into one hipGraph and replays it.
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

#include "../kernels/kernels.h"

namespace jr {

using TList = c10::List<c10::optional<at::Tensor>>;
using IList = std::vector<int64_t>;
using Launch = std::function<int(hipStream_t, int)>;

static inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

static inline at::Tensor opt(const TList& t, size_t i) {
  if (i >= t.size()) return at::Tensor();
  c10::optional<at::Tensor> v = t.get(i);
  return v.has_value() ? *v : at::Tensor();
}
static inline void* ptr(const at::Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }
static inline int cs(const at::Tensor& t) { return t.defined() ? (int)t.size(-1) : 0; }

#define JR_CHECK_OK(expr)                                                                 \
  do {                                                                                    \
    int e__ = (expr);                                                                     \
    TORCH_CHECK(e__ == 0, "jax_raft_amd kernel launch failed: ", hipGetErrorString((hipError_t)e__)); \
  } while (0)

static void check_bf16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.defined(), name, " must be defined");
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
static void check_f32(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.defined(), name, " must be defined");
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// ----------------------------------------------------------------------- conv
// t = [x, w, bias, y, y2, res, h32, zbuf, coords, flow32, y3, bmap(, tapw)]
// i = [N, H, W, x_coff, cin8, KH, KW, SH, SW, PH, PW, cout, act, split,
//      y_coff, y2_coff, res_coff, hidden, y3_coff, epi, cfg, res_post
//      (, OH_override, OW_override, log2 dil_h, log2 dil_w (, bmap_coff))]
static int64_t check_flow_out(const at::Tensor& out, int B, int h, int w);

static void conv_train_extras(ConvParams& p, int epi, const TList& tx, const IList& ix, std::vector<at::Tensor>* keep);

static ConvParams build_conv(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep,
                             const TList* tx, const IList* ix, int* epi_out, int* cfg_out) {
  TORCH_CHECK(i.size() == 22 || i.size() == 26 || i.size() == 27, "conv: expected 22, 26 or 27 ints");
  at::Tensor x = opt(t, 0), w = opt(t, 1), bias = opt(t, 2), y = opt(t, 3), y2 = opt(t, 4), res = opt(t, 5);
  at::Tensor h32 = opt(t, 6), zbuf = opt(t, 7), coords = opt(t, 8), flow32 = opt(t, 9), y3 = opt(t, 10);
  at::Tensor bmap = opt(t, 11), tapw;
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_f32(bias, "bias");
  TORCH_CHECK(y.defined() && y.is_contiguous(), "conv: y must be contiguous");
  ConvParams p{};
  p.x = x.data_ptr();
  p.N = (int)i[0]; p.H = (int)i[1]; p.W = (int)i[2];
  p.x_cstride = cs(x); p.x_coff = (int)i[3]; p.cin8 = (int)i[4];
  p.KH = (int)i[5]; p.KW = (int)i[6]; p.SH = (int)i[7]; p.SW = (int)i[8]; p.PH = (int)i[9]; p.PW = (int)i[10];
  p.dsh = i.size() >= 26 ? (int)i[24] : 0;
  p.dsw = i.size() >= 26 ? (int)i[25] : 0;
  TORCH_CHECK(p.dsh >= 0 && p.dsh <= 3 && p.dsw >= 0 && p.dsw <= 3, "conv: dilation must be 1, 2, 4 or 8");
  p.OH = ((p.H << p.dsh) - ((1 << p.dsh) - 1) + 2 * p.PH - p.KH) / p.SH + 1;
  p.OW = ((p.W << p.dsw) - ((1 << p.dsw) - 1) + 2 * p.PW - p.KW) / p.SW + 1;
  if (i.size() >= 26 && i[22] > 0) p.OH = (int)i[22];
  if (i.size() >= 26 && i[23] > 0) p.OW = (int)i[23];
  p.M = p.N * p.OH * p.OW;
  p.x_bytes = x.numel() * 2;
  p.w_bytes = w.numel() * 2;
  TORCH_CHECK(p.x_bytes <= (1LL << 31) && p.w_bytes <= (1LL << 31), "conv: operand larger than 2 GiB");
  p.w = w.data_ptr(); p.kpad = (int)w.size(1); p.cout_pad = (int)w.size(0);
  p.nkc = p.KH * p.KW * p.cin8 / 8;
  p.cout = (int)i[11]; p.bias = bias.data_ptr<float>(); p.alpha = (float)alpha;
  p.act = (int)i[12]; p.split = (int)i[13];
  p.y = y.data_ptr(); p.y_cstride = cs(y); p.y_coff = (int)i[14]; p.y_fp32 = y.scalar_type() == at::kFloat;
  p.y2 = ptr(y2); p.y2_cstride = cs(y2); p.y2_coff = (int)i[15];
  p.res = ptr(res); p.res_cstride = cs(res); p.res_coff = (int)i[16]; p.res_post = (int)i[21];
  p.h32 = h32.defined() ? h32.data_ptr<float>() : nullptr; p.hidden = (int)i[17];
  p.zbuf = ptr(zbuf);
  p.coords = coords.defined() ? coords.data_ptr<float>() : nullptr;
  p.flow32 = flow32.defined() ? flow32.data_ptr<float>() : nullptr;
  p.y3 = ptr(y3); p.y3_cstride = cs(y3); p.y3_coff = (int)i[18];
  p.bmap = ptr(bmap);
  p.bmap_cstride = bmap.defined() ? cs(bmap) : 0;
  p.bmap_coff = i.size() >= 27 ? (int)i[26] : 0;
  p.bmap_bf16 = bmap.defined() && bmap.scalar_type() == at::kBFloat16;
  p.z_bf16 = zbuf.defined() && zbuf.scalar_type() == at::kBFloat16;
  if (bmap.defined()) {
    TORCH_CHECK(bmap.is_cuda() && bmap.is_contiguous() &&
                    (bmap.scalar_type() == at::kFloat || bmap.scalar_type() == at::kBFloat16),
                "conv: bias map must be a contiguous fp32 / bf16 GPU tensor");
    TORCH_CHECK(p.bmap_cstride % 8 == 0 && p.bmap_coff % 8 == 0 && p.bmap_coff + p.cout <= p.bmap_cstride,
                "conv: bias map channel slice must be 8-aligned and inside the tensor");
    TORCH_CHECK(bmap.numel() >= (int64_t)p.M * p.bmap_cstride, "conv: bias map too small");
  }
  const int epi = (int)i[19];
  {
    const int taps = p.KH * p.KW;
    p.fast = p.dsh == 0 && p.dsw == 0 && taps <= 32 && (taps == 1 || p.cin8 % 64 == 0);
  }
  int cfg = (int)i[20];
  // Timing-only ablation (tools/microbench.py --ablate): cfg bits 8/9 give the
  // X / W buffer descriptors zero records, so every load through them is
  // dropped by the range check while the instruction stream stays the same.
  // Lowering variants (same results; tests and microbench A/B): bit 10 = XCD-aware tile
  // order (conv_igemm.h:tile_of_block; measured -0.5..1.4 % on the RAFT convs, whose inputs
  // are MALL-resident, so off by default), bit 11 = the generic im2col loader instead of FAST.
  if (cfg >> 8) {
    if ((cfg >> 8) & 1) p.x_bytes = 0;
    if ((cfg >> 8) & 2) p.w_bytes = 0;
    p.xcd_remap = (cfg >> 10) & 1;
    if ((cfg >> 11) & 1) p.fast = 0;
    cfg &= 255;
  }
  // Shape / alignment contract of conv_igemm.hip.
  TORCH_CHECK(p.cin8 % 8 == 0 && p.cin8 > 0, "conv: cin8 must be a positive multiple of 8");
  TORCH_CHECK(p.x_cstride % 8 == 0 && p.x_coff % 8 == 0 && p.x_coff + p.cin8 <= p.x_cstride,
              "conv: input channel slice must be 8-aligned and inside the tensor");
  TORCH_CHECK((int64_t)p.N * p.H * p.W * p.x_cstride <= x.numel(), "conv: input tensor too small");
  TORCH_CHECK(p.kpad % 64 == 0 && p.kpad >= p.KH * p.KW * p.cin8, "conv: packed weight K mismatch");
  TORCH_CHECK(p.cout_pad % 64 == 0 && p.cout_pad >= p.cout && bias.numel() >= p.cout, "conv: packed weight rows (64-row groups)");
  TORCH_CHECK(p.OH > 0 && p.OW > 0, "conv: empty output");
  TORCH_CHECK(p.y_cstride % 8 == 0, "conv: output channel stride must be a multiple of 8");
  TORCH_CHECK((int64_t)p.M * p.y_cstride <= y.numel(), "conv: output tensor too small");
  if (epi == EPI_STD) {
    TORCH_CHECK(p.y_coff % 8 == 0 && p.y_coff + p.cout <= p.y_cstride, "conv: output slice");
    TORCH_CHECK(y.scalar_type() == at::kBFloat16 || y.scalar_type() == at::kFloat, "conv: output dtype");
    if (y2.defined()) { check_bf16(y2, "y2"); TORCH_CHECK(p.y2_cstride % 8 == 0 && p.y2_coff % 8 == 0, "y2 align"); }
    if (res.defined()) { check_bf16(res, "res"); TORCH_CHECK(p.res_cstride % 8 == 0 && p.res_coff % 8 == 0, "res align"); }
    if (h32.defined()) { check_f32(h32, "h32"); TORCH_CHECK(h32.numel() >= (int64_t)p.M * p.hidden, "h32 size"); }
  } else if (epi == EPI_GRU_A) {
    if (h32.defined()) check_f32(h32, "h32");
    else TORCH_CHECK(p.OH == p.H && p.OW == p.W && p.dsh == 0 && p.dsw == 0 && p.x_coff + p.hidden <= p.x_cstride,
                     "GRU-A without h32 reads h from its stride-1 input [h | ...]");
    check_bf16(y, "y");
    TORCH_CHECK(zbuf.defined() && zbuf.is_cuda() && zbuf.is_contiguous() &&
                    (zbuf.scalar_type() == at::kFloat || zbuf.scalar_type() == at::kBFloat16) &&
                    zbuf.numel() >= (int64_t)p.M * p.hidden, "GRU: zbuf must be an fp32 / bf16 [M][hidden] GPU tensor");
    TORCH_CHECK(p.cout == 2 * p.hidden && p.hidden % 16 == 0, "GRU-A: cout must be 2*hidden, hidden % 16 == 0");
    TORCH_CHECK(p.y_coff % 8 == 0, "GRU-A align");
  } else if (epi == EPI_GRU_B) {
    check_f32(h32, "h32"); check_bf16(y, "y");
    TORCH_CHECK(zbuf.defined() && zbuf.is_cuda() && zbuf.is_contiguous() &&
                    (zbuf.scalar_type() == at::kFloat || zbuf.scalar_type() == at::kBFloat16) &&
                    zbuf.numel() >= (int64_t)p.M * p.hidden, "GRU: zbuf must be an fp32 / bf16 [M][hidden] GPU tensor");
    TORCH_CHECK(p.cout == p.hidden && p.hidden % 16 == 0, "GRU-B: cout must be hidden");
    TORCH_CHECK(p.y_coff % 8 == 0, "GRU-B align");
    if (y2.defined()) { check_bf16(y2, "y2"); TORCH_CHECK(p.y2_coff % 8 == 0, "y2 align"); }
  } else if (epi == EPI_BWD) {
    TORCH_CHECK(tx != nullptr, "EPI_BWD needs the training operands (conv_train)");
    TORCH_CHECK(!bmap.defined() && !res.defined(), "EPI_BWD: no bias map / residual");
    TORCH_CHECK(p.hidden >= 0 && p.hidden % 16 == 0 && p.hidden <= p.cout, "EPI_BWD: split must be a multiple of 16 <= cout");
  } else if (epi == EPI_TAPS) {
    tapw = opt(t, 12);
    check_f32(y, "y (taps)");
    check_bf16(tapw, "tapw");
    TORCH_CHECK(tapw.numel() == 4 * 2 * 2 * 64 * 8 && reinterpret_cast<uintptr_t>(tapw.data_ptr()) % 16 == 0,
                "TAPS: tap weights must be pack_taps_epi's [4][2][2][64][8] bf16");
    TORCH_CHECK(p.cout == 256 && p.y_coff == 0 && p.y_cstride >= 18 && p.y_cstride % 4 == 0 && !bmap.defined() &&
                    !res.defined() && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
                "TAPS: 256 channels in, fp32 taps [M][>=18] out, no bias map / residual");
    TORCH_CHECK(cfg == 22 || cfg == 34 || cfg == 35 || cfg == 38, "TAPS: tile config ", cfg,
                " is not a 256-channel 16-wave 64x32 tiling");
    p.tapw = tapw.data_ptr();
  } else {
    TORCH_CHECK(false, "conv: unknown epilogue ", epi);
  }
  TORCH_CHECK(cfg >= 0 && cfg <= 43 && !(cfg >= 29 && cfg <= 32), "conv: unknown tile config ", cfg);
  if (tx) conv_train_extras(p, epi, *tx, *ix, keep);
  if (keep) for (auto& v : {x, w, bias, y, y2, res, h32, zbuf, coords, flow32, y3, bmap, tapw}) if (v.defined()) keep->push_back(v);
  *epi_out = epi;
  *cfg_out = cfg;
  return p;
}

// Tile configs >= kHaloCfg0 select the halo 3x3 kernel (conv_halo.hip, table index cfg - kHaloCfg0)
// for an EPI_STD 3x3 / stride-1 / pad-1 conv; its weights (ops/native.py:pack_gru_halo of the
// kernel, cout padded to 32) come as t[12].  Optional t[13]: per-channel statistics partials.
constexpr int kHaloCfg0 = 100;

bool conv_halo_ok_cfg(int64_t cfg, int64_t cin8, int64_t cout) {
  int c[6];
  if (!jr_conv_halo_cfg((int)(cfg - kHaloCfg0), c) || jr_conv_halo_ks((int)(cfg - kHaloCfg0)) != 3) return false;
  return c[0] == cin8 && cout <= 512 && jr_conv_halo_lds((int)(cfg - kHaloCfg0)) <= 160 * 1024;
}

static Launch make_conv_halo(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep) {
  TORCH_CHECK(i.size() >= 22, "conv: expected >= 22 ints");
  const int cfg = (int)i[20] - kHaloCfg0;
  int c[6];
  TORCH_CHECK(jr_conv_halo_cfg(cfg, c), "conv_halo: unknown tile config ", i[20]);
  at::Tensor x = opt(t, 0), bias = opt(t, 2), y = opt(t, 3), y2 = opt(t, 4), res = opt(t, 5), wh = opt(t, 12),
             part = opt(t, 13);
  check_bf16(x, "x"); check_f32(bias, "bias"); check_bf16(y, "y"); check_bf16(wh, "halo weights");
  const int N = (int)i[0], H = (int)i[1], W = (int)i[2], xoff = (int)i[3], cin8 = (int)i[4];
  const int KH = (int)i[5], KW = (int)i[6], SH = (int)i[7], SW = (int)i[8], PH = (int)i[9], PW = (int)i[10];
  const int cout = (int)i[11], act = (int)i[12], epi = (int)i[19];
  // kernel size 3 (pad 1) or 4: the space-to-depth stem, pads 2 (top / left) and 1, i.e. a
  // 4x4 / pad-2 spec whose output size is forced to the input's (out_hw = (H, W))
  const int ks = jr_conv_halo_ks(cfg);
  const bool geom3 = ks == 3 && PH == 1 && PW == 1 && (i.size() < 26 || (i[22] <= 0 && i[23] <= 0));
  const bool geom4 = ks == 4 && PH == 2 && PW == 2 && i.size() >= 26 && i[22] == H && i[23] == W;
  TORCH_CHECK(KH == ks && KW == ks && SH == 1 && SW == 1 && (geom3 || geom4) && epi == EPI_STD &&
                  (act == 0 || act == 1) && alpha == 1.0 && !opt(t, 11).defined() &&   // ACT_NONE / ACT_RELU
                  !opt(t, 6).defined() && (i.size() < 26 || (i[24] == 0 && i[25] == 0)),
              "conv_halo: a 3x3 / stride-1 / pad-1 (or stem 4x4 / pad-2, output = input size) EPI_STD conv "
              "(relu / none, no alpha / bias map / state)");
  TORCH_CHECK(c[0] == cin8 && cin8 % 16 == 0, "conv_halo: config ", i[20], " is for ", c[0], " input channels, got ", cin8);
  const int cpad = (cout + 31) / 32 * 32;
  TORCH_CHECK(wh.numel() == (int64_t)cpad * ks * ks * cin8, "conv_halo: halo weights (pack_gru_halo, cout padded to 32)");
  TORCH_CHECK(cs(x) % 8 == 0 && xoff % 8 == 0 && xoff + cin8 <= cs(x) && x.numel() >= (int64_t)N * H * W * cs(x),
              "conv_halo: input channel slice");
  const int64_t M = (int64_t)N * H * W;
  TORCH_CHECK(cs(y) % 8 == 0 && (int)i[14] % 8 == 0 && (int)i[14] + cout <= cs(y) && y.numel() >= M * cs(y), "conv_halo: y");
  ConvHaloParams p{};
  p.x = x.data_ptr(); p.xcs = cs(x); p.xoff = xoff; p.N = N; p.H = H; p.W = W; p.cin = cin8;
  p.w = wh.data_ptr(); p.w_bytes = (long)wh.numel() * 2;
  p.bias = bias.data_ptr<float>(); p.cout = cout; p.act = act;
  p.y = y.data_ptr(); p.ycs = cs(y); p.yoff = (int)i[14];
  if (y2.defined()) {
    check_bf16(y2, "y2");
    TORCH_CHECK(cs(y2) % 8 == 0 && (int)i[15] % 8 == 0 && (int)i[15] + cout <= cs(y2) && y2.numel() >= M * cs(y2), "conv_halo: y2");
    p.y2 = y2.data_ptr(); p.y2cs = cs(y2); p.y2off = (int)i[15];
  }
  if (res.defined()) {
    check_bf16(res, "res");
    TORCH_CHECK(cs(res) % 8 == 0 && (int)i[16] % 8 == 0 && (int)i[16] + cout <= cs(res) && res.numel() >= M * cs(res),
                "conv_halo: residual");
    p.res = res.data_ptr(); p.rcs = cs(res); p.roff = (int)i[16]; p.res_post = (int)i[21];
  }
  p.TR = c[4]; p.TC = c[5];
  p.tiles_y = (H + p.TR - 1) / p.TR; p.tiles_x = (W + p.TC - 1) / p.TC;
  const int64_t nt = (int64_t)N * p.tiles_y * p.tiles_x;
  TORCH_CHECK(nt < (1LL << 31), "conv_halo: too many tiles");
  p.ntiles = (int)nt;
  if (part.defined()) {
    check_f32(part, "stats partials");
    TORCH_CHECK(part.numel() >= (int64_t)N * p.tiles_y * p.tiles_x * c[2] * cout * 2, "conv_halo: stats partials too small");
    p.stats_part = part.data_ptr<float>();
  }
  // optional t[14]: stats of the input ([N][cin][2] sums) -> instance norm (+ relu) on load;
  // i[27..28] (after the 27-int form): in_relu, in_hw; eps 1e-5 (the encoders' InstanceNorm)
  at::Tensor ist = opt(t, 14);
  if (ist.defined()) {
    check_f32(ist, "input stats");
    TORCH_CHECK(i.size() >= 29, "conv_halo: the input norm needs [.., in_relu, in_hw]");
    TORCH_CHECK(ist.numel() >= (int64_t)N * cin8 * 2 && i[28] > 0, "conv_halo: input stats [N][cin][2]");
    p.in_stats = ist.data_ptr<float>(); p.in_relu = (int)i[27]; p.in_hw = (int)i[28]; p.in_eps = 1e-5f;
    if (keep) keep->push_back(ist);
  }
  // optional t[15..17]: the input's residual (bf16 [N][H][W][>= cin], channel offset 0), its
  // stats ([N][cin][2], instance-normalised if given), the write-back of the built input
  at::Tensor ires = opt(t, 15), irst = opt(t, 16), xn = opt(t, 17);
  if (ires.defined() || irst.defined() || xn.defined()) {
    TORCH_CHECK(ist.defined(), "conv_halo: an input residual / write-back needs the input norm");
    const int64_t M = (int64_t)N * H * W;
    if (ires.defined()) {
      check_bf16(ires, "input residual");
      TORCH_CHECK(cs(ires) % 8 == 0 && cs(ires) >= cin8 && ires.numel() >= M * cs(ires) &&
                  (int64_t)ires.numel() * 2 <= (1LL << 31), "conv_halo: input residual [N][H][W][>= cin]");
      p.in_res = ires.data_ptr(); p.in_rcs = cs(ires); p.in_res_bytes = (long)ires.numel() * 2;
      if (keep) keep->push_back(ires);
    }
    if (irst.defined()) {
      TORCH_CHECK(ires.defined(), "conv_halo: residual stats without a residual");
      check_f32(irst, "residual stats");
      TORCH_CHECK(irst.numel() >= (int64_t)N * cin8 * 2, "conv_halo: residual stats [N][cin][2]");
      p.in_res_stats = irst.data_ptr<float>();
      if (keep) keep->push_back(irst);
    }
    if (xn.defined()) {
      check_bf16(xn, "input write-back");
      TORCH_CHECK(cs(xn) % 8 == 0 && cs(xn) >= cin8 && xn.numel() >= M * cs(xn), "conv_halo: xn [N][H][W][>= cin]");
      TORCH_CHECK(!(xn.data_ptr() == x.data_ptr()) && !(ires.defined() && xn.data_ptr() == ires.data_ptr()),
                  "conv_halo: xn must not alias the input or its residual (neighbouring tiles read them)");
      p.xn = xn.data_ptr(); p.xncs = cs(xn);
      if (keep) keep->push_back(xn);
    }
  }
  p.x_bytes = (long)x.numel() * 2;
  TORCH_CHECK(p.x_bytes < (1LL << 31), "conv_halo: input larger than 2 GiB");
  for (const at::Tensor* v : {&x, &wh, &y})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(v->data_ptr()) % 16 == 0, "conv_halo: 16-byte aligned operands");
  if (keep) for (auto& v : {x, bias, y, y2, res, wh, part}) if (v.defined()) keep->push_back(v);
  return [p, cfg](hipStream_t s, int) { return jr_conv_halo(&p, cfg, s); };
}

static Launch make_conv(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep,
                        const TList* tx = nullptr, const IList* ix = nullptr) {
  if (i.size() >= 22 && (i[20] & 255) >= kHaloCfg0 && tx == nullptr) return make_conv_halo(t, i, alpha, keep);
  int epi = 0, cfg = 0;
  const ConvParams p = build_conv(t, i, alpha, keep, tx, ix, &epi, &cfg);
  return [p, epi, cfg](hipStream_t s, int) { return jr_conv_forward(&p, cfg, epi, s); };
}

// A conv whose input on ODD loop iterations is x_alt (same shape as x): the reader of a state
// that ping-pongs between two buffers (raft_small's FlowHead after the single-stage halo GRU).
static Launch make_conv_alt(const TList& t, const IList& i, double alpha, const at::Tensor& x_alt,
                            std::vector<at::Tensor>* keep) {
  if (i.size() >= 22 && (i[20] & 255) >= kHaloCfg0) {   // halo kernel: two launch closures (cfg bits 8+: igemm variants)
    TList t2 = t.copy();
    t2.set(0, c10::optional<at::Tensor>(x_alt));
    Launch a = make_conv_halo(t, i, alpha, keep), b = make_conv_halo(t2, i, alpha, keep);
    return [a, b](hipStream_t s, int it) { return (it & 1) ? b(s, it) : a(s, it); };
  }
  int epi = 0, cfg = 0;
  const ConvParams p = build_conv(t, i, alpha, keep, nullptr, nullptr, &epi, &cfg);
  const at::Tensor x = opt(t, 0);
  check_bf16(x_alt, "x_alt");
  TORCH_CHECK(x_alt.sizes() == x.sizes(), "conv_alt: x_alt must have x's shape");
  ConvParams q = p;
  q.x = x_alt.data_ptr();
  if (keep) keep->push_back(x_alt);
  return [p, q, epi, cfg](hipStream_t s, int it) { return jr_conv_forward((it & 1) ? &q : &p, cfg, epi, s); };
}

// Two independent EPI_STD convs with the same tile config as ONE grid (conv_igemm.h:
// conv_grouped_kernel; configs of conv_fam_grp.hip), e.g. the one-lane loop's convcorr2 +
// convflow2 at batch 1.
static Launch make_conv_group(const TList& t1, const IList& i1, double a1, const TList& t2, const IList& i2,
                              double a2, std::vector<at::Tensor>* keep) {
  int e1 = 0, c1 = 0, e2 = 0, c2 = 0;
  const ConvParams p1 = build_conv(t1, i1, a1, keep, nullptr, nullptr, &e1, &c1);
  const ConvParams p2 = build_conv(t2, i2, a2, keep, nullptr, nullptr, &e2, &c2);
  TORCH_CHECK(e1 == EPI_STD && e2 == EPI_STD && c1 == c2 && p1.fast == p2.fast && jr_conv_grouped_ok(c1),
              "conv_group: two STD-epilogue convs with the same grouped-launch tile config and loader");
  return [p1, p2, c1](hipStream_t s, int) { return jr_conv_grouped(&p1, &p2, c1, s); };
}

// Training operands of a conv (op conv_train / Plan.add_conv_train):
// tx = [rbuf, qbuf, h32o, gz, gr, gq, ghp, gdq, gdzr,
//       seg0.gin, seg0.mask, seg0.out, seg1.gin, seg1.mask, seg1.out]
// ix = [seg0.mode, seg0.gin_coff, seg0.mask_coff, seg0.valid, seg0.out_coff,  (same for seg1)]
// Channel strides are the tensors' last dims.  GRU operands are [M][hidden]
// (gdzr [M][2 hidden]); see BwdSeg (kernels.h) for the segment semantics.
static void conv_train_extras(ConvParams& p, int epi, const TList& tx, const IList& ix, std::vector<at::Tensor>* keep) {
  TORCH_CHECK(tx.size() == 15 && ix.size() == 10, "conv_train: expected 15 tensors and 10 ints");
  std::vector<at::Tensor> ts;
  for (size_t k = 0; k < 15; ++k) ts.push_back(opt(tx, k));
  const int64_t M = p.M;
  auto need_bf16 = [&](const at::Tensor& v, int64_t n, const char* nm) {
    check_bf16(v, nm);
    TORCH_CHECK(v.numel() >= n, "conv_train: ", nm, " too small");
  };
  auto need_f32 = [&](const at::Tensor& v, int64_t n, const char* nm) {
    check_f32(v, nm);
    TORCH_CHECK(v.numel() >= n, "conv_train: ", nm, " too small");
  };
  const int hd = p.hidden;
  if (ts[0].defined()) { TORCH_CHECK(epi == EPI_GRU_A, "rbuf: GRU-A only"); need_bf16(ts[0], M * hd, "rbuf"); p.rbuf = ts[0].data_ptr(); }
  if (ts[1].defined()) { TORCH_CHECK(epi == EPI_GRU_B, "qbuf: GRU-B only"); need_bf16(ts[1], M * hd, "qbuf"); p.qbuf = ts[1].data_ptr(); }
  if (ts[2].defined()) { TORCH_CHECK(epi == EPI_GRU_B, "h32o: GRU-B only"); need_f32(ts[2], M * hd, "h32o"); p.h32o = ts[2].data_ptr<float>(); }
  if (epi == EPI_BWD) {
    bool gru = false;
    for (int s = 0; s < 2; ++s) {
      BwdSeg& g = p.seg[s];
      const int b = 5 * s;
      const int lo = s ? hd : 0, hi = s ? p.cout : hd;
      const int width = hi - lo;
      g.mode = (int)ix[b];
      TORCH_CHECK(g.mode >= 0 && g.mode <= 2, "conv_train: segment mode 0..2");
      TORCH_CHECK(!(s == 1 && g.mode != 0), "conv_train: segment 1 is mode 0");
      if (width <= 0) continue;
      const at::Tensor &gin = ts[9 + 3 * s], &mask = ts[10 + 3 * s], &out = ts[11 + 3 * s];
      TORCH_CHECK(out.defined() && out.is_cuda() && out.is_contiguous() &&
                      (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16),
                  "conv_train: segment output must be a contiguous fp32 / bf16 GPU tensor");
      g.out = out.data_ptr(); g.out_cs = cs(out); g.out_coff = (int)ix[b + 4];
      g.out_f32 = out.scalar_type() == at::kFloat;
      TORCH_CHECK(g.out_cs % 8 == 0 && g.out_coff % 8 == 0 && g.out_coff + width <= g.out_cs &&
                      out.numel() >= M * g.out_cs, "conv_train: segment output slice");
      if (gin.defined()) {
        g.gin_bf16 = gin.scalar_type() == at::kBFloat16;
        if (g.gin_bf16) check_bf16(gin, "gin");
        else need_f32(gin, 0, "gin");
        g.gin = gin.data_ptr(); g.gin_cs = cs(gin); g.gin_coff = (int)ix[b + 1];
        const int ga = g.gin_bf16 ? 8 : 4;   // 16-byte vector loads
        TORCH_CHECK(g.gin_cs % ga == 0 && g.gin_coff % ga == 0 && g.gin_coff + width <= g.gin_cs &&
                        gin.numel() >= M * g.gin_cs, "conv_train: segment gradient-input slice");
      }
      if (mask.defined()) {
        TORCH_CHECK(g.mode == 0, "conv_train: ReLU mask in mode 0 only");
        need_bf16(mask, 0, "mask");
        g.mask = mask.data_ptr(); g.mask_cs = cs(mask); g.mask_coff = (int)ix[b + 2];
        TORCH_CHECK(g.mask_cs % 8 == 0 && g.mask_coff % 8 == 0 && g.mask_coff + width <= g.mask_cs &&
                        mask.numel() >= M * g.mask_cs, "conv_train: segment mask slice");
      }
      g.valid = (int)ix[b + 3];
      if (g.mode != 0) {
        gru = true;
        TORCH_CHECK(g.out_f32 && g.out_cs == hd && g.out_coff == 0, "conv_train: GRU segment output is fp32 [M][hidden]");
        if (g.mode == 2) TORCH_CHECK(!gin.defined(), "conv_train: reset-gate segment takes no gradient input");
      }
      if (keep) for (auto* v : {&gin, &mask, &out}) if (v->defined()) keep->push_back(*v);
    }
    if (gru) {
      TORCH_CHECK(hd > 0, "conv_train: GRU segment needs hidden > 0");
      const bool m1 = p.seg[0].mode == 1;
      if (m1) { need_bf16(ts[3], M * hd, "gz"); need_bf16(ts[5], M * hd, "gq"); need_bf16(ts[7], M * hd, "gdq"); }
      else need_bf16(ts[4], M * hd, "gr");
      need_f32(ts[6], M * hd, "ghp");
      need_bf16(ts[8], M * 2 * hd, "gdzr");
      p.gz = ptr(ts[3]); p.gr = ptr(ts[4]); p.gq = ptr(ts[5]);
      p.ghp = ts[6].data_ptr<float>(); p.gdq = ptr(ts[7]); p.gdzr = ts[8].data_ptr();
    }
  }
  if (keep) for (auto& v : ts) if (v.defined()) keep->push_back(v);
}

// t = [mask, flow, gout, dmask, taps], i = [B, h, w], alpha
static Launch make_upsample_convex_bwd(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep) {
  at::Tensor mask = opt(t, 0), flow = opt(t, 1), g = opt(t, 2), dm = opt(t, 3), taps = opt(t, 4);
  TORCH_CHECK(i.size() == 3, "upsample_convex_bwd: expected 3 ints");
  check_bf16(mask, "mask"); check_f32(flow, "flow"); check_f32(g, "gout"); check_bf16(dm, "dmask"); check_f32(taps, "taps");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2];
  const int64_t M = (int64_t)B * h * w;
  TORCH_CHECK(cs(mask) >= 576 && mask.numel() >= M * cs(mask), "upsample_convex_bwd: mask [M][>=576]");
  TORCH_CHECK(cs(dm) >= 576 && dm.numel() >= M * cs(dm), "upsample_convex_bwd: dmask [M][>=576]");
  TORCH_CHECK(flow.numel() >= 2 * M && g.numel() >= 128 * M && taps.numel() >= 18 * M, "upsample_convex_bwd: sizes");
  if (keep) for (auto& v : {mask, flow, g, dm, taps}) keep->push_back(v);
  const void* mp = mask.data_ptr();
  const float* fp = flow.data_ptr<float>();
  const float* gp = g.data_ptr<float>();
  void* dp = dm.data_ptr();
  float* tp = taps.data_ptr<float>();
  const int mcs = cs(mask), dcs = cs(dm);
  const float a = (float)alpha;
  return [=](hipStream_t s, int) { return jr_upsample_convex_bwd(mp, mcs, fp, gp, B, h, w, a, dp, dcs, tp, s); };
}

// t = [gout, om?, y, stats?, gamma?, beta?, red?, partial?, dy, gres?], i = [mode, relu, N, HW, C]
static Launch make_norm_bwd(const TList& t, const IList& i, double eps, std::vector<at::Tensor>* keep) {
  at::Tensor g = opt(t, 0), om = opt(t, 1), y = opt(t, 2), st = opt(t, 3), gam = opt(t, 4), bet = opt(t, 5);
  at::Tensor red = opt(t, 6), part = opt(t, 7), dy = opt(t, 8), gres = opt(t, 9);
  TORCH_CHECK(i.size() == 5, "norm_bwd: expected [mode, relu, N, HW, C]");
  const int mode = (int)i[0], relu = (int)i[1], N = (int)i[2], HW = (int)i[3], C = (int)i[4];
  const int64_t n = (int64_t)N * HW * C;
  TORCH_CHECK(mode >= 0 && mode <= 2 && C % 8 == 0 && C <= 2048, "norm_bwd: mode 0..2, C % 8 == 0");
  check_bf16(g, "gout"); check_bf16(y, "y"); check_bf16(dy, "dy");
  TORCH_CHECK(g.numel() >= n && y.numel() >= n && dy.numel() >= n && cs(g) == C && cs(y) == C && cs(dy) == C,
              "norm_bwd: [N][HW][C] tensors");
  if (om.defined()) { check_bf16(om, "om"); TORCH_CHECK(om.numel() >= n && cs(om) == C, "norm_bwd: om"); }
  if (gres.defined()) {   // fp32, or bf16 (the masked gradient gout * [om > 0] is exact in bf16)
    TORCH_CHECK(gres.is_cuda() && gres.is_contiguous() &&
                    (gres.scalar_type() == at::kFloat || gres.scalar_type() == at::kBFloat16), "norm_bwd: gres dtype");
    TORCH_CHECK(gres.numel() >= n && cs(gres) == C, "norm_bwd: gres");
  }
  if (mode) {
    check_f32(st, "stats");
    TORCH_CHECK(st.numel() >= (int64_t)N * C * 2, "norm_bwd: stats");
    check_f32(red, "red");
    TORCH_CHECK(red.numel() >= (int64_t)N * C * 2, "norm_bwd: red");
    const int64_t need = (int64_t)jr_norm_bwd_partials(N, HW, C) * C * 2;
    if (!part.defined()) part = at::empty({need}, st.options());
    check_f32(part, "partial");
    TORCH_CHECK(part.numel() >= need, "norm_bwd: partial workspace too small");
  }
  for (auto* v : {&gam, &bet}) if (v->defined()) { check_f32(*v, "affine"); TORCH_CHECK(v->numel() >= C, "norm_bwd: affine"); }
  if (keep) for (auto& v : {g, om, y, st, gam, bet, red, part, dy, gres}) if (v.defined()) keep->push_back(v);
  auto fp = [](const at::Tensor& v) -> float* { return v.defined() ? v.data_ptr<float>() : nullptr; };
  const void *gp = g.data_ptr(), *op = ptr(om), *yp = y.data_ptr();
  const float *sp = fp(st), *gmp = fp(gam), *btp = fp(bet);
  float *rp = fp(red), *pp = fp(part);
  void* grp = gres.defined() ? gres.data_ptr() : nullptr;
  const int gbf = gres.defined() && gres.scalar_type() == at::kBFloat16;
  void* dp = dy.data_ptr();
  const float e = (float)eps;
  return [=](hipStream_t s, int) {
    return jr_norm_bwd(gp, op, yp, sp, mode, gmp, btp, relu, N, HW, C, e, rp, pp, dp, grp, gbf, s);
  };
}

// t = [table (int64 [n][16] device), *sources, *destinations (kept alive)], i = [n, max_elems]
static Launch make_pack(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor tab = opt(t, 0);
  TORCH_CHECK(i.size() == 2, "pack: expected [n, max_elems]");
  TORCH_CHECK(tab.defined() && tab.is_cuda() && tab.is_contiguous() && tab.scalar_type() == at::kLong &&
                  tab.numel() == i[0] * 16, "pack: table must be a contiguous int64 [n][16] GPU tensor");
  if (keep) for (size_t k = 0; k < t.size(); ++k) { at::Tensor v = opt(t, k); if (v.defined()) keep->push_back(v); }
  const void* tp = tab.data_ptr();
  const int n = (int)i[0];
  const long me = (long)i[1];
  return [=](hipStream_t s, int) { return jr_pack_pieces(tp, n, me, s); };
}

// t = [x, dy, dw (fp32 HWIO), db?, part?, bpart?],
// i = [N, H, W, xoff, cin8, KH, KW, SH, SW, PH, PW, yoff, OH, OW, cout, cin]
static Launch make_wgrad(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), dy = opt(t, 1), dw = opt(t, 2), db = opt(t, 3), part = opt(t, 4), bpart = opt(t, 5);
  TORCH_CHECK(i.size() == 16, "wgrad: expected 16 ints");
  check_bf16(x, "x"); check_bf16(dy, "dy"); check_f32(dw, "dw");
  const int N = (int)i[0], H = (int)i[1], W = (int)i[2], xoff = (int)i[3], cin8 = (int)i[4], KH = (int)i[5];
  const int KW = (int)i[6], SH = (int)i[7], SW = (int)i[8], PH = (int)i[9], PW = (int)i[10], yoff = (int)i[11];
  const int OH = (int)i[12], OW = (int)i[13], cout = (int)i[14], cin = (int)i[15];
  const int xcs = cs(x), ycs = cs(dy);
  TORCH_CHECK(cin8 % 8 == 0 && cin <= cin8 && xoff % 8 == 0 && xcs % 8 == 0 && xoff + cin8 <= xcs, "wgrad: input slice");
  TORCH_CHECK(yoff % 8 == 0 && ycs % 8 == 0 && yoff + cout <= ycs, "wgrad: gradient slice");
  TORCH_CHECK(x.numel() >= (int64_t)N * H * W * xcs && dy.numel() >= (int64_t)N * OH * OW * ycs, "wgrad: sizes");
  TORCH_CHECK(OH == (H + 2 * PH - KH) / SH + 1 && OW == (W + 2 * PW - KW) / SW + 1, "wgrad: output size");
  TORCH_CHECK(dw.numel() == (int64_t)KH * KW * cin * cout, "wgrad: dw must be [KH][KW][cin][cout]");
  TORCH_CHECK(x.numel() * 2 < (1LL << 31) && dy.numel() * 2 < (1LL << 31), "wgrad: operand larger than 2 GiB");
  if (db.defined()) { check_f32(db, "db"); TORCH_CHECK(db.numel() == cout, "wgrad: db"); }
  int S, cp, kp;
  const int64_t M = (int64_t)N * OH * OW;
  jr_wgrad_plan_geom(N, H, W, cin8, KH, KW, SH, SW, PH, PW, OH, OW, cout, &S, &cp, &kp);
  if (!part.defined()) part = at::empty({(int64_t)S * cp * kp}, dw.options());
  if (!bpart.defined()) bpart = at::empty({(int64_t)S * cp}, dw.options());
  check_f32(part, "part"); check_f32(bpart, "bpart");
  TORCH_CHECK(part.numel() >= (int64_t)S * cp * kp && bpart.numel() >= (int64_t)S * cp, "wgrad: workspace");
  if (keep) for (auto& v : {x, dy, dw, db, part, bpart}) if (v.defined()) keep->push_back(v);
  const void *xp = x.data_ptr(), *yp = dy.data_ptr();
  float *dwp = dw.data_ptr<float>(), *dbp = db.defined() ? db.data_ptr<float>() : nullptr;
  float *pp = part.data_ptr<float>(), *bp = bpart.data_ptr<float>();
  const long xb = x.numel() * 2, yb = dy.numel() * 2;
  return [=](hipStream_t s, int) {
    return jr_wgrad(xp, xcs, xoff, N, H, W, cin8, KH, KW, SH, SW, PH, PW, yp, ycs, yoff, OH, OW, cout, cin, pp, bp, S,
                    dwp, dbp, xb, yb, s);
  };
}

// t = [table (int64 [n][8] device), *referenced tensors (kept alive)], i = [n, max_c]
static Launch make_bn_table(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor tab = opt(t, 0);
  TORCH_CHECK(i.size() == 2, "bn_table: expected [n, max_c]");
  TORCH_CHECK(tab.defined() && tab.is_cuda() && tab.is_contiguous() && tab.scalar_type() == at::kLong &&
                  tab.numel() == i[0] * 8, "bn_table: table must be a contiguous int64 [n][8] GPU tensor");
  if (keep) for (size_t k = 0; k < t.size(); ++k) { at::Tensor v = opt(t, k); if (v.defined()) keep->push_back(v); }
  const void* tp = tab.data_ptr();
  const int n = (int)i[0], mc = (int)i[1];
  return [=](hipStream_t s, int) { return jr_bn_table(tp, n, mc, s); };
}

// t = [taps, dflow], i = [N, h, w]
static Launch make_flow_gather_bwd(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor taps = opt(t, 0), df = opt(t, 1);
  TORCH_CHECK(i.size() == 3, "flow_gather_bwd: expected 3 ints");
  check_f32(taps, "taps"); check_bf16(df, "dflow");
  const int N = (int)i[0], h = (int)i[1], w = (int)i[2];
  const int64_t M = (int64_t)N * h * w;
  TORCH_CHECK(cs(taps) >= 18 && cs(taps) % 2 == 0 && taps.numel() >= M * cs(taps), "flow_gather_bwd: taps");
  TORCH_CHECK(cs(df) >= 2 && df.numel() >= M * cs(df), "flow_gather_bwd: dflow");
  if (keep) { keep->push_back(taps); keep->push_back(df); }
  const float* tp = taps.data_ptr<float>();
  void* dp = df.data_ptr();
  const int tcs = cs(taps), dcs = cs(df);
  return [=](hipStream_t s, int) { return jr_flow_gather_bwd(tp, tcs, N, h, w, dp, dcs, s); };
}

// t = [gout, dflow], i = [B, h, w]
static Launch make_upsample_bilinear_bwd(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor g = opt(t, 0), df = opt(t, 1);
  TORCH_CHECK(i.size() == 3, "upsample_bilinear_bwd: expected 3 ints");
  check_f32(g, "gout"); check_bf16(df, "dflow");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2];
  const int64_t M = (int64_t)B * h * w;
  TORCH_CHECK(g.numel() >= 128 * M && cs(df) >= 2 && df.numel() >= M * cs(df), "upsample_bilinear_bwd: sizes");
  if (keep) { keep->push_back(g); keep->push_back(df); }
  const float* gp = g.data_ptr<float>();
  void* dp = df.data_ptr();
  const int dcs = cs(df);
  return [=](hipStream_t s, int) { return jr_upsample_bilinear_bwd(gp, B, h, w, dp, dcs, s); };
}


// ------------------------------------------------------------------ flow taps
// t = [taps (fp32 [M][tcs]), bias (fp32 [2]), coords, flow32, hx, qx?, flow8?]
// i = [N, h, w, hx_off, qx_off]
static Launch make_flow_taps(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor tp = opt(t, 0), bias = opt(t, 1), coords = opt(t, 2), flow32 = opt(t, 3), hx = opt(t, 4), qx = opt(t, 5),
             f8 = opt(t, 6);
  TORCH_CHECK(i.size() == 5, "flow_taps: expected 5 ints");
  check_f32(tp, "taps"); check_f32(bias, "bias"); check_f32(coords, "coords"); check_f32(flow32, "flow32");
  check_bf16(hx, "hx");
  const int N = (int)i[0], h = (int)i[1], w = (int)i[2], hx_off = (int)i[3], qx_off = (int)i[4];
  const int64_t M = (int64_t)N * h * w;
  TORCH_CHECK(cs(tp) >= 18 && cs(tp) % 2 == 0 && tp.numel() >= M * cs(tp), "flow_taps: taps [M][>=18]");
  TORCH_CHECK(bias.numel() >= 2 && coords.numel() >= 2 * M && flow32.numel() >= 2 * M, "flow_taps: bias / coords / flow32");
  TORCH_CHECK(hx.numel() >= M * cs(hx) && hx_off + 2 <= cs(hx), "flow_taps: hx");
  if (qx.defined()) { check_bf16(qx, "qx"); TORCH_CHECK(qx.numel() >= M * cs(qx) && qx_off + 2 <= cs(qx), "flow_taps: qx"); }
  if (f8.defined()) { check_bf16(f8, "flow8"); TORCH_CHECK(f8.numel() >= M * cs(f8) && cs(f8) >= 2, "flow_taps: flow8"); }
  if (keep) for (auto& v : {tp, bias, coords, flow32, hx, qx, f8}) if (v.defined()) keep->push_back(v);
  const float* tpp = tp.data_ptr<float>();
  const float* bp = bias.data_ptr<float>();
  float* cp = coords.data_ptr<float>();
  float* f32p = flow32.data_ptr<float>();
  void* hp = hx.data_ptr();
  void* qp = ptr(qx);
  void* f8p = ptr(f8);
  const int tcs = cs(tp), hcs = cs(hx), qcs = qx.defined() ? cs(qx) : 0, f8cs = f8.defined() ? cs(f8) : 0;
  // optional t[7]: flow32 of ODD iterations (parity-buffered, see make_lookup)
  float* f32b = nullptr;
  if (at::Tensor fb = opt(t, 7); fb.defined()) {
    check_f32(fb, "flow32 (odd)");
    TORCH_CHECK(fb.numel() >= 2 * M, "flow_taps: odd-iteration flow32 [M][2]");
    f32b = fb.data_ptr<float>();
    if (keep) keep->push_back(fb);
  }
  return [=](hipStream_t s, int it) {
    float* f = (f32b && (it & 1)) ? f32b : f32p;
    return jr_flow_taps(tpp, tcs, bp, N, h, w, cp, f, hp, hcs, hx_off, qp, qcs, qx_off, f8p, f8cs, s);
  };
}

// t = [x (bf16 [M][cs]), wpk (bf16, pack_conv1x1), bias (fp32 [cout]), y (bf16 [M][ycs])],
// i = [M, kvalid, kpad, cout, act, y_coff]
static Launch make_conv1x1(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), wpk = opt(t, 1), bias = opt(t, 2), y = opt(t, 3);
  check_bf16(x, "x"); check_bf16(wpk, "wpk"); check_f32(bias, "bias"); check_bf16(y, "y");
  TORCH_CHECK(i.size() == 6, "conv1x1: expected 6 ints");
  const int64_t M = i[0];
  const int kvalid = (int)i[1], kpad = (int)i[2], cout = (int)i[3], act = (int)i[4], ycoff = (int)i[5];
  TORCH_CHECK(cout % 64 == 0 && kpad % 32 == 0 && kvalid <= kpad && kvalid % 8 == 0 && kvalid <= cs(x),
              "conv1x1: shapes");
  TORCH_CHECK(cs(x) % 8 == 0 && x.numel() >= M * cs(x) && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "conv1x1: x [M][cs], 16-byte rows");
  TORCH_CHECK(wpk.numel() == (int64_t)cout * kpad && reinterpret_cast<uintptr_t>(wpk.data_ptr()) % 16 == 0,
              "conv1x1: packed weights (pack_conv1x1)");
  TORCH_CHECK(bias.numel() >= cout && reinterpret_cast<uintptr_t>(bias.data_ptr()) % 16 == 0, "conv1x1: bias");
  TORCH_CHECK(cs(y) % 8 == 0 && ycoff % 8 == 0 && ycoff + cout <= cs(y) && y.numel() >= M * cs(y) &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "conv1x1: y [M][cs] with a 16-byte aligned cout-channel slice");
  if (keep) { keep->push_back(x); keep->push_back(wpk); keep->push_back(bias); keep->push_back(y); }
  const void* xp = x.data_ptr();
  const void* wp = wpk.data_ptr();
  const float* bp = bias.data_ptr<float>();
  void* yp = y.data_ptr();
  const int xcs = cs(x), ycs = cs(y);
  return [=](hipStream_t s, int) {
    return jr_conv1x1_lds(xp, xcs, kvalid, kpad, wp, bp, act, yp, ycs, ycoff, cout, (int)M, s);
  };
}

bool gru_fused_fits(int64_t H, int64_t W, int64_t vertical) {
  if (!vertical) return W >= 1 && W <= 128;
  const int J = 2 * H <= 128 && W % 2 == 0 ? 2 : 1;
  return H >= 1 && J * H <= 128 && J * (H + 4) <= 136 && W % J == 0;
}

// Fused ConvGRU stage (gru_fused.hip).  t = [hx (bf16 [M][256]: h | x), wa (pack_weight of [z | r],
// [256][1280]), wb (pack_weight of q, [128][1280]), bmap ([M][>=384] fp32 / bf16: z | r | q context
// share), h32 (fp32 [M][128], in place), y (bf16 [M][ycs], channels [0, 128)), y2 (optional copy)],
// i = [N, H, W, vertical(, g2all)].  Tiles: a row (1x5, W <= 128) or J = 2 / 1 columns (5x1, J * H <= 128).
// g2all (default 1): GEMM 2 on all 16 waves with z through LDS; 0: on the 8 z waves, z in registers
// (measured 334-341 vs 335 pairs/s at the headline, profiles/r3_gru_fused_ab.txt; kept for the tests).
static Launch make_gru_fused(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor hx = opt(t, 0), wa = opt(t, 1), wb = opt(t, 2), bmap = opt(t, 3), h32 = opt(t, 4), y = opt(t, 5),
             y2 = opt(t, 6), dbg = opt(t, 7);
  check_bf16(hx, "hx"); check_bf16(wa, "wa"); check_bf16(wb, "wb"); check_f32(h32, "h32"); check_bf16(y, "y");
  TORCH_CHECK(i.size() == 4 || i.size() == 5, "gru_fused: expected 4 or 5 ints");
  GruFusedParams p{};
  p.N = (int)i[0]; p.H = (int)i[1]; p.W = (int)i[2]; p.vertical = (int)i[3];
  p.g2all = i.size() == 5 ? (int)(i[4] != 0) : 1;
  const int64_t M = (int64_t)p.N * p.H * p.W;
  TORCH_CHECK(gru_fused_fits(p.H, p.W, p.vertical), "gru_fused: the tile geometry does not fit (", p.H, "x", p.W, ")");
  TORCH_CHECK(cs(hx) == 256 && hx.numel() >= M * 256 && reinterpret_cast<uintptr_t>(hx.data_ptr()) % 16 == 0,
              "gru_fused: hx must be [M][256] ([h 128 | x 128])");
  TORCH_CHECK(wa.numel() == 256 * 1280 && wb.numel() == 128 * 1280 &&
                  reinterpret_cast<uintptr_t>(wa.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(wb.data_ptr()) % 16 == 0,
              "gru_fused: packed weights [256][1280] / [128][1280]");
  TORCH_CHECK(bmap.defined() && bmap.is_cuda() && bmap.is_contiguous() &&
                  (bmap.scalar_type() == at::kFloat || bmap.scalar_type() == at::kBFloat16) && cs(bmap) >= 384 &&
                  cs(bmap) % 8 == 0 && bmap.numel() >= M * cs(bmap) && reinterpret_cast<uintptr_t>(bmap.data_ptr()) % 16 == 0,
              "gru_fused: bias map [M][>=384] fp32 / bf16");
  TORCH_CHECK(h32.numel() >= M * 128 && cs(h32) == 128 && reinterpret_cast<uintptr_t>(h32.data_ptr()) % 16 == 0,
              "gru_fused: h32 [M][128]");
  TORCH_CHECK(cs(y) % 8 == 0 && cs(y) >= 128 && y.numel() >= M * cs(y) && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "gru_fused: y [M][>=128]");
  if (y2.defined()) {
    check_bf16(y2, "y2");
    TORCH_CHECK(cs(y2) % 8 == 0 && cs(y2) >= 128 && y2.numel() >= M * cs(y2) &&
                    reinterpret_cast<uintptr_t>(y2.data_ptr()) % 16 == 0, "gru_fused: y2 [M][>=128]");
  }
  p.hx = hx.data_ptr(); p.hx_cs = 256; p.wa = wa.data_ptr(); p.wb = wb.data_ptr();
  p.bmap = bmap.data_ptr(); p.bmap_cs = cs(bmap); p.bmap_bf16 = bmap.scalar_type() == at::kBFloat16;
  p.h32 = h32.data_ptr<float>(); p.y = y.data_ptr(); p.y_cs = cs(y); p.y2 = ptr(y2); p.y2_cs = y2.defined() ? cs(y2) : 0;
  if (!p.vertical) { p.L = p.W; p.J = 1; p.tiles_per_img = p.H; }
  else { p.L = p.H; p.J = 2 * p.H <= 128 && p.W % 2 == 0 ? 2 : 1; p.tiles_per_img = p.W / p.J; }
  p.ntiles = p.N * p.tiles_per_img;
  if (dbg.defined()) {   // phase timestamps (tools/gru_phases.py)
    TORCH_CHECK(dbg.is_cuda() && dbg.scalar_type() == at::kLong && dbg.numel() >= (int64_t)p.ntiles * 6, "gru_fused: dbg");
    p.dbg = (long long*)dbg.data_ptr();
  }
  p.hx_bytes = (long)hx.numel() * 2; p.wa_bytes = (long)wa.numel() * 2; p.wb_bytes = (long)wb.numel() * 2;
  TORCH_CHECK(p.hx_bytes < (1LL << 31), "gru_fused: hx larger than 2 GiB");
  if (keep) for (auto& v : {hx, wa, wb, bmap, h32, y, y2}) if (v.defined()) keep->push_back(v);
  // optional t[8]: the y2 copy of ODD loop iterations (a parity-buffered h copy for the mask lane,
  // runtime/engine.py: the lane reads iteration i's copy while iteration i+1 writes the other one)
  at::Tensor y2b = opt(t, 8);
  if (y2b.defined()) {
    TORCH_CHECK(y2.defined(), "gru_fused: an odd-iteration y2 needs y2");
    check_bf16(y2b, "y2 (odd)");
    TORCH_CHECK(y2b.sizes() == y2.sizes() && reinterpret_cast<uintptr_t>(y2b.data_ptr()) % 16 == 0,
                "gru_fused: odd-iteration y2 must have y2's shape");
    GruFusedParams q = p;
    q.y2 = y2b.data_ptr();
    if (keep) keep->push_back(y2b);
    return [p, q](hipStream_t s, int it) { return jr_gru_fused((it & 1) ? &q : &p, s); };
  }
  return [p](hipStream_t s, int) { return jr_gru_fused(&p, s); };
}

// Halo-tiled fused ConvGRU stage (gru_halo.hip).
// t = [hsrc (bf16 [M][cs]: h = channels [0, hd)), xsrc (bf16 [M][cs]: x = [hd, cs)), wa, wb
//      (ops/native.py:pack_gru_halo of [z | r] / q), bmap (bf16 [M][>= 3 hd]), h32 (fp32 [M][hd],
//      in place), y (bf16 [M][ycs], h' -> channels [0, hd)), y2?],
// i = [N, H, W, mode, axis, TR, TC, nb1, nb2].  cs = 2 hd (hd 128: mode 0 = a 5-tap run, TR = 1,
// TC = run length; hd 96: mode 1 = a TR x TC block of the 3x3 GRU).
bool gru_halo_geom_ok(int64_t hd, int64_t mode, int64_t TR, int64_t TC, int64_t nb1, int64_t nb2) {
  if (TR < 1 || TC < 1) return false;
  const int64_t nreg = mode == 0 ? TC + 4 : (TR + 2) * (TC + 2);
  const int64_t nout = TR * TC;
  if ((mode == 0 && (TR != 1 || hd != 128)) || (mode == 1 && hd != 96) || mode < 0 || mode > 1) return false;
  if (nreg > 32 * nb1 || nout > 32 * nb2) return false;
  return jr_gru_halo_lds((int)hd, (int)mode, (int)TR, (int)TC, (int)nb1, (int)nb2) > 0 &&
         jr_gru_halo_lds((int)hd, (int)mode, (int)TR, (int)TC, (int)nb1, (int)nb2) <= 160 * 1024;
}

static Launch make_gru_halo(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor hs = opt(t, 0), xs = opt(t, 1), wa = opt(t, 2), wb = opt(t, 3), bmap = opt(t, 4), h32 = opt(t, 5),
             y = opt(t, 6), y2 = opt(t, 7);
  check_bf16(hs, "hsrc"); check_bf16(xs, "xsrc"); check_bf16(wa, "wa"); check_bf16(wb, "wb"); check_bf16(bmap, "bmap");
  check_f32(h32, "h32"); check_bf16(y, "y");
  TORCH_CHECK(i.size() == 9, "gru_halo: expected [N, H, W, mode, axis, TR, TC, nb1, nb2]");
  GruHaloParams p{};
  p.N = (int)i[0]; p.H = (int)i[1]; p.W = (int)i[2]; p.mode = (int)i[3]; p.axis = (int)i[4];
  p.TR = (int)i[5]; p.TC = (int)i[6]; p.nb1 = (int)i[7]; p.nb2 = (int)i[8];
  const int64_t M = (int64_t)p.N * p.H * p.W;
  const int cs_ = cs(hs), hd = cs_ / 2;
  const int taps = p.mode == 0 ? 5 : 9;
  TORCH_CHECK(p.N >= 1 && p.H >= 1 && p.W >= 1 && M < (1LL << 31), "gru_halo: map size");
  TORCH_CHECK(gru_halo_geom_ok(hd, p.mode, p.TR, p.TC, p.nb1, p.nb2), "gru_halo: unsupported tile (hd ", hd, ", mode ",
              p.mode, ", ", p.TR, "x", p.TC, ", blocks ", p.nb1, "/", p.nb2, ")");
  TORCH_CHECK(p.mode == 1 || p.axis == 0 || p.axis == 1, "gru_halo: axis must be 0 (1x5) or 1 (5x1)");
  TORCH_CHECK(cs(xs) == cs_ && hs.numel() >= M * cs_ && xs.numel() >= M * cs_ && hs.numel() == xs.numel(),
              "gru_halo: hsrc / xsrc must be [M][2 hd] with one shape");
  TORCH_CHECK(hs.data_ptr() != y.data_ptr(), "gru_halo: y must not alias hsrc (neighbouring tiles read h)");
  TORCH_CHECK(wa.numel() == (int64_t)2 * hd * taps * cs_ && wb.numel() == (int64_t)hd * taps * cs_,
              "gru_halo: packed weights (pack_gru_halo) of [z | r] and q");
  TORCH_CHECK(cs(bmap) >= 3 * hd && cs(bmap) % 8 == 0 && bmap.numel() >= M * cs(bmap), "gru_halo: bias map [M][>= 3 hd]");
  TORCH_CHECK(cs(h32) == hd && h32.numel() >= M * hd, "gru_halo: h32 [M][hd]");
  TORCH_CHECK(cs(y) % 8 == 0 && cs(y) >= hd && y.numel() >= M * cs(y), "gru_halo: y [M][>= hd]");
  for (const at::Tensor* v : {&hs, &xs, &wa, &wb, &bmap, &h32, &y})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(v->data_ptr()) % 16 == 0, "gru_halo: operands must be 16-byte aligned");
  if (y2.defined()) {
    check_bf16(y2, "y2");
    TORCH_CHECK(cs(y2) % 8 == 0 && cs(y2) >= hd && y2.numel() >= M * cs(y2) &&
                    reinterpret_cast<uintptr_t>(y2.data_ptr()) % 16 == 0, "gru_halo: y2 [M][>= hd]");
  }
  p.hsrc = hs.data_ptr(); p.xsrc = xs.data_ptr(); p.cs = cs_;
  p.wa = wa.data_ptr(); p.wb = wb.data_ptr();
  p.bmap = bmap.data_ptr(); p.bmap_cs = cs(bmap);
  p.h32 = h32.data_ptr<float>(); p.y = y.data_ptr(); p.y_cs = cs(y); p.y2 = ptr(y2); p.y2_cs = y2.defined() ? cs(y2) : 0;
  if (p.mode == 0) {
    const int len = p.axis ? p.H : p.W, lines = p.axis ? p.W : p.H;
    p.tiles_y = lines;
    p.tiles_x = (len + p.TC - 1) / p.TC;
  } else {
    p.tiles_y = (p.H + p.TR - 1) / p.TR;
    p.tiles_x = (p.W + p.TC - 1) / p.TC;
  }
  const int64_t nt = (int64_t)p.N * p.tiles_y * p.tiles_x;
  TORCH_CHECK(nt < (1LL << 31), "gru_halo: too many tiles");
  p.ntiles = (int)nt;
  p.src_bytes = (long)hs.numel() * 2; p.wa_bytes = (long)wa.numel() * 2; p.wb_bytes = (long)wb.numel() * 2;
  TORCH_CHECK(p.src_bytes < (1LL << 31), "gru_halo: loop buffers larger than 2 GiB");
  if (keep) for (auto& v : {hs, xs, wa, wb, bmap, h32, y, y2}) if (v.defined()) keep->push_back(v);
  // optional t[11..15] (training forward, train/fused.py): h32in (fp32 [M][hd]: h is read there and
  // h' written to h32), and the saved gates zo / ro / qo (bf16 [M][hd]) + r*h into rh (bf16 [M][>= hd])
  {
    at::Tensor h32in = opt(t, 11), zo = opt(t, 12), ro = opt(t, 13), qo = opt(t, 14), rh = opt(t, 15);
    if (h32in.defined()) {
      check_f32(h32in, "h32in");
      TORCH_CHECK(cs(h32in) == hd && h32in.numel() >= M * hd && h32in.data_ptr() != h32.data_ptr() &&
                      reinterpret_cast<uintptr_t>(h32in.data_ptr()) % 16 == 0, "gru_halo: h32in [M][hd], not h32");
      p.h32in = h32in.data_ptr<float>();
      if (keep) keep->push_back(h32in);
    }
    const bool any = zo.defined() || ro.defined() || qo.defined() || rh.defined();
    if (any) {
      TORCH_CHECK(zo.defined() && ro.defined() && qo.defined() && rh.defined(), "gru_halo: saved gates: all four or none");
      for (const at::Tensor* v : {&zo, &ro, &qo}) {
        check_bf16(*v, "saved gate");
        TORCH_CHECK(cs(*v) == hd && v->numel() >= M * hd && reinterpret_cast<uintptr_t>(v->data_ptr()) % 16 == 0,
                    "gru_halo: saved gates are bf16 [M][hd]");
      }
      check_bf16(rh, "rh");
      TORCH_CHECK(cs(rh) % 8 == 0 && cs(rh) >= hd && rh.numel() >= M * cs(rh) &&
                      reinterpret_cast<uintptr_t>(rh.data_ptr()) % 16 == 0 && rh.data_ptr() != hs.data_ptr() &&
                      rh.data_ptr() != xs.data_ptr(), "gru_halo: rh [M][>= hd], not a source");
      p.zo = zo.data_ptr(); p.ro = ro.data_ptr(); p.qo = qo.data_ptr(); p.rh = rh.data_ptr(); p.rh_cs = cs(rh);
      if (keep) for (auto& v : {zo, ro, qo, rh}) keep->push_back(v);
    }
  }
  // optional t[8..10] = hsrc / xsrc / y of ODD loop iterations: a single-stage GRU (raft_small)
  // ping-pongs h between two loop buffers (it cannot update h in place, see the kernel)
  at::Tensor hs2 = opt(t, 8), xs2 = opt(t, 9), y_2 = opt(t, 10);
  if (hs2.defined() || xs2.defined() || y_2.defined()) {
    TORCH_CHECK(hs2.defined() && xs2.defined() && y_2.defined(), "gru_halo: odd-iteration operands: all three or none");
    for (const at::Tensor* v : {&hs2, &xs2, &y_2}) {
      check_bf16(*v, "odd-iteration operand");
      TORCH_CHECK(v->sizes() == hs.sizes() && reinterpret_cast<uintptr_t>(v->data_ptr()) % 16 == 0,
                  "gru_halo: odd-iteration operands must have the loop buffers' shape");
    }
    TORCH_CHECK(hs2.data_ptr() != y_2.data_ptr(), "gru_halo: odd-iteration y must not alias its hsrc");
    GruHaloParams q = p;
    q.hsrc = hs2.data_ptr(); q.xsrc = xs2.data_ptr(); q.y = y_2.data_ptr(); q.y_cs = cs(y_2);
    if (keep) for (auto& v : {hs2, xs2, y_2}) keep->push_back(v);
    return [p, q](hipStream_t s, int it) { return jr_gru_halo((it & 1) ? &q : &p, s); };
  }
  return [p](hipStream_t s, int) { return jr_gru_halo(&p, s); };
}

// t = [fm (bf16 [M][cs]), wpk (bf16, pack_taps), taps (fp32 [M][>=24])], i = [M, K, fcoff]
static Launch make_taps_gemm(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor fm = opt(t, 0), wpk = opt(t, 1), taps = opt(t, 2);
  check_bf16(fm, "fm"); check_bf16(wpk, "wpk"); check_f32(taps, "taps");
  TORCH_CHECK(i.size() == 3, "taps_gemm: expected 3 ints");
  const int64_t M = i[0];
  const int K = (int)i[1], fcoff = (int)i[2];
  TORCH_CHECK(K == 128 || K == 256, "taps_gemm: K must be 128 or 256");
  TORCH_CHECK(cs(fm) % 8 == 0 && fcoff % 8 == 0 && fcoff >= 0 && fcoff + K <= cs(fm) && fm.numel() >= M * cs(fm) &&
                  reinterpret_cast<uintptr_t>(fm.data_ptr()) % 16 == 0,
              "taps_gemm: fm [M][cs] with a 16-byte aligned K-channel slice");
  TORCH_CHECK(wpk.numel() == (int64_t)K / 32 * 2 * 64 * 8 && reinterpret_cast<uintptr_t>(wpk.data_ptr()) % 16 == 0,
              "taps_gemm: packed weights (pack_taps)");
  TORCH_CHECK(cs(taps) >= 24 && cs(taps) % 4 == 0 && taps.numel() >= M * cs(taps) &&
                  reinterpret_cast<uintptr_t>(taps.data_ptr()) % 16 == 0,
              "taps_gemm: taps [M][>=24], 16-byte rows");
  if (keep) { keep->push_back(fm); keep->push_back(wpk); keep->push_back(taps); }
  const void* fp = fm.data_ptr();
  const void* wp = wpk.data_ptr();
  float* tp = taps.data_ptr<float>();
  const int fcs = cs(fm), tcs = cs(taps);
  return [=](hipStream_t s, int) { return jr_taps_gemm(fp, fcs, fcoff, K, wp, tp, tcs, (int)M, s); };
}

// ---------------------------------------------------------------- direct conv
// t = [x (bf16 NHWC, 2 channels used), w (bf16 A fragments [cout/16][NKC][64][8]), bias (fp32 [cout]), y (bf16)]
// i = [N, H, W, cin, KH, KW, PH, PW, cout, relu, y_coff]   (stride 1, output H x W)
static Launch make_conv_direct(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), w = opt(t, 1), bias = opt(t, 2), y = opt(t, 3);
  TORCH_CHECK(i.size() == 11, "conv_direct: expected 11 ints");
  check_bf16(x, "x"); check_bf16(w, "w"); check_f32(bias, "bias"); check_bf16(y, "y");
  const int N = (int)i[0], H = (int)i[1], W = (int)i[2], cin = (int)i[3], KH = (int)i[4], KW = (int)i[5];
  const int PH = (int)i[6], PW = (int)i[7], cout = (int)i[8], relu = (int)i[9], y_coff = (int)i[10];
  const int64_t M = (int64_t)N * H * W;
  TORCH_CHECK(cs(x) >= cin && x.numel() >= M * cs(x), "conv_direct: x [N*H*W][>=cin]");
  const int kwp = KW <= 4 ? 4 : 8, nkc = (KH * kwp * 2 + 31) / 32;
  TORCH_CHECK(cin == 2 && w.numel() == (int64_t)cout * nkc * 32 && bias.numel() >= cout, "conv_direct: w / bias");
  TORCH_CHECK(y.numel() >= M * cs(y) && y_coff + cout <= cs(y), "conv_direct: y");
  if (keep) for (auto& v : {x, w, bias, y}) keep->push_back(v);
  const void* xp = x.data_ptr();
  const void* wp = w.data_ptr();
  const float* bp = bias.data_ptr<float>();
  void* yp = y.data_ptr();
  const int xcs = cs(x), ycs = cs(y);
  return [=](hipStream_t s, int) {
    return jr_conv_direct(xp, xcs, N, H, W, cin, KH, KW, PH, PW, wp, bp, cout, relu, yp, ycs, y_coff, s);
  };
}

// The 7x7 flow conv (as make_conv_direct) merged with the DEFERRED x8 upsampling of the
// previous iteration (merged.hip).  t = [x, w, bias, y, flow32, out, out_slot?(, feat, wpk, cbias)],
// i = [N, H, W, 2, 7, 7, PH, PW, cout, relu, y_coff, mode (1 bilinear / 2 convex head), out_iter_stride,
// out_slot_off, feat_coff].  Iteration 0 runs the flow conv alone (nothing to upsample yet); iteration
// it > 0 upsamples iteration it - 1, as a deferred op would.
// t = [x, w, bias, y, flow32, out, out_slot, feat?, wpk?, cbias?,  (c1x, c1w, c1b, c1y)?]
// i = [conv_direct's 11 ints, mode, stride, slot_off, feat_coff,  (M, kvalid, kpad, cout, act, ycoff)?]
// With the conv1x1 operands (mode 2): the correlation features' 1x1 conv runs in the same grid,
// every iteration (iteration 0: with the flow conv alone).
static Launch make_flowin_dual(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep) {
  Launch conv = make_conv_direct(t, IList(i.begin(), i.begin() + 11), keep);
  TORCH_CHECK((i.size() == 15 || i.size() == 21) && i[4] == 7 && i[5] == 7,
              "flowin_dual: expected 15 (+6) ints, a 7x7 flow conv");
  const bool has_c1 = i.size() == 21;
  Conv1x1Args c1a{};
  if (has_c1) {
    TORCH_CHECK(i[11] == 2 && i[17] == 352, "flowin_dual: the 1x1 conv part needs mode 2 and K padded to 352");
    TList t1;
    for (size_t k = 10; k < 14; ++k) t1.push_back(c10::optional<at::Tensor>(opt(t, k)));
    (void)make_conv1x1(t1, IList(i.begin() + 15, i.end()), keep);   // validates (and keeps) the operands
    at::Tensor x1 = opt(t, 10), w1 = opt(t, 11), b1 = opt(t, 12), y1 = opt(t, 13);
    c1a = Conv1x1Args{x1.data_ptr(), (int)cs(x1), (int)i[16], (int)i[17], w1.data_ptr(), b1.data_ptr<float>(),
                      (int)i[19], y1.data_ptr(), (int)cs(y1), (int)i[20], (int)i[18], (int)i[15]};
  }
  at::Tensor x = opt(t, 0), w = opt(t, 1), bias = opt(t, 2), y = opt(t, 3), flow = opt(t, 4), out = opt(t, 5),
             slot = opt(t, 6), feat = opt(t, 7), wpk = opt(t, 8), cb = opt(t, 9);
  const int N = (int)i[0], H = (int)i[1], W = (int)i[2], PH = (int)i[6], PW = (int)i[7], cout = (int)i[8];
  const int relu = (int)i[9], y_coff = (int)i[10], mode = (int)i[11], fcoff = (int)i[14];
  const int64_t stride = i[12], slot_off = i[13];
  check_f32(flow, "flow32");
  TORCH_CHECK(mode == 1 || mode == 2, "flowin_dual: mode 1 (bilinear) or 2 (convex head)");
  TORCH_CHECK(flow.numel() >= (int64_t)N * H * W * 2, "flowin_dual: flow [M][2]");
  TORCH_CHECK(!slot.defined() || (slot.is_cuda() && slot.scalar_type() == at::kLong && slot.numel() == 1),
              "flowin_dual: out_slot must be one device int64");
  const int64_t cap = check_flow_out(out, N, H, W);
  TORCH_CHECK(stride >= 0 && stride % 8 == 0, "flowin_dual: iteration stride");
  int fcs = 0;
  if (mode == 2) {
    check_bf16(feat, "feat"); check_bf16(wpk, "wpk"); check_f32(cb, "cbias");
    fcs = cs(feat);
    TORCH_CHECK(fcs % 8 == 0 && fcoff % 8 == 0 && fcoff >= 0 && fcoff + 256 <= fcs &&
                    feat.numel() >= (int64_t)N * H * W * fcs && reinterpret_cast<uintptr_t>(feat.data_ptr()) % 16 == 0,
                "flowin_dual: feat [M][cs], 16-byte aligned 256-channel slice");
    TORCH_CHECK(wpk.numel() == 576 * 256 && cb.numel() == 576 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 32 == 0,
                "flowin_dual: convex head operands");
  }
  if (keep) for (auto& v : {flow, out, slot, feat, wpk, cb}) if (v.defined()) keep->push_back(v);
  const void* xp = x.data_ptr();
  const void* wp = w.data_ptr();
  const float* bp = bias.data_ptr<float>();
  void* yp = y.data_ptr();
  const int xcs = cs(x), ycs = cs(y);
  const float* fp = flow.data_ptr<float>();
  float* op = out.data_ptr<float>();
  const void* sp = slot.defined() ? slot.data_ptr() : nullptr;
  const void* featp = ptr(feat);
  const void* wpkp = ptr(wpk);
  const float* cbp = cb.defined() ? cb.data_ptr<float>() : nullptr;
  const float a = (float)alpha;
  const int64_t per_iter = mode == 1 ? (int64_t)N * 64 * H * W * 2 : (int64_t)N * H * W * 128;
  return [=](hipStream_t s, int it) {
    if (it == 0 && !has_c1) return conv(s, it);
    if (it == 0)
      return jr_flowin_dual(xp, xcs, N, H, W, PH, PW, wp, bp, cout, relu, yp, ycs, y_coff, mode, featp, fcs, fcoff,
                            wpkp, cbp, a, fp, nullptr, nullptr, 0, &c1a, s);
    const int64_t off = stride * (it - 1);
    if (off + per_iter > cap) return (int)hipErrorInvalidValue;
    return jr_flowin_dual(xp, xcs, N, H, W, PH, PW, wp, bp, cout, relu, yp, ycs, y_coff, mode, featp, fcs, fcoff, wpkp,
                          cbp, a, fp, op + off, sp, (long)(slot_off + off), has_c1 ? &c1a : nullptr, s);
  };
}

// ------------------------------------------------------------------ flow head
// t = [fm, wt (bf16 [2][9][cin]), bias (fp32 [2]), coords, flow32, hx, qx?, flow8?]
// i = [N, h, w, cin, fm_coff, hx_off, qx_off]
// t = [f1, f2, l0, l1, l2, l3], i = [B, h, w, C, num_levels]; levels all fp32 or all bf16
static void check_level(const at::Tensor& v, at::ScalarType dt) {
  TORCH_CHECK(v.defined() && v.is_cuda() && v.is_contiguous(), "pyramid level must be a contiguous GPU tensor");
  TORCH_CHECK(v.scalar_type() == dt && (dt == at::kFloat || dt == at::kBFloat16), "pyramid levels: fp32 or bf16, one dtype");
}

static Launch make_corr(const TList& t, const IList& i, double scale, std::vector<at::Tensor>* keep) {
  at::Tensor f1 = opt(t, 0), f2 = opt(t, 1);
  check_bf16(f1, "f1"); check_bf16(f2, "f2");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2], C = (int)i[3], L = (int)i[4];
  // optional i[5]: query pixels per image in f1 (a slab of query rows; default all h*w);
  // optional i[6]: 1 = blocked level layout (kernels.h), 2 = blocked + the persistent kernel at any batch
  const int nq = i.size() > 5 ? (int)i[5] : h * w;
  const int blocked = i.size() > 6 ? (int)i[6] : 0;
  TORCH_CHECK(!blocked || (w % 16 == 0 && (h * w) % 8 == 0 && nq == h * w),
              "corr: the blocked level layout needs w % 16 == 0 and whole query maps");
  const int nty = (h + 7) / 8, ntx = (w + 15) / 16;
  TORCH_CHECK(L >= 1 && L <= 4, "corr: 1..4 levels");
  TORCH_CHECK(C % 64 == 0, "corr: feature channels must be a multiple of 64");
  TORCH_CHECK(nq >= 1 && f1.numel() >= (int64_t)B * nq * cs(f1) && f2.numel() >= (int64_t)B * h * w * cs(f2) &&
              cs(f1) == cs(f2), "corr: fmap shapes");
  void* lv[4] = {nullptr, nullptr, nullptr, nullptr};
  at::Tensor l0 = opt(t, 2);
  TORCH_CHECK(l0.defined(), "corr: level 0 missing");
  const at::ScalarType dt = l0.scalar_type();
  int hl = h, wl = w;
  for (int l = 0; l < L; ++l) {
    at::Tensor v = opt(t, 2 + l);
    check_level(v, dt);
    TORCH_CHECK(!blocked || dt == at::kBFloat16, "corr: the blocked level layout is bf16");
    const int64_t per_q = (blocked && l < 2) ? (int64_t)nty * ntx * (128 >> (2 * l)) : (int64_t)hl * wl;
    TORCH_CHECK(v.numel() >= (int64_t)B * nq * per_q, "corr: level ", l, " too small");
    lv[l] = v.data_ptr();
    if (keep) keep->push_back(v);
    hl >>= 1; wl >>= 1;
  }
  if (keep) { keep->push_back(f1); keep->push_back(f2); }
  const void* a = f1.data_ptr();
  const void* b = f2.data_ptr();
  const int fcs = cs(f1);
  const float sc = (float)scale;
  const int obf = dt == at::kBFloat16;
  return [=](hipStream_t s, int) {
    return jr_corr_pyramid(a, b, B, h, w, nq, C, fcs, lv[0], lv[1], lv[2], lv[3], L, sc, obf, blocked, s);
  };
}

// t = [coords, out, l0, l1, l2, l3], i = [num_levels, B, h, w, radius]
static Launch make_lookup(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor coords = opt(t, 0), out = opt(t, 1);
  check_f32(coords, "coords"); check_bf16(out, "out");
  const int L = (int)i[0], B = (int)i[1], h = (int)i[2], w = (int)i[3], r = (int)i[4];
  const int nq = i.size() > 5 ? (int)i[5] : h * w;  // queries per image (slab of rows) vs level-0 map h x w
  const int blocked = i.size() > 6 ? (int)i[6] : 0;  // blocked level layout (kernels.h)
  const int nty = (h + 7) / 8, ntx = (w + 15) / 16;
  const int S = 2 * r + 1;
  TORCH_CHECK(L >= 1 && L <= 4 && r >= 1 && r <= 6 && nq >= 1, "lookup: levels 1..4, radius 1..6");
  TORCH_CHECK(cs(out) % 8 == 0 && cs(out) >= L * S * S, "lookup: output channel stride");
  TORCH_CHECK(out.numel() >= (int64_t)B * nq * cs(out) && coords.numel() >= (int64_t)B * nq * 2, "lookup: sizes");
  std::vector<const void*> lv(4, nullptr);
  at::Tensor l0 = opt(t, 2);
  TORCH_CHECK(l0.defined(), "lookup: level 0 missing");
  const at::ScalarType dt = l0.scalar_type();
  int hl = h, wl = w;
  for (int l = 0; l < L; ++l) {
    at::Tensor v = opt(t, 2 + l);
    check_level(v, dt);
    TORCH_CHECK(hl >= 2 && wl >= 2, "lookup: pyramid level too small");
    const int64_t per_q = (blocked && l < 2) ? (int64_t)nty * ntx * (128 >> (2 * l)) : (int64_t)hl * wl;
    TORCH_CHECK(v.numel() >= (int64_t)B * nq * per_q, "lookup: level size");
    lv[l] = v.data_ptr();
    if (keep) keep->push_back(v);
    hl >>= 1; wl >>= 1;
  }
  if (keep) { keep->push_back(coords); keep->push_back(out); }
  const float* cp = coords.data_ptr<float>();
  void* op = out.data_ptr();
  const int ocs = cs(out);
  const int lbf = dt == at::kBFloat16;
  // optional fused flow update (t[6..11] = taps, bias, flow32, hx, qx?, flow8?; i[7..8] = hx_off, qx_off):
  // applied in loop iterations > 0 (iteration i's lookup applies iteration i-1's FlowHead taps)
  TapsUpd upd{};
  at::Tensor tp = opt(t, 6);
  if (tp.defined()) {
    at::Tensor bias = opt(t, 7), f32 = opt(t, 8), hx = opt(t, 9), qx = opt(t, 10), f8 = opt(t, 11);
    TORCH_CHECK(i.size() >= 9, "lookup: the fused flow update needs [.., hx_off, qx_off]");
    check_f32(tp, "taps"); check_f32(bias, "bias"); check_f32(f32, "flow32"); check_bf16(hx, "hx");
    const int64_t M = (int64_t)B * nq;
    TORCH_CHECK(nq == h * w && cs(tp) >= 18 && tp.numel() >= M * cs(tp) && bias.numel() >= 2 && f32.numel() >= 2 * M,
                "lookup: fused update needs whole maps, taps [M][>=18], bias [2], flow32 [M][2]");
    const int hx_off = (int)i[7], qx_off = (int)i[8];
    TORCH_CHECK(hx.numel() >= M * cs(hx) && hx_off + 2 <= cs(hx), "lookup: hx");
    if (qx.defined()) { check_bf16(qx, "qx"); TORCH_CHECK(qx.numel() >= M * cs(qx) && qx_off + 2 <= cs(qx), "lookup: qx"); }
    if (f8.defined()) { check_bf16(f8, "flow8"); TORCH_CHECK(f8.numel() >= M * cs(f8) && cs(f8) >= 2, "lookup: flow8"); }
    upd = TapsUpd{tp.data_ptr<float>(), cs(tp), bias.data_ptr<float>(), coords.data_ptr<float>(), f32.data_ptr<float>(),
                  hx.data_ptr(), cs(hx), hx_off, ptr(qx), cs(qx), qx_off, ptr(f8), cs(f8), 1};
    if (keep) for (auto& v : {tp, bias, f32, hx, qx, f8}) if (v.defined()) keep->push_back(v);
  }
  // optional t[12]: flow32 of ODD iterations (parity-buffered for the mask lane's convex head)
  float* f32b = nullptr;
  if (at::Tensor fb = opt(t, 12); fb.defined()) {
    TORCH_CHECK(upd.on, "lookup: an odd-iteration flow32 needs the fused update");
    check_f32(fb, "flow32 (odd)");
    TORCH_CHECK(fb.numel() >= (int64_t)B * nq * 2, "lookup: odd-iteration flow32 [M][2]");
    f32b = fb.data_ptr<float>();
    if (keep) keep->push_back(fb);
  }
  return [=](hipStream_t s, int it) {
    TapsUpd u = upd;
    u.on = upd.on && it > 0;
    if (f32b && (it & 1)) u.flow32 = f32b;
    return jr_corr_lookup(lv.data(), L, B, h, w, nq, r, cp, op, ocs, lbf, blocked, s, &u);
  };
}

// ------------------------------------------------------------------ upsample
// Upsampled-flow output: a view whose trailing (B, 8h, 8w, 2) block is dense
// (the engine passes out[:, b0:b1] of the (iters, B_total, H, W, 2) buffer).
// Returns the float capacity from the view's first element to the end of its
// storage, which bounds every per-iteration write.
static int64_t check_flow_out(const at::Tensor& out, int B, int h, int w) {
  TORCH_CHECK(out.defined() && out.is_cuda() && out.scalar_type() == at::kFloat, "out must be a CUDA float32 tensor");
  TORCH_CHECK(out.dim() >= 4 && out.size(-1) == 2 && out.size(-2) == 8 * w && out.size(-3) == 8 * h &&
                  out.size(-4) == B && out.stride(-1) == 1 && out.stride(-2) == 2 && out.stride(-3) == 16 * w &&
                  out.stride(-4) == 128 * (int64_t)h * w,
              "out: trailing (B, 8h, 8w, 2) block must be dense");
  return (int64_t)(out.storage().nbytes() / sizeof(float)) - out.storage_offset();
}

// t = [mask, flow, out], i = [B, h, w, out_iter_stride]
static Launch make_upsample_convex(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor mask = opt(t, 0), flow = opt(t, 1), out = opt(t, 2);
  check_bf16(mask, "mask"); check_f32(flow, "flow");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2];
  const int64_t stride = i[3];
  TORCH_CHECK(cs(mask) >= 576, "upsample: mask needs 576 channels");
  const int64_t cap = check_flow_out(out, B, h, w);
  if (keep) { keep->push_back(mask); keep->push_back(flow); keep->push_back(out); }
  const void* mp = mask.data_ptr();
  const float* fp = flow.data_ptr<float>();
  float* op = out.data_ptr<float>();
  const int mcs = cs(mask);
  return [=](hipStream_t s, int it) {
    const int64_t off = stride * it;
    if (off + (int64_t)B * 64 * h * w * 2 > cap) return (int)hipErrorInvalidValue;
    return jr_upsample_convex(mp, mcs, fp, B, h, w, op + off, s);
  };
}

// t = [feat, wpk, bias, flow, out, out_slot?], i = [B, h, w, feat_coff, out_iter_stride(, tiles per wave: 0 =
// auto(, out_slot offset in floats))].  out_slot: device int64 holding the output base address at run time
// (the engine points it at a fresh tensor per call); `out` (same shape) bounds the writes.
static Launch make_convex_head(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep) {
  at::Tensor feat = opt(t, 0), wpk = opt(t, 1), bias = opt(t, 2), flow = opt(t, 3), out = opt(t, 4), slot = opt(t, 5);
  check_bf16(feat, "feat"); check_bf16(wpk, "wpk"); check_f32(bias, "bias"); check_f32(flow, "flow");
  TORCH_CHECK(i.size() >= 5 && i.size() <= 7, "convex_head: expected 5 to 7 ints");
  const int tiles = i.size() >= 6 ? (int)i[5] : 0;
  const int64_t slot_off = i.size() >= 7 ? i[6] : 0;
  TORCH_CHECK(!slot.defined() || (slot.is_cuda() && slot.scalar_type() == at::kLong && slot.numel() == 1),
              "convex_head: out_slot must be one device int64");
  TORCH_CHECK(tiles == 0 || tiles == 1 || tiles == 2, "convex_head: tiles per wave 0/1/2");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2], coff = (int)i[3];
  const int64_t stride = i[4];
  const int64_t M = (int64_t)B * h * w;
  const int fcs = cs(feat);
  TORCH_CHECK(fcs % 8 == 0 && coff % 8 == 0 && coff >= 0 && coff + 256 <= fcs && feat.numel() >= M * fcs &&
                  reinterpret_cast<uintptr_t>(feat.data_ptr()) % 16 == 0,
              "convex_head: feat must be [M][cs] with a 16-byte aligned 256-channel slice");
  TORCH_CHECK(wpk.numel() == 576 * 256 && reinterpret_cast<uintptr_t>(wpk.data_ptr()) % 16 == 0,
              "convex_head: packed weights (pack_convex_head)");
  TORCH_CHECK(bias.numel() == 576 && reinterpret_cast<uintptr_t>(bias.data_ptr()) % 16 == 0, "convex_head: bias [576]");
  TORCH_CHECK(flow.numel() >= 2 * M, "convex_head: flow [M][2]");
  TORCH_CHECK(stride >= 0 && stride % 8 == 0, "convex_head: iteration stride");
  const int64_t cap = check_flow_out(out, B, h, w);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 32 == 0, "convex_head: out must be 32-byte aligned");
  if (keep) { keep->push_back(feat); keep->push_back(wpk); keep->push_back(bias); keep->push_back(flow); keep->push_back(out); }
  if (keep && slot.defined()) keep->push_back(slot);
  const void* sp = slot.defined() ? slot.data_ptr() : nullptr;
  const void* fp = feat.data_ptr();
  const void* wp = wpk.data_ptr();
  const float* bp = bias.data_ptr<float>();
  const float* flp = flow.data_ptr<float>();
  float* op = out.data_ptr<float>();
  const float a = (float)alpha;
  // optional t[6]: the parity-buffered flow (runtime/engine.py): the flow of iteration it was written by
  // the update of iteration it + 1 (lookup / flow_taps), into t[6] when it + 1 is odd, else into t[3]
  const float* flb = nullptr;
  if (at::Tensor fb = opt(t, 6); fb.defined()) {
    check_f32(fb, "flow (odd)");
    TORCH_CHECK(fb.numel() >= 2 * M, "convex_head: odd flow [M][2]");
    flb = fb.data_ptr<float>();
    if (keep) keep->push_back(fb);
  }
  return [=](hipStream_t s, int it) {
    const int64_t off = stride * it;
    if (off + M * 128 > cap) return (int)hipErrorInvalidValue;
    const float* f = (flb && ((it + 1) & 1)) ? flb : flp;
    return jr_convex_head(fp, fcs, coff, wp, bp, a, f, B, h, w, op + off, sp, (long)(slot_off + off), tiles, s);
  };
}

// t = [flow, out], i = [B, h, w, out_iter_stride]
// (t[2]: optional out_slot, i[4]: its offset in floats; see make_convex_head)
static Launch make_upsample_bilinear(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor flow = opt(t, 0), out = opt(t, 1), slot = opt(t, 2);
  check_f32(flow, "flow");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2];
  const int64_t stride = i[3];
  const int64_t slot_off = i.size() > 4 ? i[4] : 0;
  TORCH_CHECK(!slot.defined() || (slot.is_cuda() && slot.scalar_type() == at::kLong && slot.numel() == 1),
              "upsample_bilinear: out_slot must be one device int64");
  const int64_t cap = check_flow_out(out, B, h, w);
  if (keep) { keep->push_back(flow); keep->push_back(out); if (slot.defined()) keep->push_back(slot); }
  const float* fp = flow.data_ptr<float>();
  float* op = out.data_ptr<float>();
  const void* sp = slot.defined() ? slot.data_ptr() : nullptr;
  return [=](hipStream_t s, int it) {
    const int64_t off = stride * it;
    if (off + (int64_t)B * 64 * h * w * 2 > cap) return (int)hipErrorInvalidValue;
    return jr_upsample_bilinear(fp, B, h, w, op + off, sp, (long)(slot_off + off), s);
  };
}

// ---------------------------------------------------------------------- norm
// t = [x, stats, partial?], i = [N, HW, C]; the partial workspace is allocated
// here when not given (eager use), never inside a launch (capture safety).
static Launch make_stats(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), st = opt(t, 1), part = opt(t, 2);
  check_bf16(x, "x"); check_f32(st, "stats");
  const int N = (int)i[0], HW = (int)i[1], C = (int)i[2];
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && cs(x) == C && x.numel() >= (int64_t)N * HW * C, "stats: shape");
  TORCH_CHECK(st.numel() >= (int64_t)N * C * 2, "stats: buffer too small");
  const int64_t need = (int64_t)jr_channel_stats_partials(N, HW, C) * C * 2;
  // (A one-launch form -- the last block per image reducing the partials behind
  // an integer ticket -- measured 0.9 ms/step SLOWER at raft_large batch 4: the
  // device-scope release fence before each block's ticket writes back the
  // whole XCD L2 while the other lanes' encoder convs have it full of dirty lines.)
  if (!part.defined()) part = at::empty({need}, st.options());
  check_f32(part, "partial");
  TORCH_CHECK(part.numel() >= need, "stats: partial workspace too small");
  if (keep) { keep->push_back(x); keep->push_back(st); keep->push_back(part); }
  const void* xp = x.data_ptr();
  float* sp = st.data_ptr<float>();
  float* pp = part.data_ptr<float>();
  return [=](hipStream_t s, int) { return jr_channel_stats(xp, N, HW, C, sp, pp, s); };
}

// t = [x, sx, gx, bx, r, sr, gr, br, y], i = [mode_x, mode_r, N, HW, C, relu]
static Launch make_norm_act(const TList& t, const IList& i, double eps, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), sx = opt(t, 1), gx = opt(t, 2), bx = opt(t, 3);
  at::Tensor r = opt(t, 4), sr = opt(t, 5), gr = opt(t, 6), br = opt(t, 7), y = opt(t, 8);
  check_bf16(x, "x"); check_bf16(y, "y");
  const int mx = (int)i[0], mr = (int)i[1], N = (int)i[2], HW = (int)i[3], C = (int)i[4], relu = (int)i[5];
  TORCH_CHECK(C % 8 == 0 && cs(x) == C && cs(y) == C && x.numel() >= (int64_t)N * HW * C && y.numel() >= (int64_t)N * HW * C,
              "norm_act: shape");
  if (mx) check_f32(sx, "sx");
  if (r.defined()) { check_bf16(r, "res"); TORCH_CHECK(cs(r) == C, "norm_act: residual channels"); if (mr) check_f32(sr, "sr"); }
  for (auto* v : {&gx, &bx, &gr, &br}) if (v->defined()) check_f32(*v, "affine");
  if (keep) for (auto& v : {x, sx, gx, bx, r, sr, gr, br, y}) if (v.defined()) keep->push_back(v);
  auto fp = [](const at::Tensor& v) -> const float* { return v.defined() ? v.data_ptr<float>() : nullptr; };
  const void* xp = x.data_ptr();
  const void* rp = ptr(r);
  void* yp = y.data_ptr();
  const float *sxp = fp(sx), *gxp = fp(gx), *bxp = fp(bx), *srp = fp(sr), *grp = fp(gr), *brp = fp(br);
  const float e = (float)eps;
  return [=](hipStream_t s, int) {
    return jr_norm_act(xp, sxp, mx, gxp, bxp, rp, srp, mr, grp, brp, yp, N, HW, C, e, relu, s);
  };
}

// ---------------------------------------------------------------------- misc
// t = [img1, img2, out], i = [B, H, W]
// uint8 frames: t = [img1, img2 (uint8 [B][H0][W0][3]), out, lut (fp32 [256])],
// i = [B, H, W, s2d, H0, W0, pt, pl] (K14: normalise + replicate pad + layout, jr_prep_u8)
static Launch make_prep_u8(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1), out = opt(t, 2), lut = opt(t, 3);
  TORCH_CHECK(a.defined() && b.defined() && a.scalar_type() == at::kByte && b.scalar_type() == at::kByte &&
                  a.is_cuda() && b.is_cuda() && a.is_contiguous() && b.is_contiguous(), "prep: uint8 frames");
  check_bf16(out, "out"); check_f32(lut, "lut");
  TORCH_CHECK(i.size() == 8 && lut.numel() == 256, "prep: uint8 frames need [B, H, W, s2d, H0, W0, pt, pl] and a 256 table");
  const int B = (int)i[0], H = (int)i[1], W = (int)i[2], s2d = (int)i[3], H0 = (int)i[4], W0 = (int)i[5];
  const int pt = (int)i[6], pl = (int)i[7];
  TORCH_CHECK(H0 >= 1 && W0 >= 1 && H >= H0 && W >= W0 && pt >= 0 && pl >= 0 && pt <= H - H0 && pl <= W - W0,
              "prep: padded size / offsets");
  TORCH_CHECK(a.numel() == (int64_t)B * H0 * W0 * 3 && b.numel() == a.numel(), "prep: uint8 frame shape");
  if (s2d) {
    TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && out.numel() >= 2LL * B * H * W * 4 && cs(out) == 16, "prep: s2d output");
  } else {
    TORCH_CHECK(out.numel() >= 2LL * B * H * W * 8 && cs(out) == 8, "prep: output");
  }
  if (keep) for (auto& v : {a, b, out, lut}) keep->push_back(v);
  const void* ap = a.data_ptr();
  const void* bp = b.data_ptr();
  const float* lp = lut.data_ptr<float>();
  void* op = out.data_ptr();
  return [=](hipStream_t s, int) { return jr_prep_u8(ap, bp, lp, B, H0, W0, H, W, pt, pl, s2d, op, s); };
}

static Launch make_prep(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  if (opt(t, 0).defined() && opt(t, 0).scalar_type() == at::kByte) return make_prep_u8(t, i, keep);
  at::Tensor a = opt(t, 0), b = opt(t, 1), out = opt(t, 2);
  check_f32(a, "img1"); check_f32(b, "img2"); check_bf16(out, "out");
  const int B = (int)i[0], H = (int)i[1], W = (int)i[2];
  const bool s2d = i.size() > 3 && i[3];   // 2x2 space-to-depth layout for the s2d stem
  TORCH_CHECK(a.numel() == (int64_t)B * H * W * 3 && b.numel() == a.numel(), "prep: image shape");
  if (s2d) {
    TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && out.numel() >= 2LL * B * H * W * 4 && cs(out) == 16, "prep: s2d output");
  } else {
    TORCH_CHECK(out.numel() >= 2LL * B * H * W * 8 && cs(out) == 8, "prep: output");
  }
  if (keep) { keep->push_back(a); keep->push_back(b); keep->push_back(out); }
  const float* ap = a.data_ptr<float>();
  const float* bp = b.data_ptr<float>();
  void* op = out.data_ptr();
  if (s2d) return [=](hipStream_t s, int) { return jr_prep_images_s2d(ap, bp, B, H, W, op, s); };
  return [=](hipStream_t s, int) { return jr_prep_images(ap, bp, B, H, W, op, s); };
}

// t = [coords], i = [B, h, w]
static Launch make_init_coords(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor c = opt(t, 0);
  check_f32(c, "coords");
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2];
  TORCH_CHECK(c.numel() >= (int64_t)B * h * w * 2, "init_coords: size");
  if (keep) keep->push_back(c);
  float* cp = c.data_ptr<float>();
  return [=](hipStream_t s, int) { return jr_init_coords(cp, B, h, w, s); };
}

// t = [x]
static Launch make_memset(const TList& t, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0);
  TORCH_CHECK(x.defined() && x.is_cuda() && x.is_contiguous(), "memset: tensor");
  if (keep) keep->push_back(x);
  void* p = x.data_ptr();
  const size_t bytes = x.numel() * x.element_size();
  TORCH_CHECK(((uintptr_t)p & 15) == 0 && bytes % 4 == 0, "memset: 16-B aligned, 4-B multiple tensors only");
  return [=](hipStream_t s, int) { return jr_zero_fill(p, (long)bytes, s); };
}

// t = [src, dst]
static Launch make_copy(const TList& t, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1);
  TORCH_CHECK(a.defined() && b.defined() && a.is_contiguous() && b.is_contiguous(), "copy: tensors");
  TORCH_CHECK(a.numel() * a.element_size() == b.numel() * b.element_size(), "copy: byte size mismatch");
  if (keep) { keep->push_back(a); keep->push_back(b); }
  const void* ap = a.data_ptr();
  void* bp = b.data_ptr();
  const size_t bytes = a.numel() * a.element_size();
  return [=](hipStream_t s, int) { return (int)hipMemcpyAsync(bp, ap, bytes, hipMemcpyDeviceToDevice, s); };
}

// t = [src, dst], i = [s_coff, d_coff, M, C]
static Launch make_copy_channels(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1);
  check_bf16(a, "src"); check_bf16(b, "dst");
  const int so = (int)i[0], dof = (int)i[1], M = (int)i[2], C = (int)i[3];
  TORCH_CHECK(so + C <= cs(a) && dof + C <= cs(b) && a.numel() >= (int64_t)M * cs(a) && b.numel() >= (int64_t)M * cs(b),
              "copy_channels: shape");
  if (keep) { keep->push_back(a); keep->push_back(b); }
  const void* ap = a.data_ptr();
  void* bp = b.data_ptr();
  const int acs = cs(a), bcs = cs(b);
  return [=](hipStream_t s, int) { return jr_copy_channels(ap, acs, so, bp, bcs, dof, M, C, s); };
}

// t = [a (bf16 [T][M][Ca]), b (bf16 [T][M][Cb]), out (bf16 [M][Ca + Cb])], i = [T, M]
static Launch make_sum_iters(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1), o = opt(t, 2);
  check_bf16(a, "a"); check_bf16(b, "b"); check_bf16(o, "out");
  const int T = (int)i[0];
  const int64_t M = i[1];
  const int Ca = cs(a), Cb = cs(b);
  TORCH_CHECK(T >= 1 && a.numel() == T * M * Ca && b.numel() == T * M * Cb && o.numel() == M * (Ca + Cb) &&
                  Ca % 8 == 0 && Cb % 8 == 0,
              "sum_iters: shapes");
  if (keep) for (auto& v : {a, b, o}) keep->push_back(v);
  const void *ap = a.data_ptr(), *bp = b.data_ptr();
  void* op = o.data_ptr();
  return [=](hipStream_t s, int) { return jr_sum_iters(ap, bp, T, (long)M, Ca, Cb, op, s); };
}

// t = [coords, gout, dl0, dl1, dl2, dl3], i = [num_levels, B, h, w, radius]
static Launch make_lookup_bwd(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor coords = opt(t, 0), g = opt(t, 1);
  check_f32(coords, "coords");
  TORCH_CHECK(g.defined() && g.is_cuda() && g.is_contiguous() &&
              (g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16), "lookup_bwd: grad");
  const int L = (int)i[0], B = (int)i[1], h = (int)i[2], w = (int)i[3], r = (int)i[4];
  const int nq = i.size() > 5 ? (int)i[5] : h * w;
  const int S = 2 * r + 1;
  TORCH_CHECK(L >= 1 && L <= 4 && r >= 1 && r <= 6 && nq >= 1 && cs(g) >= L * S * S, "lookup_bwd: shape");
  TORCH_CHECK(g.numel() >= (int64_t)B * nq * cs(g) && coords.numel() >= (int64_t)B * nq * 2, "lookup_bwd: grad size");
  std::vector<void*> lv(4, nullptr);
  int hl = h, wl = w;
  for (int l = 0; l < L; ++l) {
    at::Tensor v = opt(t, 2 + l);
    check_f32(v, "dlevel");
    TORCH_CHECK(v.numel() >= (int64_t)B * nq * hl * wl, "lookup_bwd: dlevel size");
    lv[l] = v.data_ptr();
    if (keep) keep->push_back(v);
    hl >>= 1; wl >>= 1;
  }
  if (keep) { keep->push_back(coords); keep->push_back(g); }
  const float* cp = coords.data_ptr<float>();
  const void* gp = g.data_ptr();
  const int gcs = cs(g);
  const int gbf = g.scalar_type() == at::kBFloat16;
  return [=](hipStream_t s, int) { return jr_corr_lookup_bwd(lv.data(), L, B, h, w, nq, r, cp, gp, gcs, gbf, s); };
}

// t = [x, col], i = [N, H, W, x_coff, cin8, KH, KW, SH, SW, PH, PW]
static Launch make_im2col(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), col = opt(t, 1);
  check_bf16(x, "x"); check_bf16(col, "col");
  const int N = (int)i[0], H = (int)i[1], W = (int)i[2], xoff = (int)i[3], cin8 = (int)i[4];
  const int KH = (int)i[5], KW = (int)i[6], SH = (int)i[7], SW = (int)i[8], PH = (int)i[9], PW = (int)i[10];
  const int OH = (H + 2 * PH - KH) / SH + 1, OW = (W + 2 * PW - KW) / SW + 1;
  const int kpad = cs(col);
  TORCH_CHECK(cin8 % 8 == 0 && xoff % 8 == 0 && cs(x) % 8 == 0 && xoff + cin8 <= cs(x), "im2col: input slice");
  TORCH_CHECK(kpad % 8 == 0 && kpad >= KH * KW * cin8, "im2col: kpad");
  TORCH_CHECK(x.numel() >= (int64_t)N * H * W * cs(x) && col.numel() >= (int64_t)N * OH * OW * kpad, "im2col: sizes");
  if (keep) { keep->push_back(x); keep->push_back(col); }
  const void* xp = x.data_ptr();
  void* cp = col.data_ptr();
  const int xcs = cs(x);
  return [=](hipStream_t s, int) {
    return jr_im2col(xp, N, H, W, xcs, xoff, cin8, KH, KW, SH, SW, PH, PW, OH, OW, kpad, cp, s);
  };
}

// ------------------------------------------------------------ fp32 parity mode
// (engine precision="fp32", runtime/engine_f32.py; kernels conv_f32.hip, f32.hip)
static void check_f32_min(const at::Tensor& t, const char* name, int64_t n) {
  check_f32(t, name);
  TORCH_CHECK(t.numel() >= n, name, ": tensor too small (", t.numel(), " < ", n, ")");
}

// t = [x, w ([cout][K] fp32), bias, y, y2, res, h32, zbuf, bmap]
// i = [N, H, W, x_coff, cin4, KH, KW, SH, SW, PH, PW, cout, act, split, y_coff, y2_coff, res_coff, res_post,
//      hidden, bmap_coff, epi, ksplit (0: automatic, n > 0: forced n-way split-K)]
static Launch make_conv_f32(const TList& t, const IList& i, double alpha, std::vector<at::Tensor>* keep) {
  TORCH_CHECK(i.size() == 22, "conv_f32: expected 22 ints");
  at::Tensor x = opt(t, 0), w = opt(t, 1), bias = opt(t, 2), y = opt(t, 3), y2 = opt(t, 4), res = opt(t, 5);
  at::Tensor h32 = opt(t, 6), zbuf = opt(t, 7), bmap = opt(t, 8);
  ConvF32Params p{};
  p.N = (int)i[0]; p.H = (int)i[1]; p.W = (int)i[2]; p.x_coff = (int)i[3]; p.cin4 = (int)i[4];
  p.KH = (int)i[5]; p.KW = (int)i[6]; p.SH = (int)i[7]; p.SW = (int)i[8]; p.PH = (int)i[9]; p.PW = (int)i[10];
  p.cout = (int)i[11]; p.act = (int)i[12]; p.split = (int)i[13];
  p.y_coff = (int)i[14]; p.y2_coff = (int)i[15]; p.res_coff = (int)i[16]; p.res_post = (int)i[17];
  p.hidden = (int)i[18]; p.bmap_coff = (int)i[19];
  const int epi = (int)i[20];
  TORCH_CHECK(epi >= 0 && epi <= 2, "conv_f32: epi 0..2");
  TORCH_CHECK(p.SH >= 1 && p.SW >= 1 && p.KH >= 1 && p.KW >= 1 && p.cout >= 1, "conv_f32: geometry");
  p.OH = (p.H + 2 * p.PH - p.KH) / p.SH + 1;
  p.OW = (p.W + 2 * p.PW - p.KW) / p.SW + 1;
  p.M = p.N * p.OH * p.OW;
  p.K = p.KH * p.KW * p.cin4;
  const int64_t M = p.M;
  check_f32(x, "x");
  p.x_cs = cs(x);
  TORCH_CHECK(p.x_coff + p.cin4 <= p.x_cs && x.numel() >= (int64_t)p.N * p.H * p.W * p.x_cs, "conv_f32: x");
  check_f32(w, "w");
  TORCH_CHECK(w.numel() == (int64_t)p.cout * p.K, "conv_f32: w must be [cout][KH*KW*cin4]");
  check_f32_min(bias, "bias", p.cout);
  check_f32(y, "y");
  p.y_cs = cs(y);
  const int ych = epi == 1 ? p.hidden : p.cout;   // GRU-A writes r*h (hidden channels) to y
  TORCH_CHECK(p.y_coff + ych <= p.y_cs && y.numel() >= M * p.y_cs, "conv_f32: y");
  if (y2.defined()) {
    check_f32(y2, "y2"); p.y2_cs = cs(y2);
    TORCH_CHECK(p.y2_coff + p.cout <= p.y2_cs && y2.numel() >= M * p.y2_cs, "conv_f32: y2");
  }
  if (res.defined()) {
    check_f32(res, "res"); p.res_cs = cs(res);
    TORCH_CHECK(p.res_coff + p.cout <= p.res_cs && res.numel() >= M * p.res_cs, "conv_f32: res");
  }
  if (h32.defined()) check_f32_min(h32, "h32", M * p.hidden);
  if (zbuf.defined()) check_f32_min(zbuf, "zbuf", M * p.hidden);
  if (epi == 0 && h32.defined()) TORCH_CHECK(p.split <= p.hidden && p.split <= p.cout, "conv_f32: h32 copy");
  if (bmap.defined()) {
    check_f32(bmap, "bmap"); p.bmap_cs = cs(bmap);
    TORCH_CHECK(p.bmap_coff + p.cout <= p.bmap_cs && bmap.numel() >= M * p.bmap_cs, "conv_f32: bmap");
  }
  p.x = x.data_ptr<float>(); p.w = w.data_ptr<float>(); p.bias = bias.data_ptr<float>(); p.alpha = (float)alpha;
  p.y = y.data_ptr<float>();
  p.y2 = y2.defined() ? y2.data_ptr<float>() : nullptr;
  p.res = res.defined() ? res.data_ptr<float>() : nullptr;
  p.h32 = h32.defined() ? h32.data_ptr<float>() : nullptr;
  p.zbuf = zbuf.defined() ? zbuf.data_ptr<float>() : nullptr;
  p.bmap = bmap.defined() ? bmap.data_ptr<float>() : nullptr;
  // split-K when the grid holds fewer than 4 blocks per CU (the batch-1 loop convs:
  // 110-440 blocks on 256 CUs, one 4-wave block per CU leaves the f32 MFMA pipe ~half
  // idle): aim at ~1536 blocks, >= 8 K stages per split.  i[21] = n > 0 forces n (tests).
  {
    const long blocks = (long)((p.M + 63) / 64) * ((p.cout + 63) / 64);
    const int nks = (p.K + 31) / 32;
    int S = 1;
    if (blocks < 1024) S = (int)std::min<long>({8L, (1536 + blocks - 1) / blocks, (long)std::max(1, nks / 8)});
    if (i[21] > 0) S = std::max(1, std::min((int)i[21], std::max(1, nks / 8)));
    p.ksplit = S;
    if (S > 1) {
      at::Tensor part = at::empty({(int64_t)S * p.M * ((p.cout + 3) / 4 * 4)}, x.options());
      p.part = part.data_ptr<float>();
      if (keep) keep->push_back(part);
      else {   // eager op: keep the workspace alive until the stream has used it
        auto launch = [=](hipStream_t s, int) { return jr_conv_f32(&p, epi, s); };
        return [launch, part](hipStream_t s, int it) { return launch(s, it); };
      }
    }
  }
  if (keep) for (auto& v : {x, w, bias, y, y2, res, h32, zbuf, bmap}) if (v.defined()) keep->push_back(v);
  return [=](hipStream_t s, int) { return jr_conv_f32(&p, epi, s); };
}

// t = [x, stats, partial?], i = [N, HW, C]
static Launch make_stats_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), st = opt(t, 1), part = opt(t, 2);
  const int N = (int)i[0], HW = (int)i[1], C = (int)i[2];
  check_f32(x, "x");
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && cs(x) == C && x.numel() >= (int64_t)N * HW * C, "stats_f32: shape");
  check_f32_min(st, "stats", (int64_t)N * C * 2);
  const int64_t need = (int64_t)jr_channel_stats_partials(N, HW, C) * C * 2;
  if (!part.defined()) part = at::empty({need}, st.options());
  check_f32_min(part, "partial", need);
  if (keep) for (auto& v : {x, st, part}) keep->push_back(v);
  const float* xp = x.data_ptr<float>();
  float* sp = st.data_ptr<float>();
  float* pp = part.data_ptr<float>();
  return [=](hipStream_t s, int) { return jr_channel_stats_f32(xp, N, HW, C, sp, pp, s); };
}

// t = [x, sx, res, sr, y], i = [mode_x, mode_r, N, HW, C, relu]
static Launch make_norm_act_f32(const TList& t, const IList& i, double eps, std::vector<at::Tensor>* keep) {
  at::Tensor x = opt(t, 0), sx = opt(t, 1), r = opt(t, 2), sr = opt(t, 3), y = opt(t, 4);
  const int mx = (int)i[0], mr = (int)i[1], N = (int)i[2], HW = (int)i[3], C = (int)i[4], relu = (int)i[5];
  const int64_t n = (int64_t)N * HW * C;
  check_f32_min(x, "x", n); check_f32_min(y, "y", n);
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && cs(x) == C && cs(y) == C, "norm_act_f32: shape");
  if (mx) check_f32_min(sx, "sx", (int64_t)N * C * 2);
  if (r.defined()) {
    check_f32_min(r, "res", n);
    TORCH_CHECK(cs(r) == C, "norm_act_f32: residual channels");
    if (mr) check_f32_min(sr, "sr", (int64_t)N * C * 2);
  }
  if (keep) for (auto& v : {x, sx, r, sr, y}) if (v.defined()) keep->push_back(v);
  auto fp = [](const at::Tensor& v) -> float* { return v.defined() ? v.data_ptr<float>() : nullptr; };
  const float *xp = fp(x), *sxp = fp(sx), *rp = fp(r), *srp = fp(sr);
  float* yp = fp(y);
  const float e = (float)eps;
  return [=](hipStream_t s, int) { return jr_norm_act_f32(xp, sxp, mx, rp, srp, mr, yp, N, HW, C, e, relu, s); };
}

// t = [img1, img2, out ([2B][H][W][4])], i = [B, H, W]
static Launch make_prep_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1), out = opt(t, 2);
  const int B = (int)i[0], H = (int)i[1], W = (int)i[2];
  check_f32(a, "img1"); check_f32(b, "img2"); check_f32(out, "out");
  TORCH_CHECK(a.numel() == (int64_t)B * H * W * 3 && b.numel() == a.numel(), "prep_f32: image shape");
  TORCH_CHECK(out.numel() >= 2LL * B * H * W * 4 && cs(out) == 4, "prep_f32: output");
  if (keep) for (auto& v : {a, b, out}) keep->push_back(v);
  const float *ap = a.data_ptr<float>(), *bp = b.data_ptr<float>();
  float* op = out.data_ptr<float>();
  return [=](hipStream_t s, int) { return jr_prep_images_f32(ap, bp, B, H, W, op, s); };
}

// t = [src, dst], i = [s_coff, d_coff, M, C]
static Launch make_copy_channels_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1);
  check_f32(a, "src"); check_f32(b, "dst");
  const int so = (int)i[0], dof = (int)i[1], M = (int)i[2], C = (int)i[3];
  TORCH_CHECK(so + C <= cs(a) && dof + C <= cs(b) && a.numel() >= (int64_t)M * cs(a) && b.numel() >= (int64_t)M * cs(b),
              "copy_channels_f32: shape");
  if (keep) { keep->push_back(a); keep->push_back(b); }
  const float* ap = a.data_ptr<float>();
  float* bp = b.data_ptr<float>();
  const int acs = cs(a), bcs = cs(b);
  return [=](hipStream_t s, int) { return jr_copy_channels_f32(ap, acs, so, bp, bcs, dof, M, C, s); };
}

// t = [mask (fp32 [M][>=576]), flow, out, out_slot?], i = [B, h, w, out_iter_stride(, slot offset)]
static Launch make_upsample_convex_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor mask = opt(t, 0), flow = opt(t, 1), out = opt(t, 2), slot = opt(t, 3);
  const int B = (int)i[0], h = (int)i[1], w = (int)i[2];
  const int64_t stride = i[3], slot_off = i.size() > 4 ? i[4] : 0;
  const int64_t M = (int64_t)B * h * w;
  check_f32_min(mask, "mask", M * 576); check_f32_min(flow, "flow", M * 2);
  TORCH_CHECK(cs(mask) >= 576 && mask.numel() >= M * cs(mask), "upsample_convex_f32: mask needs 576 channels");
  TORCH_CHECK(!slot.defined() || (slot.is_cuda() && slot.scalar_type() == at::kLong && slot.numel() == 1),
              "upsample_convex_f32: out_slot must be one device int64");
  const int64_t cap = check_flow_out(out, B, h, w);
  if (keep) for (auto& v : {mask, flow, out, slot}) if (v.defined()) keep->push_back(v);
  const float *mp = mask.data_ptr<float>(), *fp = flow.data_ptr<float>();
  float* op = out.data_ptr<float>();
  const void* sp = slot.defined() ? slot.data_ptr() : nullptr;
  const int mcs = cs(mask);
  return [=](hipStream_t s, int it) {
    const int64_t off = stride * it;
    if (off + M * 128 > cap) return (int)hipErrorInvalidValue;
    return jr_upsample_convex_f32(mp, mcs, fp, B, h, w, op + off, sp, (long)(slot_off + off), s);
  };
}

// t = [src ([M][hl][wl]), dst ([M][hl/2][wl/2])], i = [M, hl, wl]
static Launch make_corr_pool_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor a = opt(t, 0), b = opt(t, 1);
  const int64_t M = i[0];
  const int hl = (int)i[1], wl = (int)i[2];
  TORCH_CHECK(hl >= 2 && wl >= 2, "corr_pool_f32: level too small");
  check_f32_min(a, "src", M * hl * wl); check_f32_min(b, "dst", M * (hl / 2) * (wl / 2));
  if (keep) { keep->push_back(a); keep->push_back(b); }
  const float* ap = a.data_ptr<float>();
  float* bp = b.data_ptr<float>();
  return [=](hipStream_t s, int) { return jr_corr_pool_f32(ap, (long)M, hl, wl, bp, s); };
}

// t = [coords, out, l0, l1, l2, l3], i = [num_levels, B, h, w, radius(, nq: queries per image, default h*w)]
static Launch make_lookup_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor coords = opt(t, 0), out = opt(t, 1);
  const int L = (int)i[0], B = (int)i[1], h = (int)i[2], w = (int)i[3], r = (int)i[4];
  const int nq = i.size() > 5 ? (int)i[5] : h * w;
  const int S = 2 * r + 1;
  TORCH_CHECK(nq >= 1, "lookup_f32: nq");
  const int64_t M = (int64_t)B * nq;
  TORCH_CHECK(L >= 1 && L <= 4 && r >= 1 && r <= 4, "lookup_f32: levels 1..4, radius 1..4");
  check_f32_min(coords, "coords", M * 2);
  check_f32(out, "out");
  TORCH_CHECK(cs(out) >= L * S * S && out.numel() >= M * cs(out), "lookup_f32: out");
  std::vector<const float*> lv(4, nullptr);
  int hl = h, wl = w;
  for (int l = 0; l < L; ++l) {
    at::Tensor v = opt(t, 2 + l);
    TORCH_CHECK(hl >= 2 && wl >= 2, "lookup_f32: pyramid level too small");
    check_f32_min(v, "level", M * hl * wl);
    lv[l] = v.data_ptr<float>();
    if (keep) keep->push_back(v);
    hl >>= 1; wl >>= 1;
  }
  if (keep) { keep->push_back(coords); keep->push_back(out); }
  const float* cp = coords.data_ptr<float>();
  float* op = out.data_ptr<float>();
  const int ocs = cs(out);
  return [=](hipStream_t s, int) { return jr_corr_lookup_f32(lv.data(), L, B, h, w, nq, r, cp, op, ocs, s); };
}

// t = [delta ([M][dcs]), coords, flow32, hx, qx?, flow4?], i = [N, h, w, hx_off, qx_off]
static Launch make_flow_update_f32(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor d = opt(t, 0), coords = opt(t, 1), f32 = opt(t, 2), hx = opt(t, 3), qx = opt(t, 4), f4 = opt(t, 5);
  const int N = (int)i[0], h = (int)i[1], w = (int)i[2], hx_off = (int)i[3], qx_off = (int)i[4];
  const int64_t M = (int64_t)N * h * w;
  check_f32(d, "delta");
  TORCH_CHECK(cs(d) >= 2 && d.numel() >= M * cs(d), "flow_update_f32: delta");
  check_f32_min(coords, "coords", 2 * M); check_f32_min(f32, "flow32", 2 * M);
  check_f32(hx, "hx");
  TORCH_CHECK(hx_off + 2 <= cs(hx) && hx.numel() >= M * cs(hx), "flow_update_f32: hx");
  if (qx.defined()) { check_f32(qx, "qx"); TORCH_CHECK(qx_off + 2 <= cs(qx) && qx.numel() >= M * cs(qx), "flow_update_f32: qx"); }
  if (f4.defined()) { check_f32_min(f4, "flow4", 4 * M); TORCH_CHECK(cs(f4) == 4, "flow_update_f32: flow4 [M][4]"); }
  if (keep) for (auto& v : {d, coords, f32, hx, qx, f4}) if (v.defined()) keep->push_back(v);
  auto fp = [](const at::Tensor& v) -> float* { return v.defined() ? v.data_ptr<float>() : nullptr; };
  const float* dp = fp(d);
  float *cp = fp(coords), *fl = fp(f32), *hp = fp(hx), *qp = fp(qx), *f4p = fp(f4);
  const int dcs = cs(d), hcs = cs(hx), qcs = qx.defined() ? cs(qx) : 0;
  return [=](hipStream_t s, int) {
    return jr_flow_update_f32(dp, dcs, N, h, w, cp, fl, hp, hcs, hx_off, qp, qcs, qx_off, f4p, s);
  };
}

static void run_now(const Launch& l) { JR_CHECK_OK(l(cur_stream(), 0)); }

// ------------------------------------------------------------- sequence loss
// t = [pred (fp32 [N][P][2]), gt (fp32 [P][2]), valid? (fp32 [P]), part (fp32 [blocks][37])], i = [P, N]
void seq_loss_op(const TList& t, IList i, double max_flow) {
  at::Tensor pred = opt(t, 0), gt = opt(t, 1), valid = opt(t, 2), part = opt(t, 3);
  TORCH_CHECK(i.size() == 2, "seq_loss: expected [P, N]");
  check_f32(pred, "pred"); check_f32(gt, "gt"); check_f32(part, "part");
  const int64_t P = i[0];
  const int N = (int)i[1];
  TORCH_CHECK(N >= 1 && N <= 32, "seq_loss: 1..32 predictions");
  TORCH_CHECK(pred.numel() == (int64_t)N * P * 2 && gt.numel() == P * 2, "seq_loss: shapes");
  TORCH_CHECK(part.numel() >= (int64_t)jr_seq_loss_blocks(P) * 37, "seq_loss: partials");
  if (valid.defined()) { check_f32(valid, "valid"); TORCH_CHECK(valid.numel() == P, "seq_loss: valid"); }
  JR_CHECK_OK(jr_seq_loss(pred.data_ptr<float>(), gt.data_ptr<float>(),
                          valid.defined() ? valid.data_ptr<float>() : nullptr, P, N, (float)max_flow,
                          part.data_ptr<float>(), cur_stream()));
}
int64_t seq_loss_blocks_op(int64_t P) { return jr_seq_loss_blocks(P); }
// t = [pred, gt, valid?, scale (fp32 [N]), grad (fp32 [N][P][2])], i = [P, N]
void seq_loss_bwd_op(const TList& t, IList i, double max_flow) {
  at::Tensor pred = opt(t, 0), gt = opt(t, 1), valid = opt(t, 2), scale = opt(t, 3), grad = opt(t, 4);
  TORCH_CHECK(i.size() == 2, "seq_loss_bwd: expected [P, N]");
  check_f32(pred, "pred"); check_f32(gt, "gt"); check_f32(scale, "scale"); check_f32(grad, "grad");
  const int64_t P = i[0];
  const int N = (int)i[1];
  TORCH_CHECK(pred.numel() == (int64_t)N * P * 2 && gt.numel() == P * 2 && grad.numel() == pred.numel() &&
              scale.numel() >= N, "seq_loss_bwd: shapes");
  if (valid.defined()) { check_f32(valid, "valid"); TORCH_CHECK(valid.numel() == P, "seq_loss_bwd: valid"); }
  JR_CHECK_OK(jr_seq_loss_bwd(pred.data_ptr<float>(), gt.data_ptr<float>(),
                              valid.defined() ? valid.data_ptr<float>() : nullptr, P, N, (float)max_flow,
                              scale.data_ptr<float>(), grad.data_ptr<float>(), cur_stream()));
}

// ---------------------------------------------------------------- eager ops
void conv_op(const TList& t, IList i, double alpha) { run_now(make_conv(t, i, alpha, nullptr)); }
void conv_f32_op(const TList& t, IList i, double alpha) { run_now(make_conv_f32(t, i, alpha, nullptr)); }
void stats_f32_op(const TList& t, IList i) { run_now(make_stats_f32(t, i, nullptr)); }
void norm_act_f32_op(const TList& t, IList i, double eps) { run_now(make_norm_act_f32(t, i, eps, nullptr)); }
void prep_f32_op(const TList& t, IList i) { run_now(make_prep_f32(t, i, nullptr)); }
void copy_channels_f32_op(const TList& t, IList i) { run_now(make_copy_channels_f32(t, i, nullptr)); }
void upsample_convex_f32_op(const TList& t, IList i) { run_now(make_upsample_convex_f32(t, i, nullptr)); }
void corr_pool_f32_op(const TList& t, IList i) { run_now(make_corr_pool_f32(t, i, nullptr)); }
void lookup_f32_op(const TList& t, IList i) { run_now(make_lookup_f32(t, i, nullptr)); }
void flow_update_f32_op(const TList& t, IList i) { run_now(make_flow_update_f32(t, i, nullptr)); }

void corr_op(const TList& t, IList i, double scale) { run_now(make_corr(t, i, scale, nullptr)); }
// a stand-alone lookup applies its fused flow update when one is given (in a
// plan the update is skipped in loop iteration 0, which has no previous taps)
void lookup_op(const TList& t, IList i) { JR_CHECK_OK(make_lookup(t, i, nullptr)(cur_stream(), 1)); }
void upsample_convex_op(const TList& t, IList i) { run_now(make_upsample_convex(t, i, nullptr)); }
void convex_head_op(const TList& t, IList i, double alpha) { run_now(make_convex_head(t, i, alpha, nullptr)); }
void upsample_bilinear_op(const TList& t, IList i) { run_now(make_upsample_bilinear(t, i, nullptr)); }
void stats_op(const TList& t, IList i) {
  std::vector<at::Tensor> keep;  // keeps an internally allocated workspace alive until the launch is queued
  run_now(make_stats(t, i, &keep));
}
void norm_act_op(const TList& t, IList i, double eps) { run_now(make_norm_act(t, i, eps, nullptr)); }
void prep_op(const TList& t, IList i) { run_now(make_prep(t, i, nullptr)); }
void init_coords_op(const TList& t, IList i) { run_now(make_init_coords(t, i, nullptr)); }
void copy_channels_op(const TList& t, IList i) { run_now(make_copy_channels(t, i, nullptr)); }
void sum_iters_op(const TList& t, IList i) { run_now(make_sum_iters(t, i, nullptr)); }
void lookup_bwd_op(const TList& t, IList i) { run_now(make_lookup_bwd(t, i, nullptr)); }
void im2col_op(const TList& t, IList i) { run_now(make_im2col(t, i, nullptr)); }
void flow_taps_op(const TList& t, IList i) { run_now(make_flow_taps(t, i, nullptr)); }
void taps_gemm_op(const TList& t, IList i) { run_now(make_taps_gemm(t, i, nullptr)); }
void gru_fused_op(const TList& t, IList i) { run_now(make_gru_fused(t, i, nullptr)); }
void gru_halo_op(const TList& t, IList i) { run_now(make_gru_halo(t, i, nullptr)); }
bool conv_halo_ok_op(int64_t cfg, int64_t cin8, int64_t cout) { return conv_halo_ok_cfg(cfg, cin8, cout); }
// t = [part (fp32 [N][nb][C][2]), stats (fp32 [N][C][2])], i = [N, nb, C]
static Launch make_stats_final(const TList& t, const IList& i, std::vector<at::Tensor>* keep) {
  at::Tensor part = opt(t, 0), st = opt(t, 1);
  check_f32(part, "partials"); check_f32(st, "stats");
  TORCH_CHECK(i.size() == 3, "stats_final: expected [N, nb, C]");
  const int N = (int)i[0], nb = (int)i[1], C = (int)i[2];
  TORCH_CHECK(part.numel() >= (int64_t)N * nb * C * 2 && st.numel() >= (int64_t)N * C * 2, "stats_final: sizes");
  if (keep) { keep->push_back(part); keep->push_back(st); }
  const float* pp = part.data_ptr<float>();
  float* sp = st.data_ptr<float>();
  return [=](hipStream_t s, int) { return jr_channel_stats_final(pp, N, nb, C, sp, s); };
}
void stats_final_op(const TList& t, IList i) { run_now(make_stats_final(t, i, nullptr)); }
std::vector<int64_t> conv_halo_cfg_op(int64_t cfg) {
  int c[6];
  if (!jr_conv_halo_cfg((int)(cfg - kHaloCfg0), c)) return {};
  return {c[0], c[1], c[2], c[3], c[4], c[5]};
}
bool conv_grouped_ok_op(int64_t cfg) { return jr_conv_grouped_ok((int)cfg) != 0; }

// Batched GEMM (bgemm.hip).  t = [A (bf16 [batch][M][K] or [batch][K][M]), B (bf16 [batch][K][N]),
// C (fp32 / bf16 [batch][M][N])], i = [M, N, K, a_kmajor]
void bgemm_op(const TList& t, IList i, double alpha) {
  at::Tensor a = opt(t, 0), b = opt(t, 1), c = opt(t, 2);
  check_bf16(a, "A"); check_bf16(b, "B");
  TORCH_CHECK(i.size() == 4, "bgemm: expected [M, N, K, a_kmajor]");
  const int64_t M = i[0], N = i[1], K = i[2];
  const int ak = (int)i[3];
  TORCH_CHECK(c.defined() && c.is_cuda() && c.is_contiguous() &&
                  (c.scalar_type() == at::kFloat || c.scalar_type() == at::kBFloat16), "bgemm: C fp32 / bf16 contiguous");
  TORCH_CHECK(M % 128 == 0 && N % 128 == 0 && K % 64 == 0 && M > 0 && N > 0 && K > 0, "bgemm: M, N % 128, K % 64");
  TORCH_CHECK(a.dim() == 3 && b.dim() == 3 && c.dim() == 3 && a.size(0) == b.size(0) && a.size(0) == c.size(0),
              "bgemm: batched 3-d operands");
  TORCH_CHECK((ak ? (a.size(1) == K && a.size(2) == M) : (a.size(1) == M && a.size(2) == K)) && b.size(1) == K &&
                  b.size(2) == N && c.size(1) == M && c.size(2) == N, "bgemm: shapes");
  TORCH_CHECK(M * K * 2 < (1LL << 31) && K * N * 2 < (1LL << 31), "bgemm: one batch's operand must stay below 2 GiB");
  const bool f32 = c.scalar_type() == at::kFloat;
  JR_CHECK_OK(jr_bgemm(a.data_ptr(), (long)(M * K), (int)(ak ? M : K), ak, b.data_ptr(), (long)(K * N), (int)N,
                       (int)a.size(0), (int)M, (int)N, (int)K, (float)alpha, f32 ? c.data_ptr<float>() : nullptr,
                       f32 ? nullptr : c.data_ptr(), (long)(M * N), (int)N, cur_stream()));
}
void conv1x1_op(const TList& t, IList i) { run_now(make_conv1x1(t, i, nullptr)); }
void conv_direct_op(const TList& t, IList i) { run_now(make_conv_direct(t, i, nullptr)); }
void conv_train_op(const TList& t, IList i, double alpha, const TList& tx, IList ix) {
  run_now(make_conv(t, i, alpha, nullptr, &tx, &ix));
}
void upsample_convex_bwd_op(const TList& t, IList i, double alpha) { run_now(make_upsample_convex_bwd(t, i, alpha, nullptr)); }
// t = [dc (bf16 [M][h][w]), g0, g1?, g2?, g3?], i = [L, M, h, w]
void pyr_bwd_dc_op(const TList& t, IList i, double scale) {
  at::Tensor dc = opt(t, 0);
  TORCH_CHECK(i.size() == 4, "pyr_bwd_dc: expected [L, M, h, w]");
  const int L = (int)i[0], h = (int)i[2], w = (int)i[3];
  const int64_t M = i[1];
  check_bf16(dc, "dc");
  TORCH_CHECK(L >= 1 && L <= 4 && dc.numel() >= M * h * w, "pyr_bwd_dc: shapes");
  const float* g[4] = {nullptr, nullptr, nullptr, nullptr};
  int hl = h, wl = w;
  for (int l = 0; l < L; ++l) {
    at::Tensor v = opt(t, 1 + l);
    check_f32(v, "level gradient");
    TORCH_CHECK(v.numel() >= M * hl * wl, "pyr_bwd_dc: level ", l, " size");
    g[l] = v.data_ptr<float>();
    hl >>= 1; wl >>= 1;
  }
  JR_CHECK_OK(jr_pyr_bwd_dc(g[0], g[1], g[2], g[3], L, M, h, w, (float)scale, dc.data_ptr(), cur_stream()));
}
void wgrad_op(const TList& t, IList i) {
  std::vector<at::Tensor> keep;
  run_now(make_wgrad(t, i, &keep));
}
void pack_op(const TList& t, IList i) {
  std::vector<at::Tensor> keep;
  run_now(make_pack(t, i, &keep));
}
void norm_bwd_op(const TList& t, IList i, double eps) {
  std::vector<at::Tensor> keep;
  run_now(make_norm_bwd(t, i, eps, &keep));
}
void flow_gather_bwd_op(const TList& t, IList i) { run_now(make_flow_gather_bwd(t, i, nullptr)); }
void upsample_bilinear_bwd_op(const TList& t, IList i) { run_now(make_upsample_bilinear_bwd(t, i, nullptr)); }

// --------------------------------------------------------------------- Plan
// A Plan is the lowered RAFT forward: three segments (prologue, loop body run
// n_iters times with the iteration index, epilogue) of launch closures.  Ops
// are placed on "lanes": lane 0 is the caller's stream, lanes 1..kMaxLanes-1
// are private non-blocking streams, and record/wait ops on numbered events
// express the cross-lane dependencies of the model's DAG (independent
// branches such as the context encoder vs. the feature encoder + correlation
// pyramid, or the mask head + upsampling of iteration i vs. iteration i+1).
// Every side lane is forked from lane 0 at the start of an enqueue and joined
// back at its end, so run() is ordered like a single-stream launch and
// capture() records one hipGraph whose parallel branches the runtime may
// execute concurrently.  A wait on an event not yet recorded during the
// current enqueue is skipped (e.g. the first iteration's wait on the previous
// iteration's mask head), which also keeps graph capture self-contained.
// Lane 0 runs on a private stream of the device's greatest priority (forked
// from / joined to the caller's stream): the model's critical path (lookup ->
// motion encoder -> GRU -> flow head) wins the dispatcher over the side lanes'
// work, which only fills the CUs the critical path leaves idle.
struct RangeGuard {
  explicit RangeGuard(const char* name) { roctxRangePushA(name); }
  ~RangeGuard() { roctxRangePop(); }
};

class Plan : public torch::CustomClassHolder {
 public:
  static constexpr int kMaxLanes = 8;
  static constexpr int kMaxEvents = 64;
  Plan() = default;
  ~Plan() override {
    reset_graph();
    for (auto e : events_) if (e) (void)hipEventDestroy(e);
    for (auto e : join_) if (e) (void)hipEventDestroy(e);
    if (fork_) (void)hipEventDestroy(fork_);
    for (auto st : lanes_) if (st) (void)hipStreamDestroy(st);
    if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
  }

  // Segment 3 is the second half of the loop body (enqueued right after segment 1 in
  // every iteration): a context-parallel engine runs the two halves separately, with
  // the all-gather of the correlation features in between (run_segment).
  void set_segment(int64_t s) {
    TORCH_CHECK(s >= 0 && s <= 3, "segment must be 0 (prologue), 1 (loop), 2 (epilogue) or 3 (loop, second half)");
    seg_ = (int)s;
    defer_ = 0;
    reset_graph();
  }
  // Deferred ops (set_defer 1, loop body / epilogue): the work of the PREVIOUS
  // iteration -- skipped in loop iteration 0 and called with iteration index
  // it - 1; in the epilogue (called with n_iters) they finish the last
  // iteration.  Used when iteration i's flow update is fused into iteration
  // i+1's lookup, so iteration i's mask head / upsampling run one iteration later.
  void set_defer(int64_t d) {
    TORCH_CHECK(d == 0 || d == 1, "defer must be 0 or 1");
    TORCH_CHECK(d == 0 || seg_ != 0, "deferred ops belong to the loop body or the epilogue");
    defer_ = (int)d;
  }
  void set_lane(int64_t l) {
    TORCH_CHECK(l >= 0 && l < kMaxLanes, "lane must be in [0, ", kMaxLanes, ")");
    lane_ = (int)l;
    used_lanes_ = std::max(used_lanes_, lane_ + 1);
  }
  void add_record(int64_t ev) { push_sync(OP_RECORD, ev, "record"); }
  void add_wait(int64_t ev) { push_sync(OP_WAIT, ev, "wait"); }
  void add_conv(TList t, IList i, double alpha) { push(make_conv(t, i, alpha, &keep_), "conv"); }
  void add_conv_alt(TList t, IList i, double alpha, at::Tensor x_alt) {
    push(make_conv_alt(t, i, alpha, x_alt, &keep_), "conv");
  }
  void add_conv_group(TList t1, IList i1, double a1, TList t2, IList i2, double a2) {
    push(make_conv_group(t1, i1, a1, t2, i2, a2, &keep_), "conv_group");
  }
  void add_corr(TList t, IList i, double scale) { push(make_corr(t, i, scale, &keep_), "corr"); }
  void add_lookup(TList t, IList i) { push(make_lookup(t, i, &keep_), "lookup"); }
  void add_upsample_convex(TList t, IList i) { push(make_upsample_convex(t, i, &keep_), "upsample_convex"); }
  void add_convex_head(TList t, IList i, double alpha) { push(make_convex_head(t, i, alpha, &keep_), "convex_head"); }
  void add_upsample_bilinear(TList t, IList i) { push(make_upsample_bilinear(t, i, &keep_), "upsample_bilinear"); }
  void add_stats(TList t, IList i) { push(make_stats(t, i, &keep_), "stats"); }
  void add_norm_act(TList t, IList i, double eps) { push(make_norm_act(t, i, eps, &keep_), "norm_act"); }
  void add_prep(TList t, IList i) { push(make_prep(t, i, &keep_), "prep"); }
  void add_init_coords(TList t, IList i) { push(make_init_coords(t, i, &keep_), "init_coords"); }
  void add_memset(TList t) { push(make_memset(t, &keep_), "memset"); }
  void add_copy(TList t) { push(make_copy(t, &keep_), "copy"); }
  void add_copy_channels(TList t, IList i) { push(make_copy_channels(t, i, &keep_), "copy_channels"); }
  void add_flow_taps(TList t, IList i) { push(make_flow_taps(t, i, &keep_), "flow_taps"); }
  void add_taps_gemm(TList t, IList i) { push(make_taps_gemm(t, i, &keep_), "taps_gemm"); }
  void add_gru_fused(TList t, IList i) { push(make_gru_fused(t, i, &keep_), "gru_fused"); }
  void add_gru_halo(TList t, IList i) { push(make_gru_halo(t, i, &keep_), "gru_halo"); }
  void add_stats_final(TList t, IList i) { push(make_stats_final(t, i, &keep_), "stats_final"); }
  void add_conv1x1(TList t, IList i) { push(make_conv1x1(t, i, &keep_), "conv1x1"); }
  void add_conv_direct(TList t, IList i) { push(make_conv_direct(t, i, &keep_), "conv_direct"); }
  void add_flowin_dual(TList t, IList i, double alpha) { push(make_flowin_dual(t, i, alpha, &keep_), "flowin_dual"); }
  void add_conv_train(TList t, IList i, double alpha, TList tx, IList ix) {
    push(make_conv(t, i, alpha, &keep_, &tx, &ix), "conv_train");
  }
  void add_upsample_convex_bwd(TList t, IList i, double alpha) {
    push(make_upsample_convex_bwd(t, i, alpha, &keep_), "upsample_convex_bwd");
  }
  void add_bn_table(TList t, IList i) { push(make_bn_table(t, i, &keep_), "bn_table"); }
  void add_wgrad(TList t, IList i) { push(make_wgrad(t, i, &keep_), "wgrad"); }
  void add_pack(TList t, IList i) { push(make_pack(t, i, &keep_), "pack"); }
  void add_norm_bwd(TList t, IList i, double eps) { push(make_norm_bwd(t, i, eps, &keep_), "norm_bwd"); }
  void add_flow_gather_bwd(TList t, IList i) { push(make_flow_gather_bwd(t, i, &keep_), "flow_gather_bwd"); }
  void add_upsample_bilinear_bwd(TList t, IList i) { push(make_upsample_bilinear_bwd(t, i, &keep_), "upsample_bilinear_bwd"); }
  void add_lookup_bwd(TList t, IList i) { push(make_lookup_bwd(t, i, &keep_), "lookup_bwd"); }
  void add_im2col(TList t, IList i) { push(make_im2col(t, i, &keep_), "im2col"); }
  void add_conv_f32(TList t, IList i, double alpha) { push(make_conv_f32(t, i, alpha, &keep_), "conv_f32"); }
  void add_stats_f32(TList t, IList i) { push(make_stats_f32(t, i, &keep_), "stats_f32"); }
  void add_norm_act_f32(TList t, IList i, double eps) { push(make_norm_act_f32(t, i, eps, &keep_), "norm_act_f32"); }
  void add_prep_f32(TList t, IList i) { push(make_prep_f32(t, i, &keep_), "prep_f32"); }
  void add_copy_channels_f32(TList t, IList i) { push(make_copy_channels_f32(t, i, &keep_), "copy_channels_f32"); }
  void add_upsample_convex_f32(TList t, IList i) { push(make_upsample_convex_f32(t, i, &keep_), "upsample_convex_f32"); }
  void add_corr_pool_f32(TList t, IList i) { push(make_corr_pool_f32(t, i, &keep_), "corr_pool_f32"); }
  void add_lookup_f32(TList t, IList i) { push(make_lookup_f32(t, i, &keep_), "lookup_f32"); }
  void add_flow_update_f32(TList t, IList i) { push(make_flow_update_f32(t, i, &keep_), "flow_update_f32"); }

  int64_t num_ops(int64_t seg) const { return (int64_t)segs_[seg].size(); }
  std::vector<std::string> op_names(int64_t seg) const {
    std::vector<std::string> out;
    for (const auto& o : segs_[seg]) out.push_back(o.name + (o.lane ? "@" + std::to_string(o.lane) : std::string()));
    return out;
  }
  int64_t num_lanes() const { return used_lanes_; }

  // Launch prologue, n_iters x loop body, epilogue (lane 0 = current stream).
  void run(int64_t n_iters) { JR_CHECK_OK(enqueue(cur_stream(), (int)n_iters)); }
  // Launch one segment alone with iteration index `it` (eager; host-driven loops
  // that interleave collectives with the segments, runtime/engine.py context parallelism).
  void run_segment(int64_t seg, int64_t it) {
    TORCH_CHECK(seg >= 0 && seg <= 3, "segment must be 0..3");
    JR_CHECK_OK(enqueue(cur_stream(), (int)it, false, -1, (int)seg));
  }
  // Enqueue into a stream that an outer capture is recording (e.g. a whole
  // training step captured by torch.cuda.graph): lane 0 is the caller's stream
  // itself, as in capture(), so the origin stream never holds only fork / join
  // event nodes (which crashes hipStreamEndCapture on this ROCm); no per-op
  // checks (no synchronisation inside a capture).
  void run_inline(int64_t n_iters) { JR_CHECK_OK(enqueue(cur_stream(), (int)n_iters, true)); }

  // Capture the same sequence into one hipGraph (on a private stream: the
  // legacy default stream cannot be captured) and instantiate it.
  void capture(int64_t n_iters) {
    reset_graph();
    capture_into(n_iters, -1, &graph_, &exec_);
    captured_iters_ = n_iters;
  }
  // Capture one phase as its own hipGraph: part 0 = the prologue (encoders +
  // correlation pyramid), part 1 = n_iters loop iterations + the epilogue.
  // Replayed on different streams, the prologue of batch i+1 overlaps the
  // refinement loop of batch i (cross-batch pipelining, runtime/engine.py).
  void capture_part(int64_t part, int64_t n_iters) {
    TORCH_CHECK(part == 0 || part == 1, "part must be 0 (prologue) or 1 (loop + epilogue)");
    reset_part(part);
    capture_into(n_iters, (int)part, &pgraph_[part], &pexec_[part]);
    pcaptured_[part] = n_iters;
  }
  int64_t captured_part_iters(int64_t part) const { return pcaptured_[part & 1]; }
  void replay_part(int64_t part) {
    TORCH_CHECK((part == 0 || part == 1) && pexec_[part] != nullptr, "plan: part ", part, " not captured");
    hipError_t e = hipGraphLaunch(pexec_[part], cur_stream());
    TORCH_CHECK(e == hipSuccess, "graph launch failed: ", hipGetErrorString(e));
  }

  // Software-pipelined step: ONE hipGraph holding this plan's refinement loop
  // + epilogue (batch i) and `next`'s prologue (encoders + correlation pyramid
  // of batch i+1, a plan with its own buffers) as independent branches.  The
  // loop is latency-bound (one workgroup per CU, ~220 of 256 CUs per kernel);
  // the throughput-bound encoder convs fill the idle SIMD slots.  Two graphs
  // launched on two streams serialise on this ROCm (measured 196 pairs/s,
  // engine.submit), the branches of one graph do not.  The loop branch is
  // enqueued first, so its nodes come first in the graph's launch order.
  void capture_pipelined(c10::intrusive_ptr<Plan> next, int64_t n_iters) {
    TORCH_CHECK(next.get() != this, "capture_pipelined: the next plan must have its own buffers");
    reset_pipe();
    // The two phases are captured on their own (capture_part) and their nodes
    // copied, with their dependency edges, into one graph with no edge between
    // the two: every lane of both stays a parallel branch.  (Enqueueing both
    // into one stream capture -- the next plan's lanes forked from this one's
    // capture stream -- crashed hipStreamEndCapture on this ROCm whenever both
    // plans use several lanes (batch 4); a child-graph node runs its graph's
    // nodes in order on one stream, i.e. without the lanes.)
    if (pcaptured_[1] != n_iters) capture_part(1, n_iters);
    if (next->pcaptured_[0] != n_iters) next->capture_part(0, n_iters);
    debug_ = std::getenv("JR_PLAN_DEBUG") != nullptr;
    hipGraph_t g = nullptr;
    TORCH_CHECK(hipGraphCreate(&g, 0) == hipSuccess, "graph create");
    pipe_graph_ = g;
    // loop nodes first (the executor launches in creation order; the prologue's first
    // measured batch 1 157 -> 78 pairs/s, the two phases then run one after the other).
    // (The prologue as one child-graph node, i.e. its nodes in order on one stream,
    // measured 264 vs 289 pairs/s at batch 4.)
    // One empty root node ahead of both branches: the executor forks a node's successors
    // onto parallel streams, but runs disconnected components in creation order on the
    // launch stream (measured: 21.6 us of a 3.2 ms raft_small batch-1 step concurrent;
    // with the root raft_small b1 12 it 788 vs 713 pairs/s, profiles/r5_pipeline_fork_ab.txt).
    hipGraphNode_t root = nullptr;
    TORCH_CHECK(hipGraphAddEmptyNode(&root, g, nullptr, 0) == hipSuccess, "graph root");
    append_graph(g, pgraph_[1], root);
    append_graph(g, next->pgraph_[0], root);
    hipError_t e3 = hipGraphInstantiate(&pipe_exec_, g, nullptr, nullptr, 0);
    if (debug_) fprintf(stderr, "[plan] pipelined instantiate %d\n", (int)e3);
    TORCH_CHECK(e3 == hipSuccess, "graph instantiate failed: ", hipGetErrorString(e3));
    pipe_iters_ = n_iters;
    pipe_next_ = next.get();
  }
  // Copy every node of src (kernel / empty nodes: what a plan capture holds)
  // into dst in dependency order, keeping src's edges.
  static void append_graph(hipGraph_t dst, hipGraph_t src, hipGraphNode_t root = nullptr) {
    size_t n = 0;
    TORCH_CHECK(hipGraphGetNodes(src, nullptr, &n) == hipSuccess, "graph nodes");
    std::vector<hipGraphNode_t> nodes(n);
    TORCH_CHECK(hipGraphGetNodes(src, nodes.data(), &n) == hipSuccess, "graph nodes");
    std::unordered_map<hipGraphNode_t, size_t> index;
    for (size_t i = 0; i < n; ++i) index[nodes[i]] = i;
    std::vector<std::vector<size_t>> deps(n), users(n);
    std::vector<size_t> missing(n, 0);
    for (size_t i = 0; i < n; ++i) {
      size_t nd = 0;
      TORCH_CHECK(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd) == hipSuccess, "node deps");
      std::vector<hipGraphNode_t> d(nd);
      if (nd) TORCH_CHECK(hipGraphNodeGetDependencies(nodes[i], d.data(), &nd) == hipSuccess, "node deps");
      for (auto x : d) {
        const size_t j = index.at(x);
        deps[i].push_back(j);
        users[j].push_back(i);
      }
      missing[i] = deps[i].size();
    }
    std::vector<hipGraphNode_t> copy(n, nullptr);
    // ready nodes are copied in src creation order: the executor maps a node's
    // successors onto its streams in creation order, and a depth-first copy of
    // the forward graph measured 6 % slower (profiles/r2_pipelined_graph_ab.txt)
    std::vector<size_t> ready;
    for (size_t i = 0; i < n; ++i) if (!missing[i]) ready.push_back(i);
    size_t done = 0;
    while (!ready.empty()) {
      const auto it = std::min_element(ready.begin(), ready.end());
      const size_t i = *it;
      ready.erase(it);
      std::vector<hipGraphNode_t> d;
      for (size_t j : deps[i]) d.push_back(copy[j]);
      if (d.empty() && root) d.push_back(root);
      hipGraphNodeType type;
      TORCH_CHECK(hipGraphNodeGetType(nodes[i], &type) == hipSuccess, "node type");
      hipError_t e = hipSuccess;
      if (type == hipGraphNodeTypeKernel) {
        hipKernelNodeParams kp;
        e = hipGraphKernelNodeGetParams(nodes[i], &kp);
        if (e == hipSuccess) e = hipGraphAddKernelNode(&copy[i], dst, d.data(), d.size(), &kp);
      } else if (type == hipGraphNodeTypeEmpty) {
        e = hipGraphAddEmptyNode(&copy[i], dst, d.data(), d.size());
      } else {
        TORCH_CHECK(false, "capture_pipelined: unsupported graph node type ", (int)type);
      }
      TORCH_CHECK(e == hipSuccess, "capture_pipelined: node copy failed: ", hipGetErrorString(e));
      ++done;
      for (size_t u : users[i]) if (--missing[u] == 0) ready.push_back(u);
    }
    TORCH_CHECK(done == n, "capture_pipelined: cyclic graph");
  }
  // Batch parts as ONE graph: every part plan's full-forward capture (own
  // buffers, own lanes) copied into a single graph with no edge between the
  // parts, so their in-order chains interleave on the GPU without any
  // cross-stream edge (separate graphs on separate streams serialise on this
  // ROCm).  merge_reset(); merge_add(part) for every part; merge_finish(n);
  // replay_pipelined().
  void merge_reset() {
    reset_pipe();
    TORCH_CHECK(hipGraphCreate(&pipe_graph_, 0) == hipSuccess, "graph create");
    // one root: the parts fork (capture_pipelined)
    TORCH_CHECK(hipGraphAddEmptyNode(&pipe_root_, pipe_graph_, nullptr, 0) == hipSuccess, "graph root");
  }
  void merge_add(c10::intrusive_ptr<Plan> part, int64_t n_iters) {
    TORCH_CHECK(pipe_graph_ != nullptr && pipe_exec_ == nullptr, "merge_add: call merge_reset() first");
    if (part->captured_iters_ != n_iters) {
      // capture() resets this plan's graphs, the merge in progress included
      hipGraph_t merging = pipe_graph_;
      pipe_graph_ = nullptr;
      part->capture(n_iters);
      pipe_graph_ = merging;
    }
    append_graph(pipe_graph_, part->graph_, pipe_root_);
  }
  void merge_finish(int64_t n_iters) {
    TORCH_CHECK(pipe_graph_ != nullptr && pipe_exec_ == nullptr, "merge_finish: call merge_reset() first");
    hipError_t e = hipGraphInstantiate(&pipe_exec_, pipe_graph_, nullptr, nullptr, 0);
    TORCH_CHECK(e == hipSuccess, "graph instantiate failed: ", hipGetErrorString(e));
    pipe_iters_ = n_iters;
    pipe_next_ = this;
  }
  int64_t merged_iters() const { return pipe_next_ == this ? pipe_iters_ : -1; }

  // n_iters of the pipelined graph if it was captured with `next`, else -1.
  int64_t pipelined_iters(c10::intrusive_ptr<Plan> next) const {
    return pipe_next_ == next.get() ? pipe_iters_ : -1;
  }
  void replay_pipelined() {
    TORCH_CHECK(pipe_exec_ != nullptr, "plan: no pipelined graph captured");
    hipError_t e = hipGraphLaunch(pipe_exec_, cur_stream());
    TORCH_CHECK(e == hipSuccess, "graph launch failed: ", hipGetErrorString(e));
  }

 private:
  void reset_pipe() {
    if (pipe_exec_) { (void)hipGraphExecDestroy(pipe_exec_); pipe_exec_ = nullptr; }
    if (pipe_graph_) { (void)hipGraphDestroy(pipe_graph_); pipe_graph_ = nullptr; }
    pipe_root_ = nullptr;
    pipe_iters_ = -1;
    pipe_next_ = nullptr;
  }
  hipStream_t ensure_cap_stream() {
    if (!cap_stream_) {
      int least = 0, greatest = 0;
      TORCH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess, "priority range");
      TORCH_CHECK(hipStreamCreateWithPriority(&cap_stream_, hipStreamNonBlocking, greatest) == hipSuccess, "stream");
    }
    return cap_stream_;
  }
  void reset_part(int64_t part) {
    if (pexec_[part]) { (void)hipGraphExecDestroy(pexec_[part]); pexec_[part] = nullptr; }
    if (pgraph_[part]) { (void)hipGraphDestroy(pgraph_[part]); pgraph_[part] = nullptr; }
    pcaptured_[part] = -1;
  }
  void capture_into(int64_t n_iters, int part, hipGraph_t* graph_out, hipGraphExec_t* exec_out) {
    hipStream_t s = ensure_cap_stream();
    debug_ = std::getenv("JR_PLAN_DEBUG") != nullptr;
    // order the capture after work already queued on the current stream
    TORCH_CHECK(hipStreamSynchronize(cur_stream()) == hipSuccess, "sync");
    TORCH_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess, "begin capture");
    int err = enqueue(s, (int)n_iters, true, part);
    if (debug_) fprintf(stderr, "[plan] enqueue done err=%d\n", err);
    hipGraph_t g = nullptr;
    hipError_t e2 = hipStreamEndCapture(s, &g);
    if (debug_) fprintf(stderr, "[plan] end capture %d\n", (int)e2);
    TORCH_CHECK(err == 0, "launch failed during capture: ", hipGetErrorString((hipError_t)err));
    TORCH_CHECK(e2 == hipSuccess && g != nullptr, "end capture failed: ", hipGetErrorString(e2));
    *graph_out = g;
    hipError_t e3 = hipGraphInstantiate(exec_out, g, nullptr, nullptr, 0);
    if (debug_) fprintf(stderr, "[plan] instantiate %d\n", (int)e3);
    TORCH_CHECK(e3 == hipSuccess, "graph instantiate failed: ", hipGetErrorString(e3));
  }

 public:
  int64_t captured_iters() const { return captured_iters_; }
  void replay() {
    TORCH_CHECK(exec_ != nullptr, "plan: no captured graph");
    hipError_t e = hipGraphLaunch(exec_, cur_stream());
    TORCH_CHECK(e == hipSuccess, "graph launch failed: ", hipGetErrorString(e));
  }
  void reset_graph() {
    if (exec_) { (void)hipGraphExecDestroy(exec_); exec_ = nullptr; }
    if (graph_) { (void)hipGraphDestroy(graph_); graph_ = nullptr; }
    captured_iters_ = -1;
    reset_part(0);
    reset_part(1);
    reset_pipe();
  }

 private:
  enum OpKind { OP_LAUNCH = 0, OP_RECORD = 1, OP_WAIT = 2 };
  struct Op {
    Launch l;
    int lane;
    int kind;
    int ev;
    std::string name;
    int defer;   // 1: previous iteration's work (see set_defer)
  };
  void push(Launch l, const char* name) {
    segs_[seg_].push_back(Op{std::move(l), lane_, OP_LAUNCH, -1, name, defer_});
    reset_graph();
  }
  void push_sync(int kind, int64_t ev, const char* name) {
    TORCH_CHECK(ev >= 0 && ev < kMaxEvents, "event id out of range");
    segs_[seg_].push_back(Op{Launch(), lane_, kind, (int)ev, std::string(name) + std::to_string(ev), defer_});
    reset_graph();
  }
  static int create_event(hipEvent_t* e) {
    return (int)hipEventCreateWithFlags(e, hipEventDisableTiming);
  }
  int ensure_resources() {
    if (events_.empty()) {
      events_.assign(kMaxEvents, nullptr);
      for (auto& e : events_) if (int r = create_event(&e)) return r;
    }
    if (!fork_) if (int r = create_event(&fork_)) return r;
    int least = 0, greatest = 0;
    if (int r = (int)hipDeviceGetStreamPriorityRange(&least, &greatest)) return r;
    if (!lanes_[0]) if (int r = (int)hipStreamCreateWithPriority(&lanes_[0], hipStreamNonBlocking, greatest)) return r;
    if (!join_[0]) if (int r = create_event(&join_[0])) return r;
    for (int l = 1; l < used_lanes_; ++l) {
      if (!lanes_[l]) if (int r = (int)hipStreamCreateWithPriority(&lanes_[l], hipStreamNonBlocking, least)) return r;
      if (!join_[l]) if (int r = create_event(&join_[l])) return r;
    }
    return 0;
  }
  // recorded[ev] = 1 + lane of the event's latest record in this enqueue (0: not recorded).
  // A wait on an event last recorded on the same lane is already satisfied by stream
  // order and is skipped (a same-stream record/wait pair on a forked capture stream
  // also crashes hipStreamEndCapture on this ROCm).
  int exec_op(const Op& o, hipStream_t* st, int it, std::vector<char>& recorded) {
    if (o.defer) {
      if (it == 0) return 0;
      --it;
    }
    hipStream_t s = st[o.lane];
    if (debug_) fprintf(stderr, "[plan] it=%d lane=%d %s stream=%p\n", it, o.lane, o.name.c_str(), (void*)s);
    switch (o.kind) {
      case OP_LAUNCH: {
        const int r = o.l(s, it);
        // JR_PLAN_CHECK=1 (eager run only): synchronise after every launch so an asynchronous
        // fault or launch error is attributed to the op that caused it (fault localisation,
        // SURVEY.md 5.2); the failing op's segment index, lane, iteration and name are reported.
        if (check_ && !capturing_) {
          hipError_t e = r ? (hipError_t)r : hipStreamSynchronize(s);
          if (e == hipSuccess) e = hipGetLastError();
          if (e != hipSuccess) {
            fprintf(stderr, "[plan check] op '%s' (lane %d, iteration %d) failed: %s\n", o.name.c_str(), o.lane, it,
                    hipGetErrorString(e));
            return (int)e;
          }
        }
        return r;
      }
      case OP_RECORD: recorded[o.ev] = (char)(1 + o.lane); return (int)hipEventRecord(events_[o.ev], s);
      default:
        if (!recorded[o.ev] || recorded[o.ev] == 1 + o.lane) return 0;
        return (int)hipStreamWaitEvent(s, events_[o.ev], 0);
    }
  }
  // part: -1 = the whole forward, 0 = prologue only, 1 = loop + epilogue only.
  // only_seg >= 0: just that segment, with iteration index n_iters.
  int enqueue(hipStream_t s, int n_iters, bool capturing = false, int part = -1, int only_seg = -1) {
    if (int r = ensure_resources()) return r;
    check_ = std::getenv("JR_PLAN_CHECK") != nullptr && std::getenv("JR_PLAN_CHECK")[0] == '1';
    capturing_ = capturing;
    // Eager: lane 0 is the private high-priority stream, forked from the caller's.
    // Capture: lane 0 is the capture stream itself (created with the greatest
    // priority); a capture whose origin stream holds only the fork/join event
    // nodes crashes hipStreamEndCapture on this ROCm.
    const int l0 = capturing ? 1 : 0;
    hipStream_t st[kMaxLanes] = {};
    st[0] = s;
    // fork / join only the lanes that hold ops in the enqueued segments: a forked
    // capture stream holding nothing but the fork wait and the join record
    // crashes hipStreamEndCapture on this ROCm (e.g. the context-encoder lane in
    // a loop-only capture, capture_part(1))
    bool used[kMaxLanes] = {};
    used[0] = true;
    for (int sg = 0; sg < 4; ++sg) {
      if ((sg == 0 && part == 1) || (sg != 0 && part == 0)) continue;
      if (only_seg >= 0 && sg != only_seg) continue;
      for (const auto& o : segs_[sg]) used[o.lane] = true;
    }
    if (int r = (int)hipEventRecord(fork_, s)) return r;
    for (int l = l0; l < used_lanes_; ++l) {
      if (!used[l]) continue;
      st[l] = lanes_[l];
      if (int r = (int)hipStreamWaitEvent(st[l], fork_, 0)) return r;
    }
    std::vector<char> recorded(kMaxEvents, 0);
    // roctx ranges (visible in rocprofv3 --marker-trace) bracket the host-side
    // enqueue of each phase: encoders + correlation pyramid, every refinement
    // iteration, the epilogue.
    RangeGuard all("raft.plan");
    if (only_seg >= 0) {
      RangeGuard r("raft.segment");
      for (auto& o : segs_[only_seg]) if (int e = exec_op(o, st, n_iters, recorded)) return e;
    } else {
    if (part != 1) {
      RangeGuard r("raft.prologue");
      for (auto& o : segs_[0]) if (int e = exec_op(o, st, 0, recorded)) return e;
    }
    for (int it = 0; part != 0 && it < n_iters; ++it) {
      RangeGuard r("raft.iteration");
      for (auto& o : segs_[1]) if (int e = exec_op(o, st, it, recorded)) return e;
      for (auto& o : segs_[3]) if (int e = exec_op(o, st, it, recorded)) return e;
    }
    if (part != 0) {
      RangeGuard r("raft.epilogue");
      for (auto& o : segs_[2]) if (int e = exec_op(o, st, n_iters, recorded)) return e;
    }
    }
    for (int l = l0; l < used_lanes_; ++l) {
      if (!used[l]) continue;
      if (int r = (int)hipEventRecord(join_[l], st[l])) return r;
      if (int r = (int)hipStreamWaitEvent(s, join_[l], 0)) return r;
    }
    return 0;
  }
  std::vector<Op> segs_[4];
  std::vector<at::Tensor> keep_;
  int seg_ = 0;
  int lane_ = 0;
  int defer_ = 0;
  int used_lanes_ = 1;
  std::vector<hipEvent_t> events_;
  hipEvent_t fork_ = nullptr;
  hipEvent_t join_[kMaxLanes] = {};
  hipStream_t lanes_[kMaxLanes] = {};
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  int64_t captured_iters_ = -1;
  hipGraph_t pgraph_[2] = {};
  hipGraphExec_t pexec_[2] = {};
  int64_t pcaptured_[2] = {-1, -1};
  hipGraph_t pipe_graph_ = nullptr;
  hipGraphNode_t pipe_root_ = nullptr;
  hipGraphExec_t pipe_exec_ = nullptr;
  int64_t pipe_iters_ = -1;
  const Plan* pipe_next_ = nullptr;
  bool debug_ = false;
  bool check_ = false;
  bool capturing_ = false;
};

}  // namespace jr

TORCH_LIBRARY(jax_raft_amd, m) {
  m.def("conv(Tensor?[] t, int[] i, float alpha) -> ()", &jr::conv_op);
  m.def("corr(Tensor?[] t, int[] i, float scale) -> ()", &jr::corr_op);
  m.def("lookup(Tensor?[] t, int[] i) -> ()", &jr::lookup_op);
  m.def("upsample_convex(Tensor?[] t, int[] i) -> ()", &jr::upsample_convex_op);
  m.def("convex_head(Tensor?[] t, int[] i, float alpha) -> ()", &jr::convex_head_op);
  m.def("upsample_bilinear(Tensor?[] t, int[] i) -> ()", &jr::upsample_bilinear_op);
  m.def("stats(Tensor?[] t, int[] i) -> ()", &jr::stats_op);
  m.def("norm_act(Tensor?[] t, int[] i, float eps) -> ()", &jr::norm_act_op);
  m.def("prep(Tensor?[] t, int[] i) -> ()", &jr::prep_op);
  m.def("init_coords(Tensor?[] t, int[] i) -> ()", &jr::init_coords_op);
  m.def("copy_channels(Tensor?[] t, int[] i) -> ()", &jr::copy_channels_op);
  m.def("sum_iters(Tensor?[] t, int[] i) -> ()", &jr::sum_iters_op);
  m.def("lookup_bwd(Tensor?[] t, int[] i) -> ()", &jr::lookup_bwd_op);
  m.def("im2col(Tensor?[] t, int[] i) -> ()", &jr::im2col_op);
  m.def("flow_taps(Tensor?[] t, int[] i) -> ()", &jr::flow_taps_op);
  m.def("taps_gemm(Tensor?[] t, int[] i) -> ()", &jr::taps_gemm_op);
  m.def("gru_fused(Tensor?[] t, int[] i) -> ()", &jr::gru_fused_op);
  m.def("bgemm(Tensor?[] t, int[] i, float alpha) -> ()", &jr::bgemm_op);
  m.def("conv_grouped_ok(int cfg) -> bool", &jr::conv_grouped_ok_op);
  m.def("gru_fused_fits(int H, int W, int vertical) -> bool", &jr::gru_fused_fits);
  m.def("gru_halo(Tensor?[] t, int[] i) -> ()", &jr::gru_halo_op);
  m.def("conv_halo_ok(int cfg, int cin8, int cout) -> bool", &jr::conv_halo_ok_op);
  m.def("stats_final(Tensor?[] t, int[] i) -> ()", &jr::stats_final_op);
  m.def("conv_halo_cfg(int cfg) -> int[]", &jr::conv_halo_cfg_op);
  m.def("gru_halo_geom_ok(int hd, int mode, int TR, int TC, int nb1, int nb2) -> bool", &jr::gru_halo_geom_ok);
  m.def("conv1x1(Tensor?[] t, int[] i) -> ()", &jr::conv1x1_op);
  m.def("conv_direct(Tensor?[] t, int[] i) -> ()", &jr::conv_direct_op);
  m.def("conv_train(Tensor?[] t, int[] i, float alpha, Tensor?[] tx, int[] ix) -> ()", &jr::conv_train_op);
  m.def("upsample_convex_bwd(Tensor?[] t, int[] i, float alpha) -> ()", &jr::upsample_convex_bwd_op);
  m.def("flow_gather_bwd(Tensor?[] t, int[] i) -> ()", &jr::flow_gather_bwd_op);
  m.def("norm_bwd(Tensor?[] t, int[] i, float eps) -> ()", &jr::norm_bwd_op);
  m.def("pack(Tensor?[] t, int[] i) -> ()", &jr::pack_op);
  m.def("wgrad(Tensor?[] t, int[] i) -> ()", &jr::wgrad_op);
  m.def("pyr_bwd_dc(Tensor?[] t, int[] i, float scale) -> ()", &jr::pyr_bwd_dc_op);
  m.def("upsample_bilinear_bwd(Tensor?[] t, int[] i) -> ()", &jr::upsample_bilinear_bwd_op);
  m.def("seq_loss(Tensor?[] t, int[] i, float max_flow) -> ()", &jr::seq_loss_op);
  m.def("seq_loss_blocks(int P) -> int", &jr::seq_loss_blocks_op);
  m.def("seq_loss_bwd(Tensor?[] t, int[] i, float max_flow) -> ()", &jr::seq_loss_bwd_op);
  m.def("conv_f32(Tensor?[] t, int[] i, float alpha) -> ()", &jr::conv_f32_op);
  m.def("stats_f32(Tensor?[] t, int[] i) -> ()", &jr::stats_f32_op);
  m.def("norm_act_f32(Tensor?[] t, int[] i, float eps) -> ()", &jr::norm_act_f32_op);
  m.def("prep_f32(Tensor?[] t, int[] i) -> ()", &jr::prep_f32_op);
  m.def("copy_channels_f32(Tensor?[] t, int[] i) -> ()", &jr::copy_channels_f32_op);
  m.def("upsample_convex_f32(Tensor?[] t, int[] i) -> ()", &jr::upsample_convex_f32_op);
  m.def("corr_pool_f32(Tensor?[] t, int[] i) -> ()", &jr::corr_pool_f32_op);
  m.def("lookup_f32(Tensor?[] t, int[] i) -> ()", &jr::lookup_f32_op);
  m.def("flow_update_f32(Tensor?[] t, int[] i) -> ()", &jr::flow_update_f32_op);
  m.class_<jr::Plan>("Plan")
      .def(torch::init<>())
      .def("set_segment", &jr::Plan::set_segment)
      .def("capture_pipelined", &jr::Plan::capture_pipelined)
      .def("pipelined_iters", &jr::Plan::pipelined_iters)
      .def("replay_pipelined", &jr::Plan::replay_pipelined)
      .def("merge_reset", &jr::Plan::merge_reset)
      .def("merge_add", &jr::Plan::merge_add)
      .def("merge_finish", &jr::Plan::merge_finish)
      .def("merged_iters", &jr::Plan::merged_iters)
      .def("set_lane", &jr::Plan::set_lane)
      .def("set_defer", &jr::Plan::set_defer)
      .def("add_record", &jr::Plan::add_record)
      .def("add_wait", &jr::Plan::add_wait)
      .def("num_lanes", &jr::Plan::num_lanes)
      .def("add_conv", &jr::Plan::add_conv)
      .def("add_conv_alt", &jr::Plan::add_conv_alt)
      .def("add_corr", &jr::Plan::add_corr)
      .def("add_lookup", &jr::Plan::add_lookup)
      .def("add_upsample_convex", &jr::Plan::add_upsample_convex)
      .def("add_convex_head", &jr::Plan::add_convex_head)
      .def("add_upsample_bilinear", &jr::Plan::add_upsample_bilinear)
      .def("add_stats", &jr::Plan::add_stats)
      .def("add_norm_act", &jr::Plan::add_norm_act)
      .def("add_prep", &jr::Plan::add_prep)
      .def("add_init_coords", &jr::Plan::add_init_coords)
      .def("add_memset", &jr::Plan::add_memset)
      .def("add_copy", &jr::Plan::add_copy)
      .def("add_copy_channels", &jr::Plan::add_copy_channels)
      .def("add_flow_taps", &jr::Plan::add_flow_taps)
      .def("add_taps_gemm", &jr::Plan::add_taps_gemm)
      .def("add_gru_fused", &jr::Plan::add_gru_fused)
      .def("add_gru_halo", &jr::Plan::add_gru_halo)
      .def("add_stats_final", &jr::Plan::add_stats_final)
      .def("add_flowin_dual", &jr::Plan::add_flowin_dual)
      .def("add_conv_group", &jr::Plan::add_conv_group)
      .def("add_conv1x1", &jr::Plan::add_conv1x1)
      .def("add_conv_direct", &jr::Plan::add_conv_direct)
      .def("add_conv_train", &jr::Plan::add_conv_train)
      .def("add_upsample_convex_bwd", &jr::Plan::add_upsample_convex_bwd)
      .def("add_flow_gather_bwd", &jr::Plan::add_flow_gather_bwd)
      .def("add_norm_bwd", &jr::Plan::add_norm_bwd)
      .def("add_pack", &jr::Plan::add_pack)
      .def("add_wgrad", &jr::Plan::add_wgrad)
      .def("add_bn_table", &jr::Plan::add_bn_table)
      .def("add_upsample_bilinear_bwd", &jr::Plan::add_upsample_bilinear_bwd)
      .def("add_lookup_bwd", &jr::Plan::add_lookup_bwd)
      .def("add_im2col", &jr::Plan::add_im2col)
      .def("add_conv_f32", &jr::Plan::add_conv_f32)
      .def("add_stats_f32", &jr::Plan::add_stats_f32)
      .def("add_norm_act_f32", &jr::Plan::add_norm_act_f32)
      .def("add_prep_f32", &jr::Plan::add_prep_f32)
      .def("add_copy_channels_f32", &jr::Plan::add_copy_channels_f32)
      .def("add_upsample_convex_f32", &jr::Plan::add_upsample_convex_f32)
      .def("add_corr_pool_f32", &jr::Plan::add_corr_pool_f32)
      .def("add_lookup_f32", &jr::Plan::add_lookup_f32)
      .def("add_flow_update_f32", &jr::Plan::add_flow_update_f32)
      .def("num_ops", &jr::Plan::num_ops)
      .def("op_names", &jr::Plan::op_names)
      .def("run", &jr::Plan::run)
      .def("run_segment", &jr::Plan::run_segment)
      .def("run_inline", &jr::Plan::run_inline)
      .def("capture", &jr::Plan::capture)
      .def("captured_iters", &jr::Plan::captured_iters)
      .def("replay", &jr::Plan::replay)
      .def("capture_part", &jr::Plan::capture_part)
      .def("captured_part_iters", &jr::Plan::captured_part_iters)
      .def("replay_part", &jr::Plan::replay_part)
      .def("reset_graph", &jr::Plan::reset_graph);
}
