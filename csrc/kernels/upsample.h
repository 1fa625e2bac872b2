// Bilinear x8 upsampling of the flow (align_corners, reference jax_raft/model.py:69-82 via
// upsample_flow without a mask): one output pixel per thread -- shared by elementwise.hip and
// the merged launches of merged.hip.
#pragma once
#include "common.h"

namespace {

JR_DEVICE void upsample_bilinear_elem(const float* __restrict__ flow, int B, int h, int w, float* __restrict__ out,
                                      const long long* __restrict__ out_slot, long out_off, long idx) {
  if (out_slot) out = (float*)(*out_slot) + out_off;  // output address supplied at run time
  const int H8 = 8 * h, W8 = 8 * w;
  const long total = (long)B * H8 * W8;
  if (idx >= total) return;
  const int X = idx % W8;
  const long t = idx / W8;
  const int Y = t % H8;
  const int b = t / H8;
  const float sx = (w > 1) ? (float)(w - 1) / (float)(W8 - 1) : 0.f;
  const float sy = (h > 1) ? (float)(h - 1) / (float)(H8 - 1) : 0.f;
  const float xi = X * sx, yi = Y * sy;
  int x0 = (int)floorf(xi), y0 = (int)floorf(yi);
  x0 = min(max(x0, 0), w - 1);
  y0 = min(max(y0, 0), h - 1);
  const int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, h - 1);
  const float wx = xi - x0, wy = yi - y0;
  const float2* f = (const float2*)flow + (long)b * h * w;
  const float2 a = f[y0 * w + x0], c = f[y0 * w + x1], d = f[y1 * w + x0], e = f[y1 * w + x1];
  const float top_x = a.x + wx * (c.x - a.x), top_y = a.y + wx * (c.y - a.y);
  const float bot_x = d.x + wx * (e.x - d.x), bot_y = d.y + wx * (e.y - d.y);
  ((float2*)out)[idx] = make_float2(8.f * (top_x + wy * (bot_x - top_x)), 8.f * (top_y + wy * (bot_y - top_y)));
}

}  // namespace
