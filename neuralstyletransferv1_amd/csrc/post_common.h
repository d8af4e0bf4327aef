// post_common.h — device helpers shared by the post-chain kernels (nst_ops.hip, region_ops.hip):
// the io_preset output decode and the bilinear fit of a raw model output to the content size.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace nst {

// output decode (pipeline.py:1445-1486): v = (((y[perm[c]] + p) * q) / r) + s, clamp(0,1).
// NST_PRESET_NONE (p=0, q=1, r=1, s=0) is the identity on values already in [0,1].
struct DecodeConsts {
  float p[3], q[3], r[3], s[3];
  int perm[3];
};

__device__ __forceinline__ float decode01(const float* y, int ch, const DecodeConsts& d) {
  float v = (((y[d.perm[ch]] + d.p[ch]) * d.q[ch]) / d.r[ch]) + d.s[ch];
  return fminf(fmaxf(v, 0.f), 1.f);
}

// decoded value of the f32 NCHW plane set yb ([3][h][w]) at output pixel (oy, ox) of an oh x ow fit:
// F.interpolate(bilinear, align_corners=False) of the decoded image (each tap decoded then
// interpolated, pipeline.py:1512-1516); the identity when the sizes agree.
__device__ __forceinline__ void decode_fit(const float* yb, int h, int w, const DecodeConsts& d, int oy, int ox,
                                           int oh, int ow, float* v) {
  const size_t plane = (size_t)h * w;
  if (oh == h && ow == w) {
    const size_t i = (size_t)oy * w + ox;
    const float yy[3] = {yb[i], yb[plane + i], yb[2 * plane + i]};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) v[ch] = decode01(yy, ch, d);
    return;
  }
  const float sh = (float)h / (float)oh, sw = (float)w / (float)ow;
  float fy = sh * ((float)oy + 0.5f) - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  float fx = sw * ((float)ox + 0.5f) - 0.5f;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  const size_t i00 = (size_t)y0 * w + x0, i01 = (size_t)y0 * w + x1, i10 = (size_t)y1 * w + x0, i11 = (size_t)y1 * w + x1;
  float t00[3], t01[3], t10[3], t11[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    t00[ch] = yb[ch * plane + i00]; t01[ch] = yb[ch * plane + i01];
    t10[ch] = yb[ch * plane + i10]; t11[ch] = yb[ch * plane + i11];
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float c00 = decode01(t00, ch, d), c01 = decode01(t01, ch, d), c10 = decode01(t10, ch, d),
                c11 = decode01(t11, ch, d);
    v[ch] = ly0 * (lx0 * c00 + lx1 * c01) + ly1 * (lx0 * c10 + lx1 * c11);
  }
}

}  // namespace nst
