// seg_ops.hip — the non-GEMM stages of the DeepLab v3+ mask program (configs[4]):
// the stem's normalised im2col, max / average pooling, align_corners=True bilinear resizes written
// into concatenation buffers, the final upsample + argmax, the class-id selection, the binary
// morphology and the two image resamplers of the mask path (Pillow LANCZOS for the working-size
// downscale, OpenCV INTER_LINEAR for the mask's upscale).  All NHWC, one thread per output element
// or 16-byte channel group; HBM-bound streaming kernels.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "nst_hip.h"
#include "seg_internal.h"

namespace nst {

namespace {

// activations in the compute dtype dt (NST_DT_F32 / NST_DT_BF16 / NST_DT_F16)
__device__ __forceinline__ float ld_act(const void* p, size_t i, int dt) {
  if (dt == NST_DT_F32) return ((const float*)p)[i];
  const uint16_t v = ((const uint16_t*)p)[i];
  return dt == NST_DT_F16 ? (float)__builtin_bit_cast(_Float16, v) : __uint_as_float((uint32_t)v << 16);
}
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ uint16_t h16_rne(float f, int dt) {  // to the 16-bit format dt, round to nearest even
  return dt == NST_DT_F16 ? __builtin_bit_cast(uint16_t, (_Float16)f) : bf16_rne(f);
}
__device__ __forceinline__ void st_act(void* p, size_t i, float v, int dt) {
  if (dt == NST_DT_F32) ((float*)p)[i] = v;
  else ((uint16_t*)p)[i] = h16_rne(v, dt);
}
inline unsigned blocks_for(size_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

// ---- stem im2col (sky_swap.py:179-183 preprocess_pil fused for u8 frames) ----
// u8: float32(u8) / 255 in float32, then (x - mean) / std in float64 (numpy promotes the float32
// array against the float64 tuples), then .float() -> float32 — reproduced operation for operation.
__global__ __launch_bounds__(256) void stem_im2col_kernel(const void* __restrict__ x, int x_u8, int dt, int n, int h,
                                                          int w, int ho, int wo, int kp, void* __restrict__ col) {
  // one thread = one output pixel x 8 consecutive columns (one 16-byte bf16 / two 16-byte fp32 stores;
  // consecutive threads write consecutive chunks of a pixel's row).  u8 frames go through a per-block table
  // of the 3 x 256 normalised values, each computed once with the reference's float32 / float64 steps.
  __shared__ float lut[3][256];
  if (x_u8) {
    const double mean[3] = {0.485, 0.456, 0.406}, sd[3] = {0.229, 0.224, 0.225};
    for (int i = threadIdx.x; i < 768; i += blockDim.x) {
      const int c = i >> 8, v = i & 255;
      lut[c][v] = (float)(((double)((float)v / 255.0f) - mean[c]) / sd[c]);
    }
    __syncthreads();
  }
  const int chunks = kp >> 3;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)n * ho * wo * chunks;
  if (e >= total) return;
  const int k0 = (int)(e % chunks) * 8;
  const size_t px = e / chunks;
  const int ox = (int)(px % wo);
  const int oy = (int)((px / wo) % ho);
  const int img = (int)(px / ((size_t)wo * ho));
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = k0 + q;
    v[q] = 0.f;
    if (k < 147) {
      const int c = k % 3, tap = k / 3, ky = tap / 7, kx = tap - ky * 7;
      const int iy = oy * 2 - 3 + ky, ix = ox * 2 - 3 + kx;
      if (iy >= 0 && iy < h && ix >= 0 && ix < w) {
        if (x_u8) v[q] = lut[c][((const uint8_t*)x)[(((size_t)img * h + iy) * w + ix) * 3 + c]];
        else v[q] = ((const float*)x)[(((size_t)img * 3 + c) * h + iy) * w + ix];
      }
    }
  }
  const size_t o = px * kp + k0;
  if (dt == NST_DT_F32) {
    *(float4*)((float*)col + o) = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)((float*)col + o + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    uint4 u;
    u.x = (uint32_t)h16_rne(v[0], dt) | ((uint32_t)h16_rne(v[1], dt) << 16);
    u.y = (uint32_t)h16_rne(v[2], dt) | ((uint32_t)h16_rne(v[3], dt) << 16);
    u.z = (uint32_t)h16_rne(v[4], dt) | ((uint32_t)h16_rne(v[5], dt) << 16);
    u.w = (uint32_t)h16_rne(v[6], dt) | ((uint32_t)h16_rne(v[7], dt) << 16);
    *(uint4*)((uint16_t*)col + o) = u;
  }
}

// ---- MaxPool2d(3, stride 2, padding 1) (resnet.py:65), NHWC ----
__global__ __launch_bounds__(256) void maxpool_kernel(const void* __restrict__ in, int dt, int n, int h, int w, int c,
                                                      void* __restrict__ out, int ho, int wo) {
  // one thread = one output pixel x 8 consecutive channels
  const int groups = c >> 3;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)n * ho * wo * groups;
  if (e >= total) return;
  const int ch = (int)(e % groups) * 8;
  const size_t px = e / groups;
  const int ox = (int)(px % wo), oy = (int)((px / wo) % ho), img = (int)(px / ((size_t)wo * ho));
  float m[8];
  bool any = false;
  for (int dy = 0; dy < 3; ++dy) {
    const int iy = oy * 2 - 1 + dy;
    if (iy < 0 || iy >= h) continue;
    for (int dx = 0; dx < 3; ++dx) {
      const int ix = ox * 2 - 1 + dx;
      if (ix < 0 || ix >= w) continue;
      const size_t b = (((size_t)img * h + iy) * w + ix) * c + ch;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = ld_act(in, b + q, dt);
        m[q] = any ? fmaxf(m[q], v) : v;
      }
      any = true;
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) st_act(out, px * c + ch + q, m[q], dt);
}

// ---- AdaptiveAvgPool2d(1) (aspp.py:55): torch takes the mean over (h, w).  Block = 64 channels x 4 pixel
// lanes (coalesced 64-channel rows), fp64 sums combined in fixed lane order ----
__global__ __launch_bounds__(256) void avgpool_kernel(const void* __restrict__ in, int dt, int hw, int c, int cs,
                                                      void* __restrict__ out) {
  __shared__ double part[4][64];
  const int t = threadIdx.x, cl = t & 63, lane = t >> 6;
  const int ch = blockIdx.x * 64 + cl, img = blockIdx.y;
  double s = 0.0;
  if (ch < c) {
    const size_t base = (size_t)img * hw * cs + ch;
    for (int i = lane; i < hw; i += 4) s += (double)ld_act(in, base + (size_t)i * cs, dt);
  }
  part[lane][cl] = s;
  __syncthreads();
  if (lane == 0 && ch < c) {
    const double tot = ((part[0][cl] + part[1][cl]) + part[2][cl]) + part[3][cl];
    st_act(out, (size_t)img * cs + ch, (float)(tot / hw), dt);
  }
}

// ---- bilinear, align_corners=True (deeplab.py:31, aspp.py:71, decoder.py:39): torch's CPU
// arithmetic — scale = (in-1)/(out-1) in float, src = scale*dst, i0 = floor, lambda in float,
// v = (v00*l0x + v01*l1x)*l0y + (v10*l0x + v11*l1x)*l1y ----
struct AcAxis {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ AcAxis ac_axis(int dst, int in, int out) {
  const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float real = scale * (float)dst;
  int i0 = min((int)floorf(real), in - 1);
  const float lam = fminf(fmaxf(real - (float)i0, 0.f), 1.f);
  AcAxis a;
  a.i0 = i0;
  a.i1 = i0 + (i0 < in - 1 ? 1 : 0);
  a.l1 = lam;
  a.l0 = 1.f - lam;
  return a;
}

__global__ __launch_bounds__(256) void resize_ac_kernel(const void* __restrict__ in, int dt, int n, int h, int w,
                                                        int c, int cs_in, void* __restrict__ out, int oh, int ow,
                                                        int cs_out, int off) {
  // one thread = one output pixel x 8 consecutive channels
  const int groups = c >> 3;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)n * oh * ow * groups;
  if (e >= total) return;
  const int ch = (int)(e % groups) * 8;
  const size_t px = e / groups;
  const int ox = (int)(px % ow), oy = (int)((px / ow) % oh), img = (int)(px / ((size_t)ow * oh));
  const AcAxis ay = ac_axis(oy, h, oh), ax = ac_axis(ox, w, ow);
  const size_t b = (size_t)img * h * w;
  const size_t i00 = (b + (size_t)ay.i0 * w + ax.i0) * cs_in + ch, i01 = (b + (size_t)ay.i0 * w + ax.i1) * cs_in + ch;
  const size_t i10 = (b + (size_t)ay.i1 * w + ax.i0) * cs_in + ch, i11 = (b + (size_t)ay.i1 * w + ax.i1) * cs_in + ch;
  const size_t o = px * cs_out + off + ch;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float t0 = ld_act(in, i00 + q, dt) * ax.l0 + ld_act(in, i01 + q, dt) * ax.l1;
    const float t1 = ld_act(in, i10 + q, dt) * ax.l0 + ld_act(in, i11 + q, dt) * ax.l1;
    st_act(out, o + q, t0 * ay.l0 + t1 * ay.l1, dt);
  }
}

// ---- final upsample (deeplab.py:31) + argmax over classes (sky_swap.py:193: first maximum wins) ----
__global__ __launch_bounds__(256) void upsample_argmax_kernel(const float* __restrict__ lg, int n, int h4, int w4,
                                                              int nc, int ncs, int h, int w, uint8_t* __restrict__ pred,
                                                              float* __restrict__ lout) {
  const size_t px = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (px >= (size_t)n * h * w) return;
  const int ox = (int)(px % w), oy = (int)((px / w) % h), img = (int)(px / ((size_t)w * h));
  const AcAxis ay = ac_axis(oy, h4, h), ax = ac_axis(ox, w4, w);
  const size_t b = (size_t)img * h4 * w4;
  const float* p00 = lg + (b + (size_t)ay.i0 * w4 + ax.i0) * ncs;
  const float* p01 = lg + (b + (size_t)ay.i0 * w4 + ax.i1) * ncs;
  const float* p10 = lg + (b + (size_t)ay.i1 * w4 + ax.i0) * ncs;
  const float* p11 = lg + (b + (size_t)ay.i1 * w4 + ax.i1) * ncs;
  float best = 0.f;
  int arg = 0;
  for (int c = 0; c < nc; ++c) {
    const float t0 = p00[c] * ax.l0 + p01[c] * ax.l1;
    const float t1 = p10[c] * ax.l0 + p11[c] * ax.l1;
    const float v = t0 * ay.l0 + t1 * ay.l1;
    if (c == 0 || v > best) {
      best = v;
      arg = c;
    }
    if (lout) lout[(((size_t)img * nc + c) * h + oy) * w + ox] = v;
  }
  if (pred) pred[px] = (uint8_t)arg;
}

__global__ __launch_bounds__(256) void select_kernel(const uint8_t* __restrict__ pred, size_t npix, SegIdSet ids,
                                                     uint8_t* __restrict__ mask) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int c = pred[p];
  mask[p] = ((ids.bits[c >> 5] >> (c & 31)) & 1u) ? 255 : 0;
}

// ---- rectangle morphology (cv2.dilate / cv2.erode with ones(k, k), anchor at the centre, default
// border = ignored): separable, rows then columns ----
__global__ __launch_bounds__(256) void morph_pass_kernel(const uint8_t* __restrict__ in, int n, int h, int w, int k,
                                                         int op, int vertical, uint8_t* __restrict__ out) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (size_t)n * h * w) return;
  const int x = (int)(p % w), y = (int)((p / w) % h);
  const size_t img = p / ((size_t)w * h);
  const int a = k / 2;
  int m = op == 0 ? 0 : 255;
  const int lo = (vertical ? y : x) - a, len = vertical ? h : w;
  for (int i = 0; i < k; ++i) {
    const int q = lo + i;
    if (q < 0 || q >= len) continue;
    const int v = vertical ? in[(img * h + q) * w + x] : in[(img * h + y) * w + q];
    m = op == 0 ? max(m, v) : min(m, v);
  }
  out[p] = (uint8_t)m;
}

// ---- cv2.resize INTER_LINEAR on u8 (OpenCV's fixed-point path: 11-bit taps, horizontal sums as
// int, vertical ((b0*(S0>>4))>>16 + (b1*(S1>>4))>>16 + 2) >> 2) ----
__global__ __launch_bounds__(256) void resize_linear_cv_kernel(const uint8_t* __restrict__ in, int n, int h, int w,
                                                               int c, uint8_t* __restrict__ out, int oh, int ow,
                                                               const int* __restrict__ xofs,
                                                               const short* __restrict__ xa,
                                                               const int* __restrict__ yofs,
                                                               const short* __restrict__ yb) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)n * oh * ow * c) return;
  const int ch = (int)(e % c);
  const size_t px = e / c;
  const int dx = (int)(px % ow), dy = (int)((px / ow) % oh);
  const size_t img = px / ((size_t)ow * oh);
  const int sx = xofs[dx], sx1 = min(sx + 1, w - 1);
  const int a0 = xa[2 * dx], a1 = xa[2 * dx + 1];
  const int sy = yofs[dy];
  const int r0 = min(max(sy, 0), h - 1), r1 = min(max(sy + 1, 0), h - 1);
  const uint8_t* row0 = in + (img * h + r0) * (size_t)w * c;
  const uint8_t* row1 = in + (img * h + r1) * (size_t)w * c;
  const int S0 = row0[sx * c + ch] * a0 + row0[sx1 * c + ch] * a1;
  const int S1 = row1[sx * c + ch] * a0 + row1[sx1 * c + ch] * a1;
  const int b0 = yb[2 * dy], b1 = yb[2 * dy + 1];
  const int v = (((b0 * (S0 >> 4)) >> 16) + ((b1 * (S1 >> 4)) >> 16) + 2) >> 2;
  out[e] = (uint8_t)min(max(v, 0), 255);
}

// ---- Pillow Image.resize(LANCZOS) on RGB (libImaging/Resample.c 8bpc passes: 22-bit integer taps,
// accumulator seeded with 1 << 21, >> 22, clip to 0..255) ----
__device__ __forceinline__ uint8_t clip8_pil(int ss) {
  const int v = ss >> 22;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}
__global__ __launch_bounds__(256) void pil_h_kernel(const uint8_t* __restrict__ in, int h, int w, int y0, int th,
                                                    uint8_t* __restrict__ out, int ow, const int* __restrict__ xb,
                                                    const int* __restrict__ xk, int kx, int n) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (size_t)n * th * ow) return;
  const int xx = (int)(p % ow), yy = (int)((p / ow) % th);
  const size_t img = p / ((size_t)ow * th);
  const int xmin = xb[2 * xx], xmax = xb[2 * xx + 1];
  const int* k = xk + (size_t)xx * kx;
  const uint8_t* row = in + ((img * h) + y0 + yy) * (size_t)w * 3;
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int x = 0; x < xmax; ++x) {
    const uint8_t* q = row + (size_t)(x + xmin) * 3;
    s0 += q[0] * k[x];
    s1 += q[1] * k[x];
    s2 += q[2] * k[x];
  }
  uint8_t* o = out + p * 3;
  o[0] = clip8_pil(s0);
  o[1] = clip8_pil(s1);
  o[2] = clip8_pil(s2);
}
// one source row per block: the row is staged in LDS with coalesced byte loads, then each thread produces output
// pixels of that row from LDS (the per-pixel kernel above re-reads every source byte ~2 * support * scale times
// from global memory: 1080p -> 256 px, 45 taps x 3 byte loads per output).  Same integer arithmetic.
__global__ __launch_bounds__(256) void pil_h_rows_kernel(const uint8_t* __restrict__ in, int h, int w, int y0, int th,
                                                         uint8_t* __restrict__ out, int ow, const int* __restrict__ xb,
                                                         const int* __restrict__ xk, int kx) {
  extern __shared__ uint8_t srow[];
  const int r = blockIdx.x;  // image * th + row
  const int img = r / th, yy = r - img * th;
  const uint8_t* row = in + ((size_t)img * h + y0 + yy) * (size_t)w * 3;
  for (int i = threadIdx.x; i < w * 3; i += blockDim.x) srow[i] = row[i];
  __syncthreads();
  uint8_t* orow = out + (size_t)r * ow * 3;
  for (int xx = threadIdx.x; xx < ow; xx += blockDim.x) {
    const int xmin = xb[2 * xx], xmax = xb[2 * xx + 1];
    const int* k = xk + (size_t)xx * kx;
    const uint8_t* q = srow + xmin * 3;
    int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
    for (int x = 0; x < xmax; ++x) {
      const int kk = k[x];
      s0 += q[3 * x] * kk;
      s1 += q[3 * x + 1] * kk;
      s2 += q[3 * x + 2] * kk;
    }
    orow[3 * xx] = clip8_pil(s0);
    orow[3 * xx + 1] = clip8_pil(s1);
    orow[3 * xx + 2] = clip8_pil(s2);
  }
}
__global__ __launch_bounds__(256) void pil_v_kernel(const uint8_t* __restrict__ in, int h, int w,
                                                    uint8_t* __restrict__ out, int oh, const int* __restrict__ yb,
                                                    const int* __restrict__ yk, int ky, int n) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (size_t)n * oh * w) return;
  const int xx = (int)(p % w), yy = (int)((p / w) % oh);
  const size_t img = p / ((size_t)w * oh);
  const int ymin = yb[2 * yy], ymax = yb[2 * yy + 1];
  const int* k = yk + (size_t)yy * ky;
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int y = 0; y < ymax; ++y) {
    const uint8_t* q = in + ((img * h + ymin + y) * (size_t)w + xx) * 3;
    s0 += q[0] * k[y];
    s1 += q[1] * k[y];
    s2 += q[2] * k[y];
  }
  uint8_t* o = out + p * 3;
  o[0] = clip8_pil(s0);
  o[1] = clip8_pil(s1);
  o[2] = clip8_pil(s2);
}

}  // namespace

hipError_t launch_seg_stem_im2col(int dtype, const void* x, int x_u8, int n, int h, int w, int ho, int wo, int kp,
                                  void* col, hipStream_t st) {
  if (kp < 147 || kp % 8) return hipErrorInvalidValue;
  const size_t total = (size_t)n * ho * wo * (kp / 8);
  hipLaunchKernelGGL(stem_im2col_kernel, dim3(blocks_for(total)), dim3(256), 0, st, x, x_u8, dtype,
                     n, h, w, ho, wo, kp, col);
  return hipGetLastError();
}

hipError_t launch_seg_maxpool(int dtype, const void* in, int n, int h, int w, int c, void* out, int ho, int wo,
                              hipStream_t st) {
  if (c % 8) return hipErrorInvalidValue;
  const size_t total = (size_t)n * ho * wo * (c / 8);
  hipLaunchKernelGGL(maxpool_kernel, dim3(blocks_for(total)), dim3(256), 0, st, in, dtype, n, h,
                     w, c, out, ho, wo);
  return hipGetLastError();
}

hipError_t launch_seg_avgpool(int dtype, const void* in, int n, int hw, int c, int cs, void* out, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_kernel, dim3((unsigned)((c + 63) / 64), (unsigned)n), dim3(256), 0, st, in,
                     dtype, hw, c, cs, out);
  return hipGetLastError();
}

hipError_t launch_seg_resize_ac(int dtype, const void* in, int n, int h, int w, int c, int cs_in, void* out, int oh,
                                int ow, int cs_out, int off, hipStream_t st) {
  if (c % 8 || cs_in % 8 || cs_out % 8 || off % 8) return hipErrorInvalidValue;
  const size_t total = (size_t)n * oh * ow * (c / 8);
  hipLaunchKernelGGL(resize_ac_kernel, dim3(blocks_for(total)), dim3(256), 0, st, in, dtype, n,
                     h, w, c, cs_in, out, oh, ow, cs_out, off);
  return hipGetLastError();
}

hipError_t launch_seg_upsample_argmax(const float* logits, int n, int h4, int w4, int nc, int ncs, int h, int w,
                                      uint8_t* pred, float* logits_out, hipStream_t st) {
  const size_t total = (size_t)n * h * w;
  hipLaunchKernelGGL(upsample_argmax_kernel, dim3(blocks_for(total)), dim3(256), 0, st, logits, n, h4, w4, nc, ncs, h,
                     w, pred, logits_out);
  return hipGetLastError();
}

hipError_t launch_seg_select(const uint8_t* pred, size_t npix, SegIdSet ids, uint8_t* mask, hipStream_t st) {
  hipLaunchKernelGGL(select_kernel, dim3(blocks_for(npix)), dim3(256), 0, st, pred, npix, ids, mask);
  return hipGetLastError();
}

hipError_t launch_seg_morph(const uint8_t* in, int n, int h, int w, int k, int op, uint8_t* tmp, uint8_t* out,
                            hipStream_t st) {
  const size_t total = (size_t)n * h * w;
  hipLaunchKernelGGL(morph_pass_kernel, dim3(blocks_for(total)), dim3(256), 0, st, in, n, h, w, k, op, 0, tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(morph_pass_kernel, dim3(blocks_for(total)), dim3(256), 0, st, (const uint8_t*)tmp, n, h, w, k, op,
                     1, out);
  return hipGetLastError();
}

hipError_t launch_resize_linear_cv_u8(const uint8_t* in, int n, int h, int w, int c, uint8_t* out, int oh, int ow,
                                      const int* xofs, const short* xalpha, const int* yofs, const short* ybeta,
                                      hipStream_t st) {
  const size_t total = (size_t)n * oh * ow * c;
  hipLaunchKernelGGL(resize_linear_cv_kernel, dim3(blocks_for(total)), dim3(256), 0, st, in, n, h, w, c, out, oh, ow,
                     xofs, xalpha, yofs, ybeta);
  return hipGetLastError();
}

hipError_t launch_resize_pil_u8(const uint8_t* in, int n, int h, int w, uint8_t* tmp, int y0, int th, uint8_t* out,
                                int oh, int ow, const int* xb, const int* xk, int kx, const int* yb, const int* yk,
                                int ky, int need_h, int need_v, hipStream_t st) {
  const uint8_t* vsrc = in;
  int vh = h;
  if (need_h) {
    uint8_t* hdst = need_v ? tmp : out;
    const size_t row_b = (size_t)w * 3;
    if (row_b <= 48 * 1024)
      hipLaunchKernelGGL(pil_h_rows_kernel, dim3((unsigned)(n * th)), dim3(256), row_b, st, in, h, w, y0, th, hdst, ow,
                         xb, xk, kx);
    else
      hipLaunchKernelGGL(pil_h_kernel, dim3(blocks_for((size_t)n * th * ow)), dim3(256), 0, st, in, h, w, y0, th, hdst,
                         ow, xb, xk, kx, n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !need_v) return e;
    vsrc = tmp;
    vh = th;
  }
  if (need_v) {
    hipLaunchKernelGGL(pil_v_kernel, dim3(blocks_for((size_t)n * oh * ow)), dim3(256), 0, st, vsrc, vh, ow, out, oh,
                       yb, yk, ky, n);
  }
  return hipGetLastError();
}

}  // namespace nst
