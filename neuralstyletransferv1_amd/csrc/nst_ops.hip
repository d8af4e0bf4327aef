// nst_ops.hip — the non-conv kernels of the hot path: InstanceNorm finalize, residual add,
// output decode + bilinear fit, LAB temporal smoothing, original/mask blend, Gram matrix.
// All fp32 elementwise arithmetic is written op-by-op in the reference's order and the
// library is built with -ffp-contract=off, so no FMA contraction changes a rounding.
#include <algorithm>
#include <cstdlib>

#include "nst_internal.h"
#include "seg_internal.h"
#include "nst_hip.h"
#include "post_common.h"
#include "conv_impl.h"

namespace nst {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// InstanceNorm2d(affine=True, eps=1e-5, track_running_stats=False) statistics:
// per-(n,c) mean and BIASED variance over H*W (transformer_net.py:9 etc; frozen eval
// semantics identical to train for IN).  Reduces the conv epilogue's per-tile partial sums
// in fp64 and emits the affine {scale, shift} the consumer's prologue applies:
//   y = x*scale + shift, scale = gamma/sqrt(var+eps), shift = beta - mean*scale.
// Two deterministic stages (fixed summation order, no atomics):
//   stage 1  grid (n, cstride/CH, nseg), block 256 = CH channels x 256/CH tile phases: each block
//            sums a contiguous segment of tiles in fp64 -> seg[n][s][c] (double2)
//   stage 2  grid (n, cstride/CH), block 256: sums the nseg segments, emits {scale, shift}.
//   (r06: blocks of CH channels x 256/CH phases -- stage 1 CH = 16, stage 2 CH = 4 -- instead of 64 x 4: the 32- and
//   64-channel full-resolution layers kept half of their lanes idle and ran few blocks; the phases of a wave are
//   combined by xor shuffles, the four waves through LDS in wave order: deterministic)
template <int CH>
__global__ __launch_bounds__(256) void in_partial_reduce_kernel(const float* __restrict__ partial, int tiles,
                                                                int cstride, int per_seg,
                                                                double2* __restrict__ seg) {
  constexpr int PH = 256 / CH;
  __shared__ double red[4][CH][2];
  const int n = blockIdx.x, s = blockIdx.z;
  const int cl = threadIdx.x & (CH - 1), q = threadIdx.x / CH;
  const int c = blockIdx.y * CH + cl;
  const int t0 = s * per_seg, t1 = min(tiles, t0 + per_seg);
  double s1 = 0.0, s2 = 0.0;
  if (c < cstride) {
    const float2* p = (const float2*)partial + (size_t)n * tiles * cstride + c;
    int t = t0 + q;
    for (; t + 3 * PH < t1; t += 4 * PH) {
      const float2 a = p[(size_t)t * cstride], b = p[(size_t)(t + PH) * cstride];
      const float2 d = p[(size_t)(t + 2 * PH) * cstride], e = p[(size_t)(t + 3 * PH) * cstride];
      s1 += (double)a.x + (double)b.x + (double)d.x + (double)e.x;
      s2 += (double)a.y + (double)b.y + (double)d.y + (double)e.y;
    }
    for (; t < t1; t += PH) {
      const float2 a = p[(size_t)t * cstride];
      s1 += a.x;
      s2 += a.y;
    }
  }
#pragma unroll
  for (int o = CH; o < 64; o <<= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < CH) {
    red[wv][cl][0] = s1;
    red[wv][cl][1] = s2;
  }
  __syncthreads();
  if (threadIdx.x < CH && c < cstride) {
    s1 = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
    s2 = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
    seg[((size_t)n * gridDim.z + s) * cstride + c] = make_double2(s1, s2);
  }
}

template <int CH>
__global__ __launch_bounds__(256) void in_finalize_kernel(const double2* __restrict__ seg, int nseg, int cstride,
                                                          double count, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, int frn,
                                                          float2* __restrict__ out) {
  // CH channels x 256/CH segment phases per block (the segments' loads in flight together), the wave's phases by
  // xor shuffles, then a fixed-order LDS combine: deterministic
  constexpr int PH = 256 / CH;
  __shared__ double red[4][CH][2];
  const int n = blockIdx.x;
  const int cl = threadIdx.x & (CH - 1), q = threadIdx.x / CH;
  const int c = blockIdx.y * CH + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < cstride) {
    for (int s = q; s < nseg; s += PH) {
      const double2 v = seg[((size_t)n * nseg + s) * cstride + c];
      s1 += v.x;
      s2 += v.y;
    }
  }
#pragma unroll
  for (int o = CH; o < 64; o <<= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < CH) {
    red[wv][cl][0] = s1;
    red[wv][cl][1] = s2;
  }
  __syncthreads();
  if (threadIdx.x >= CH || c >= cstride) return;
  s1 = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
  s2 = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
  // FRN (frn.py:71-74): nu2 = mean(x^2), x * rsqrt(nu2 + |eps|), then weight * x + bias
  const double mean = frn ? 0.0 : s1 / count;
  double var = s2 / count - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  const double rstd = 1.0 / sqrt(var + (double)eps);
  const double scale = (double)gamma[c] * rstd;
  out[(size_t)n * cstride + c] = make_float2((float)scale, (float)((double)beta[c] - mean * scale));
}
constexpr int IN_RED_CH = 16, IN_FIN_CH = 4;

// One-launch form for layers with few tiles per frame (the 270x480 trunk: ~1k): grid (n, cstride/CH), block
// 1024 = CH channels x 1024/CH tile phases, each thread sums tiles phase, phase + 1024/CH, ... in fp64 (all its loads
// in flight), a wave's phases by xor shuffles, the 16 waves through LDS in wave order, then the finalize.
// Deterministic; half the launches of the two-stage form, whose second launch is pure latency at this size.
constexpr int IN_ONE_MAX_TILES = 2048;
template <int CH>
__global__ __launch_bounds__(1024) void in_stats_kernel(const float* __restrict__ partial, int tiles, int cstride,
                                                        double count, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, int frn,
                                                        float2* __restrict__ out) {
  constexpr int PH = 1024 / CH, NL = IN_ONE_MAX_TILES / PH;
  __shared__ double red[16][CH][2];
  const int n = blockIdx.x;
  const int cl = threadIdx.x & (CH - 1), q = threadIdx.x / CH;
  const int c = min(blockIdx.y * CH + cl, cstride - 1);
  const float2* p = (const float2*)partial + (size_t)n * tiles * cstride + c;
  // every load in flight at once: indices clamped into range (always a valid address), the extra ones zeroed after
  float2 v[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) v[k] = p[(size_t)min(q + k * PH, tiles - 1) * cstride];
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const bool in = q + k * PH < tiles;
    s1 += in ? (double)v[k].x : 0.0;
    s2 += in ? (double)v[k].y : 0.0;
  }
  // the wave's 64 / CH tile phases (lanes cl, cl + CH, ...), then the 16 waves in LDS, fixed order
#pragma unroll
  for (int o = CH; o < 64; o <<= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < CH) {
    red[wv][cl][0] = s1;
    red[wv][cl][1] = s2;
  }
  __syncthreads();
  if (threadIdx.x >= CH || blockIdx.y * CH + cl >= cstride) return;
  s1 = red[0][cl][0];
  s2 = red[0][cl][1];
  for (int w = 1; w < 16; ++w) {
    s1 += red[w][cl][0];
    s2 += red[w][cl][1];
  }
  const double mean = frn ? 0.0 : s1 / count;  // FRN: mean(x^2) only (frn.py:71-74)
  double var = s2 / count - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  const double rstd = 1.0 / sqrt(var + (double)eps);
  const double scale = (double)gamma[c] * rstd;
  out[(size_t)n * cstride + c] = make_float2((float)scale, (float)((double)beta[c] - mean * scale));
}

// channels per block of the one-launch form: 4 (r06: 9.2 -> 5.9 µs per trunk layer against 16, four times the
// blocks in flight; `profiles/r06_in_one_ab.txt`); NST_IN_ONE_CH = 2, 8 or 16 for A/B runs
static int in_one_ch() {
  static const int v = [] {
    const char* e = std::getenv("NST_IN_ONE_CH");
    const int x = e ? std::atoi(e) : 4;
    return (x == 2 || x == 8 || x == 16) ? x : 4;
  }();
  return v;
}

int in_finalize_segments(int tiles) { return max(1, min(IN_MAX_SEGMENTS, tiles / 64)); }

// range check (nst_set_range_check): any non-finite value among n floats raises *flag.  An activation outside the
// fp16 range turns into inf in the 16-bit and split modes' operand conversions and then into a non-finite InstanceNorm
// statistic, so the layers' IN tables and the raw output are what is checked
__global__ __launch_bounds__(256) void check_finite_kernel(const float* __restrict__ v, size_t n, int* __restrict__ flag) {
  bool bad = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    bad |= !__builtin_isfinite(v[i]);
  if (bad) atomicOr(flag, 1);
}
hipError_t launch_check_finite(const float* v, size_t n, int* flag, hipStream_t st) {
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(check_finite_kernel, dim3(std::max(1u, blocks)), dim3(256), 0, st, v, n, flag);
  return hipGetLastError();
}

hipError_t launch_in_finalize(const float* partial, int n, int tiles, int cstride, double count,
                              const float* gamma, const float* beta, float eps, int frn, float2* out,
                              void* seg_ws, hipStream_t st) {
  if (tiles <= IN_ONE_MAX_TILES) {
    const int ch = in_one_ch();
    const dim3 grid(n, (cstride + ch - 1) / ch);
    if (ch == 2)
      hipLaunchKernelGGL(in_stats_kernel<2>, grid, dim3(1024), 0, st, partial, tiles, cstride, count, gamma, beta, eps, frn, out);
    else if (ch == 4)
      hipLaunchKernelGGL(in_stats_kernel<4>, grid, dim3(1024), 0, st, partial, tiles, cstride, count, gamma, beta, eps, frn, out);
    else if (ch == 8)
      hipLaunchKernelGGL(in_stats_kernel<8>, grid, dim3(1024), 0, st, partial, tiles, cstride, count, gamma, beta, eps, frn, out);
    else
      hipLaunchKernelGGL(in_stats_kernel<16>, grid, dim3(1024), 0, st, partial, tiles, cstride, count, gamma, beta, eps, frn, out);
    return hipGetLastError();
  }
  const int nseg = in_finalize_segments(tiles);
  const int per_seg = (tiles + nseg - 1) / nseg;
  hipLaunchKernelGGL(in_partial_reduce_kernel<IN_RED_CH>, dim3(n, (cstride + IN_RED_CH - 1) / IN_RED_CH, nseg),
                     dim3(256), 0, st, partial, tiles, cstride, per_seg, (double2*)seg_ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(in_finalize_kernel<IN_FIN_CH>, dim3(n, (cstride + IN_FIN_CH - 1) / IN_FIN_CH), dim3(256), 0, st,
                     (const double2*)seg_ws, nseg, cstride, count, gamma, beta, eps, frn, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Residual add:  out = IN(y) + r  (ResidualBlock.forward, transformer_net.py:71-76 /
// transformer_net_nst.py:138-142), r either materialised or itself IN+ReLU of a raw conv
// output (the first block's input, never materialised); ReCoNet ResLayer applies ReLU after
// the add (model.py:55-60).  16 bytes per thread, NHWC.
// Thread layout: a block covers tpp pixels x CV channel vectors (CV = c / CPC) per sweep, so each
// thread keeps ONE channel vector (its IN constants loaded once) and walks RES_UNROLL pixels with
// all loads issued before use.
constexpr int RES_UNROLL = 4;
template <typename T>
__global__ __launch_bounds__(256) void residual_kernel(const T* __restrict__ y, const float2* __restrict__ ys,
                                                       const T* r, const float2* __restrict__ rs,
                                                       int r_relu, int relu_out, T* out, int hw, int c) {
  constexpr int CPC = 16 / (int)sizeof(T);
  const int cv_n = c / CPC;
  const int tpp = blockDim.x / cv_n;  // pixels per sweep
  const int cv = threadIdx.x % cv_n, pl = threadIdx.x / cv_n;
  const int n = blockIdx.y;
  const int ch0 = cv * CPC;
  float ysc[CPC], ysh[CPC], rsc[CPC], rsh[CPC];
#pragma unroll
  for (int j = 0; j < CPC; ++j) {
    const float2 a = ys[(size_t)n * c + ch0 + j];
    ysc[j] = a.x; ysh[j] = a.y;
    rsc[j] = 1.f; rsh[j] = 0.f;
    if (rs) { const float2 b = rs[(size_t)n * c + ch0 + j]; rsc[j] = b.x; rsh[j] = b.y; }
  }
  const size_t base = (size_t)n * hw * c + ch0;
  const int px0 = blockIdx.x * tpp * RES_UNROLL + pl;
  uint4 va[RES_UNROLL], vb[RES_UNROLL];
#pragma unroll
  for (int u = 0; u < RES_UNROLL; ++u) {
    const int px = px0 + u * tpp;
    if (px < hw) {
      va[u] = *(const uint4*)(y + base + (size_t)px * c);
      vb[u] = *(const uint4*)(r + base + (size_t)px * c);
    }
  }
#pragma unroll
  for (int u = 0; u < RES_UNROLL; ++u) {
    const int px = px0 + u * tpp;
    if (px >= hw) continue;
    float vy[CPC], vr[CPC];
    if constexpr (sizeof(T) == 2) {
      const uint32_t wa[4] = {va[u].x, va[u].y, va[u].z, va[u].w}, wb[4] = {vb[u].x, vb[u].y, vb[u].z, vb[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vy[2 * j] = lo16<T>(wa[j]);
        vy[2 * j + 1] = hi16<T>(wa[j]);
        vr[2 * j] = lo16<T>(wb[j]);
        vr[2 * j + 1] = hi16<T>(wb[j]);
      }
    } else {
      vy[0] = __uint_as_float(va[u].x); vy[1] = __uint_as_float(va[u].y);
      vy[2] = __uint_as_float(va[u].z); vy[3] = __uint_as_float(va[u].w);
      vr[0] = __uint_as_float(vb[u].x); vr[1] = __uint_as_float(vb[u].y);
      vr[2] = __uint_as_float(vb[u].z); vr[3] = __uint_as_float(vb[u].w);
    }
    float o[CPC];
#pragma unroll
    for (int j = 0; j < CPC; ++j) {
      float rr = vr[j];
      if (rs) {
        // as a normalising fill stages it (conv_impl.h norm_chunk): one fma, rounded to T
        if constexpr (sizeof(T) == 2)
          rr = lo16<T>(pack16<T>(__builtin_fmaf(rr, rsc[j], rsh[j]), 0.f));
        else
          rr = rr * rsc[j] + rsh[j];
        if (r_relu) rr = fmaxf(rr, 0.f);
      }
      float v = vy[j] * ysc[j] + ysh[j];
      v = rr + v;
      if (relu_out) v = fmaxf(v, 0.f);
      o[j] = v;
    }
    T* dst = out + base + (size_t)px * c;
    if constexpr (sizeof(T) == 2) {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = pack16<T>(o[2 * j], o[2 * j + 1]);
      *(uint4*)dst = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      *(float4*)dst = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

hipError_t launch_residual(int dtype, const void* y, const float2* ys, const void* r, const float2* rs,
                           int r_relu, int relu_out, void* out, int n, int hw, int c, hipStream_t st) {
  const int cpc = f32_storage(dtype) ? 4 : 8;
  const int cv_n = c / cpc;
  if (c % cpc != 0 || cv_n > 256) return hipErrorInvalidValue;
  const int tpp = 256 / cv_n;
  const dim3 grid((unsigned)((hw + tpp * RES_UNROLL - 1) / (tpp * RES_UNROLL)), (unsigned)n);
  const dim3 block((unsigned)(tpp * cv_n));
  if (dtype == NST_DT_BF16)
    hipLaunchKernelGGL(residual_kernel<__bf16>, grid, block, 0, st, (const __bf16*)y, ys, (const __bf16*)r, rs,
                       r_relu, relu_out, (__bf16*)out, hw, c);
  else if (dtype == NST_DT_F16)
    hipLaunchKernelGGL(residual_kernel<_Float16>, grid, block, 0, st, (const _Float16*)y, ys, (const _Float16*)r, rs,
                       r_relu, relu_out, (_Float16*)out, hw, c);
  else
    hipLaunchKernelGGL(residual_kernel<float>, grid, block, 0, st, (const float*)y, ys, (const float*)r, rs, r_relu,
                       relu_out, (float*)out, hw, c);
  return hipGetLastError();
}

// y, r fp32 -> out fp16, 8 channels per thread (two 16-B loads of each input, one 16-B store); the fp32
// arithmetic of residual_kernel<float> (product, then sum, no contraction), one RNE rounding to fp16
__global__ __launch_bounds__(256) void residual_f32_to_f16_kernel(const float* __restrict__ y, const float2* __restrict__ ys,
                                                                  const float* __restrict__ r, const float2* __restrict__ rs,
                                                                  int r_relu, int relu_out, _Float16* __restrict__ out,
                                                                  int hw, int c) {
  const int cv_n = c / 8;
  const int tpp = blockDim.x / cv_n;
  const int cv = threadIdx.x % cv_n, pl = threadIdx.x / cv_n;
  const int n = blockIdx.y, ch0 = cv * 8;
  float ysc[8], ysh[8], rsc[8], rsh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 a = ys[(size_t)n * c + ch0 + j];
    ysc[j] = a.x; ysh[j] = a.y;
    rsc[j] = 1.f; rsh[j] = 0.f;
    if (rs) { const float2 b = rs[(size_t)n * c + ch0 + j]; rsc[j] = b.x; rsh[j] = b.y; }
  }
  const size_t base = (size_t)n * hw * c + ch0;
  for (int px = blockIdx.x * tpp + pl; px < hw; px += gridDim.x * tpp) {
    const float4* yp = (const float4*)(y + base + (size_t)px * c);
    const float4* rp = (const float4*)(r + base + (size_t)px * c);
    const float4 y0 = yp[0], y1 = yp[1], r0 = rp[0], r1 = rp[1];
    const float vy[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
    const float vr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float o[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        float rr = vr[j + k];
        if (rs) {
          rr = rr * rsc[j + k] + rsh[j + k];
          if (r_relu) rr = fmaxf(rr, 0.f);
        }
        float v = vy[j + k] * ysc[j + k] + ysh[j + k];
        v = rr + v;
        if (relu_out) v = fmaxf(v, 0.f);
        o[k] = v;
      }
      w[j / 2] = pack16<_Float16>(o[0], o[1]);
    }
    *(uint4*)(out + base + (size_t)px * c) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

hipError_t launch_residual_f32_to_f16(const void* y, const float2* ys, const void* r, const float2* rs, int r_relu,
                                      int relu_out, void* out, int n, int hw, int c, hipStream_t st) {
  const int cv_n = c / 8;
  if (c % 8 != 0 || cv_n > 256) return hipErrorInvalidValue;
  const int tpp = 256 / cv_n;
  const int blocks = std::min((hw + tpp - 1) / tpp, 2048);
  hipLaunchKernelGGL(residual_f32_to_f16_kernel, dim3((unsigned)blocks, (unsigned)n), dim3((unsigned)(tpp * cv_n)), 0, st,
                     (const float*)y, ys, (const float*)r, rs, r_relu, relu_out, (_Float16*)out, hw, c);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Output fit: preset decode + clamp(0,1) of the raw model output (pipeline.py:1445-1486),
// bilinear resize to the content size with align_corners=False (pipeline.py:1512-1516,
// PyTorch upsample_bilinear2d index math), ToPILImage truncation to uint8 NHWC.
__global__ __launch_bounds__(256) void decode_resize_kernel(const float* __restrict__ y, int n, int h, int w,
                                                            DecodeConsts d, uint8_t* __restrict__ out,
                                                            int oh, int ow) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)n * oh * ow;
  if (i >= total) return;
  const int ox = (int)(i % ow);
  const int oy = (int)((i / ow) % oh);
  const int b = (int)(i / ((size_t)ow * oh));
  const size_t plane = (size_t)h * w;
  const float* yb = y + (size_t)b * 3 * plane;
  uint8_t* o = out + i * 3;
  if (oh == h && ow == w) {
    const float yy[3] = {yb[(size_t)oy * w + ox], yb[plane + (size_t)oy * w + ox], yb[2 * plane + (size_t)oy * w + ox]};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) o[ch] = (uint8_t)(decode01(yy, ch, d) * 255.0f);
    return;
  }
  const float sh = (float)h / (float)oh, sw = (float)w / (float)ow;
  float fy = sh * ((float)oy + 0.5f) - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  float fx = sw * ((float)ox + 0.5f) - 0.5f;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1;
  const float lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  float c00[3], c01[3], c10[3], c11[3];
  const size_t i00 = (size_t)y0 * w + x0, i01 = (size_t)y0 * w + x1, i10 = (size_t)y1 * w + x0,
               i11 = (size_t)y1 * w + x1;
  float t00[3], t01[3], t10[3], t11[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    t00[ch] = yb[ch * plane + i00];
    t01[ch] = yb[ch * plane + i01];
    t10[ch] = yb[ch * plane + i10];
    t11[ch] = yb[ch * plane + i11];
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    c00[ch] = decode01(t00, ch, d);
    c01[ch] = decode01(t01, ch, d);
    c10[ch] = decode01(t10, ch, d);
    c11[ch] = decode01(t11, ch, d);
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float v = ly0 * (lx0 * c00[ch] + lx1 * c01[ch]) + ly1 * (lx0 * c10[ch] + lx1 * c11[ch]);
    o[ch] = (uint8_t)(v * 255.0f);
  }
}

hipError_t launch_decode_resize_u8(const float* y, int n, int h, int w, const float* p, const float* q,
                                   const float* r, const float* s, const int* perm, uint8_t* out, int oh,
                                   int ow, hipStream_t st) {
  DecodeConsts d;
  for (int c = 0; c < 3; ++c) {
    d.p[c] = p[c]; d.q[c] = q[c]; d.r[c] = r[c]; d.s[c] = s[c]; d.perm[c] = perm[c];
  }
  const size_t total = (size_t)n * oh * ow;
  hipLaunchKernelGGL(decode_resize_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, y, n, h,
                     w, d, out, oh, ow);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Multi-model RGB blend (pipeline.py:1872-1879): out01 = zeros; out01 += w_i * out_i (in slot order);
// clamp(0,1); ToPILImage truncation.  out_i = decode_i(y_i) clamped (each slot's own io_preset),
// fitted bilinearly to the content size like model A's (pipeline.py:1512-1516).
struct ModelSet {
  const float* y[NST_MAX_MODELS];
  DecodeConsts d[NST_MAX_MODELS];
  float w[NST_MAX_MODELS];
  int m;
};

__global__ __launch_bounds__(256) void blend_models_kernel(ModelSet ms, int n, int h, int w, uint8_t* __restrict__ out,
                                                           int oh, int ow) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)n * oh * ow;
  if (i >= total) return;
  const int ox = (int)(i % ow), oy = (int)((i / ow) % oh), b = (int)(i / ((size_t)ow * oh));
  float acc[3] = {0.f, 0.f, 0.f};
  for (int k = 0; k < ms.m; ++k) {
    float v[3];
    decode_fit(ms.y[k] + (size_t)b * 3 * h * w, h, w, ms.d[k], oy, ox, oh, ow, v);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float t = ms.w[k] * v[ch];
      acc[ch] = acc[ch] + t;
    }
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) out[i * 3 + ch] = (uint8_t)(fminf(fmaxf(acc[ch], 0.f), 1.f) * 255.0f);
}

hipError_t launch_blend_models_u8(const float* const* ys, const float (*dp)[3], const float (*dq)[3],
                                  const float (*dr)[3], const float (*ds)[3], const int (*perm)[3], const float* wts,
                                  int m, int n, int h, int w, uint8_t* out, int oh, int ow, hipStream_t st) {
  ModelSet ms;
  ms.m = m;
  for (int k = 0; k < m; ++k) {
    ms.y[k] = ys[k];
    ms.w[k] = wts[k];
    for (int c = 0; c < 3; ++c) {
      ms.d[k].p[c] = dp[k][c]; ms.d[k].q[c] = dq[k][c]; ms.d[k].r[c] = dr[k][c]; ms.d[k].s[c] = ds[k][c];
      ms.d[k].perm[c] = perm[k][c];
    }
  }
  const size_t total = (size_t)n * oh * ow;
  hipLaunchKernelGGL(blend_models_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, ms, n, h, w, out,
                     oh, ow);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// LAB temporal smoothing (pipeline.py:1942-1978): Pillow RGB->LAB, float32 EMA of L (and
// optionally a/b bytes), np.clip(0,255), astype(uint8) truncation, LAB->RGB.  The two
// LittleCMS transforms are exact 2^24-entry LUT gathers (tables made from Pillow itself), held on
// the device as 4-byte entries {x, y, z, 0} so one dword load is one lookup.
// A thread owns 4 consecutive pixels (three aligned dwords of each frame) and walks the batch in
// frame order in chunks of LAB_NF frames: the chunk's loads and rgb->lab gathers are issued
// together (independent across frames), then the sequential EMA (registers only), then the
// lab->rgb gathers and stores together -- three dependent memory rounds per chunk instead of two
// per frame.  The ragged tail (hw % 4) takes the same arithmetic one pixel at a time.
constexpr int LAB_NF = 8;

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[3], int i) {  // byte i of 12 packed bytes
  return (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
}

struct LabEma {
  int sl, sc;
  float a, oma, ca, coma;
  // one pixel, one frame: lab (x = L, y = a, z = b bytes) -> smoothed lab index; state updated
  __device__ __forceinline__ uint32_t step(uint32_t lab, bool seed, float& pL, float& pa, float& pb) const {
    float L = (float)(lab & 0xffu), A = (float)((lab >> 8) & 0xffu), Bc = (float)((lab >> 16) & 0xffu);
    if (sl) {
      if (seed) pL = L;
      const float t0 = a * L;
      const float t1 = oma * pL;
      const float Ls = t0 + t1;
      pL = Ls;
      L = fminf(fmaxf(Ls, 0.f), 255.f);
    }
    if (sc) {
      if (seed) { pa = A; pb = Bc; }
      const float as = ca * A + coma * pa;
      const float bs = ca * Bc + coma * pb;
      pa = as;
      pb = bs;
      A = fminf(fmaxf(as, 0.f), 255.f);
      Bc = fminf(fmaxf(bs, 0.f), 255.f);
    }
    return ((uint32_t)(uint8_t)L << 16) | ((uint32_t)(uint8_t)A << 8) | (uint32_t)(uint8_t)Bc;
  }
};

__global__ __launch_bounds__(256) void lab_ema_kernel(const uint32_t* __restrict__ rgb2lab,
                                                      const uint32_t* __restrict__ lab2rgb, const uint8_t* in,
                                                      uint8_t* out, int n, int hw, LabEma e,
                                                      float* __restrict__ state, int first) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int p0 = 4 * t;
  if (p0 >= hw) return;
  const int np = min(4, hw - p0);
  float pL[4], pa[4], pb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = min(p0 + k, hw - 1);
    pL[k] = e.sl ? state[p] : 0.f;
    pa[k] = e.sc ? state[hw + p] : 0.f;
    pb[k] = e.sc ? state[2 * hw + p] : 0.f;
  }
  if (np == 4 && (hw & 3) == 0) {  // every frame's 4-pixel groups dword-aligned
    for (int f0 = 0; f0 < n; f0 += LAB_NF) {
      const int nf = min(LAB_NF, n - f0);
      uint32_t w[LAB_NF][3], lab[LAB_NF][4];
#pragma unroll
      for (int f = 0; f < LAB_NF; ++f) {
        if (f < nf) {
          const uint32_t* src = (const uint32_t*)(in + ((size_t)(f0 + f) * hw + p0) * 3);
          w[f][0] = src[0]; w[f][1] = src[1]; w[f][2] = src[2];
        }
      }
#pragma unroll
      for (int f = 0; f < LAB_NF; ++f) {
        if (f < nf) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            lab[f][k] = rgb2lab[(byte_of(w[f], 3 * k) << 16) | (byte_of(w[f], 3 * k + 1) << 8) | byte_of(w[f], 3 * k + 2)];
        }
      }
#pragma unroll
      for (int f = 0; f < LAB_NF; ++f) {
        if (f < nf) {
#pragma unroll
          for (int k = 0; k < 4; ++k) lab[f][k] = e.step(lab[f][k], first && f0 + f == 0, pL[k], pa[k], pb[k]);
        }
      }
#pragma unroll
      for (int f = 0; f < LAB_NF; ++f) {
        if (f < nf) {
          uint32_t rgb[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) rgb[k] = lab2rgb[lab[f][k]];
          // 4 pixels x {r, g, b} -> 12 bytes
          uint32_t o[3] = {0u, 0u, 0u};
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const int i = 3 * k + c;
              o[i >> 2] |= ((rgb[k] >> (8 * c)) & 0xffu) << (8 * (i & 3));
            }
          uint32_t* dst = (uint32_t*)(out + ((size_t)(f0 + f) * hw + p0) * 3);
          dst[0] = o[0]; dst[1] = o[1]; dst[2] = o[2];
        }
      }
    }
  } else {
    for (int k = 0; k < np; ++k) {
      for (int f = 0; f < n; ++f) {
        const size_t idx = ((size_t)f * hw + p0 + k) * 3;
        const volatile uint8_t* v = in + idx;  // single bytes (see the note on byte merging below)
        const uint32_t r = v[0], g = v[1], b = v[2];
        const uint32_t li = e.step(rgb2lab[(r << 16) | (g << 8) | b], first && f == 0, pL[k], pa[k], pb[k]);
        const uint32_t rgb = lab2rgb[li];
        out[idx] = (uint8_t)(rgb & 0xffu);
        out[idx + 1] = (uint8_t)((rgb >> 8) & 0xffu);
        out[idx + 2] = (uint8_t)((rgb >> 16) & 0xffu);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < np) {
      if (e.sl) state[p0 + k] = pL[k];
      if (e.sc) { state[hw + p0 + k] = pa[k]; state[2 * hw + p0 + k] = pb[k]; }
    }
  }
}
// Note on byte merging: with ordinary uint8_t loads of adjacent bytes hipcc (ROCm 7.2) once merged
// them into one 16-bit load and shifted the pair left by 16 without masking the upper byte,
// corrupting a 24-bit table index; the tail reads single bytes through volatile pointers, the main
// path extracts bytes from dwords explicitly.

hipError_t launch_lab_ema(const uint32_t* rgb2lab, const uint32_t* lab2rgb, const uint8_t* in, uint8_t* out,
                          int n, int hw, int sl, float a, float oma, int sc, float ca, float coma,
                          float* state, int first, hipStream_t st) {
  const LabEma e{sl, sc, a, oma, ca, coma};
  const int threads = (hw + 3) / 4;
  hipLaunchKernelGGL(lab_ema_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, rgb2lab, lab2rgb,
                     in, out, n, hw, e, state, first);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// The same EMA split in three stages for the --gpus N video pipeline (frames.py): the frame's owner
// extracts the LAB planes the EMA reads (lab_planes_kernel: L, and a / b with chroma smoothing), rank 0
// runs the ordered EMA over those planes alone (lab_ema_planes_kernel: 1-3 bytes per pixel cross xGMI
// instead of the RGB frame), and the owner rebuilds RGB from its own frame with the smoothed planes
// substituted (lab_merge_kernel).  Same tables, same LabEma::step arithmetic: bit-identical to
// lab_ema_kernel.  Planes: uint8 [n][np][hw], np = sl + 2 sc, in the order L, a, b.
__global__ __launch_bounds__(256) void lab_planes_kernel(const uint32_t* __restrict__ rgb2lab, const uint8_t* in,
                                                         uint8_t* __restrict__ planes, int n, int hw, int sl, int sc) {
  const int np = sl + 2 * sc;
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // (frame, 4-pixel group)
  const int groups = (hw + 3) / 4;
  if (q >= (size_t)n * groups) return;
  const int f = (int)(q / groups), p0 = (int)(q % groups) * 4;
  const int cnt = min(4, hw - p0);
  const uint8_t* src = in + ((size_t)f * hw + p0) * 3;
  uint32_t lab[4];
  if (cnt == 4 && (hw & 3) == 0) {
    const uint32_t* s = (const uint32_t*)src;
    const uint32_t w[3] = {s[0], s[1], s[2]};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      lab[k] = rgb2lab[(byte_of(w, 3 * k) << 16) | (byte_of(w, 3 * k + 1) << 8) | byte_of(w, 3 * k + 2)];
  } else {
    const volatile uint8_t* v = src;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      lab[k] = k < cnt ? rgb2lab[((uint32_t)v[3 * k] << 16) | ((uint32_t)v[3 * k + 1] << 8) | (uint32_t)v[3 * k + 2]] : 0u;
  }
  uint8_t* dst = planes + (size_t)f * np * hw + p0;
  int pl = 0;
  for (int c = 0; c < 3; ++c) {
    if (c == 0 ? !sl : !sc) continue;
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) o |= ((lab[k] >> (8 * c)) & 0xffu) << (8 * k);
    uint8_t* d = dst + (size_t)pl * hw;
    if (cnt == 4 && (hw & 3) == 0) {
      *(uint32_t*)d = o;
    } else {
      for (int k = 0; k < cnt; ++k) d[k] = (uint8_t)(o >> (8 * k));
    }
    ++pl;
  }
}

__global__ __launch_bounds__(256) void lab_ema_planes_kernel(const uint8_t* in, uint8_t* out, int n, int hw, LabEma e,
                                                             float* __restrict__ state, int first) {
  const int np = e.sl + 2 * e.sc;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= hw) return;
  float pL = e.sl ? state[p] : 0.f;
  float pa = e.sc ? state[hw + p] : 0.f;
  float pb = e.sc ? state[2 * hw + p] : 0.f;
  for (int f = 0; f < n; ++f) {
    const uint8_t* s = in + (size_t)f * np * hw + p;
    uint32_t lab = 0;
    int pl = 0;
    if (e.sl) lab |= (uint32_t)s[(size_t)(pl++) * hw];
    if (e.sc) {
      lab |= (uint32_t)s[(size_t)(pl++) * hw] << 8;
      lab |= (uint32_t)s[(size_t)(pl++) * hw] << 16;
    }
    const uint32_t li = e.step(lab, first && f == 0, pL, pa, pb);  // (L << 16) | (a << 8) | b
    uint8_t* d = out + (size_t)f * np * hw + p;
    pl = 0;
    if (e.sl) d[(size_t)(pl++) * hw] = (uint8_t)(li >> 16);
    if (e.sc) {
      d[(size_t)(pl++) * hw] = (uint8_t)(li >> 8);
      d[(size_t)(pl++) * hw] = (uint8_t)li;
    }
  }
  if (e.sl) state[p] = pL;
  if (e.sc) { state[hw + p] = pa; state[2 * hw + p] = pb; }
}

__global__ __launch_bounds__(256) void lab_merge_kernel(const uint32_t* __restrict__ rgb2lab,
                                                        const uint32_t* __restrict__ lab2rgb, const uint8_t* in,
                                                        const uint8_t* __restrict__ planes, uint8_t* out, int n,
                                                        int hw, int sl, int sc) {
  const int np = sl + 2 * sc;
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int groups = (hw + 3) / 4;
  if (q >= (size_t)n * groups) return;
  const int f = (int)(q / groups), p0 = (int)(q % groups) * 4;
  const int cnt = min(4, hw - p0);
  const bool vec = cnt == 4 && (hw & 3) == 0;
  const uint8_t* src = in + ((size_t)f * hw + p0) * 3;
  uint32_t lab[4];
  if (vec) {
    const uint32_t* s = (const uint32_t*)src;
    const uint32_t w[3] = {s[0], s[1], s[2]};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      lab[k] = rgb2lab[(byte_of(w, 3 * k) << 16) | (byte_of(w, 3 * k + 1) << 8) | byte_of(w, 3 * k + 2)];
  } else {
    const volatile uint8_t* v = src;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      lab[k] = k < cnt ? rgb2lab[((uint32_t)v[3 * k] << 16) | ((uint32_t)v[3 * k + 1] << 8) | (uint32_t)v[3 * k + 2]] : 0u;
  }
  const uint8_t* pp = planes + (size_t)f * np * hw + p0;
  uint32_t pw[3] = {0u, 0u, 0u};
  for (int pl = 0; pl < np; ++pl) {
    if (vec) {
      pw[pl] = *(const uint32_t*)(pp + (size_t)pl * hw);
    } else {
      for (int k = 0; k < cnt; ++k) pw[pl] |= (uint32_t)pp[(size_t)pl * hw + k] << (8 * k);
    }
  }
  uint32_t rgb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t L = lab[k] & 0xffu, A = (lab[k] >> 8) & 0xffu, B = (lab[k] >> 16) & 0xffu;
    int pl = 0;
    if (sl) L = (pw[pl++] >> (8 * k)) & 0xffu;
    if (sc) {
      A = (pw[pl++] >> (8 * k)) & 0xffu;
      B = (pw[pl++] >> (8 * k)) & 0xffu;
    }
    rgb[k] = lab2rgb[(L << 16) | (A << 8) | B];
  }
  uint8_t* dst = out + ((size_t)f * hw + p0) * 3;
  if (vec) {
    uint32_t o[3] = {0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int i = 3 * k + c;
        o[i >> 2] |= ((rgb[k] >> (8 * c)) & 0xffu) << (8 * (i & 3));
      }
    uint32_t* d = (uint32_t*)dst;
    d[0] = o[0]; d[1] = o[1]; d[2] = o[2];
  } else {
    for (int k = 0; k < cnt; ++k)
      for (int c = 0; c < 3; ++c) dst[3 * k + c] = (uint8_t)((rgb[k] >> (8 * c)) & 0xffu);
  }
}

hipError_t launch_lab_planes(const uint32_t* rgb2lab, const uint8_t* in, uint8_t* planes, int n, int hw, int sl, int sc,
                             hipStream_t st) {
  const size_t threads = (size_t)n * ((hw + 3) / 4);
  hipLaunchKernelGGL(lab_planes_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, rgb2lab, in, planes,
                     n, hw, sl, sc);
  return hipGetLastError();
}

hipError_t launch_lab_ema_planes(const uint8_t* in, uint8_t* out, int n, int hw, int sl, float a, float oma, int sc,
                                 float ca, float coma, float* state, int first, hipStream_t st) {
  const LabEma e{sl, sc, a, oma, ca, coma};
  hipLaunchKernelGGL(lab_ema_planes_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, in, out, n, hw, e,
                     state, first);
  return hipGetLastError();
}

hipError_t launch_lab_merge(const uint32_t* rgb2lab, const uint32_t* lab2rgb, const uint8_t* in, const uint8_t* planes,
                            uint8_t* out, int n, int hw, int sl, int sc, hipStream_t st) {
  const size_t threads = (size_t)n * ((hw + 3) / 4);
  hipLaunchKernelGGL(lab_merge_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, rgb2lab, lab2rgb, in,
                     planes, out, n, hw, sl, sc);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Multi-model LAB blend (pipeline.py:1841-1870): L from model A; a/b = clip(wL*a_A + wab*mix, 0, 255)
// with mix = sum_i w_i * a_i over models B.. in order (float32 accumulation starting from 0), all on
// the raw LAB bytes (Pillow keeps the signed a/b as uint8, so the reference mixes the wrapped
// bytes); astype(uint8) truncation; LAB -> RGB.  Two LittleCMS table gathers per model and pixel.
struct LabBlendArgs {
  const uint8_t* f[NST_MAX_MODELS];  // f[0] = model A's uint8 frame, f[1..] = the others
  float w[NST_MAX_MODELS];           // w[i] multiplies f[i + 1]
};
__global__ __launch_bounds__(256) void lab_blend_kernel(const uint32_t* __restrict__ rgb2lab,
                                                        const uint32_t* __restrict__ lab2rgb, LabBlendArgs a,
                                                        int nrest, float wL, float wab, size_t npix, uint8_t* out) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  auto lab_of = [&](const uint8_t* f, uint32_t& L, uint32_t& A, uint32_t& B) {
    const volatile uint8_t* v = f + p * 3;
    const uint32_t r = v[0], g = v[1], b = v[2];
    const uint32_t lab = rgb2lab[(r << 16) | (g << 8) | b];
    L = lab & 0xffu;
    A = (lab >> 8) & 0xffu;
    B = (lab >> 16) & 0xffu;
  };
  uint32_t La, Aa, Ba;
  lab_of(a.f[0], La, Aa, Ba);
  float am = 0.f, bm = 0.f;
  for (int i = 0; i < nrest; ++i) {
    uint32_t Li, Ai, Bi;
    lab_of(a.f[i + 1], Li, Ai, Bi);
    am = am + a.w[i] * (float)Ai;
    bm = bm + a.w[i] * (float)Bi;
  }
  const float A = fminf(fmaxf(wL * (float)Aa + wab * am, 0.f), 255.f);
  const float B = fminf(fmaxf(wL * (float)Ba + wab * bm, 0.f), 255.f);
  const uint32_t li = (La << 16) | ((uint32_t)(uint8_t)A << 8) | (uint32_t)(uint8_t)B;
  const uint32_t rgb = lab2rgb[li];
  out[p * 3] = (uint8_t)(rgb & 0xffu);
  out[p * 3 + 1] = (uint8_t)((rgb >> 8) & 0xffu);
  out[p * 3 + 2] = (uint8_t)((rgb >> 16) & 0xffu);
}

hipError_t launch_lab_blend(const uint32_t* rgb2lab, const uint32_t* lab2rgb, const uint8_t* const* frames,
                            const float* wrest, int nrest, float wL, float wab, size_t npix, uint8_t* out,
                            hipStream_t st) {
  if (nrest < 0 || nrest + 1 > NST_MAX_MODELS) return hipErrorInvalidValue;
  LabBlendArgs a;
  for (int i = 0; i < NST_MAX_MODELS; ++i) {
    a.f[i] = i <= nrest ? frames[i] : nullptr;
    a.w[i] = i < nrest ? wrest[i] : 0.f;
  }
  hipLaunchKernelGGL(lab_blend_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, rgb2lab, lab2rgb, a,
                     nrest, wL, wab, npix, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Mask feather (pipeline.py:349-351: cv2.GaussianBlur(m, (0, 0), sigmaX = sigmaY = feather_px * 0.5)
// on the uint8 mask), restated from OpenCV's documented semantics: ksize = round(6*sigma + 1) | 1
// for 8-bit data, taps exp(-x^2 / (2 sigma^2)) normalised to 1 (computed in double, as
// getGaussianKernel), separable rows-then-columns, BORDER_REFLECT_101, round to uint8; then
// alpha = m / 255 (pipeline.py:353).  cv2 is not importable here: parity unpinned (OpenCV's 8-bit
// path quantises the taps to fixed point, which can move a rounding boundary by 1 LSB).
constexpr int FEATHER_MAX_R = 1023;
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}
__device__ void feather_taps(float* k, int r, double sigma) {
  __shared__ double part[256];
  double s = 0.0;
  for (int i = threadIdx.x; i <= 2 * r; i += blockDim.x) {
    const double x = (double)(i - r);
    s += exp(-(x * x) / (2.0 * sigma * sigma));
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  const double inv = 1.0 / part[0];
  for (int i = threadIdx.x; i <= 2 * r; i += blockDim.x) {
    const double x = (double)(i - r);
    k[i] = (float)(exp(-(x * x) / (2.0 * sigma * sigma)) * inv);
  }
  __syncthreads();
}
__global__ __launch_bounds__(256) void feather_rows_kernel(const uint8_t* __restrict__ m, int h, int w, int r,
                                                           double sigma, float* __restrict__ tmp) {
  __shared__ float k[2 * FEATHER_MAX_R + 1];
  feather_taps(k, r, sigma);
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  const size_t f = (size_t)blockIdx.z * h * w;
  if (x >= w) return;
  float s = 0.f;
  for (int i = -r; i <= r; ++i) s += k[i + r] * (float)m[f + (size_t)y * w + reflect101(x + i, w)];
  tmp[f + (size_t)y * w + x] = s;
}
__global__ __launch_bounds__(256) void feather_cols_kernel(const float* __restrict__ tmp, int h, int w, int r,
                                                           double sigma, float* __restrict__ alpha,
                                                           uint8_t* __restrict__ out_u8) {
  __shared__ float k[2 * FEATHER_MAX_R + 1];
  feather_taps(k, r, sigma);
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  const size_t f = (size_t)blockIdx.z * h * w;
  if (x >= w) return;
  float s = 0.f;
  for (int i = -r; i <= r; ++i) s += k[i + r] * tmp[f + (size_t)reflect101(y + i, h) * w + x];
  const float u8 = fminf(fmaxf(rintf(s), 0.f), 255.f);  // saturate_cast<uchar>
  if (out_u8) out_u8[f + (size_t)y * w + x] = (uint8_t)u8;  // the blurred mask itself (sky_swap.py:213-215)
  else alpha[f + (size_t)y * w + x] = u8 / 255.0f;
}

int feather_radius(float sigma) {
  const int ksize = ((int)lrint((double)sigma * 6.0 + 1.0)) | 1;
  return ksize / 2;
}

hipError_t launch_mask_feather(const uint8_t* m, int n, int h, int w, float sigma, float* tmp, float* alpha,
                               hipStream_t st) {
  const int r = feather_radius(sigma);
  if (r > FEATHER_MAX_R || !(sigma > 0.f)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)n);
  hipLaunchKernelGGL(feather_rows_kernel, grid, dim3(256), 0, st, m, h, w, r, (double)sigma, tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(feather_cols_kernel, grid, dim3(256), 0, st, tmp, h, w, r, (double)sigma, alpha, nullptr);
  return hipGetLastError();
}

// the same blur with the uint8 result kept (the DeepLab mask's feather, sky_swap.py:213-215)
hipError_t launch_seg_gauss_u8(const uint8_t* m, int n, int h, int w, float sigma, float* tmp, uint8_t* out,
                               hipStream_t st) {
  const int r = feather_radius(sigma);
  if (r > FEATHER_MAX_R || !(sigma > 0.f)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)n);
  hipLaunchKernelGGL(feather_rows_kernel, grid, dim3(256), 0, st, m, h, w, r, (double)sigma, tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(feather_cols_kernel, grid, dim3(256), 0, st, tmp, h, w, r, (double)sigma, nullptr, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Mask composite (pipeline.py:2040-2043) + uniform blend with the original (pipeline.py:2087-2092)
// + ToPILImage truncation.  S = styled/255, O = original/255 (to_tensor).
struct BlendOp {
  const float* mask;
  const uint8_t* mask8;
  int mode;
  float b, omb;
  // one channel value of pixel p: styled byte sv, original byte ov -> output byte
  __device__ __forceinline__ uint32_t operator()(uint32_t sv, uint32_t ov, size_t p) const {
    const float S = (float)sv / 255.0f;
    const float O = (float)ov / 255.0f;
    float C = S;
    if (mask || mask8) {  // alpha = the fp32 mask, or an 8-bit mask read as m / 255 (pipeline.py:353)
      const float al = mask ? mask[p] : (float)mask8[p] / 255.0f;
      const float oal = 1.0f - al;
      const float v = mode == 0 ? (al * S + oal * O) : (oal * S + al * O);
      C = fminf(fmaxf(v, 0.f), 1.f);
    }
    float v = C;
    if (b >= 0.f && b < 1.f) {
      const float t0 = b * C;
      const float t1 = omb * O;
      v = fminf(fmaxf(t0 + t1, 0.f), 1.f);
    }
    return (uint32_t)(uint8_t)(v * 255.0f);
  }
};

__global__ __launch_bounds__(256) void blend1_kernel(const uint8_t* __restrict__ s, const uint8_t* __restrict__ o,
                                                     BlendOp op, uint8_t* out, size_t npix) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) out[p * 3 + ch] = (uint8_t)op(s[p * 3 + ch], o[p * 3 + ch], p);
}

// 4 pixels (12 bytes: three aligned dwords of each frame buffer) per thread; the last ragged pixels one at a time
// (the same per-channel arithmetic either way)
__global__ __launch_bounds__(256) void blend_kernel(const uint8_t* __restrict__ s, const uint8_t* __restrict__ o,
                                                    BlendOp op, uint8_t* out, size_t npix) {
  const size_t p0 = 4 * ((size_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (p0 >= npix) return;
  if (p0 + 4 <= npix) {
    const uint32_t* s4 = (const uint32_t*)(s + p0 * 3);
    const uint32_t* o4 = (const uint32_t*)(o + p0 * 3);
    const uint32_t sw[3] = {s4[0], s4[1], s4[2]}, ow[3] = {o4[0], o4[1], o4[2]};
    uint32_t r[3] = {0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const uint32_t v = op((sw[i >> 2] >> (8 * (i & 3))) & 0xffu, (ow[i >> 2] >> (8 * (i & 3))) & 0xffu, p0 + i / 3);
      r[i >> 2] |= v << (8 * (i & 3));
    }
    uint32_t* d4 = (uint32_t*)(out + p0 * 3);
    d4[0] = r[0]; d4[1] = r[1]; d4[2] = r[2];
    return;
  }
  for (size_t p = p0; p < npix; ++p)
    for (int ch = 0; ch < 3; ++ch) out[p * 3 + ch] = (uint8_t)op(s[p * 3 + ch], o[p * 3 + ch], p);
}

hipError_t launch_blend(const uint8_t* s, const uint8_t* o, const float* mask, int mode, float b, float omb,
                        uint8_t* out, int n, int hw, hipStream_t st, const uint8_t* mask8) {
  const size_t npix = (size_t)n * hw;
  const BlendOp op{mask, mask8, mode, b, omb};
  if (((uintptr_t)s | (uintptr_t)o | (uintptr_t)out) & 3) {  // unaligned buffers: one pixel per thread
    hipLaunchKernelGGL(blend1_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, s, o, op, out, npix);
    return hipGetLastError();
  }
  const size_t threads = (npix + 3) / 4;
  hipLaunchKernelGGL(blend_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, s, o, op, out, npix);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Gram matrix G = F F^T / (c*h*w)  (utils.py:80-83) on MFMA, deterministic.
// F per batch element: [c][hw] (GRAM_CHW, the reference's layout) or [hw][c] (GRAM_HWC, the engine's
// NHWC activations).  Workgroup = one TI x TI tile of G over one K slice (hw range) of KB-pixel
// fills: the fill is staged channel-major in LDS ([row][KB pixels], padded rows: conflict-free
// fragment reads; an HWC fill is transposed on its way in), the next fill prefetched into
// registers during the MFMAs.  8 waves in a 2 x 4 grid of (TI/2) x (TI/4) sub-blocks.  K slices
// write fp32 partial tiles; a second pass sums the slices in fixed order and divides by c*hw (one
// slice: the first pass writes G directly).  No atomics: bit-identical across runs.
template <typename T>
struct GramT;
template <>
struct GramT<__bf16> {
  static constexpr int KM = 32, VEC = 8, KB = 64, RS = 160;  // MFMA K, elements per 16 B, pixels per fill, row bytes
};
template <>
struct GramT<float> {
  static constexpr int KM = 4, VEC = 4, KB = 64, RS = 272;
};

// ds_read_b64_tr_b16 (gfx950): per 16-lane group a 4-row x 16-column block of 16-bit elements, delivered column-major
__device__ __forceinline__ uint2 tr_read16(const char* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
  return __builtin_bit_cast(uint2, v);
}

template <typename T, int TI, bool HWC, bool RELU>
__global__ __launch_bounds__(512) void gram_kernel(const T* __restrict__ F, int c, int hw, int kslice,
                                                   float* __restrict__ out, size_t slice_stride) {
  using GT = GramT<T>;
  constexpr int KB = GT::KB, RS = GT::RS, VEC = GT::VEC, KM = GT::KM;
  constexpr int MI = TI / 32, MJ = TI / 64;                // 16 x 16 fragments per wave
  constexpr int CPS = TI * KB / VEC;                        // 16-B chunks per side and fill
  constexpr int CPT = (CPS + 511) / 512;                    // per thread
  // 16-bit HWC side image: KB pixel rows x TI channels, row pitch = 32 mod 256 bytes, so the 8 rows of a 32-lane
  // half's transposed read (4 per 16-lane group) fall on 8 distinct 8-bank groups
  constexpr int RST = TI * 2 + 32;
  constexpr bool TR = HWC && sizeof(T) == 2;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tt = (c + TI - 1) / TI;
  const int ti = blockIdx.x / tt, tj = blockIdx.x % tt;
  const int b = blockIdx.z;
  const bool diag = ti == tj;
  const int i0 = ti * TI, j0 = tj * TI;
  const int k0 = blockIdx.y * kslice, k1 = min(hw, k0 + kslice);
  const T* Fb = F + (size_t)b * c * hw;
  char* sa = gsm;
  char* sb = diag ? gsm : gsm + (TR ? KB * RST : TI * RS);

  // chunk q of a side: CHW: row q / (KB/VEC), pixels (q % (KB/VEC)) * VEC ..; HWC: pixel q / (TI/VEC),
  // channels (q % (TI/VEC)) * VEC ..
  auto load = [&](int r0, int k, int q) -> uint4 {
    int row, px;
    if constexpr (HWC) { px = q / (TI / VEC); row = (q % (TI / VEC)) * VEC; }
    else { row = q / (KB / VEC); px = (q % (KB / VEC)) * VEC; }
    const int gr = r0 + row, gk = k + px;
    if (q >= CPS || gr >= c || gk >= k1) return make_uint4(0u, 0u, 0u, 0u);  // hw % VEC == 0 (checked)
    const T* src = HWC ? Fb + (size_t)gk * c + gr : Fb + (size_t)gr * hw + gk;
    return *(const uint4*)src;
  };
  auto store = [&](char* side, int q, uint4 v) {
    if (q >= CPS) return;
    if constexpr (RELU) {  // Gram of ReLU(F) (the VGG program stores pre-activations)
      if constexpr (sizeof(T) == 2) {
        typedef short s2 __attribute__((ext_vector_type(2)));
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          w[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, w[j]), (s2){0, 0}));
        v = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        v = make_uint4(__float_as_uint(fmaxf(__uint_as_float(v.x), 0.f)), __float_as_uint(fmaxf(__uint_as_float(v.y), 0.f)),
                       __float_as_uint(fmaxf(__uint_as_float(v.z), 0.f)), __float_as_uint(fmaxf(__uint_as_float(v.w), 0.f)));
      }
    }
    if constexpr (HWC) {
      const int px = q / (TI / VEC), row = (q % (TI / VEC)) * VEC;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      if constexpr (sizeof(T) == 2) {
        // 16-bit HWC: the fill keeps the [pixel][channel] rows (one 16-B write); the fragments are read
        // transposed (ds_read_b64_tr_b16, below)
        *(uint4*)(side + px * RST + row * 2) = v;
        (void)w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) *(uint32_t*)(side + (row + e) * RS + px * 4) = w[e];
      }
    } else {
      const int row = q / (KB / VEC), px = (q % (KB / VEC)) * VEC;
      *(uint4*)(side + row * RS + px * (int)sizeof(T)) = v;
    }
  };

  const int wr = wv >> 2, wc = wv & 3;
  const int ra = wr * (TI / 2), cb = wc * (TI / 4);  // this wave's rows / cols inside the tile
  const int row = lane & 15, g = lane >> 4;
  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int m = 0; m < MI; ++m)
#pragma unroll
    for (int n = 0; n < MJ; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  uint4 pa[CPT], pb[CPT];
#pragma unroll
  for (int t = 0; t < CPT; ++t) {
    pa[t] = load(i0, k0, t * 512 + tid);
    if (!diag) pb[t] = load(j0, k0, t * 512 + tid);
  }
  for (int k = k0; k < k1; k += KB) {
    __syncthreads();  // the previous fill's fragment reads are done
#pragma unroll
    for (int t = 0; t < CPT; ++t) {
      store(sa, t * 512 + tid, pa[t]);
      if (!diag) store(sb, t * 512 + tid, pb[t]);
    }
    __syncthreads();
    if (k + KB < k1) {
#pragma unroll
      for (int t = 0; t < CPT; ++t) {
        pa[t] = load(i0, k + KB, t * 512 + tid);
        if (!diag) pb[t] = load(j0, k + KB, t * 512 + tid);
      }
    }
#pragma unroll
    for (int kk = 0; kk < KB; kk += KM) {
      if constexpr (TR) {
        // transposed reads of the [pixel][channel] image: lane 4q + p of 16-lane group g addresses pixel row
        // kk + 16h + 4g + q, channels c0 + 4p .. +3, and receives channel c0 + (lane & 15) of those 4 pixels.
        // K element e of group g is pixel kk + 16 (e >> 2) + 4g + (e & 3) for both operands (a permutation of
        // the 32 pixels of the step: the same products are summed)
        const int q = (lane & 15) >> 2, pp = lane & 3;
        uint4 fa[MI], fb[MJ];
#pragma unroll
        for (int m = 0; m < MI; ++m) {
          const char* a0 = sa + (kk + 4 * g + q) * RST + (ra + 16 * m + 4 * pp) * 2;
          const uint2 lo = tr_read16(a0), hi = tr_read16(a0 + 16 * RST);
          fa[m] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
#pragma unroll
        for (int n = 0; n < MJ; ++n) {
          const char* b0 = sb + (kk + 4 * g + q) * RST + (cb + 16 * n + 4 * pp) * 2;
          const uint2 lo = tr_read16(b0), hi = tr_read16(b0 + 16 * RST);
          fb[n] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
#pragma unroll
        for (int m = 0; m < MI; ++m)
#pragma unroll
          for (int n = 0; n < MJ; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[m]),
                                                                __builtin_bit_cast(bf16x8_t, fb[n]), acc[m][n], 0, 0, 0);
      } else if constexpr (sizeof(T) == 2) {
        uint4 fa[MI], fb[MJ];
#pragma unroll
        for (int m = 0; m < MI; ++m) fa[m] = *(const uint4*)(sa + (ra + 16 * m + row) * RS + (kk + 8 * g) * 2);
#pragma unroll
        for (int n = 0; n < MJ; ++n) fb[n] = *(const uint4*)(sb + (cb + 16 * n + row) * RS + (kk + 8 * g) * 2);
#pragma unroll
        for (int m = 0; m < MI; ++m)
#pragma unroll
          for (int n = 0; n < MJ; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[m]),
                                                                __builtin_bit_cast(bf16x8_t, fb[n]), acc[m][n], 0, 0, 0);
      } else {
        float fa[MI], fb[MJ];
#pragma unroll
        for (int m = 0; m < MI; ++m) fa[m] = *(const float*)(sa + (ra + 16 * m + row) * RS + (kk + g) * 4);
#pragma unroll
        for (int n = 0; n < MJ; ++n) fb[n] = *(const float*)(sb + (cb + 16 * n + row) * RS + (kk + g) * 4);
#pragma unroll
        for (int m = 0; m < MI; ++m)
#pragma unroll
          for (int n = 0; n < MJ; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[m], fb[n], acc[m][n], 0, 0, 0);
      }
    }
  }
  // C[4g + r][lane & 15] of fragment (m, n): G row i0 + ra + 16m + 4g + r, col j0 + cb + 16n + (lane & 15)
  float* o = out + (size_t)blockIdx.y * slice_stride + (size_t)b * c * c;
#pragma unroll
  for (int m = 0; m < MI; ++m)
#pragma unroll
    for (int n = 0; n < MJ; ++n) {
      const int j = j0 + cb + 16 * n + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + ra + 16 * m + 4 * g + r;
        if (i < c && j < c) o[(size_t)i * c + j] = acc[m][n][r];
      }
    }
}

// G = (sum over the K slices) / (c*hw), in a fixed order (bit-identical across runs): a 1024-thread block owns 64
// consecutive entries; its 16 lane groups each sum a contiguous 1/16 of the slices with four interleaved
// accumulators (independent loads in flight: the slices are read at HBM rate instead of one dependent load at a
// time), combined ((a0 + a1) + (a2 + a3)), then the 16 group sums are added in group order.
// DELTA (the Gatys style loss, vgg_gatys.cpp): also Mb = bf16(k (G - A)) and one partial of sum (G - A)^2 per block
// (a fixed-order xor tree over the block's 64 entries), which launch_vgg_sum_parts adds in block order
template <bool DELTA>
__global__ __launch_bounds__(1024) void gram_reduce_kernel(const float* __restrict__ part, int slices,
                                                           size_t slice_stride, float denom, float* __restrict__ G,
                                                           GramDelta gd) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const size_t e = (size_t)blockIdx.x * 64 + lane;
  const int per = (slices + 15) / 16;
  const int s0 = grp * per, s1 = min(slices, s0 + per);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (e < slice_stride) {
    int sidx = s0;
    for (; sidx + 4 <= s1; sidx += 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += part[(size_t)(sidx + j) * slice_stride + e];
    }
    for (int j = 0; sidx < s1; ++sidx, ++j) a[j] += part[(size_t)sidx * slice_stride + e];
  }
  red[grp][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (grp == 0) {
    float d2 = 0.f;
    if (e < slice_stride) {
      float t = red[0][lane];
      for (int g = 1; g < 16; ++g) t += red[g][lane];
      G[e] = t / denom;
      if constexpr (DELTA) {
        const float d = t / denom - gd.A[e];
        gd.Mb[e] = (__bf16)(gd.k * d);
        d2 = d * d;
      }
    }
    if constexpr (DELTA) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) d2 = d2 + __shfl_xor(d2, o);
      if (lane == 0) gd.parts[blockIdx.x] = d2;
    }
  }
}

// The float4 form (n c^2 % 4 == 0 and 16-byte aligned buffers: every VGG style layer).  A 256-thread block is
// G slice groups x L = 256 / G lanes, each lane owning 4 consecutive entries; group g sums its contiguous share of
// the slices with four interleaved accumulators, the G group sums are added in group order.  The host sizes G so
// that a thread reads at most 8 (16 at G = 32) slices: the 1024-thread, 64-entry blocks of gram_reduce_kernel
// left 12 of 16 groups idle at 4 slices and launched 4,096 blocks for a c = 512 Gram (11.7-13.9 us for 4-16 MiB)
template <int G, bool DELTA>
__global__ __launch_bounds__(256) void gram_reduce4_kernel(const float4* part, int slices, size_t n4,
                                                           float denom, float4* Gout, GramDelta gd) {
  constexpr int L = 256 / G;
  __shared__ float4 red[G > 1 ? G : 1][L];
  __shared__ float wsum[4];
  const int lane = threadIdx.x % L, grp = threadIdx.x / L;
  const size_t e = (size_t)blockIdx.x * L + lane;
  const int per = (slices + G - 1) / G;
  const int s0 = grp * per, s1 = min(slices, s0 + per);
  float4 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n4) {
    int s = s0;
#pragma unroll 2
    for (; s + 4 <= s1; s += 4) {
      float4 x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = part[(size_t)(s + j) * n4 + e];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)  // the tail (static indices: a dynamic a[j] would live in scratch)
      if (s + j < s1) a[j] += part[(size_t)(s + j) * n4 + e];
  }
  float4 t = (a[0] + a[1]) + (a[2] + a[3]);
  if constexpr (G > 1) {
    red[grp][lane] = t;
    __syncthreads();
    if (grp == 0) {
      t = red[0][lane];
#pragma unroll 4
      for (int g = 1; g < G; ++g) t += red[g][lane];
    }
  }
  float d2 = 0.f;
  if (grp == 0 && e < n4) {
    const float4 gv = make_float4(t.x / denom, t.y / denom, t.z / denom, t.w / denom);
    Gout[e] = gv;
    if constexpr (DELTA) {
      const float4 av = ((const float4*)gd.A)[e];
      const float d[4] = {gv.x - av.x, gv.y - av.y, gv.z - av.z, gv.w - av.w};
      __bf16 m[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        m[j] = (__bf16)(gd.k * d[j]);
        d2 += d[j] * d[j];
      }
      *(uint2*)(gd.Mb + 4 * e) = __builtin_bit_cast(uint2, m);
    }
  }
  if constexpr (DELTA) {
    // fixed-order tree: xor within each wave, then the 4 wave sums in wave order
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) d2 = d2 + __shfl_xor(d2, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = d2;
    __syncthreads();
    if (threadIdx.x == 0) gd.parts[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
  }
}

namespace {
struct GramPlan {
  int ti, tt, slices, kslice;
  size_t ws_bytes;
};
// the float4 reduce's slice groups per block (0: the scalar gram_reduce_kernel)
int gram_reduce_groups(size_t slice, int slices) {
  if (slice % 4) return 0;
  int G = 1;
  while (G < 32 && (slices + G - 1) / G > 8) G *= 2;
  while (G > 1 && (slice / 4 + 256 / G - 1) / (256 / G) > (size_t)GRAM_DELTA_MAX_PARTS) G /= 2;
  return G;
}
size_t gram_reduce_blocks(size_t slice, int slices) {
  const int G = gram_reduce_groups(slice, slices);
  return G ? (slice / 4 + 256 / G - 1) / (256 / G) : (slice + 63) / 64;
}
GramPlan gram_plan(int n, int c, int hw) {
  GramPlan g;
  // 128-channel tiles above 64 channels: the 256 tile left a c = 512 Gram with 4 output tiles, so all of its
  // parallelism had to come from split-K partials of 1 MiB each
  g.ti = c <= 64 ? 64 : 128;
  g.tt = (c + g.ti - 1) / g.ti;
  const int blocks = g.tt * g.tt * n;
  const int fills = (hw + 63) / 64;
  // enough K slices to fill the chip (~512 workgroups), but their fp32 partials (c*c*4 B each) no more than
  // four times the bytes of F (bf16) itself: beyond that the split-K traffic costs more than it buys
  static const int capx = [] {
    const char* e = std::getenv("NST_GRAM_CAP");  // tuning sweeps only
    return e ? std::max(1, std::atoi(e)) : 4;
  }();
  const int cap = std::max(1, (int)(((size_t)capx * 2 * hw) / ((size_t)4 * c)));
  g.slices = std::max(1, std::min(std::min(fills, cap), (512 + blocks - 1) / blocks));
  g.kslice = ((fills + g.slices - 1) / g.slices) * 64;
  g.slices = (hw + g.kslice - 1) / g.kslice;
  g.ws_bytes = g.slices > 1 ? (size_t)g.slices * n * c * c * sizeof(float) : 0;
  return g;
}
}  // namespace

size_t gram_workspace_bytes(int n, int c, int hw) { return gram_plan(n, c, hw).ws_bytes; }

int gram_delta_parts(int n, int c, int hw) {
  return (int)gram_reduce_blocks((size_t)n * c * c, gram_plan(n, c, hw).slices);
}

hipError_t launch_gram(const void* F, int dtype, int layout_hwc, int n, int c, int hw, float* G, void* ws,
                       hipStream_t st, int relu, const GramDelta* delta) {
  const GramPlan g = gram_plan(n, c, hw);
  const size_t slice = (size_t)n * c * c;
  const float denom = (float)((double)c * (double)hw);
  float* dst = g.slices > 1 ? (float*)ws : G;  // one slice: the reduce pass divides G in place
  dim3 grid(g.tt * g.tt, g.slices, n);
  const int rs = dtype == NST_DT_BF16 ? GramT<__bf16>::RS : GramT<float>::RS;
  const size_t lds = std::max((size_t)2 * g.ti * rs, (size_t)2 * 64 * (g.ti * 2 + 32));  // CHW / 16-bit HWC images
#define NST_GRAM_GO(T, TI, HWC, RL)                                                                      \
  do {                                                                                                   \
    static const hipError_t attr = hipFuncSetAttribute((const void*)gram_kernel<T, TI, HWC, RL>,        \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
    (void)attr;                                                                                          \
    hipLaunchKernelGGL((gram_kernel<T, TI, HWC, RL>), grid, dim3(512), lds, st, (const T*)F, c, hw, g.kslice, dst, slice); \
  } while (0)
#define NST_GRAM_TI(T, HWC, RL)                      \
  do {                                               \
    if (g.ti == 64) NST_GRAM_GO(T, 64, HWC, RL);     \
    else if (g.ti == 128) NST_GRAM_GO(T, 128, HWC, RL); \
    else NST_GRAM_GO(T, 256, HWC, RL);               \
  } while (0)
  if (dtype == NST_DT_BF16) {
    if (layout_hwc) {
      if (relu) NST_GRAM_TI(__bf16, true, true); else NST_GRAM_TI(__bf16, true, false);
    } else {
      NST_GRAM_TI(__bf16, false, false);
    }
  } else {
    if (layout_hwc) NST_GRAM_TI(float, true, false); else NST_GRAM_TI(float, false, false);
  }
#undef NST_GRAM_TI
#undef NST_GRAM_GO
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  const int rg = (al16(dst) && al16(G) && (!delta || (al16(delta->A) && ((uintptr_t)delta->Mb & 7) == 0)))
                     ? gram_reduce_groups(slice, g.slices) : 0;
  const unsigned nb = (unsigned)(rg ? gram_reduce_blocks(slice, g.slices) : (slice + 63) / 64);
  // the delta mode's loss partials are counted by gram_delta_parts (the float4 reduce): the scalar reduce writes
  // a different number of them, so a caller summing gram_delta_parts() partials would undercount -- refuse it
  if (delta && (!rg || nb != (unsigned)gram_delta_parts(n, c, hw))) return hipErrorInvalidValue;
  if (delta && nb > (unsigned)GRAM_DELTA_MAX_PARTS) return hipErrorInvalidValue;
  if (rg) {
#define NST_GRED4(GG)                                                                                          \
  case GG:                                                                                                     \
    if (delta)                                                                                                 \
      hipLaunchKernelGGL((gram_reduce4_kernel<GG, true>), dim3(nb), dim3(256), 0, st, (const float4*)dst,     \
                         g.slices, slice / 4, denom, (float4*)G, *delta);                                      \
    else                                                                                                       \
      hipLaunchKernelGGL((gram_reduce4_kernel<GG, false>), dim3(nb), dim3(256), 0, st, (const float4*)dst,    \
                         g.slices, slice / 4, denom, (float4*)G, GramDelta{});                                 \
    break;
    switch (rg) {
      NST_GRED4(1) NST_GRED4(2) NST_GRED4(4) NST_GRED4(8) NST_GRED4(16) NST_GRED4(32)
      default: return hipErrorInvalidValue;
    }
#undef NST_GRED4
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return delta && delta->loss_out ? launch_vgg_sum_parts(delta->parts, (int)nb, delta->loss_out, st) : hipSuccess;
  }
  if (delta) {
    hipLaunchKernelGGL(gram_reduce_kernel<true>, dim3(nb), dim3(1024), 0, st, dst, g.slices, slice, denom, G, *delta);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return delta->loss_out ? launch_vgg_sum_parts(delta->parts, (int)nb, delta->loss_out, st) : hipSuccess;
  }
  hipLaunchKernelGGL(gram_reduce_kernel<false>, dim3(nb), dim3(1024), 0, st, dst, g.slices, slice, denom, G, GramDelta{});
  return hipGetLastError();
}

}  // namespace nst
