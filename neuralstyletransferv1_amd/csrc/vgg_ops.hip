// vgg_ops.hip — the non-conv kernels of the Gatys loop (configs[2], vgg_gatys.cpp): 2x2 max-pool
// forward / backward, ReLU backward with the content-loss gradient, the Gram (style-loss) gradient
// as an MFMA GEMM against the feature map, the loss reductions and the Adam update of the image.
// Activations are bf16 NHWC pre-activations z (the ReLU is applied where they are read); gradients
// are bf16 NHWC, accumulated in fp32 inside each kernel.  Reductions run in a fixed order.
//
// The reference has no VGG / Gatys loop; the pieces follow the usual definitions:
// torchvision VGG-19 features (conv3x3 + ReLU, MaxPool2d(2)), Gram = utils.py:80-83, MSE losses,
// torch.optim.Adam's update rule.
#include <cstdlib>
#include <algorithm>

#include "nst_internal.h"
#include "nst_hip.h"

namespace nst {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t bf_pack(float lo, float hi) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf2));
}
__device__ __forceinline__ void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) { f[2 * j] = bf_lo(w[j]); f[2 * j + 1] = bf_hi(w[j]); }
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(bf_pack(f[0], f[1]), bf_pack(f[2], f[3]), bf_pack(f[4], f[5]), bf_pack(f[6], f[7]));
}

// ---- MaxPool2d(2) of ReLU(z): z [h][w][c] -> out [h/2][w/2][c]; 8 channels per thread ----
__global__ __launch_bounds__(256) void vgg_pool_kernel(const uint4* __restrict__ z, int h, int w, int c,
                                                       uint4* __restrict__ out) {
  const int cv = c / 8, ho = h / 2, wo = w / 2;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)ho * wo * cv) return;
  const int q = (int)(i % cv);
  const size_t px = i / cv;
  const int oy = (int)(px / wo), ox = (int)(px % wo);
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = 0.f;  // ReLU: max(0, window)
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      float f[8];
      unpack8(z[((size_t)(2 * oy + dy) * w + 2 * ox + dx) * cv + q], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
    }
  out[i] = pack8(m);
}

// ---- MaxPool2d backward + ReLU backward: gz[y][x] = gp[y/2][x/2] at the window's first maximum of
// ReLU(z) when z > 0, else 0 (max_pool2d routes the gradient to the first maximum in scan order) ----
__global__ __launch_bounds__(256) void vgg_pool_bwd_kernel(const uint4* __restrict__ z, const uint4* __restrict__ gp,
                                                           int h, int w, int c, uint4* __restrict__ gz) {
  const int cv = c / 8, ho = h / 2, wo = w / 2;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)ho * wo * cv) return;
  const int q = (int)(i % cv);
  const size_t px = i / cv;
  const int oy = (int)(px / wo), ox = (int)(px % wo);
  float v[4][8], g[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) unpack8(z[((size_t)(2 * oy + (k >> 1)) * w + 2 * ox + (k & 1)) * cv + q], v[k]);
  unpack8(gp[i], g);
  float o[4][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float best = fmaxf(v[0][j], 0.f);
    int arg = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float r = fmaxf(v[k][j], 0.f);
      if (r > best) { best = r; arg = k; }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k][j] = (k == arg && v[k][j] > 0.f) ? g[j] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) gz[((size_t)(2 * oy + (k >> 1)) * w + 2 * ox + (k & 1)) * cv + q] = pack8(o[k]);
}

// ---- ReLU backward (+ content gradient): gz = z > 0 ? ga + cw * (ReLU(z) - P) : 0 ----
__global__ __launch_bounds__(256) void vgg_relu_bwd_kernel(const uint4* __restrict__ z, const uint4* __restrict__ ga,
                                                           const uint4* __restrict__ P, float cw, size_t nvec,
                                                           uint4* __restrict__ gz) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  float f[8], g[8], t[8], o[8];
  unpack8(z[i], f);
  unpack8(ga[i], g);
  if (P) unpack8(P[i], t);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = g[j];
    if (P) v = v + cw * (fmaxf(f[j], 0.f) - t[j]);
    o[j] = f[j] > 0.f ? v : 0.f;
  }
  gz[i] = pack8(o);
}

// ---- Gram (style) gradient, fused with the ReLU backward and the other gradient terms:
//   gz[p][i] = z[p][i] > 0 ? ga[p][i] + sum_j ReLU(z[p][j]) M[j][i] + cw * (ReLU(z[p][i]) - P[p][i]) : 0
// M = 4 beta w_l (G - A) / (c^3 hw), symmetric (so row i of M is column i).  MFMA 16x16x32 bf16 with M as the A
// operand (16 channels x 32) and ReLU(z) as B (32 x 16 pixels): lane (pixel, g) ends with 4 consecutive channels of
// one pixel.  Workgroup = 4 waves = 64 pixels x 64 channels, each wave 16 pixels x 64 channels.  The product goes
// through an LDS tile [64 px][64 ch] so the fused epilogue reads z / ga / P and writes gz as whole 16-byte
// chunks (8 channels of a pixel per thread, full 128-B channel runs per pixel), not 2-byte elements.
template <int C>
__global__ __launch_bounds__(256) void vgg_gram_bwd_kernel(const __bf16* __restrict__ z, const __bf16* __restrict__ ga,
                                                           const __bf16* __restrict__ P, float cw,
                                                           const __bf16* __restrict__ Mb, int hw,
                                                           __bf16* __restrict__ gz) {
  constexpr int TP = 64 + 4;  // floats per staged pixel row (16-B pad: the float4 writes of a 16-lane group spread)
  __shared__ __attribute__((aligned(16))) float tile[64 * TP];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int p0 = blockIdx.x * 64 + wv * 16;
  const int i0 = blockIdx.y * 64;
  const int pb = min(p0 + col, hw - 1);  // B column (pixel) of this lane
  f32x4_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // the whole K loop unrolled (C / 32 steps): every step's loads are independent of the MFMAs, so they
  // issue ahead of them instead of one load latency per step
#pragma unroll
  for (int k = 0; k < C; k += 32) {
    float f[8];
    unpack8(*(const uint4*)(z + (size_t)pb * C + k + 8 * g), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    const uint4 b = pack8(f);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint4 a = *(const uint4*)(Mb + (size_t)(i0 + 16 * t + col) * C + k + 8 * g);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                       acc[t], 0, 0, 0);
    }
  }
  // D[16t + 4g + r][col]: channel i0 + 16t + 4g + r of pixel p0 + col
#pragma unroll
  for (int t = 0; t < 4; ++t) *(f32x4_t*)(tile + (wv * 16 + col) * TP + 16 * t + 4 * g) = acc[t];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = k * 256 + threadIdx.x;  // 64 pixels x 8 chunks of 8 channels
    const int pl = q >> 3, cq = q & 7;
    const int p = blockIdx.x * 64 + pl;
    if (p >= hw) continue;
    const size_t o = (size_t)p * C + i0 + 8 * cq;
    float zv[8], gv[8], pv[8], o8[8];
    unpack8(*(const uint4*)(z + o), zv);
    if (ga) unpack8(*(const uint4*)(ga + o), gv);
    if (P) unpack8(*(const uint4*)(P + o), pv);
    const f32x4_t m0 = *(const f32x4_t*)(tile + pl * TP + 8 * cq), m1 = *(const f32x4_t*)(tile + pl * TP + 8 * cq + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = j < 4 ? m0[j] : m1[j - 4];
      if (ga) v = v + gv[j];
      if (P) v = v + cw * (fmaxf(zv[j], 0.f) - pv[j]);
      o8[j] = zv[j] > 0.f ? v : 0.f;
    }
    *(uint4*)(gz + o) = pack8(o8);
  }
}

// The same product with ReLU(z) staged once per workgroup in LDS: wave w owns channels i0 + 16w .. +15 for all 64
// pixels (4 pixel subtiles), reading its 16 rows of M straight from memory and the 64 pixels from LDS.  The form
// above reads the workgroup's 64 rows of M in every wave (4x the M traffic: 64 KiB per wave at C = 512) and leaves
// each lane one dependent load chain per K step; here each M row is read once per workgroup.  Same products, same
// K order per output: bit-identical results
template <int C>
__global__ __launch_bounds__(256) void vgg_gram_bwd_lds_kernel(const __bf16* __restrict__ z, const __bf16* __restrict__ ga,
                                                               const __bf16* __restrict__ P, float cw,
                                                               const __bf16* __restrict__ Mb, int hw,
                                                               __bf16* __restrict__ gz) {
  constexpr int ZS = C * 2 + 16;  // bytes per staged pixel row (16-B pad: a 16-lane group's rows spread over banks)
  constexpr int TP = 64 + 4;      // floats per pixel row of the product tile (aliases the staged rows)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int i0 = blockIdx.y * 64;
  constexpr int CQ = C / 8;  // 16-B chunks per pixel
#pragma unroll
  for (int it = 0; it < 64 * CQ / 256; ++it) {
    const int q = it * 256 + threadIdx.x;
    const int pl = q / CQ, cq = q - pl * CQ;
    const int p = blockIdx.x * 64 + pl;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (p < hw) {
      float f[8];
      unpack8(*(const uint4*)(z + (size_t)p * C + 8 * cq), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
      v = pack8(f);
    }
    *(uint4*)(smem + pl * ZS + 16 * cq) = v;
  }
  __syncthreads();
  f32x4_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const __bf16* mrow = Mb + (size_t)(i0 + 16 * wv + col) * C + 8 * g;
#pragma unroll
  for (int k = 0; k < C; k += 32) {
    const uint4 a = *(const uint4*)(mrow + k);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint4 b = *(const uint4*)(smem + (16 * t + col) * ZS + (k + 8 * g) * 2);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                       acc[t], 0, 0, 0);
    }
  }
  __syncthreads();  // the staged rows are dead: the product tile reuses the space
  float* tile = (float*)smem;
  // D[4g + r][col] of subtile t: channel i0 + 16 wv + 4g + r of pixel 16t + col
#pragma unroll
  for (int t = 0; t < 4; ++t) *(f32x4_t*)(tile + (16 * t + col) * TP + 16 * wv + 4 * g) = acc[t];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = k * 256 + threadIdx.x;  // 64 pixels x 8 chunks of 8 channels
    const int pl = q >> 3, cq = q & 7;
    const int p = blockIdx.x * 64 + pl;
    if (p >= hw) continue;
    const size_t o = (size_t)p * C + i0 + 8 * cq;
    float zv[8], gv[8], pv[8], o8[8];
    unpack8(*(const uint4*)(z + o), zv);
    if (ga) unpack8(*(const uint4*)(ga + o), gv);
    if (P) unpack8(*(const uint4*)(P + o), pv);
    const f32x4_t m0 = *(const f32x4_t*)(tile + pl * TP + 8 * cq), m1 = *(const f32x4_t*)(tile + pl * TP + 8 * cq + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = j < 4 ? m0[j] : m1[j - 4];
      if (ga) v = v + gv[j];
      if (P) v = v + cw * (fmaxf(zv[j], 0.f) - pv[j]);
      o8[j] = zv[j] > 0.f ? v : 0.f;
    }
    *(uint4*)(gz + o) = pack8(o8);
  }
}
template <int C>
constexpr size_t gram_bwd_lds_bytes() {
  return std::max((size_t)64 * (C * 2 + 16), (size_t)64 * 68 * 4);
}

// ---- block partials summed in block order (deterministic): the style loss (gram_reduce_kernel<true>) and the
// content loss ----
__global__ __launch_bounds__(256) void vgg_sum_parts_kernel(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s = s + part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

// ---- content loss: partial sums of (ReLU(z) - P)^2 per block, then one block sums them ----
__global__ __launch_bounds__(256) void vgg_content_partial_kernel(const uint4* __restrict__ z, const uint4* __restrict__ P,
                                                                  size_t nvec, float* __restrict__ part) {
  __shared__ float red[256];
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
    float f[8], t[8];
    unpack8(z[i], f);
    unpack8(P[i], t);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = fmaxf(f[j], 0.f) - t[j];
      s = s + d * d;
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// losses[0] = total, [1] = content = alpha * mean, [2] = style = beta * sum_l w_l * mean_l
struct LossArgs {
  float cscale;          // alpha / numel(content features)
  float sscale[5];       // beta * w_l / c_l^2
  int snparts[5];        // spart: each style layer's Gram-reduce block partials (vgg_sum_parts_kernel's sums)
  int sstride;
};
// spart: the style layers' raw sums are summed here from their block partials (one launch instead of one
// vgg_sum_parts_kernel per layer, the same fixed-order arithmetic) and written to style_raw; else style_raw is read
__global__ __launch_bounds__(256) void vgg_loss_final_kernel(const float* __restrict__ part, int nparts,
                                                             const float* __restrict__ spart, float* __restrict__ style_raw,
                                                             LossArgs a, float* __restrict__ losses) {
  __shared__ float red[256];
  if (spart != nullptr) {
    for (int l = 0; l < 5; ++l) {
      float s = 0.f;
      for (int i = threadIdx.x; i < a.snparts[l]; i += 256) s = s + spart[l * a.sstride + i];
      red[threadIdx.x] = s;
      __syncthreads();
      for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
        __syncthreads();
      }
      if (threadIdx.x == 0) style_raw[l] = red[0];
      __syncthreads();
    }
  }
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s = s + part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float lc = a.cscale * red[0];
    float ls = 0.f;
    for (int l = 0; l < 5; ++l) ls = ls + a.sscale[l] * style_raw[l];
    losses[0] = lc + ls;
    losses[1] = lc;
    losses[2] = ls;
  }
}

// ---- Adam on the image (torch.optim.Adam, no weight decay): the gradient arrives with respect to
// the normalised image (conv1_1's input); d/dx = g / std[c].  Optional clamp to [0, 1] ----
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ x, const float* __restrict__ gn,
                                                   float* __restrict__ m, float* __restrict__ v, int hw, int n,
                                                   float3 inv_std, float lr, float b1, float b2, float eps,
                                                   float bc1, float bc2, int clamp01) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int ch = (i / hw) % 3;
  const float g = gn[i] * (ch == 0 ? inv_std.x : (ch == 1 ? inv_std.y : inv_std.z));
  const float mi = b1 * m[i] + (1.f - b1) * g;
  const float vi = b2 * v[i] + (1.f - b2) * g * g;
  m[i] = mi;
  v[i] = vi;
  const float mh = mi / bc1, vh = vi / bc2;
  float xi = x[i] - lr * mh / (sqrtf(vh) + eps);
  if (clamp01) xi = fminf(fmaxf(xi, 0.f), 1.f);
  x[i] = xi;
}

hipError_t launch_vgg_pool(const void* z, int h, int w, int c, void* out, hipStream_t st) {
  const size_t n = (size_t)(h / 2) * (w / 2) * (c / 8);
  hipLaunchKernelGGL(vgg_pool_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const uint4*)z, h, w, c,
                     (uint4*)out);
  return hipGetLastError();
}
hipError_t launch_vgg_pool_bwd(const void* z, const void* gp, int h, int w, int c, void* gz, hipStream_t st) {
  const size_t n = (size_t)(h / 2) * (w / 2) * (c / 8);
  hipLaunchKernelGGL(vgg_pool_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const uint4*)z,
                     (const uint4*)gp, h, w, c, (uint4*)gz);
  return hipGetLastError();
}
hipError_t launch_vgg_relu_bwd(const void* z, const void* ga, const void* P, float cw, size_t elems, void* gz,
                               hipStream_t st) {
  const size_t n = elems / 8;
  hipLaunchKernelGGL(vgg_relu_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const uint4*)z,
                     (const uint4*)ga, (const uint4*)P, cw, n, (uint4*)gz);
  return hipGetLastError();
}
hipError_t launch_vgg_gram_bwd(const void* z, const void* ga, const void* P, float cw, const void* Mb, int hw, int c,
                               void* gz, hipStream_t st) {
  const dim3 grid((unsigned)((hw + 63) / 64), (unsigned)(c / 64));
  const __bf16 *zz = (const __bf16*)z, *gg = (const __bf16*)ga, *pp = (const __bf16*)P, *mm = (const __bf16*)Mb;
  __bf16* out = (__bf16*)gz;
  static const bool lds = [] {
    const char* e = std::getenv("NST_GRAM_BWD_LDS");  // A/B switch: 0 = the register form
    return !e || std::atoi(e) != 0;
  }();
#define NST_GBWD_LDS(CC)                                                                                        \
  case CC: {                                                                                                    \
    static const hipError_t attr = hipFuncSetAttribute((const void*)vgg_gram_bwd_lds_kernel<CC>,               \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
    (void)attr;                                                                                                 \
    hipLaunchKernelGGL(vgg_gram_bwd_lds_kernel<CC>, grid, dim3(256), gram_bwd_lds_bytes<CC>(), st, zz, gg, pp, cw, \
                       mm, hw, out);                                                                            \
    return hipGetLastError();                                                                                   \
  }
  if (lds) {
    switch (c) {
      NST_GBWD_LDS(64) NST_GBWD_LDS(128) NST_GBWD_LDS(256) NST_GBWD_LDS(512)
      default: return hipErrorInvalidValue;
    }
  }
#undef NST_GBWD_LDS
  switch (c) {
    case 64: hipLaunchKernelGGL(vgg_gram_bwd_kernel<64>, grid, dim3(256), 0, st, zz, gg, pp, cw, mm, hw, out); break;
    case 128: hipLaunchKernelGGL(vgg_gram_bwd_kernel<128>, grid, dim3(256), 0, st, zz, gg, pp, cw, mm, hw, out); break;
    case 256: hipLaunchKernelGGL(vgg_gram_bwd_kernel<256>, grid, dim3(256), 0, st, zz, gg, pp, cw, mm, hw, out); break;
    case 512: hipLaunchKernelGGL(vgg_gram_bwd_kernel<512>, grid, dim3(256), 0, st, zz, gg, pp, cw, mm, hw, out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_vgg_sum_parts(const float* parts, int n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(vgg_sum_parts_kernel, dim3(1), dim3(256), 0, st, parts, n, out);
  return hipGetLastError();
}
int vgg_content_parts(size_t elems) { return (int)std::min<size_t>(512, (elems / 8 + 255) / 256); }
hipError_t launch_vgg_losses(const void* z, const void* P, size_t elems, float* part, float* style_raw,
                             float cscale, const float* sscale, float* losses, hipStream_t st, const float* spart,
                             const int* snparts, int sstride) {
  const int parts = vgg_content_parts(elems);
  hipLaunchKernelGGL(vgg_content_partial_kernel, dim3(parts), dim3(256), 0, st, (const uint4*)z, (const uint4*)P,
                     elems / 8, part);
  LossArgs a;
  a.cscale = cscale;
  for (int l = 0; l < 5; ++l) {
    a.sscale[l] = sscale[l];
    a.snparts[l] = spart ? snparts[l] : 0;
  }
  a.sstride = sstride;
  hipLaunchKernelGGL(vgg_loss_final_kernel, dim3(1), dim3(256), 0, st, part, parts, spart, style_raw, a, losses);
  return hipGetLastError();
}
hipError_t launch_adam(float* x, const float* g, float* m, float* v, int hw, int n, const float* inv_std, float lr,
                       float b1, float b2, float eps, float bc1, float bc2, int clamp01, hipStream_t st) {
  const float3 is = make_float3(inv_std[0], inv_std[1], inv_std[2]);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, g, m, v, hw, n, is, lr, b1,
                     b2, eps, bc1, bc2, clamp01);
  return hipGetLastError();
}

}  // namespace nst
