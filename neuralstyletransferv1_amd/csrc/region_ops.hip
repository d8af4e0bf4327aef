// region_ops.hip — the region-blend compositor (region_blend.py, pipeline.py:1120-1407 / 1720-1839) on the GPU.
//
// Masks are fp32 planes [K][H][W] in HBM (one per region, 8.3 MB each at 1080p), generated from the
// host-drawn geometry (the reference's random.Random draws stay on the host so the same seed gives the
// same regions), feathered by a separable Gaussian, and consumed by two composite kernels that read each
// source pixel once:
//   * full frame (composite_regions / composite_regions_advanced, region_blend.py:1049-1108, 1589-1679):
//     result = sum_k (sum_j w_kj * src_j) * m_k, ws = sum_k m_k, out = clamp(result / max(ws, 1e-6), 0, 1)
//   * crops (composite_from_crops, region_blend.py:2186-2294): the same sum restricted to each region's
//     padded bbox with per-crop styled sources, then the coverage-gap fill (original frame, or iterative
//     max-pool dilation) and the normalisation.
// Sources are raw model outputs decoded with their io_preset and bilinearly fitted on the fly
// (post_common.h decode_fit), so no decoded full-frame copy is materialised.  Every fp32 operation is
// written in the reference's order (the library is built with -ffp-contract=off); the ToPILImage
// truncation (pipeline.py:1943) is fused into the store.
#include <math.h>

#include "region_internal.h"

namespace nst {

enum { RGK_RECTS = 0, RGK_DIAGONAL = 1, RGK_VORONOI = 2, RGK_RADIAL = 3, RGK_WAVES = 4, RGK_SPIRAL = 5,
       RGK_CONCENTRIC = 6 };

// torch.remainder(a, b) for b > 0 (fmod, then moved into [0, b) when the signs differ)
__device__ __forceinline__ float py_mod(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.f && m < 0.f) m = m + b;
  return m;
}

// waves (region_blend.py:404-447): the band coordinate before its min/max normalisation
__device__ __forceinline__ float wave_position(const RegionGeomDev& g, int x, int y, int h, int w) {
  const float yc = (float)y / (float)h, xc = (float)x / (float)w;
  const float two = 2.0f, pi = (float)M_PI;
  if (g.i0 == 0) {  // horizontal
    const float wave = sinf((((xc * g.f0) * two) * pi) + g.f2) * g.f1;
    return yc + wave;
  }
  if (g.i0 == 1) {  // vertical
    const float wave = sinf((((yc * g.f0) * two) * pi) + g.f2) * g.f1;
    return xc + wave;
  }
  const float diag = (xc + yc) / 2.0f;
  const float wave = sinf((((diag * g.f0) * two) * pi) + g.f2) * g.f1;
  return diag + wave;
}

__global__ __launch_bounds__(256) void wave_minmax_kernel(RegionGeomDev g, int h, int w, float* __restrict__ pos,
                                                          float2* __restrict__ part) {
  __shared__ float smin[256], smax[256];
  const size_t hw = (size_t)h * w;
  float mn = INFINITY, mx = -INFINITY;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < hw; i += (size_t)gridDim.x * 256) {
    const float p = wave_position(g, (int)(i % w), (int)(i / w), h, w);
    pos[i] = p;
    mn = fminf(mn, p);
    mx = fmaxf(mx, p);
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = make_float2(smin[0], smax[0]);
}

__global__ __launch_bounds__(256) void wave_minmax_final_kernel(const float2* __restrict__ part, int nb,
                                                                float2* __restrict__ mm) {
  __shared__ float smin[256], smax[256];
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nb; i += 256) {
    mn = fminf(mn, part[i].x);
    mx = fmaxf(mx, part[i].y);
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *mm = make_float2(smin[0], smax[0]);
}

// hard masks of generate_region_masks (feather applied afterwards): each pixel computes its pattern
// coordinate once and writes all K planes; masks k >= n_gen repeat the last region (region_blend.py:977-978)
__global__ __launch_bounds__(256) void region_masks_kernel(RegionGeomDev g, int h, int w,
                                                           const float* __restrict__ wave_pos,
                                                           const float2* __restrict__ wave_mm,
                                                           float* __restrict__ masks) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= hw) return;
  const int x = (int)(i % w), y = (int)(i / w);
  float t = 0.f;   // band coordinate (band modes)
  int nearest = 0; // voronoi
  const float pi = (float)M_PI, two_pi = (float)(2 * M_PI);
  switch (g.kind) {
    case RGK_DIAGONAL: {  // region_blend.py:150-162
      const float d = g.i0 ? (float)x + (float)y : ((float)(w - 1) - (float)x) + (float)y;
      t = d / g.f3;
      break;
    }
    case RGK_VORONOI: {  // region_blend.py:198-228: argmin keeps the first of equal distances
      float best = INFINITY;
      for (int k = 0; k < g.n_gen; ++k) {
        const float dx = (float)x - g.px[k], dy = (float)y - g.py[k];
        float d = sqrtf((dx * dx) + (dy * dy));
        if (g.pdiv[k] != 0.f) d = d / g.pdiv[k];
        if (d < best) { best = d; nearest = k; }
      }
      break;
    }
    case RGK_RADIAL: {  // region_blend.py:384-389
      const float yc = (float)y - (float)g.i1, xc = (float)x - (float)g.i0;
      t = py_mod((atan2f(yc, xc) + pi) + g.f0, two_pi);
      break;
    }
    case RGK_WAVES: {  // region_blend.py:437
      const float2 mm = *wave_mm;
      t = (wave_pos[i] - mm.x) / ((mm.y - mm.x) + 1e-6f);
      break;
    }
    case RGK_SPIRAL: {  // region_blend.py:466-475
      const float yc = (float)y - (float)g.i1, xc = (float)x - (float)g.i0;
      const float r = sqrtf((xc * xc) + (yc * yc));
      const float theta = (atan2f(yc, xc) + pi) + g.f1;
      t = py_mod(theta + ((((r / g.f2) * g.f0) * 2.0f) * pi), two_pi) / two_pi;
      break;
    }
    case RGK_CONCENTRIC: {  // region_blend.py:501-506
      const float yc = (float)y - (float)g.i1, xc = (float)x - (float)g.i0;
      t = sqrtf((xc * xc) + (yc * yc)) / g.f3;
      break;
    }
    default: break;
  }
  for (int k = 0; k < g.count; ++k) {
    const int r = k < g.n_gen ? k : g.n_gen - 1;
    float v;
    if (r < 0) {
      v = 1.f;  // no region generated: torch.ones
    } else if (g.kind == RGK_RECTS) {
      v = (y >= g.rect[r][0] && y < g.rect[r][1] && x >= g.rect[r][2] && x < g.rect[r][3]) ? 1.f : 0.f;
    } else if (g.kind == RGK_VORONOI) {
      v = nearest == r ? 1.f : 0.f;
    } else {
      v = (t >= g.lo[r] && t < g.hi[r]) ? 1.f : 0.f;
    }
    masks[(size_t)k * hw + i] = v;
  }
}

hipError_t launch_region_masks(const RegionGeomDev& g, int h, int w, float* masks, float* scratch, hipStream_t st) {
  const size_t hw = (size_t)h * w;
  float* pos = nullptr;
  float2* mm = nullptr;
  if (g.kind == RGK_WAVES) {  // scratch: hw floats + 1024 float2 partials + the final pair
    pos = scratch;
    float2* part = (float2*)(scratch + ((hw + 3) & ~(size_t)3));
    mm = part + 1024;
    const int nb = (int)std::min<size_t>(1024, (hw + 255) / 256);
    hipLaunchKernelGGL(wave_minmax_kernel, dim3(nb), dim3(256), 0, st, g, h, w, pos, part);
    hipLaunchKernelGGL(wave_minmax_final_kernel, dim3(1), dim3(256), 0, st, part, nb, mm);
  }
  hipLaunchKernelGGL(region_masks_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, g, h, w, pos, mm,
                     masks);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// feather_mask (region_blend.py:69-102): F.pad(reflect) + conv2d with the outer product of the 1-D
// Gaussian taps, computed here as a row pass then a column pass (the taps are the host's fp32 copies of
// the reference's torch taps).  Row tiles of 256 pixels + halo staged in LDS.
struct FeatherTaps {
  int ks;
  float t[RG_MAX_TAPS];
};

__device__ __forceinline__ int reflect101(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - 2 - p : p;
}

__global__ __launch_bounds__(256) void feather_row_kernel(const float* __restrict__ in, int h, int w, FeatherTaps tp,
                                                          float* __restrict__ out) {
  extern __shared__ float row[];  // 256 + ks - 1 entries
  const int pad = tp.ks / 2;
  const size_t plane = (size_t)blockIdx.z * h * w;
  const int y = blockIdx.y, x0 = blockIdx.x * 256;
  const float* src = in + plane + (size_t)y * w;
  for (int j = threadIdx.x; j < 256 + tp.ks - 1; j += 256) {
    const int xs = x0 + j - pad;
    row[j] = (xs < w + pad) ? src[reflect101(xs, w)] : 0.f;
  }
  __syncthreads();
  const int x = x0 + threadIdx.x;
  if (x >= w) return;
  float acc = 0.f;
  for (int j = 0; j < tp.ks; ++j) acc = acc + tp.t[j] * row[threadIdx.x + j];
  out[plane + (size_t)y * w + x] = acc;
}

__global__ __launch_bounds__(256) void feather_col_kernel(const float* __restrict__ in, int h, int w, FeatherTaps tp,
                                                          float* __restrict__ out) {
  const int pad = tp.ks / 2;
  const size_t plane = (size_t)blockIdx.z * h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  float acc = 0.f;
  for (int i = 0; i < tp.ks; ++i) acc = acc + tp.t[i] * in[plane + (size_t)reflect101(y + i - pad, h) * w + x];
  out[plane + (size_t)y * w + x] = acc;
}

hipError_t launch_region_feather(float* masks, int k, int h, int w, const float* taps, int ks, float* scratch,
                                 hipStream_t st) {
  FeatherTaps tp;
  tp.ks = ks;
  for (int i = 0; i < ks; ++i) tp.t[i] = taps[i];
  const dim3 grid((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)k);
  hipLaunchKernelGGL(feather_row_kernel, grid, dim3(256), (256 + ks - 1) * sizeof(float), st, masks, h, w, tp,
                     scratch);
  hipLaunchKernelGGL(feather_col_kernel, grid, dim3(256), 0, st, scratch, h, w, tp, masks);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// rotate_all_masks (region_blend.py:25-66): cv2.warpAffine(m, getRotationMatrix2D((W/2, H/2), angle, 1),
// (W, H), INTER_LINEAR, BORDER_REPLICATE) restated (cv2 is absent here: parity unpinned): the forward
// matrix is inverted (invertAffineTransform), source coordinates in 1/1024 fixed point with per-column
// deltas cvRound(M00*x*1024) and per-row bases, quantised to 1/32 pixel (INTER_BITS 5), bilinear weights
// from the 32x32 float table, taps clamped to the frame.  Then every pixel is normalised by the fp32 sum
// of the rotated masks clamped to 1e-6 (region_blend.py:56-64).
struct Affine {
  double m[6];
};

__global__ __launch_bounds__(256) void rotate_kernel(const float* __restrict__ in, int k, int h, int w, Affine A,
                                                     float* __restrict__ out) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= hw) return;
  const int x = (int)(i % w), y = (int)(i / w);
  const int X0 = (int)rint((A.m[1] * y + A.m[2]) * 1024.0) + 16;
  const int Y0 = (int)rint((A.m[4] * y + A.m[5]) * 1024.0) + 16;
  const int X = (X0 + (int)rint(A.m[0] * x * 1024.0)) >> 5;
  const int Y = (Y0 + (int)rint(A.m[3] * x * 1024.0)) >> 5;
  const int sx = X >> 5, sy = Y >> 5;
  const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
  const float w00 = (1.f - fy) * (1.f - fx), w01 = (1.f - fy) * fx, w10 = fy * (1.f - fx), w11 = fy * fx;
  const int x0 = min(max(sx, 0), w - 1), x1 = min(max(sx + 1, 0), w - 1);
  const int y0 = min(max(sy, 0), h - 1), y1 = min(max(sy + 1, 0), h - 1);
  float r[RG_MAX];
  float sum = 0.f;
  for (int j = 0; j < k; ++j) {
    const float* p = in + (size_t)j * hw;
    const float t0 = p[(size_t)y0 * w + x0] * w00 + p[(size_t)y0 * w + x1] * w01;
    const float t1 = p[(size_t)y1 * w + x0] * w10 + p[(size_t)y1 * w + x1] * w11;
    r[j] = t0 + t1;
    sum = sum + r[j];
  }
  sum = fmaxf(sum, 1e-6f);
  for (int j = 0; j < k; ++j) out[(size_t)j * hw + i] = r[j] / sum;
}

hipError_t launch_region_rotate(const float* in, int k, int h, int w, const double* M, float* out, hipStream_t st) {
  Affine A;
  for (int i = 0; i < 6; ++i) A.m[i] = M[i];
  const size_t hw = (size_t)h * w;
  hipLaunchKernelGGL(rotate_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, in, k, h, w, A, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// compute_mask_bbox (region_blend.py:1969-1994): rows / columns holding a value > threshold.  One block
// per (mask, row) reduces the row; the extremes combine by atomicMin/Max (order-independent results).
// bbox[k] = {x1, y1, x2, y2} exclusive ends, initialised by the launcher to an empty box.
__global__ __launch_bounds__(256) void bbox_kernel(const float* __restrict__ masks, int h, int w, float thr,
                                                   int* __restrict__ bbox) {
  const int k = blockIdx.z, y = blockIdx.y;
  const float* row = masks + ((size_t)k * h + y) * w;
  int xmin = INT_MAX, xmax = -1;
  for (int x = threadIdx.x; x < w; x += 256)
    if (row[x] > thr) { xmin = min(xmin, x); xmax = max(xmax, x); }
  __shared__ int smin[256], smax[256];
  smin[threadIdx.x] = xmin;
  smax[threadIdx.x] = xmax;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = min(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = max(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && smax[0] >= 0) {
    atomicMin(&bbox[4 * k + 0], smin[0]);
    atomicMin(&bbox[4 * k + 1], y);
    atomicMax(&bbox[4 * k + 2], smax[0] + 1);
    atomicMax(&bbox[4 * k + 3], y + 1);
  }
}

__global__ void bbox_init_kernel(int* bbox, int k) {
  const int i = threadIdx.x;
  if (i < k) {
    bbox[4 * i + 0] = INT_MAX; bbox[4 * i + 1] = INT_MAX; bbox[4 * i + 2] = -1; bbox[4 * i + 3] = -1;
  }
}

hipError_t launch_region_bbox(const float* masks, int k, int h, int w, float thr, int* bbox, hipStream_t st) {
  hipLaunchKernelGGL(bbox_init_kernel, dim3(1), dim3(64), 0, st, bbox, k);
  hipLaunchKernelGGL(bbox_kernel, dim3(1, (unsigned)h, (unsigned)k), dim3(256), 0, st, masks, h, w, thr, bbox);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// composites
__device__ __forceinline__ void region_blend_at(const RegionSrcSet& ss, const RegionTermsDev& t, int k, int b,
                                                const uint8_t* __restrict__ orig, size_t opix, int ly, int lx,
                                                int rh, int rw, float* rb) {
  rb[0] = 0.f; rb[1] = 0.f; rb[2] = 0.f;  // region_blend = torch.zeros
  for (int j = 0; j < t.n_terms[k]; ++j) {
    const int s = t.src[k][j];
    float v[3];
    if (s < 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (float)orig[opix * 3 + c] / 255.0f;  // to_tensor
    } else {
      const RegionSrcDev& src = ss.s[s];
      decode_fit(src.y + (size_t)b * 3 * src.h * src.w, src.h, src.w, src.d, ly, lx, rh, rw, v);
    }
    const float wt = t.w[k][j];
#pragma unroll
    for (int c = 0; c < 3; ++c) rb[c] = rb[c] + wt * v[c];
  }
}

__device__ __forceinline__ void store_px(float r0, float r1, float r2, size_t o, uint8_t* out, float* out_f32,
                                         size_t hw, int b) {
  const float r[3] = {r0, r1, r2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = fminf(fmaxf(r[c], 0.f), 1.f);
    if (out) out[o * 3 + c] = (uint8_t)(v * 255.0f);  // ToPILImage: pic.mul(255).byte()
    if (out_f32) out_f32[((size_t)b * 3 + c) * hw + (o - (size_t)b * hw)] = v;
  }
}

// full-frame composite (region_blend.py:1081-1108 / 1634-1679), one thread per pixel
__global__ __launch_bounds__(256) void region_composite_kernel(RegionSrcSet ss, RegionTermsDev t,
                                                               const uint8_t* __restrict__ orig,
                                                               const float* __restrict__ masks, int n, int h, int w,
                                                               uint8_t* __restrict__ out, float* __restrict__ out_f32) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * hw) return;
  const int b = (int)(i / hw);
  const size_t p = i - (size_t)b * hw;
  const int x = (int)(p % w), y = (int)(p / w);
  float res[3] = {0.f, 0.f, 0.f}, ws = 0.f;
  for (int k = 0; k < t.n_regions; ++k) {
    const float m = masks[(size_t)k * hw + p];
    // a zero mask adds rb * 0 = +0 to non-negative sums: skipping it is exact and skips its source reads
    // (the feathered masks are exactly 0 beyond the Gaussian's radius, so most pixels touch one region)
    if (m == 0.f) continue;
    float rb[3];
    region_blend_at(ss, t, k, b, orig, i, y, x, h, w, rb);
#pragma unroll
    for (int c = 0; c < 3; ++c) res[c] = res[c] + rb[c] * m;
    ws = ws + m;
  }
  ws = fmaxf(ws, 1e-6f);
  store_px(res[0] / ws, res[1] / ws, res[2] / ws, i, out, out_f32, hw, b);
}

hipError_t launch_region_composite(const RegionSrcSet& ss, const RegionTermsDev& t, const uint8_t* orig,
                                   const float* masks, int n, int h, int w, uint8_t* out, float* out_f32,
                                   hipStream_t st) {
  const size_t total = (size_t)n * h * w;
  hipLaunchKernelGGL(region_composite_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, ss, t, orig,
                     masks, n, h, w, out, out_f32);
  return hipGetLastError();
}

// composite_from_crops accumulation: canvas [n][4][h][w] = (R, G, B, weight) (region_blend.py:2208-2256)
__global__ __launch_bounds__(256) void crops_accum_kernel(RegionSrcSet ss, RegionTermsDev t,
                                                          const uint8_t* __restrict__ orig,
                                                          const float* __restrict__ masks, int n, int h, int w,
                                                          float* __restrict__ canvas) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * hw) return;
  const int b = (int)(i / hw);
  const size_t p = i - (size_t)b * hw;
  const int x = (int)(p % w), y = (int)(p / w);
  float res[3] = {0.f, 0.f, 0.f}, ws = 0.f;
  for (int k = 0; k < t.n_regions; ++k) {
    const int x1 = t.box[k][0], y1 = t.box[k][1], x2 = t.box[k][2], y2 = t.box[k][3];
    if (x < x1 || x >= x2 || y < y1 || y >= y2) continue;
    const float m = masks[(size_t)k * hw + p];
    if (m == 0.f) continue;  // exact, as in the full-frame composite
    float rb[3];
    region_blend_at(ss, t, k, b, orig, i, y - y1, x - x1, y2 - y1, x2 - x1, rb);
#pragma unroll
    for (int c = 0; c < 3; ++c) res[c] = res[c] + rb[c] * m;
    ws = ws + m;
  }
  float* cv = canvas + (size_t)b * 4 * hw + p;
  cv[0] = res[0]; cv[hw] = res[1]; cv[2 * hw] = res[2]; cv[3 * hw] = ws;
}

// gap fill without an original (region_blend.py:2272-2289): max_pool2d(k, stride 1, pad k/2) of the four
// planes (separable, exact), taken only where weight < 0.1.  The reference stops early once no gap is left;
// a pass with no gap leaves every value unchanged (x*1 + d*0), so all three passes always run.
__global__ __launch_bounds__(256) void gap_rowmax_kernel(const float* __restrict__ cv, int h, int w, int r,
                                                         float* __restrict__ tmp) {
  const size_t plane = (size_t)blockIdx.z * h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const float* row = cv + plane + (size_t)y * w;
  float m = -INFINITY;
  for (int j = max(0, x - r); j <= min(w - 1, x + r); ++j) m = fmaxf(m, row[j]);
  tmp[plane + (size_t)y * w + x] = m;
}

__global__ __launch_bounds__(256) void gap_colmax_select_kernel(const float* __restrict__ cv,
                                                                const float* __restrict__ tmp, int h, int w, int r,
                                                                float* __restrict__ nxt) {
  const size_t hw = (size_t)h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, b = blockIdx.z;
  if (x >= w) return;
  const size_t base = (size_t)b * 4 * hw + (size_t)y * w + x;
  const float gap = cv[base + 3 * hw] < 0.1f ? 1.f : 0.f;
  for (int c = 0; c < 4; ++c) {
    const float* col = tmp + (size_t)b * 4 * hw + (size_t)c * hw + x;
    float m = -INFINITY;
    for (int j = max(0, y - r); j <= min(h - 1, y + r); ++j) m = fmaxf(m, col[(size_t)j * w]);
    const float v = cv[base + (size_t)c * hw];
    nxt[base + (size_t)c * hw] = (v * (1.f - gap)) + (m * gap);
  }
}

__global__ __launch_bounds__(256) void crops_finalize_kernel(const float* __restrict__ canvas,
                                                             const uint8_t* __restrict__ orig, int n, int h, int w,
                                                             uint8_t* __restrict__ out, float* __restrict__ out_f32) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * hw) return;
  const int b = (int)(i / hw);
  const size_t p = i - (size_t)b * hw;
  const float* cv = canvas + (size_t)b * 4 * hw + p;
  float r[3] = {cv[0], cv[hw], cv[2 * hw]}, ws = cv[3 * hw];
  if (orig) {  // region_blend.py:2267-2270: canvas + original * gap, weight + gap
    const float gap = ws < 0.1f ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) r[c] = r[c] + ((float)orig[i * 3 + c] / 255.0f) * gap;
    ws = ws + gap;
  }
  ws = fmaxf(ws, 1e-6f);
  store_px(r[0] / ws, r[1] / ws, r[2] / ws, i, out, out_f32, hw, b);
}

hipError_t launch_region_crops(const RegionSrcSet& ss, const RegionTermsDev& t, const uint8_t* orig,
                               const float* masks, int n, int h, int w, float* canvas, float* tmp, uint8_t* out,
                               float* out_f32, hipStream_t st) {
  const size_t total = (size_t)n * h * w;
  const dim3 g1((unsigned)((total + 255) / 256));
  hipLaunchKernelGGL(crops_accum_kernel, g1, dim3(256), 0, st, ss, t, orig, masks, n, h, w, canvas);
  const float* cur = canvas;
  if (!orig) {
    // canvas -> (tmp: row max) -> second half of tmp (next canvas) -> ... ping-pong through `canvas`
    float* rowmax = tmp;
    float* alt = tmp + total * 4;
    float* bufs[2] = {alt, canvas};
    const int radii[3] = {2, 5, 10};  // kernel sizes 5, 11, 21
    for (int it = 0; it < 3; ++it) {
      const dim3 gr((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)(n * 4));
      hipLaunchKernelGGL(gap_rowmax_kernel, gr, dim3(256), 0, st, cur, h, w, radii[it], rowmax);
      const dim3 gc((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)n);
      float* nxt = bufs[it & 1];
      hipLaunchKernelGGL(gap_colmax_select_kernel, gc, dim3(256), 0, st, cur, rowmax, h, w, radii[it], nxt);
      cur = nxt;
    }
  }
  hipLaunchKernelGGL(crops_finalize_kernel, g1, dim3(256), 0, st, cur, orig, n, h, w, out, out_f32);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// crop input of --region_optimize (pipeline.py:1309-1332): extract_crop of to_tensor(frame), then
// F.interpolate(bilinear, align_corners=False) to the inference size when the region scale is < 1.
// Output: f32 NCHW [n,3,oh,ow] in [0,1] (nst_forward applies the io_preset encode to it).
__global__ __launch_bounds__(256) void crop_input_kernel(const uint8_t* __restrict__ f, int n, int h, int w, int x1,
                                                         int y1, int ch, int cw, int oh, int ow, float* __restrict__ out) {
  const size_t ohw = (size_t)oh * ow;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * ohw) return;
  const int b = (int)(i / ohw);
  const size_t p = i - (size_t)b * ohw;
  const int ox = (int)(p % ow), oy = (int)(p / ow);
  const uint8_t* fb = f + (size_t)b * h * w * 3;
  float v[3];
  if (oh == ch && ow == cw) {
    const size_t s = ((size_t)(y1 + oy) * w + (x1 + ox)) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (float)fb[s + c] / 255.0f;
  } else {
    const float sh = (float)ch / (float)oh, sw = (float)cw / (float)ow;
    float fy = sh * ((float)oy + 0.5f) - 0.5f;
    fy = fy < 0.f ? 0.f : fy;
    float fx = sw * ((float)ox + 0.5f) - 0.5f;
    fx = fx < 0.f ? 0.f : fx;
    const int yy0 = (int)fy, xx0 = (int)fx;
    const int yy1 = yy0 + (yy0 < ch - 1 ? 1 : 0), xx1 = xx0 + (xx0 < cw - 1 ? 1 : 0);
    const float ly1 = fy - (float)yy0, ly0 = 1.f - ly1, lx1 = fx - (float)xx0, lx0 = 1.f - lx1;
    const size_t s00 = ((size_t)(y1 + yy0) * w + (x1 + xx0)) * 3, s01 = ((size_t)(y1 + yy0) * w + (x1 + xx1)) * 3;
    const size_t s10 = ((size_t)(y1 + yy1) * w + (x1 + xx0)) * 3, s11 = ((size_t)(y1 + yy1) * w + (x1 + xx1)) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float c00 = (float)fb[s00 + c] / 255.0f, c01 = (float)fb[s01 + c] / 255.0f;
      const float c10 = (float)fb[s10 + c] / 255.0f, c11 = (float)fb[s11 + c] / 255.0f;
      v[c] = ly0 * (lx0 * c00 + lx1 * c01) + ly1 * (lx0 * c10 + lx1 * c11);
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) out[((size_t)b * 3 + c) * ohw + p] = v[c];
}

hipError_t launch_region_crop_input(const uint8_t* frames, int n, int h, int w, int x1, int y1, int x2, int y2,
                                    int oh, int ow, float* out, hipStream_t st) {
  const size_t total = (size_t)n * oh * ow;
  hipLaunchKernelGGL(crop_input_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, frames, n, h, w, x1,
                     y1, y2 - y1, x2 - x1, oh, ow, out);
  return hipGetLastError();
}

// the pipeline's simulated low-resolution outputs (pipeline.py:1786-1796): the decoded, fitted output
// bilinearly resized to (oh, ow) -> f32 NCHW decoded values (a source with the identity preset)
__global__ __launch_bounds__(256) void resize_src_kernel(RegionSrcDev s, int n, int oh, int ow, int fh, int fw,
                                                         float* __restrict__ out) {
  const size_t ohw = (size_t)oh * ow;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * ohw) return;
  const int b = (int)(i / ohw);
  const size_t p = i - (size_t)b * ohw;
  const int ox = (int)(p % ow), oy = (int)(p / ow);
  const float* yb = s.y + (size_t)b * 3 * s.h * s.w;
  // bilinear over the fitted (fh x fw) decoded image, whose pixels are themselves decode_fit values
  const float sh = (float)fh / (float)oh, sw = (float)fw / (float)ow;
  float fy = sh * ((float)oy + 0.5f) - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  float fx = sw * ((float)ox + 0.5f) - 0.5f;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < fh - 1 ? 1 : 0), x1 = x0 + (x0 < fw - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  float c00[3], c01[3], c10[3], c11[3];
  decode_fit(yb, s.h, s.w, s.d, y0, x0, fh, fw, c00);
  decode_fit(yb, s.h, s.w, s.d, y0, x1, fh, fw, c01);
  decode_fit(yb, s.h, s.w, s.d, y1, x0, fh, fw, c10);
  decode_fit(yb, s.h, s.w, s.d, y1, x1, fh, fw, c11);
#pragma unroll
  for (int c = 0; c < 3; ++c)
    out[((size_t)b * 3 + c) * ohw + p] = ly0 * (lx0 * c00[c] + lx1 * c01[c]) + ly1 * (lx0 * c10[c] + lx1 * c11[c]);
}

hipError_t launch_region_resize_fit(const RegionSrcDev& s, int n, int fh, int fw, int oh, int ow, float* out,
                                    hipStream_t st) {
  const size_t total = (size_t)n * oh * ow;
  hipLaunchKernelGGL(resize_src_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, s, n, oh, ow, fh,
                     fw, out);
  return hipGetLastError();
}

}  // namespace nst

namespace nst {

// ---------------------------------------------------------------------------------------
// --region_morph (warp_all_masks_organic, region_blend.py:535-810).
// Noise fields (_simplex_noise_2d, :604-652): per octave o (two per field) the float64 sum
//   sin(xx*fm + ox) * cos(yy*fm + oy) + sin((xx+yy)*fm*0.7 + ox*0.8)*0.5 + cos((xx-yy)*fm*0.5 + oy*0.6)*0.3
// added into a float32 accumulator (numpy's in-place float32 += float64), xx/yy = linspace(0, frequency, W/H),
// the random offsets drawn on the host from numpy's PCG64 in the reference's order; then / total amplitude and
// the min/max normalisation in float32.  Masks are then remapped (cv2.remap INTER_LINEAR, BORDER_REFLECT,
// restated: 1/32-pixel fixed point from cvRound(map * 32), float weight table) by x + flow_x*max_disp.
struct MorphDev {
  int mode;  // 0 blob, 1 tentacle, 2 wave, 3 pulse
  int k;
  double freq, t, max_disp, step_x, step_y;  // linspace steps of the noise grid (frequency / (n - 1))
  double off[RG_MAX][2][2][2];               // [mask][field x/y][octave][offset x/y]
};

__device__ __forceinline__ double lin(int i, int n, double step, double stop) {
  return i == n - 1 ? stop : (double)i * step;  // numpy.linspace(0, stop, n)
}

__global__ __launch_bounds__(256) void morph_noise_kernel(MorphDev m, int h, int w, float* __restrict__ raw,
                                                          float2* __restrict__ part) {
  __shared__ float smin[256], smax[256];
  const size_t hw = (size_t)h * w;
  const int kf = blockIdx.y;  // mask k, field f
  const int k = kf >> 1, f = kf & 1;
  const double tf = f ? m.t * 1.3 : m.t;  // _generate_flow_field: the y field runs at time_offset * 1.3
  float mn = INFINITY, mx = -INFINITY;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < hw; i += (size_t)gridDim.x * 256) {
    const int x = (int)(i % w), y = (int)(i / w);
    const double xx = lin(x, w, m.step_x, m.freq), yy = lin(y, h, m.step_y, m.freq);
    float acc = 0.f;
    double amp = 1.0, fm = 1.0;
    for (int o = 0; o < 2; ++o) {
      const double ox = tf * (0.5 + 0.3 * o) + m.off[k][f][o][0];
      const double oy = tf * (0.3 + 0.2 * o) + m.off[k][f][o][1];
      double nz = sin(xx * fm + ox) * cos(yy * fm + oy);
      nz = nz + sin((xx + yy) * fm * 0.7 + ox * 0.8) * 0.5;
      nz = nz + cos((xx - yy) * fm * 0.5 + oy * 0.6) * 0.3;
      acc = (float)((double)acc + nz * amp);
      amp *= 0.5;
      fm *= 2.0;
    }
    acc = acc / 1.5f;  // total amplitude 1 + 0.5
    raw[(size_t)kf * hw + i] = acc;
    mn = fminf(mn, acc);
    mx = fmaxf(mx, acc);
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)kf * gridDim.x + blockIdx.x] = make_float2(smin[0], smax[0]);
}

__global__ __launch_bounds__(256) void morph_minmax_kernel(const float2* __restrict__ part, int nb,
                                                           float2* __restrict__ mm) {
  __shared__ float smin[256], smax[256];
  const int kf = blockIdx.x;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nb; i += 256) {
    mn = fminf(mn, part[(size_t)kf * nb + i].x);
    mx = fmaxf(mx, part[(size_t)kf * nb + i].y);
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) mm[kf] = make_float2(smin[0], smax[0]);
}

__device__ __forceinline__ int reflect_cv(int p, int n) {  // cv2 BORDER_REFLECT: fedcba|abcdefgh|hgfedcb
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p - 1 : 2 * n - p - 1;
  return p;
}

// cv2.remap(src, map_x, map_y, INTER_LINEAR, BORDER_REFLECT) at one pixel
__device__ __forceinline__ float remap_reflect(const float* src, int h, int w, float mx, float my) {
  const int X = (int)rintf(mx * 32.f), Y = (int)rintf(my * 32.f);
  const int sx = X >> 5, sy = Y >> 5;
  const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
  const float w00 = (1.f - fy) * (1.f - fx), w01 = (1.f - fy) * fx, w10 = fy * (1.f - fx), w11 = fy * fx;
  const int x0 = reflect_cv(sx, w), x1 = reflect_cv(sx + 1, w), y0 = reflect_cv(sy, h), y1 = reflect_cv(sy + 1, h);
  const float t0 = src[(size_t)y0 * w + x0] * w00 + src[(size_t)y0 * w + x1] * w01;
  const float t1 = src[(size_t)y1 * w + x0] * w10 + src[(size_t)y1 * w + x1] * w11;
  return t0 + t1;
}

__global__ __launch_bounds__(256) void morph_warp_kernel(MorphDev m, const float* __restrict__ in, int h, int w,
                                                         const float* __restrict__ raw, const float2* __restrict__ mm,
                                                         float* __restrict__ out) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= hw) return;
  const int x = (int)(i % w), y = (int)(i / w);
  for (int k = 0; k < m.k; ++k) {
    float mapx, mapy;
    if (m.mode <= 1) {  // blob / tentacle: float32 noise fields
      float fl[2];
      for (int f = 0; f < 2; ++f) {
        const float2 r = mm[2 * k + f];
        const float v = (raw[(size_t)(2 * k + f) * hw + i] - r.x) / ((r.y - r.x) + 1e-6f);
        fl[f] = (v * 2.f) - 1.f;
      }
      if (m.mode == 1) {  // flow_y += sin(linspace(0, 1, H) * pi * 3 + t) * 0.5 (float64, stored float32)
        const double yl = lin(y, h, h > 1 ? 1.0 / (double)(h - 1) : 0.0, 1.0);
        fl[1] = (float)((double)fl[1] + sin(yl * M_PI * 3.0 + m.t) * 0.5);
      }
      const float md = (float)m.max_disp;
      mapx = (float)x + fl[0] * md;
      mapy = (float)y + fl[1] * md;
    } else {  // wave / pulse: float64 fields
      double fx, fy;
      if (m.mode == 2) {
        const double sy = h > 1 ? M_PI * m.freq / (double)(h - 1) : 0.0, sx = w > 1 ? M_PI * m.freq / (double)(w - 1) : 0.0;
        fx = sin(lin(y, h, sy, M_PI * m.freq) + m.t * 2.0);
        fy = cos(lin(x, w, sx, M_PI * m.freq) + m.t * 1.5);
      } else {
        const double yc = (double)(y - h / 2), xc = (double)(x - w / 2);
        const double r = sqrt(xc * xc + yc * yc) + 1e-6, th = atan2(yc, xc);
        const double pu = sin(r * 0.05 - m.t * 3.0) * 0.5 + 0.5;
        fx = cos(th) * pu;
        fy = sin(th) * pu;
      }
      mapx = (float)((double)(float)x + fx * m.max_disp);
      mapy = (float)((double)(float)y + fy * m.max_disp);
    }
    out[(size_t)k * hw + i] = remap_reflect(in + (size_t)k * hw, h, w, mapx, mapy);
  }
}

// gap fill + normalisation of the warped set (region_blend.py:768-810): four max-pool dilations (5, 11, 21,
// 41) applied only where the fp32 sum of the planes is < 0.1 (a pass with no gap changes nothing, so all run),
// then each plane / clamp(sum, 1e-6)
__global__ __launch_bounds__(256) void planes_rowmax_kernel(const float* __restrict__ in, int h, int w, int r,
                                                            float* __restrict__ out) {
  const size_t plane = (size_t)blockIdx.z * h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const float* row = in + plane + (size_t)y * w;
  float m = -INFINITY;
  for (int j = max(0, x - r); j <= min(w - 1, x + r); ++j) m = fmaxf(m, row[j]);
  out[plane + (size_t)y * w + x] = m;
}

__global__ __launch_bounds__(256) void planes_fill_kernel(const float* __restrict__ cur, const float* __restrict__ rmax,
                                                          int k, int h, int w, int r, float* __restrict__ nxt) {
  const size_t hw = (size_t)h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const size_t p = (size_t)y * w + x;
  float s = 0.f;
  for (int j = 0; j < k; ++j) s = s + cur[(size_t)j * hw + p];
  const float gap = s < 0.1f ? 1.f : 0.f;
  for (int j = 0; j < k; ++j) {
    const float* col = rmax + (size_t)j * hw + x;
    float m = -INFINITY;
    for (int q = max(0, y - r); q <= min(h - 1, y + r); ++q) m = fmaxf(m, col[(size_t)q * w]);
    const float v = cur[(size_t)j * hw + p];
    nxt[(size_t)j * hw + p] = (v * (1.f - gap)) + (m * gap);
  }
}

__global__ __launch_bounds__(256) void planes_normalize_kernel(float* __restrict__ m, int k, size_t hw) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= hw) return;
  float s = 0.f;
  for (int j = 0; j < k; ++j) s = s + m[(size_t)j * hw + i];
  s = fmaxf(s, 1e-6f);
  for (int j = 0; j < k; ++j) m[(size_t)j * hw + i] = m[(size_t)j * hw + i] / s;
}

// scratch: 2*k*hw floats (noise) + 2*k*1024 float2 + 2*k float2 + 2*k*hw floats (ping-pong planes)
hipError_t launch_region_morph(const MorphDevHost& mh, const float* in, int h, int w, float* out, float* scratch,
                               hipStream_t st) {
  MorphDev m;
  m.mode = mh.mode; m.k = mh.k; m.freq = mh.freq; m.t = mh.t; m.max_disp = mh.max_disp;
  m.step_x = w > 1 ? mh.freq / (double)(w - 1) : 0.0;
  m.step_y = h > 1 ? mh.freq / (double)(h - 1) : 0.0;
  for (int j = 0; j < mh.k; ++j)
    for (int f = 0; f < 2; ++f)
      for (int o = 0; o < 2; ++o)
        for (int c = 0; c < 2; ++c) m.off[j][f][o][c] = mh.off[j][f][o][c];
  const size_t hw = (size_t)h * w;
  const int k = mh.k;
  float* raw = scratch;
  float2* part = (float2*)(scratch + 2 * (size_t)k * hw);
  float2* mm = part + (size_t)2 * k * 1024;
  float* a = (float*)(mm + 2 * k);
  const int nb = (int)std::min<size_t>(1024, (hw + 255) / 256);
  if (m.mode <= 1) {
    hipLaunchKernelGGL(morph_noise_kernel, dim3(nb, 2 * k), dim3(256), 0, st, m, h, w, raw, part);
    hipLaunchKernelGGL(morph_minmax_kernel, dim3(2 * k), dim3(256), 0, st, part, nb, mm);
  }
  const dim3 g1((unsigned)((hw + 255) / 256));
  hipLaunchKernelGGL(morph_warp_kernel, g1, dim3(256), 0, st, m, in, h, w, raw, mm, out);
  // dilation passes: out -> (raw: row max) -> a -> ... ending in out
  const int radii[4] = {2, 5, 10, 20};
  float* bufs[2] = {a, out};
  const float* cur = out;
  for (int it = 0; it < 4; ++it) {
    hipLaunchKernelGGL(planes_rowmax_kernel, dim3((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)k), dim3(256), 0,
                       st, cur, h, w, radii[it], raw);
    float* nxt = bufs[it & 1];
    hipLaunchKernelGGL(planes_fill_kernel, dim3((unsigned)((w + 255) / 256), (unsigned)h), dim3(256), 0, st, cur, raw,
                       k, h, w, radii[it], nxt);
    cur = nxt;
  }
  hipLaunchKernelGGL(planes_normalize_kernel, g1, dim3(256), 0, st, out, k, hw);
  return hipGetLastError();
}

}  // namespace nst
