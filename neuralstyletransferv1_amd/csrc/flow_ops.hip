// flow_ops.hip — the temporal stage of the frame loop (pipeline.py:1884-1940 --flow_ema, :2072-2086
// --motion_blend) on the GPU:
//   * grayscale of the content frame (pipeline.py:1100 pil_rgb.convert("L"): Pillow's integer luma)
//   * dense optical flow cv2.calcOpticalFlowFarneback(prev, next, None, 0.5, 3, 15, 3, 5, 1.1, 0) restated
//     after OpenCV's optflowgf.cpp (cv2 is not installed here: parity unpinned): per pyramid level the
//     images are Gaussian-smoothed and resized, expanded into quadratic polynomials (FarnebackPolyExp,
//     separable 1-D Gaussian-weighted moments, n = 5, sigma = 1.1), then `iterations` rounds of
//     UpdateMatrices + a 15 x 15 box blur of the 5 matrix fields + the 2x2 solve; coarse-to-fine with the
//     flow resized x 1/pyr_scale between levels;
//   * the flow-guided EMA: prev styled frame warped by cv2.remap(INTER_LINEAR, BORDER_REPLICATE) of
//     grid + flow (restated), fused = clip(a * curr + (1 - a) * warped);
//   * the motion-adaptive blend alpha: clip(|flow| / 8) blurred (cv2.GaussianBlur sigma 3), then
//     max_alpha - (max_alpha - min_alpha) * m.
// One thread per output element throughout; all planes fp32 in HBM (the box sums in fp64, as OpenCV).
#include <cfloat>
#include <math.h>

#include <algorithm>

#include "flow_internal.h"

namespace nst {

// Pillow ImagingConvert RGB -> L: L = (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16
__global__ __launch_bounds__(256) void gray_kernel(const uint8_t* __restrict__ rgb, size_t npix, uint8_t* __restrict__ g) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix) return;
  const uint32_t r = rgb[3 * i], gg = rgb[3 * i + 1], b = rgb[3 * i + 2];
  g[i] = (uint8_t)((r * 19595u + gg * 38470u + b * 7471u + 0x8000u) >> 16);
}

hipError_t launch_gray(const uint8_t* rgb, size_t npix, uint8_t* gray, hipStream_t st) {
  hipLaunchKernelGGL(gray_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, rgb, npix, gray);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void u8_to_f32_kernel(const uint8_t* __restrict__ a, size_t n, float* __restrict__ o) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) o[i] = (float)a[i];
}

// separable Gaussian with BORDER_REFLECT_101, taps in a kernel argument (cv2.GaussianBlur on a float image)
struct Taps {
  int n;
  float t[64];
};

__device__ __forceinline__ int refl101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

__global__ __launch_bounds__(256) void gauss_rows_kernel(const float* __restrict__ in, int h, int w, Taps tp,
                                                         float* __restrict__ out) {
  const size_t plane = (size_t)blockIdx.z * h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const int r = tp.n / 2;
  const float* row = in + plane + (size_t)y * w;
  float acc = 0.f;
  for (int j = 0; j < tp.n; ++j) acc = acc + tp.t[j] * row[refl101(x + j - r, w)];
  out[plane + (size_t)y * w + x] = acc;
}

__global__ __launch_bounds__(256) void gauss_cols_kernel(const float* __restrict__ in, int h, int w, Taps tp,
                                                         float* __restrict__ out) {
  const size_t plane = (size_t)blockIdx.z * h * w;
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const int r = tp.n / 2;
  float acc = 0.f;
  for (int j = 0; j < tp.n; ++j) acc = acc + tp.t[j] * in[plane + (size_t)refl101(y + j - r, h) * w + x];
  out[plane + (size_t)y * w + x] = acc;
}

// cv2.getGaussianKernel(n, sigma, CV_32F): sigma <= 0 and n <= 7 takes the fixed small table
static Taps gaussian_taps(int n, double sigma) {
  Taps tp;
  tp.n = n;
  if (sigma <= 0 && n == 3) {
    tp.t[0] = 0.25f; tp.t[1] = 0.5f; tp.t[2] = 0.25f;
    return tp;
  }
  if (sigma <= 0) sigma = ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
  const double s2 = -0.5 / (sigma * sigma);
  double sum = 0;
  double v[64];
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    v[i] = std::exp(s2 * x * x);
    sum += v[i];
  }
  for (int i = 0; i < n; ++i) tp.t[i] = (float)(v[i] / sum);
  return tp;
}

hipError_t launch_gauss(float* planes, int k, int h, int w, int ksize, double sigma, float* tmp, hipStream_t st) {
  if (ksize > 63) return hipErrorInvalidValue;
  const Taps tp = gaussian_taps(ksize, sigma);
  const dim3 g((unsigned)((w + 255) / 256), (unsigned)h, (unsigned)k);
  hipLaunchKernelGGL(gauss_rows_kernel, g, dim3(256), 0, st, planes, h, w, tp, tmp);
  hipLaunchKernelGGL(gauss_cols_kernel, g, dim3(256), 0, st, tmp, h, w, tp, planes);
  return hipGetLastError();
}

// cv2.resize(INTER_LINEAR) of float planes with c interleaved channels: fx = (dx + 0.5) * scale - 0.5, taps
// clamped at the borders (OpenCV's coefficient rule)
__device__ __forceinline__ void lin_coef(int d, double scale, int n, int& s0, float& a1) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) { s = 0; f = 0.f; }
  if (s >= n - 1) { s = n - 1; f = 0.f; }
  s0 = s;
  a1 = f;
}

__global__ __launch_bounds__(256) void resize_lin_kernel(const float* __restrict__ in, int h, int w, int c, int oh,
                                                         int ow, double sy, double sx, float mul,
                                                         float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t np = (size_t)blockIdx.z * oh * ow;
  if (i >= (size_t)oh * ow) return;
  const int x = (int)(i % ow), y = (int)(i / ow);
  int x0, y0;
  float fx, fy;
  lin_coef(x, sx, w, x0, fx);
  lin_coef(y, sy, h, y0, fy);
  const int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, h - 1);
  const float* src = in + (size_t)blockIdx.z * h * w * c;
  for (int ch = 0; ch < c; ++ch) {
    const float r0 = src[((size_t)y0 * w + x0) * c + ch] * (1.f - fx) + src[((size_t)y0 * w + x1) * c + ch] * fx;
    const float r1 = src[((size_t)y1 * w + x0) * c + ch] * (1.f - fx) + src[((size_t)y1 * w + x1) * c + ch] * fx;
    out[(np + i) * c + ch] = (r0 * (1.f - fy) + r1 * fy) * mul;
  }
}

hipError_t launch_resize_lin(const float* in, int k, int h, int w, int c, int oh, int ow, float mul, float* out,
                             hipStream_t st) {
  const size_t n = (size_t)oh * ow;
  hipLaunchKernelGGL(resize_lin_kernel, dim3((unsigned)((n + 255) / 256), 1, (unsigned)k), dim3(256), 0, st, in, h, w,
                     c, oh, ow, (double)h / oh, (double)w / ow, mul, out);
  return hipGetLastError();
}

// ---- FarnebackPolyExp (n <= 8): vertical moments [h][w][3] (clamped rows), then horizontal in double ----
struct PolyTab {
  int n;
  float g[17], xg[17], xxg[17];  // index k + n
  double ig11, ig03, ig33, ig55;
};

__global__ __launch_bounds__(256) void polyexp_v_kernel(const float* __restrict__ src, int h, int w, PolyTab pt,
                                                        float* __restrict__ row3) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t pl = (size_t)blockIdx.z * h * w;
  if (i >= (size_t)h * w) return;
  const int x = (int)(i % w), y = (int)(i / w);
  const float* s = src + pl;
  float t0 = s[(size_t)y * w + x] * pt.g[pt.n], t1 = 0.f, t2 = 0.f;
  for (int k = 1; k <= pt.n; ++k) {
    const float a = s[(size_t)max(y - k, 0) * w + x], b = s[(size_t)min(y + k, h - 1) * w + x];
    const float p = a + b;
    t0 = t0 + pt.g[pt.n + k] * p;
    t1 = t1 + pt.xg[pt.n + k] * (b - a);
    t2 = t2 + pt.xxg[pt.n + k] * p;
  }
  float* o = row3 + (pl + i) * 3;
  o[0] = t0; o[1] = t1; o[2] = t2;
}

__global__ __launch_bounds__(256) void polyexp_h_kernel(const float* __restrict__ row3, int h, int w, PolyTab pt,
                                                        float* __restrict__ R) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t pl = (size_t)blockIdx.z * h * w;
  if (i >= (size_t)h * w) return;
  const int x = (int)(i % w), y = (int)(i / w);
  const float* rw = row3 + (pl + (size_t)y * w) * 3;
  const float g0 = pt.g[pt.n];
  double b1 = rw[x * 3] * g0, b2 = 0, b3 = rw[x * 3 + 1] * g0, b4 = 0, b5 = rw[x * 3 + 2] * g0, b6 = 0;
  for (int k = 1; k <= pt.n; ++k) {
    const int xp = min(x + k, w - 1), xm = max(x - k, 0);  // the row's replicated border
    // as optflowgf.cpp types them: tg is a float sum held in a double; the other products are float
    const double tg = rw[xp * 3] + rw[xm * 3];
    b1 += tg * pt.g[pt.n + k];
    b4 += tg * pt.xxg[pt.n + k];
    b2 += (rw[xp * 3] - rw[xm * 3]) * pt.xg[pt.n + k];
    b3 += (rw[xp * 3 + 1] + rw[xm * 3 + 1]) * pt.g[pt.n + k];
    b6 += (rw[xp * 3 + 1] - rw[xm * 3 + 1]) * pt.xg[pt.n + k];
    b5 += (rw[xp * 3 + 2] + rw[xm * 3 + 2]) * pt.g[pt.n + k];
  }
  float* o = R + (pl + i) * 5;
  o[1] = (float)(b2 * pt.ig11);
  o[0] = (float)(b3 * pt.ig11);
  o[3] = (float)(b1 * pt.ig03 + b4 * pt.ig33);
  o[2] = (float)(b1 * pt.ig03 + b5 * pt.ig33);
  o[4] = (float)(b6 * pt.ig55);
}

// FarnebackPrepareGaussian: the taps and the needed entries of the inverse 6x6 moment matrix G
static PolyTab poly_tab(int n, double sigma) {
  PolyTab pt;
  pt.n = n;
  if (sigma < 1.19209290e-07) sigma = n * 0.3;
  double gd[17], s = 0;
  for (int x = -n; x <= n; ++x) {
    pt.g[x + n] = (float)std::exp(-x * x / (2 * sigma * sigma));
    s += pt.g[x + n];
  }
  s = 1. / s;
  for (int x = -n; x <= n; ++x) {
    pt.g[x + n] = (float)(pt.g[x + n] * s);
    pt.xg[x + n] = (float)(x * pt.g[x + n]);
    pt.xxg[x + n] = (float)(x * x * pt.g[x + n]);
    gd[x + n] = pt.g[x + n];
  }
  double G00 = 0, G11 = 0, G33 = 0, G55 = 0;
  for (int y = -n; y <= n; ++y)
    for (int x = -n; x <= n; ++x) {
      G00 += gd[y + n] * gd[x + n];
      G11 += gd[y + n] * gd[x + n] * x * x;
      G33 += gd[y + n] * gd[x + n] * x * x * x * x;
      G55 += gd[y + n] * gd[x + n] * x * x * y * y;
    }
  // G: [0,0]=G00, [1,1]=[2,2]=[0,3]=[0,4]=[3,0]=[4,0]=G11, [3,3]=[4,4]=G33, [3,4]=[4,3]=[5,5]=G55.  The
  // {0,3,4} block inverted in closed form; rows 1, 2, 5 are diagonal.
  const double a = G00, b = G11, c = G33, d = G55;
  // M = [[a, b, b], [b, c, d], [b, d, c]]: inverse entries (0,3) -> m01, (3,3) -> m11
  const double det = a * (c * c - d * d) - b * (b * c - b * d) + b * (b * d - c * b);
  pt.ig03 = -(b * c - b * d) / det;
  pt.ig33 = (a * c - b * b) / det;
  pt.ig11 = 1.0 / b;
  pt.ig55 = 1.0 / d;
  return pt;
}

// FarnebackUpdateMatrices
__global__ __launch_bounds__(256) void update_matrices_kernel(const float* __restrict__ R0, const float* __restrict__ R1,
                                                              const float* __restrict__ flow, int h, int w,
                                                              float* __restrict__ M) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)h * w) return;
  const int x = (int)(i % w), y = (int)(i / w);
  const float border[5] = {0.14f, 0.14f, 0.4472f, 0.4472f, 0.4472f};
  const float dx = flow[2 * i], dy = flow[2 * i + 1];
  float fx = (float)x + dx, fy = (float)y + dy;
  const int x1 = (int)floorf(fx), y1 = (int)floorf(fy);
  fx -= (float)x1;
  fy -= (float)y1;
  const float* r0 = R0 + i * 5;
  float r2, r3, r4, r5, r6;
  if ((unsigned)x1 < (unsigned)(w - 1) && (unsigned)y1 < (unsigned)(h - 1)) {
    const float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
    const float* p = R1 + ((size_t)y1 * w + x1) * 5;
    const size_t s1 = (size_t)w * 5;
    float v[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) v[c] = a00 * p[c] + a01 * p[5 + c] + a10 * p[s1 + c] + a11 * p[s1 + 5 + c];
    r2 = v[0]; r3 = v[1];
    r4 = (r0[2] + v[2]) * 0.5f;
    r5 = (r0[3] + v[3]) * 0.5f;
    r6 = (r0[4] + v[4]) * 0.25f;
  } else {
    r2 = r3 = 0.f;
    r4 = r0[2];
    r5 = r0[3];
    r6 = r0[4] * 0.5f;
  }
  r2 = (r0[0] - r2) * 0.5f;
  r3 = (r0[1] - r3) * 0.5f;
  r2 += r4 * dy + r6 * dx;
  r3 += r6 * dy + r5 * dx;
  if ((unsigned)(x - 5) >= (unsigned)(w - 10) || (unsigned)(y - 5) >= (unsigned)(h - 10)) {
    const float sc = (x < 5 ? border[x] : 1.f) * (x >= w - 5 ? border[w - x - 1] : 1.f) * (y < 5 ? border[y] : 1.f) *
                     (y >= h - 5 ? border[h - y - 1] : 1.f);
    r2 *= sc; r3 *= sc; r4 *= sc; r5 *= sc; r6 *= sc;
  }
  float* m = M + i * 5;
  m[0] = r4 * r4 + r6 * r6;
  m[1] = (r4 + r5) * r6;
  m[2] = r5 * r5 + r6 * r6;
  m[3] = r4 * r2 + r6 * r3;
  m[4] = r6 * r2 + r5 * r3;
}

// FarnebackUpdateFlow_Blur: block_size x block_size box sums of M (rows and columns clamped to the frame)
// in double, then the 2x2 solve with the 1e-3 regulariser.  As OpenCV sums them: a running vertical sum per
// column (each step adds the float difference entering - leaving row), then the horizontal window over the
// vertical sums.  Vertical: one thread per column walks a strip of BOX_ROWS rows; horizontal: a 256-pixel row
// segment and its halo staged in LDS.
constexpr int BOX_ROWS = 16;

__global__ __launch_bounds__(256) void box_v_kernel(const float* __restrict__ M, int h, int w, int m,
                                                    double* __restrict__ vs) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= w) return;
  const int y0 = blockIdx.y * BOX_ROWS, y1 = min(h, y0 + BOX_ROWS);
  auto row = [&](int q) { return M + ((size_t)min(max(q, 0), h - 1) * w + x) * 5; };
  double s[5] = {0, 0, 0, 0, 0};
  for (int q = y0 - m; q <= y0 + m; ++q) {
    const float* p = row(q);
#pragma unroll
    for (int c = 0; c < 5; ++c) s[c] += p[c];
  }
  for (int y = y0; y < y1; ++y) {
    if (y > y0) {
      const float* pa = row(y + m);
      const float* pd = row(y - m - 1);
#pragma unroll
      for (int c = 0; c < 5; ++c) s[c] += pa[c] - pd[c];
    }
    double* o = vs + ((size_t)y * w + x) * 5;
#pragma unroll
    for (int c = 0; c < 5; ++c) o[c] = s[c];
  }
}

__global__ __launch_bounds__(256) void box_h_solve_kernel(const double* __restrict__ vs, int h, int w, int m,
                                                          double scale, float* __restrict__ flow) {
  extern __shared__ double seg[];  // (256 + 2m) x 5
  const int y = blockIdx.y, x0 = blockIdx.x * 256;
  const int n = 256 + 2 * m;
  for (int j = threadIdx.x; j < n * 5; j += 256) {
    const int e = j / 5, c = j - e * 5;
    const int xs = min(max(x0 - m + e, 0), w - 1);
    seg[j] = vs[((size_t)y * w + xs) * 5 + c];
  }
  __syncthreads();
  const int x = x0 + threadIdx.x;
  if (x >= w) return;
  double s[5] = {0, 0, 0, 0, 0};
  for (int q = 0; q <= 2 * m; ++q) {
    const double* p = seg + (threadIdx.x + q) * 5;
#pragma unroll
    for (int c = 0; c < 5; ++c) s[c] += p[c];
  }
  const size_t i = (size_t)y * w + x;
  const double g11 = s[0] * scale, g12 = s[1] * scale, g22 = s[2] * scale, h1 = s[3] * scale, h2 = s[4] * scale;
  const double idet = 1. / (g11 * g22 - g12 * g12 + 1e-3);
  flow[2 * i] = (float)((g11 * h2 - g12 * h1) * idet);
  flow[2 * i + 1] = (float)((g22 * h1 - g12 * h2) * idet);
}

size_t farneback_scratch_floats(int h, int w) {
  const size_t n = (size_t)h * w;
  // img f32 x2, tmp x2, I x2, row3 x2 (3ch), R x2 (5ch), M (5ch), vs (5 doubles = 10 floats), flow x2 (2ch)
  return n * (2 + 2 + 2 + 6 + 10 + 5 + 10 + 4) + 64;
}

hipError_t launch_farneback(const uint8_t* prev, const uint8_t* next, int h, int w, double pyr_scale, int levels,
                            int winsize, int iterations, int poly_n, double poly_sigma, float* flow_out, float* scratch,
                            hipStream_t st) {
  const size_t n = (size_t)h * w;
  float* img = scratch;             // 2 planes, full resolution
  float* tmp = img + 2 * n;         // 2 planes
  float* I = tmp + 2 * n;           // 2 planes at the level size
  float* row3 = I + 2 * n;          // 2 x 3ch
  float* R = row3 + 6 * n;          // 2 x 5ch
  float* M = R + 10 * n;            // 5ch
  double* vs = (double*)(M + 5 * n + ((5 * n) & 1));  // 5 doubles per pixel (8-byte aligned)
  float* fa = (float*)(vs + 5 * n); // 2ch
  float* fb = fa + 2 * n;           // 2ch
  const int min_size = 32;
  int k;
  double scale = 1;
  for (k = 0; k < levels; ++k) {
    scale *= pyr_scale;
    if (w * scale < min_size || h * scale < min_size) break;
  }
  levels = k;
  const PolyTab pt = poly_tab(poly_n, poly_sigma);
  const int m = winsize / 2;
  const double bscale = 1. / (winsize * winsize);
  float* prev_flow = nullptr;
  int pw = 0, ph = 0;
  for (k = levels; k >= 0; --k) {
    scale = 1;
    for (int i = 0; i < k; ++i) scale *= pyr_scale;
    const double sigma = (1. / scale - 1) * 0.5;
    int ksz = ((int)std::nearbyint(sigma * 5)) | 1;
    ksz = std::max(ksz, 3);
    const int lw = (int)std::nearbyint(w * scale), lh = (int)std::nearbyint(h * scale);
    const size_t ln = (size_t)lw * lh;
    float* flow = k == 0 ? flow_out : (prev_flow == fa ? fb : fa);
    if (!prev_flow) {
      const hipError_t e0 = hipMemsetAsync(flow, 0, ln * 2 * sizeof(float), st);
      if (e0 != hipSuccess) return e0;
    } else {
      hipError_t e = launch_resize_lin(prev_flow, 1, ph, pw, 2, lh, lw, (float)(1. / pyr_scale), flow, st);
      if (e != hipSuccess) return e;
    }
    // both images: to float, GaussianBlur(ksz, sigma), resize to the level, polynomial expansion
    hipLaunchKernelGGL(u8_to_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, prev, n, img);
    hipLaunchKernelGGL(u8_to_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, next, n, img + n);
    hipError_t e = launch_gauss(img, 2, h, w, ksz, sigma, tmp, st);
    if (e != hipSuccess) return e;
    const float* lev = img;
    if (lw != w || lh != h) {
      e = launch_resize_lin(img, 2, h, w, 1, lh, lw, 1.f, I, st);
      if (e != hipSuccess) return e;
      lev = I;
    }
    const dim3 gl((unsigned)((ln + 255) / 256), 1, 2);
    hipLaunchKernelGGL(polyexp_v_kernel, gl, dim3(256), 0, st, lev, lh, lw, pt, row3);
    hipLaunchKernelGGL(polyexp_h_kernel, gl, dim3(256), 0, st, row3, lh, lw, pt, R);
    const dim3 g1((unsigned)((ln + 255) / 256));
    hipLaunchKernelGGL(update_matrices_kernel, g1, dim3(256), 0, st, R, R + 5 * ln, flow, lh, lw, M);
    const dim3 gv((unsigned)((lw + 255) / 256), (unsigned)((lh + BOX_ROWS - 1) / BOX_ROWS));
    const dim3 gh((unsigned)((lw + 255) / 256), (unsigned)lh);
    const size_t hl = (size_t)(256 + 2 * m) * 5 * sizeof(double);
    for (int it = 0; it < iterations; ++it) {
      hipLaunchKernelGGL(box_v_kernel, gv, dim3(256), 0, st, M, lh, lw, m, vs);
      hipLaunchKernelGGL(box_h_solve_kernel, gh, dim3(256), hl, st, vs, lh, lw, m, bscale, flow);
      if (it < iterations - 1)
        hipLaunchKernelGGL(update_matrices_kernel, g1, dim3(256), 0, st, R, R + 5 * ln, flow, lh, lw, M);
    }
    prev_flow = flow;
    pw = lw;
    ph = lh;
  }
  return hipGetLastError();
}

// ---- cv2.resize(src, (ow, oh), interpolation=INTER_AREA) of u8 images (--flow_downscale's grays,
// pipeline.py:1886-1892, and the DIS pyramid) — OpenCV's resize.cpp restated (cv2 absent: parity unpinned):
//   * integer scales in both axes (is_area_fast): resizeAreaFast_, the int sum of each iscale_x x iscale_y
//     block times the fp32 1/area, rounded (cvRound); at scale 2 x 2 ResizeAreaFastVec's (sum + 2) >> 2;
//   * otherwise (downscaling, scale >= 1) ResizeArea_Invoker with computeResizeAreaTab's fractional cells:
//     per destination column the source columns sx with weight alpha (fp32 of a double ratio, the partial
//     first / last cells only beyond 1e-3), per destination row the rows sy with beta; per row
//     buf = sum(S[sy][sx] * alpha) over the column's cells in order, sum = beta * buf (first row) or
//     sum += beta * buf, then cvRound + saturate.  The cell tables are recomputed per thread in double,
//     exactly as the host would (no table upload per geometry). ----
struct AreaCells {
  int sx[3], n_mid;       // first partial cell (or -1), the full cells sx1 .. sx1 + n_mid - 1, last partial cell (or -1)
  float a_first, a_mid, a_last;
  int sx1;
};
__device__ __forceinline__ AreaCells area_cells(int d, int ssize, double scale) {
  AreaCells c;
  const double fs1 = d * scale, fs2 = fs1 + scale;
  const double cell = fmin(scale, ssize - fs1);
  int s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  c.sx[0] = (s1 - fs1 > 1e-3) ? s1 - 1 : -1;
  c.a_first = (float)((s1 - fs1) / cell);
  c.sx1 = s1;
  c.n_mid = s2 - s1;
  c.a_mid = (float)(1.0 / cell);
  c.sx[2] = (fs2 - s2 > 1e-3) ? s2 : -1;
  c.a_last = (float)(fmin(fmin(fs2 - s2, 1.0), cell) / cell);
  return c;
}

__global__ __launch_bounds__(256) void area_resize_kernel(const uint8_t* __restrict__ in, int n, int h, int w, int ch,
                                                          int oh, int ow, double sx_scale, double sy_scale, int fast,
                                                          int isx, int isy, uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * oh * ow * ch) return;
  const int c = (int)(i % ch);
  size_t r = i / ch;
  const int dx = (int)(r % ow);
  r /= ow;
  const int dy = (int)(r % oh);
  const int f = (int)(r / oh);
  const uint8_t* S = in + (size_t)f * h * w * ch;
  if (fast) {
    int sum = 0;
    for (int yy = 0; yy < isy; ++yy)
      for (int xx = 0; xx < isx; ++xx) sum += S[((size_t)(dy * isy + yy) * w + dx * isx + xx) * ch + c];
    if (isx == 2 && isy == 2) {  // ResizeAreaFastVec: (sum + 2) >> 2 (halves round up), SIMD and tail alike
      out[i] = (uint8_t)((sum + 2) >> 2);
      return;
    }
    const float scale = 1.f / (float)(isx * isy);
    out[i] = (uint8_t)min(255, max(0, (int)rintf((float)sum * scale)));
    return;
  }
  const AreaCells X = area_cells(dx, w, sx_scale), Y = area_cells(dy, h, sy_scale);
  auto row_buf = [&](int sy) {
    const uint8_t* R = S + (size_t)sy * w * ch + c;
    float buf = 0.f;
    if (X.sx[0] >= 0) buf = buf + (float)R[(size_t)X.sx[0] * ch] * X.a_first;
    for (int k = 0; k < X.n_mid; ++k) buf = buf + (float)R[(size_t)(X.sx1 + k) * ch] * X.a_mid;
    if (X.sx[2] >= 0) buf = buf + (float)R[(size_t)X.sx[2] * ch] * X.a_last;
    return buf;
  };
  float sum = 0.f;
  bool first = true;
  auto add_row = [&](int sy, float beta) {
    const float b = beta * row_buf(sy);
    sum = first ? b : sum + b;
    first = false;
  };
  if (Y.sx[0] >= 0) add_row(Y.sx[0], Y.a_first);
  for (int k = 0; k < Y.n_mid; ++k) add_row(Y.sx1 + k, Y.a_mid);
  if (Y.sx[2] >= 0) add_row(Y.sx[2], Y.a_last);
  out[i] = (uint8_t)min(255, max(0, (int)rintf(sum)));
}

hipError_t launch_area_resize(const uint8_t* in, int n, int h, int w, int ch, int oh, int ow, uint8_t* out,
                              hipStream_t st) {
  // resize(): inv_scale = dsize / ssize, scale = 1 / inv_scale; is_area_fast when both are integers
  const double sx = 1. / ((double)ow / w), sy = 1. / ((double)oh / h);
  const int isx = (int)lrint(sx), isy = (int)lrint(sy);
  const int fast = fabs(sx - isx) < DBL_EPSILON && fabs(sy - isy) < DBL_EPSILON;
  const size_t total = (size_t)n * oh * ow * ch;
  hipLaunchKernelGGL(area_resize_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, n, h, w, ch, oh, ow,
                     sx, sy, fast, isx, isy, out);
  return hipGetLastError();
}

// ---- flow EMA: fused = clip(a * curr + (1 - a) * remap(prev, grid + flow, BORDER_REPLICATE)) ----
__global__ __launch_bounds__(256) void flow_fuse_kernel(const float* __restrict__ curr, const float* __restrict__ prev,
                                                        const float* __restrict__ flow, int h, int w, float a,
                                                        float oma, float* __restrict__ out) {
  const size_t hw = (size_t)h * w;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= hw) return;
  const int x = (int)(i % w), y = (int)(i / w);
  // cv2's saturate_cast<int>(map * 32) saturates (NaN -> INT_MIN); clamping the map far outside the frame first
  // gives the same replicated-border sample and keeps the int conversion defined
  const float mx = fminf(fmaxf((float)x + flow[2 * i], -2.f * w), 3.f * w);
  const float my = fminf(fmaxf((float)y + flow[2 * i + 1], -2.f * h), 3.f * h);
  const int X = (int)rintf(mx * 32.f), Y = (int)rintf(my * 32.f);
  const int sx = X >> 5, sy = Y >> 5;
  const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
  const float w00 = (1.f - fy) * (1.f - fx), w01 = (1.f - fy) * fx, w10 = fy * (1.f - fx), w11 = fy * fx;
  const int x0 = min(max(sx, 0), w - 1), x1 = min(max(sx + 1, 0), w - 1);
  const int y0 = min(max(sy, 0), h - 1), y1 = min(max(sy + 1, 0), h - 1);
  for (int c = 0; c < 3; ++c) {
    const float* p = prev + c * hw;
    const float t0 = p[(size_t)y0 * w + x0] * w00 + p[(size_t)y0 * w + x1] * w01;
    const float t1 = p[(size_t)y1 * w + x0] * w10 + p[(size_t)y1 * w + x1] * w11;
    const float v = (a * curr[c * hw + i]) + (oma * (t0 + t1));
    out[c * hw + i] = fminf(fmaxf(v, 0.f), 1.f);
  }
}

hipError_t launch_flow_fuse(const float* curr, const float* prev, const float* flow, int h, int w, float a, float oma,
                            float* out, hipStream_t st) {
  const size_t hw = (size_t)h * w;
  hipLaunchKernelGGL(flow_fuse_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, curr, prev, flow, h, w, a,
                     oma, out);
  return hipGetLastError();
}

// ---- motion-adaptive alpha (pipeline.py:2073-2080) ----
__global__ __launch_bounds__(256) void motion_mag_kernel(const float* __restrict__ flow, size_t hw, float norm,
                                                         float* __restrict__ m) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= hw) return;
  const float fx = flow[2 * i], fy = flow[2 * i + 1];
  const float mag = sqrtf(fx * fx + fy * fy);
  m[i] = fminf(fmaxf(mag / norm, 0.f), 1.f);
}

__global__ __launch_bounds__(256) void motion_alpha_kernel(float* __restrict__ m, size_t hw, float maxa, float span) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < hw) m[i] = maxa - span * m[i];
}

hipError_t launch_motion_alpha(const float* flow, int h, int w, float norm, double sigma, float max_alpha, float span,
                               float* alpha, float* tmp, hipStream_t st) {
  const size_t hw = (size_t)h * w;
  const dim3 g((unsigned)((hw + 255) / 256));
  hipLaunchKernelGGL(motion_mag_kernel, g, dim3(256), 0, st, flow, hw, norm, alpha);
  // cv2.GaussianBlur(m, (0, 0), sigma) on float: ksize = cvRound(sigma * 4 * 2 + 1) | 1
  const int ksz = ((int)std::nearbyint(sigma * 8 + 1)) | 1;
  hipError_t e = launch_gauss(alpha, 1, h, w, ksz, sigma, tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(motion_alpha_kernel, g, dim3(256), 0, st, alpha, hw, max_alpha, span);
  return hipGetLastError();
}

}  // namespace nst
