// dis_ops.hip — DIS optical flow (cv2.DISOpticalFlow_create(PRESET_FAST).calc, the reference's default
// --flow_method: pipeline.py:1904-1914) on the GPU, for a batch of frame pairs.
//
// OpenCV's DISOpticalFlowImpl (dis_flow.cpp) and VariationalRefinement (variational_refinement.cpp) restated with
// PRESET_FAST's parameters (patch 8, stride 4, finest scale 2, 16 gradient-descent iterations, 5 variational
// refinement iterations); the CPU restatement this is checked against is oracle/dis_oracle.py (cv2 is absent:
// parity unpinned).  Per pyramid level, coarsest to finest:
//   * pyramid: INTER_AREA (flow_ops.hip launch_area_resize), I1 replicate-padded by 16, Sobel 3x3 of I0 (int16);
//   * structure tensor: running box sums per patch (one thread per row, then per patch column: cv2's order);
//   * inverse search with spatial propagation: 8 stripes of patch rows (the reference's fixed stripe count), each
//     a forward and a backward sweep; a patch depends only on its left and upper (forward) neighbour, so a
//     workgroup per (stripe, frame) walks the stripe's anti-diagonals, one wave per patch: lane = pixel of the
//     8x8 patch, the patch sums are wave reductions (xor butterfly: the oracle's halving tree), the
//     Gauss-Newton iterations run in lockstep and stop together (the SSD is wave-uniform);
//   * densification: per pixel, the overlapping patches weighted by 1 / max(1, |warp error|);
//   * variational refinement: derivative planes once, then per fixed-point iteration the data term, the
//     smoothness weights and 5 red-black SOR sweeps, each a launch over all frames of the batch;
//   * cv2.resize INTER_LINEAR x 2 to the next level; finally to the frame, x 4.
// fp32 throughout in cv2's operation order (built with -ffp-contract=off: no fused multiply-adds), fp64 where
// cv2 uses double.
#include <cfloat>
#include <math.h>

#include "flow_internal.h"

namespace nst {

namespace {

constexpr int DIS_PATCH = 8, DIS_STRIDE = 4, DIS_FINEST = 2, DIS_GD = 16, DIS_BORDER = 16, DIS_STRIPES = 8;
constexpr int DIS_VR_ITER = 5, DIS_SOR = 5;
constexpr float DIS_EPS = 0.001f, DIS_INF = 1e20f;

int coarsest_scale(int h, int w) {
  return std::min((int)(std::log(std::max(w, h) / (4.0 * DIS_PATCH)) / std::log(2.0) + 0.5),
                  (int)(std::log(std::min(w, h) / (double)DIS_PATCH) / std::log(2.0)));
}

// ---------------------------------------------------------------------------------------- per-level setup
__global__ __launch_bounds__(256) void pad_rep_kernel(const uint8_t* __restrict__ in, int n, int h, int w,
                                                      uint8_t* __restrict__ out) {
  const int he = h + 2 * DIS_BORDER, we = w + 2 * DIS_BORDER;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * he * we) return;
  const int x = (int)(i % we);
  const size_t r = i / we;
  const int y = (int)(r % he), f = (int)(r / he);
  const int sy = min(max(y - DIS_BORDER, 0), h - 1), sx = min(max(x - DIS_BORDER, 0), w - 1);
  out[i] = in[((size_t)f * h + sy) * w + sx];
}

__device__ __forceinline__ int refl101(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - 2 - p : p;
}

// spatialGradient (3x3 Sobel, BORDER_REFLECT_101) -> int16
__global__ __launch_bounds__(256) void sobel_kernel(const uint8_t* __restrict__ I, int n, int h, int w,
                                                    int16_t* __restrict__ gx, int16_t* __restrict__ gy) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)n * h * w) return;
  const int x = (int)(i % w);
  const size_t r = i / w;
  const int y = (int)(r % h), f = (int)(r / h);
  const uint8_t* P = I + (size_t)f * h * w;
  const int ym = refl101(y - 1, h), yp = refl101(y + 1, h), xm = refl101(x - 1, w), xp = refl101(x + 1, w);
  auto at = [&](int yy, int xx) { return (int)P[(size_t)yy * w + xx]; };
  const int dxm = at(ym, xp) - at(ym, xm), dx0 = at(y, xp) - at(y, xm), dxp = at(yp, xp) - at(yp, xm);
  const int dym = at(yp, xm) - at(ym, xm), dy0 = at(yp, x) - at(ym, x), dyp = at(yp, xp) - at(ym, xp);
  gx[i] = (int16_t)(dxm + 2 * dx0 + dxp);
  gy[i] = (int16_t)(dym + 2 * dy0 + dyp);
}

// precomputeStructureTensor, horizontal pass: one thread per (frame, row): running sums of the 5 terms over 8
// columns, stored every stride -> aux[t][f][row][ws]
__global__ __launch_bounds__(256) void tensor_h_kernel(const int16_t* __restrict__ gx, const int16_t* __restrict__ gy,
                                                       int n, int h, int w, int ws, float* __restrict__ aux) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n * h) return;
  const int16_t* X = gx + (size_t)r * w;
  const int16_t* Y = gy + (size_t)r * w;
  const size_t plane = (size_t)n * h * ws;
  float* A = aux + (size_t)r * ws;
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  auto term = [&](int j, int t) -> int {
    const int a = X[j], b = Y[j];
    return t == 0 ? a * a : t == 1 ? b * b : t == 2 ? a * b : t == 3 ? a : b;
  };
#pragma unroll
  for (int t = 0; t < 5; ++t)
    for (int j = 0; j < DIS_PATCH; ++j) s[t] = s[t] + (float)term(j, t);
#pragma unroll
  for (int t = 0; t < 5; ++t) A[t * plane] = s[t];
  int js = 1;
  for (int j = DIS_PATCH; j < w; ++j) {
#pragma unroll
    for (int t = 0; t < 5; ++t) s[t] = s[t] + (float)(term(j, t) - term(j - DIS_PATCH, t));
    if ((j - DIS_PATCH + 1) % DIS_STRIDE == 0) {
      if (js < ws) {
#pragma unroll
        for (int t = 0; t < 5; ++t) A[t * plane + js] = s[t];
      }
      ++js;
    }
  }
}

// vertical pass: one thread per (frame, patch column) -> T[t][f][hs][ws]
__global__ __launch_bounds__(256) void tensor_v_kernel(const float* __restrict__ aux, int n, int h, int ws, int hs,
                                                       float* __restrict__ T) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n * ws) return;
  const int f = c / ws, js = c - f * ws;
  const size_t ap = (size_t)n * h * ws, tp = (size_t)n * hs * ws;
  for (int t = 0; t < 5; ++t) {
    const float* A = aux + t * ap + (size_t)f * h * ws + js;
    float* O = T + t * tp + (size_t)f * hs * ws + js;
    float v = 0.f;
    for (int i = 0; i < DIS_PATCH; ++i) v = v + A[(size_t)i * ws];
    O[0] = v;
    int is = 1;
    for (int i = DIS_PATCH; i < h; ++i) {
      v = v + (A[(size_t)i * ws] - A[(size_t)(i - DIS_PATCH) * ws]);
      if ((i - DIS_PATCH + 1) % DIS_STRIDE == 0) {
        if (is < hs) O[(size_t)is * ws] = v;
        ++is;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------- inverse search
struct SearchArgs {
  int n, h, w, hs, ws, stripe, first_level;
  const uint8_t* I0;   // [n][h][w]
  const uint8_t* I1e;  // [n][h + 32][w + 32]
  const int16_t* gx;   // [n][h][w]
  const int16_t* gy;
  const float* T;      // [5][n][hs][ws]: xx, yy, xy, x, y
  const float* Ux;     // [n][h][w] the previous level's flow (initial approximation)
  const float* Uy;
  float* Sx;           // [n][hs][ws] out
  float* Sy;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) v = v + __shfl_xor(v, k, 64);
  return v;
}

constexpr int SEARCH_WAVES = 16;
constexpr int SEARCH_LDS_FLOATS = 16384;  // 64 KB: the stripe's sparse flow (rows x ws x 2)

__global__ __launch_bounds__(64 * SEARCH_WAVES) void search_kernel(SearchArgs a) {
  __shared__ float S[SEARCH_LDS_FLOATS];
  const int s = blockIdx.x, f = blockIdx.y;
  const int r0 = min(s * a.stripe, a.hs), r1 = min((s + 1) * a.stripe, a.hs);
  const int nrows = r1 - r0;
  if (nrows <= 0) return;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pi = lane >> 3, pj = lane & 7;
  const int h = a.h, w = a.w, ws = a.ws, we = w + 2 * DIS_BORDER;
  const uint8_t* I0 = a.I0 + (size_t)f * h * w;
  const uint8_t* I1e = a.I1e + (size_t)f * (h + 2 * DIS_BORDER) * we;
  const int16_t* GX = a.gx + (size_t)f * h * w;
  const int16_t* GY = a.gy + (size_t)f * h * w;
  const size_t tp = (size_t)a.n * a.hs * ws;
  const float* Txx = a.T + (size_t)f * a.hs * ws;
  float* SX = S;                    // [nrows][ws]
  float* SY = S + nrows * ws;
  const float il = (float)(DIS_BORDER - DIS_PATCH + 1), iu = (float)(DIS_BORDER + h - 1);
  const float jl = (float)(DIS_BORDER - DIS_PATCH + 1), ju = (float)(DIS_BORDER + w - 1);
  const float n64 = 64.f;

  // per-lane diff of the bilinear I1 sample at flow (ux, uy) against I0 (INIT_BILINEAR_WEIGHTS + processPatch)
  auto diff_at = [&](int i, int j, float ux, float uy, float i0) {
    const float iI1 = fminf(fmaxf(((float)i + uy) + (float)DIS_BORDER, il), iu);
    const float jI1 = fminf(fmaxf(((float)j + ux) + (float)DIS_BORDER, jl), ju);
    const float di = iI1 - floorf(iI1), dj = jI1 - floorf(jI1);
    const float w11 = di * dj, w10 = di * (1.f - dj), w01 = (1.f - di) * dj, w00 = (1.f - di) * (1.f - dj);
    const uint8_t* p = I1e + (size_t)((int)iI1 + pi) * we + (int)jI1 + pj;
    float t = w00 * (float)p[0];
    t = t + w01 * (float)p[1];
    t = t + w10 * (float)p[we];
    t = t + w11 * (float)p[we + 1];
    return t - i0;
  };
  auto ssd = [&](int i, int j, float ux, float uy, float i0) {
    const float d = diff_at(i, j, ux, uy, i0);
    const float sd = wave_sum(d), sq = wave_sum(d * d);
    return sq - (sd * sd) / n64;
  };

  for (int pass = 0; pass < 2; ++pass) {
    const bool fwd = pass == 0;
    const int dir = fwd ? 1 : -1;
    if (pass == 0) {  // the stripe's sparse flow starts from the previous level's dense flow (iter == 0)
      for (int k = threadIdx.x; k < nrows * ws; k += 64 * SEARCH_WAVES) {
        const int rr = k / ws, js = k - rr * ws;
        const int i = (r0 + rr) * DIS_STRIDE, j = js * DIS_STRIDE;
        const size_t u = (size_t)f * h * w + (size_t)(i + DIS_PATCH / 2) * w + j + DIS_PATCH / 2;
        SX[k] = a.Ux[u];
        SY[k] = a.Uy[u];
      }
      __syncthreads();
    }
    const int nstep = ws + nrows - 1;
    for (int t = 0; t < nstep; ++t) {
      for (int r = wv; r < nrows; r += SEARCH_WAVES) {
        const int c = t - r;
        if (c < 0 || c >= ws) continue;
        const int lr = fwd ? r : nrows - 1 - r;  // row within the stripe
        const int js = fwd ? c : ws - 1 - c;
        const int is = r0 + lr;
        const int i = is * DIS_STRIDE, j = js * DIS_STRIDE;
        const float i0 = (float)I0[(size_t)(i + pi) * w + j + pj];
        const int k = lr * ws + js;
        float cx = SX[k], cy = SY[k];
        float min_ssd = ssd(i, j, cx, cy, i0);
        if (c > 0) {  // left (forward) / right (backward) neighbour in the row
          const float nx = SX[k - dir], ny = SY[k - dir];
          const float cs = ssd(i, j, nx, ny, i0);
          if (cs < min_ssd) { min_ssd = cs; cx = nx; cy = ny; }
        }
        if (r > 0) {  // upper (forward) / lower (backward) neighbour in the stripe
          const float nx = SX[k - dir * ws], ny = SY[k - dir * ws];
          const float cs = ssd(i, j, nx, ny, i0);
          if (cs < min_ssd) { min_ssd = cs; cx = nx; cy = ny; }
        }
        // inverse-compositional Gauss-Newton with the inverted structure tensor
        const size_t q = (size_t)is * ws + js;
        const float xx = Txx[q], yy = Txx[tp + q], xy = Txx[2 * tp + q], xs = Txx[3 * tp + q], ys = Txx[4 * tp + q];
        float det = xx * yy - xy * xy;
        if (fabsf(det) < DIS_EPS) det = DIS_EPS;
        const float h11 = yy / det, h12 = -xy / det, h22 = xx / det;
        const float gxl = (float)GX[(size_t)(i + pi) * w + j + pj], gyl = (float)GY[(size_t)(i + pi) * w + j + pj];
        float ux = cx, uy = cy, prev = DIS_INF;
        for (int it = 0; it < DIS_GD / 2; ++it) {
          const float d = diff_at(i, j, ux, uy, i0);
          const float sd = wave_sum(d), sq = wave_sum(d * d), sxm = wave_sum(d * gxl), sym = wave_sum(d * gyl);
          const float dux = sxm - (sd * xs) / n64;
          const float duy = sym - (sd * ys) / n64;
          const float cur = sq - (sd * sd) / n64;
          const float dx = h11 * dux + h12 * duy;
          const float dy = h12 * dux + h22 * duy;
          ux = ux - dx;
          uy = uy - dy;
          if (cur >= prev) break;
          prev = cur;
        }
        const double ex = (double)(ux - cx), ey = (double)(uy - cy);
        const bool keep = sqrt(ex * ex + ey * ey) <= (double)DIS_PATCH;
        // every lane holds the same values; one write
        if (lane == 0) {
          SX[k] = keep ? ux : cx;
          SY[k] = keep ? uy : cy;
        }
      }
      __syncthreads();
    }
  }
  for (int k = threadIdx.x; k < nrows * ws; k += 64 * SEARCH_WAVES) {
    const int rr = k / ws, js = k - rr * ws;
    a.Sx[(size_t)f * a.hs * ws + (size_t)(r0 + rr) * ws + js] = SX[k];
    a.Sy[(size_t)f * a.hs * ws + (size_t)(r0 + rr) * ws + js] = SY[k];
  }
}

// ---------------------------------------------------------------------------------------- densification
// the patch ranges covering each row / column, by Densification_ParBody's incremental rule
__global__ void ranges_kernel(int h, int w, int2* __restrict__ rows, int2* __restrict__ cols) {
  const int t = threadIdx.x;
  if (t > 1) return;
  const int n = t == 0 ? h : w;
  int2* o = t == 0 ? rows : cols;
  int s = 0, e = -1;
  for (int i = 0; i < n; ++i) {
    if (i % DIS_STRIDE == 0 && i + DIS_PATCH <= n) ++e;
    if (i - DIS_PATCH >= 0 && (i - DIS_PATCH) % DIS_STRIDE == 0 && s < e) ++s;
    o[i] = make_int2(s, e);
  }
}

__global__ __launch_bounds__(256) void densify_kernel(const uint8_t* __restrict__ I0, const uint8_t* __restrict__ I1,
                                                      const float* __restrict__ Sx, const float* __restrict__ Sy,
                                                      const int2* __restrict__ rows, const int2* __restrict__ cols,
                                                      int n, int h, int w, int hs, int ws, float* __restrict__ Ux,
                                                      float* __restrict__ Uy) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)n * h * w) return;
  const int j = (int)(idx % w);
  const size_t r = idx / w;
  const int i = (int)(r % h), f = (int)(r / h);
  const uint8_t* A = I0 + (size_t)f * h * w;
  const uint8_t* B = I1 + (size_t)f * h * w;
  const float* SX = Sx + (size_t)f * hs * ws;
  const float* SY = Sy + (size_t)f * hs * ws;
  const int2 ri = rows[i], rj = cols[j];
  const float i0 = (float)A[(size_t)i * w + j];
  const float wm = (float)(w - 1.0f) - DIS_EPS, hm = (float)(h - 1.0f) - DIS_EPS;
  float su = 0.f, sv = 0.f, sc = 0.f;
  for (int is = ri.x; is <= ri.y; ++is)
    for (int js = rj.x; js <= rj.y; ++js) {
      const float sx = SX[(size_t)is * ws + js], sy = SY[(size_t)is * ws + js];
      const float jm = fminf(fmaxf((float)j + sx, 0.f), wm);
      const float im = fminf(fmaxf((float)i + sy, 0.f), hm);
      const int jl = (int)jm, il = (int)im, ju = jl + 1, iu = il + 1;
      float t = ((jm - (float)jl) * (im - (float)il)) * (float)B[(size_t)iu * w + ju];
      t = t + (((float)ju - jm) * (im - (float)il)) * (float)B[(size_t)iu * w + jl];
      t = t + ((jm - (float)jl) * ((float)iu - im)) * (float)B[(size_t)il * w + ju];
      t = t + (((float)ju - jm) * ((float)iu - im)) * (float)B[(size_t)il * w + jl];
      const float diff = t - i0;
      const float coef = 1.f / fmaxf(1.f, fabsf(diff));
      su = su + coef * sx;
      sv = sv + coef * sy;
      sc = sc + coef;
    }
  Ux[idx] = su / sc;
  Uy[idx] = sv / sc;
}

// ---------------------------------------------------------------------------------------- variational refinement
struct VrBufs {
  float *avg, *Iz, *Ix, *Iy, *Ixz, *Iyz, *Ixx, *Ixy, *Iyy;
  float *a11, *a12, *a22, *b1, *b2, *dU, *dV, *phi;
};

// warp I1 by the flow (cv2.remap INTER_LINEAR, BORDER_REPLICATE, 1/32-pixel fixed point), the averaged image and
// the temporal difference
__global__ __launch_bounds__(256) void vr_warp_kernel(const uint8_t* __restrict__ I0, const uint8_t* __restrict__ I1,
                                                      const float* __restrict__ U, const float* __restrict__ V, int n,
                                                      int h, int w, float* __restrict__ avg, float* __restrict__ Iz) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)n * h * w) return;
  const int x = (int)(idx % w);
  const size_t r = idx / w;
  const int y = (int)(r % h), f = (int)(r / h);
  const uint8_t* P = I1 + (size_t)f * h * w;
  const float mx = fminf(fmaxf((float)x + U[idx], -2.f * w), 3.f * w);
  const float my = fminf(fmaxf((float)y + V[idx], -2.f * h), 3.f * h);
  const int X = (int)rintf(mx * 32.f), Y = (int)rintf(my * 32.f);
  const int sx = X >> 5, sy = Y >> 5;
  const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
  const int x0 = min(max(sx, 0), w - 1), x1 = min(max(sx + 1, 0), w - 1);
  const int y0 = min(max(sy, 0), h - 1), y1 = min(max(sy + 1, 0), h - 1);
  const float t0 = (float)P[(size_t)y0 * w + x0] * ((1.f - fy) * (1.f - fx)) + (float)P[(size_t)y0 * w + x1] * ((1.f - fy) * fx);
  const float t1 = (float)P[(size_t)y1 * w + x0] * (fy * (1.f - fx)) + (float)P[(size_t)y1 * w + x1] * (fy * fx);
  const float i1w = t0 + t1, i0 = (float)I0[idx];
  avg[idx] = 0.5f * i0 + 0.5f * i1w;
  Iz[idx] = i1w - i0;
}

// Sobel ksize 1 (I(x+1) - I(x-1), BORDER_REPLICATE) of src into dx and/or dy
__global__ __launch_bounds__(256) void vr_deriv_kernel(const float* __restrict__ src, int n, int h, int w,
                                                       float* __restrict__ dx, float* __restrict__ dy) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)n * h * w) return;
  const int x = (int)(idx % w);
  const int y = (int)((idx / w) % h);
  if (dx) dx[idx] = src[idx - x + min(x + 1, w - 1)] - src[idx - x + max(x - 1, 0)];
  if (dy) dy[idx] = src[idx + (size_t)(min(y + 1, h - 1) - y) * w] - src[idx - (size_t)(y - max(y - 1, 0)) * w];
}

// smoothness weight of every pixel from the current flow U + dU (forward differences, 0 past the last row/column)
__global__ __launch_bounds__(256) void vr_phi_kernel(const float* __restrict__ U, const float* __restrict__ V,
                                                     const float* __restrict__ dU, const float* __restrict__ dV, int n,
                                                     int h, int w, float alpha2, float eps2, float* __restrict__ phi) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)n * h * w) return;
  const int x = (int)(idx % w);
  const int y = (int)((idx / w) % h);
  const float tu = U[idx] + dU[idx], tv = V[idx] + dV[idx];
  float ux = 0.f, vx = 0.f, uy = 0.f, vy = 0.f;
  if (x < w - 1) {
    ux = (U[idx + 1] + dU[idx + 1]) - tu;
    vx = (V[idx + 1] + dV[idx + 1]) - tv;
  }
  if (y < h - 1) {
    uy = (U[idx + w] + dU[idx + w]) - tu;
    vy = (V[idx + w] + dV[idx + w]) - tv;
  }
  const float s2 = ux * ux + vx * vx + uy * uy + vy * vy + eps2;
  phi[idx] = alpha2 / sqrtf(s2);
}

// the linear system of one fixed-point iteration: data term (ComputeDataTerm_ParBody) + smoothness edges
__global__ __launch_bounds__(256) void vr_system_kernel(VrBufs b, const float* __restrict__ U, const float* __restrict__ V,
                                                        int n, int h, int w, float zeta2, float eps2, float delta2,
                                                        float gamma2) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)n * h * w) return;
  const int x = (int)(idx % w);
  const int y = (int)((idx / w) % h);
  const float Ix = b.Ix[idx], Iy = b.Iy[idx], Iz = b.Iz[idx];
  const float Ixx = b.Ixx[idx], Ixy = b.Ixy[idx], Iyy = b.Iyy[idx], Ixz = b.Ixz[idx], Iyz = b.Iyz[idx];
  const float du = b.dU[idx], dv = b.dV[idx];
  float dn = Ix * Ix + Iy * Iy + zeta2;
  const float k = Iz + Ix * du + Iy * dv;
  float wt = (delta2 / sqrtf(k * k / dn + eps2)) / dn;
  float a11 = wt * (Ix * Ix) + zeta2;
  float a12 = wt * (Ix * Iy);
  float a22 = wt * (Iy * Iy) + zeta2;
  float b1 = -wt * (Iz * Ix);
  float b2 = -wt * (Iz * Iy);
  const float dn1 = Ixx * Ixx + Ixy * Ixy + zeta2;
  const float dn2 = Iyy * Iyy + Ixy * Ixy + zeta2;
  const float kx = Ixz + Ixx * du + Ixy * dv;
  const float ky = Iyz + Ixy * du + Iyy * dv;
  wt = gamma2 / sqrtf(kx * kx / dn1 + ky * ky / dn2 + eps2);
  a11 = a11 + wt * (Ixx * Ixx / dn1 + Ixy * Ixy / dn2);
  a12 = a12 + wt * (Ixx * Ixy / dn1 + Ixy * Iyy / dn2);
  a22 = a22 + wt * (Ixy * Ixy / dn1 + Iyy * Iyy / dn2);
  b1 = b1 + -wt * (Ixx * Ixz / dn1 + Ixy * Iyz / dn2);
  b2 = b2 + -wt * (Ixy * Ixz / dn1 + Iyy * Iyz / dn2);
  // smoothness edges in the order left, right, up, down: right / down edges carry this pixel's weight, left / up
  // the neighbour's; b gets the edge-weighted differences of the flow the refinement started from
  const float u = U[idx], v = V[idx];
  auto edge = [&](bool has, float we, size_t q) {
    if (!has) return;
    a11 = a11 + we;
    a22 = a22 + we;
    b1 = b1 + we * (U[q] - u);
    b2 = b2 + we * (V[q] - v);
  };
  edge(x > 0, x > 0 ? b.phi[idx - 1] : 0.f, idx - 1);
  edge(x < w - 1, b.phi[idx], idx + 1);
  edge(y > 0, y > 0 ? b.phi[idx - w] : 0.f, idx - w);
  edge(y < h - 1, b.phi[idx], idx + w);
  b.a11[idx] = a11;
  b.a12[idx] = a12;
  b.a22[idx] = a22;
  b.b1[idx] = b1;
  b.b2[idx] = b2;
}

// one red-black SOR half sweep: pixels with (x + y) % 2 == color
__global__ __launch_bounds__(256) void vr_sor_kernel(VrBufs b, int n, int h, int w, int color, float omega) {
  const size_t idx2 = (size_t)blockIdx.x * 256 + threadIdx.x;  // every other pixel
  const int w2 = (w + 1) / 2;
  if (idx2 >= (size_t)n * h * w2) return;
  const int xh = (int)(idx2 % w2);
  const size_t r = idx2 / w2;
  const int y = (int)(r % h), f = (int)(r / h);
  const int x = 2 * xh + ((y + color) & 1);
  if (x >= w) return;
  const size_t idx = ((size_t)f * h + y) * w + x;
  float su = 0.f, sv = 0.f;
  auto edge = [&](bool has, float we, size_t q) {
    if (!has) return;
    su = su + we * b.dU[q];
    sv = sv + we * b.dV[q];
  };
  const float ph = b.phi[idx];
  edge(x > 0, x > 0 ? b.phi[idx - 1] : 0.f, idx - 1);
  edge(x < w - 1, ph, idx + 1);
  edge(y > 0, y > 0 ? b.phi[idx - w] : 0.f, idx - w);
  edge(y < h - 1, ph, idx + w);
  float du = b.dU[idx], dv = b.dV[idx];
  const float a12 = b.a12[idx];
  du = du + omega * ((su + b.b1[idx] - dv * a12) / b.a11[idx] - du);
  dv = dv + omega * ((sv + b.b2[idx] - du * a12) / b.a22[idx] - dv);
  b.dU[idx] = du;
  b.dV[idx] = dv;
}

__global__ __launch_bounds__(256) void vr_finish_kernel(float* __restrict__ U, float* __restrict__ V,
                                                        const float* __restrict__ dU, const float* __restrict__ dV,
                                                        size_t total) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  U[idx] = U[idx] + dU[idx];
  V[idx] = V[idx] + dV[idx];
}

__global__ __launch_bounds__(256) void interleave_kernel(const float* __restrict__ U, const float* __restrict__ V,
                                                         size_t total, float* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  out[2 * idx] = U[idx];
  out[2 * idx + 1] = V[idx];
}

dim3 g256(size_t total) { return dim3((unsigned)((total + 255) / 256)); }

}  // namespace

// ---------------------------------------------------------------------------------------- plan + driver
struct DisPlan {
  int cs = -1;
  int lh[16], lw[16];      // level sizes
  size_t off_img[16];      // I0s / I1s of level s: [2][n][h][w] u8
  size_t off_I1e, off_gx, off_gy, off_aux, off_T, off_Sx, off_Sy, off_U[4], off_vr, off_rows, off_cols, off_UV;
  size_t bytes = 0;
};

static size_t al(size_t v) { return (v + 255) / 256 * 256; }

static DisPlan dis_plan(int n, int H, int W) {
  DisPlan P;
  P.cs = coarsest_scale(H, W);
  if (P.cs < DIS_FINEST || P.cs > 15) return P;
  size_t off = 0;
  for (int s = DIS_FINEST; s <= P.cs; ++s) {
    if (s == DIS_FINEST) {
      P.lh[s] = H / (1 << s);
      P.lw[s] = W / (1 << s);
    } else {
      P.lh[s] = P.lh[s - 1] / 2;
      P.lw[s] = P.lw[s - 1] / 2;
    }
    P.off_img[s] = off;
    off += al((size_t)2 * n * P.lh[s] * P.lw[s]);
  }
  const int h = P.lh[DIS_FINEST], w = P.lw[DIS_FINEST];
  const int ws = 1 + (w - DIS_PATCH) / DIS_STRIDE, hs = 1 + (h - DIS_PATCH) / DIS_STRIDE;
  const size_t px = (size_t)n * h * w;
  P.off_I1e = off; off += al((size_t)n * (h + 2 * DIS_BORDER) * (w + 2 * DIS_BORDER));
  P.off_gx = off; off += al(px * 2);
  P.off_gy = off; off += al(px * 2);
  P.off_aux = off; off += al((size_t)5 * n * h * ws * 4);
  P.off_T = off; off += al((size_t)5 * n * hs * ws * 4);
  P.off_Sx = off; off += al((size_t)n * hs * ws * 4);
  P.off_Sy = off; off += al((size_t)n * hs * ws * 4);
  for (int k = 0; k < 4; ++k) { P.off_U[k] = off; off += al(px * 4); }
  P.off_vr = off; off += 17 * al(px * 4);
  P.off_rows = off; off += al((size_t)h * 8);
  P.off_cols = off; off += al((size_t)w * 8);
  P.off_UV = off; off += al(px * 8);
  P.bytes = off;
  return P;
}

size_t dis_scratch_bytes(int n, int h, int w) { return dis_plan(n, h, w).bytes; }

int dis_check_shape(int h, int w) {
  const DisPlan P = dis_plan(1, h, w);
  if (P.cs < DIS_FINEST) return -1;
  const int lw = P.lw[DIS_FINEST], lh = P.lh[DIS_FINEST];
  const int ws = 1 + (lw - DIS_PATCH) / DIS_STRIDE, hs = 1 + (lh - DIS_PATCH) / DIS_STRIDE;
  const int stripe = (hs + DIS_STRIPES - 1) / DIS_STRIPES;
  if (stripe * ws * 2 > SEARCH_LDS_FLOATS) return -2;
  return 0;
}

hipError_t launch_dis(const uint8_t* prev, const uint8_t* next, int n, int H, int W, float* flow, void* scratch,
                      hipStream_t st) {
  const DisPlan P = dis_plan(n, H, W);
  char* ws_ = (char*)scratch;
  auto img = [&](int s, int which) { return (uint8_t*)(ws_ + P.off_img[s]) + (size_t)which * n * P.lh[s] * P.lw[s]; };
  // pyramid (prepareBuffers): the finest level from the frames, each coarser one from the level below
  for (int s = DIS_FINEST; s <= P.cs; ++s) {
    const uint8_t* src0 = s == DIS_FINEST ? prev : img(s - 1, 0);
    const uint8_t* src1 = s == DIS_FINEST ? next : img(s - 1, 1);
    const int sh = s == DIS_FINEST ? H : P.lh[s - 1], sw = s == DIS_FINEST ? W : P.lw[s - 1];
    hipError_t e = launch_area_resize(src0, n, sh, sw, 1, P.lh[s], P.lw[s], img(s, 0), st);
    if (e == hipSuccess) e = launch_area_resize(src1, n, sh, sw, 1, P.lh[s], P.lw[s], img(s, 1), st);
    if (e != hipSuccess) return e;
  }
  uint8_t* I1e = (uint8_t*)(ws_ + P.off_I1e);
  int16_t* gx = (int16_t*)(ws_ + P.off_gx);
  int16_t* gy = (int16_t*)(ws_ + P.off_gy);
  float* aux = (float*)(ws_ + P.off_aux);
  float* T = (float*)(ws_ + P.off_T);
  float* Sx = (float*)(ws_ + P.off_Sx);
  float* Sy = (float*)(ws_ + P.off_Sy);
  float* Ucur[2] = {(float*)(ws_ + P.off_U[0]), (float*)(ws_ + P.off_U[1])};
  float* Unext[2] = {(float*)(ws_ + P.off_U[2]), (float*)(ws_ + P.off_U[3])};
  const size_t fpx = (size_t)n * P.lh[DIS_FINEST] * P.lw[DIS_FINEST];
  float* vr = (float*)(ws_ + P.off_vr);
  const size_t vstride = al(fpx * 4) / 4;
  VrBufs b;
  float** vp[17] = {&b.avg, &b.Iz, &b.Ix, &b.Iy, &b.Ixz, &b.Iyz, &b.Ixx, &b.Ixy, &b.Iyy,
                    &b.a11, &b.a12, &b.a22, &b.b1, &b.b2, &b.dU, &b.dV, &b.phi};
  for (int k = 0; k < 17; ++k) *vp[k] = vr + k * vstride;
  int2* rows = (int2*)(ws_ + P.off_rows);
  int2* cols = (int2*)(ws_ + P.off_cols);
  // the coarsest level starts from zero flow
  hipError_t e = hipMemsetAsync(Ucur[0], 0, (size_t)n * P.lh[P.cs] * P.lw[P.cs] * 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(Ucur[1], 0, (size_t)n * P.lh[P.cs] * P.lw[P.cs] * 4, st);
  if (e != hipSuccess) return e;
  const float zeta2 = 0.1f * 0.1f, eps2 = 0.001f * 0.001f;
  for (int s = P.cs; s >= DIS_FINEST; --s) {
    const int h = P.lh[s], w = P.lw[s];
    const int ws = 1 + (w - DIS_PATCH) / DIS_STRIDE, hs = 1 + (h - DIS_PATCH) / DIS_STRIDE;
    const size_t px = (size_t)n * h * w;
    const uint8_t* I0 = img(s, 0);
    const uint8_t* I1 = img(s, 1);
    hipLaunchKernelGGL(pad_rep_kernel, g256((size_t)n * (h + 2 * DIS_BORDER) * (w + 2 * DIS_BORDER)), dim3(256), 0, st, I1,
                       n, h, w, I1e);
    hipLaunchKernelGGL(sobel_kernel, g256(px), dim3(256), 0, st, I0, n, h, w, gx, gy);
    hipLaunchKernelGGL(tensor_h_kernel, g256((size_t)n * h), dim3(256), 0, st, gx, gy, n, h, w, ws, aux);
    hipLaunchKernelGGL(tensor_v_kernel, g256((size_t)n * ws), dim3(256), 0, st, aux, n, h, ws, hs, T);
    SearchArgs sa;
    sa.n = n; sa.h = h; sa.w = w; sa.hs = hs; sa.ws = ws;
    sa.stripe = (hs + DIS_STRIPES - 1) / DIS_STRIPES;
    sa.first_level = s == P.cs;
    sa.I0 = I0; sa.I1e = I1e; sa.gx = gx; sa.gy = gy; sa.T = T; sa.Ux = Ucur[0]; sa.Uy = Ucur[1]; sa.Sx = Sx; sa.Sy = Sy;
    hipLaunchKernelGGL(search_kernel, dim3(DIS_STRIPES, (unsigned)n), dim3(64 * SEARCH_WAVES), 0, st, sa);
    hipLaunchKernelGGL(ranges_kernel, dim3(1), dim3(64), 0, st, h, w, rows, cols);
    hipLaunchKernelGGL(densify_kernel, g256(px), dim3(256), 0, st, I0, I1, Sx, Sy, rows, cols, n, h, w, hs, ws, Ucur[0],
                       Ucur[1]);
    // variational refinement (calcUV)
    float* U = Ucur[0];
    float* V = Ucur[1];
    hipLaunchKernelGGL(vr_warp_kernel, g256(px), dim3(256), 0, st, I0, I1, U, V, n, h, w, b.avg, b.Iz);
    hipLaunchKernelGGL(vr_deriv_kernel, g256(px), dim3(256), 0, st, b.avg, n, h, w, b.Ix, b.Iy);
    hipLaunchKernelGGL(vr_deriv_kernel, g256(px), dim3(256), 0, st, b.Iz, n, h, w, b.Ixz, b.Iyz);
    hipLaunchKernelGGL(vr_deriv_kernel, g256(px), dim3(256), 0, st, b.Ix, n, h, w, b.Ixx, b.Ixy);
    hipLaunchKernelGGL(vr_deriv_kernel, g256(px), dim3(256), 0, st, b.Iy, n, h, w, (float*)nullptr, b.Iyy);
    e = hipMemsetAsync(b.dU, 0, px * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(b.dV, 0, px * 4, st);
    if (e != hipSuccess) return e;
    const size_t half = (size_t)n * h * ((w + 1) / 2);
    for (int it = 0; it < DIS_VR_ITER; ++it) {
      hipLaunchKernelGGL(vr_phi_kernel, g256(px), dim3(256), 0, st, U, V, b.dU, b.dV, n, h, w, 20.f / 2, eps2, b.phi);
      hipLaunchKernelGGL(vr_system_kernel, g256(px), dim3(256), 0, st, b, U, V, n, h, w, zeta2, eps2, 5.f / 2, 10.f / 2);
      for (int k = 0; k < DIS_SOR; ++k) {
        hipLaunchKernelGGL(vr_sor_kernel, g256(half), dim3(256), 0, st, b, n, h, w, 0, 1.6f);
        hipLaunchKernelGGL(vr_sor_kernel, g256(half), dim3(256), 0, st, b, n, h, w, 1, 1.6f);
      }
    }
    hipLaunchKernelGGL(vr_finish_kernel, g256(px), dim3(256), 0, st, U, V, b.dU, b.dV, px);
    if (s > DIS_FINEST) {  // resize(Ux[i], Ux[i - 1].size()) * 2
      e = launch_resize_lin(U, n, h, w, 1, P.lh[s - 1], P.lw[s - 1], 2.f, Unext[0], st);
      if (e == hipSuccess) e = launch_resize_lin(V, n, h, w, 1, P.lh[s - 1], P.lw[s - 1], 2.f, Unext[1], st);
      if (e != hipSuccess) return e;
      std::swap(Ucur[0], Unext[0]);
      std::swap(Ucur[1], Unext[1]);
    }
  }
  // merge(U, V) -> resize to the frame (INTER_LINEAR) * 2^finest
  float* UV = (float*)(ws_ + P.off_UV);
  const size_t fp = (size_t)n * P.lh[DIS_FINEST] * P.lw[DIS_FINEST];
  hipLaunchKernelGGL(interleave_kernel, g256(fp), dim3(256), 0, st, Ucur[0], Ucur[1], fp, UV);
  e = launch_resize_lin(UV, n, P.lh[DIS_FINEST], P.lw[DIS_FINEST], 2, H, W, (float)(1 << DIS_FINEST), flow, st);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

}  // namespace nst
