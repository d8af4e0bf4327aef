// region_api.cpp — C ABI of the region-blend compositor (include/nst_hip.h "Region-blend compositor").
#include <math.h>

#include <string>

#include "nst_hip.h"
#include "nst_internal.h"
#include "region_internal.h"

namespace nst {
bool decode_consts_for_preset(int preset, DecodeConsts& d);  // nst_api.cpp
}

using namespace nst;

namespace {

#define RG_LAUNCH(expr, what)                                                            \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      set_error(std::string(what) + " launch: " + hipGetErrorString(_e));                \
      return NST_E_HIP;                                                                  \
    }                                                                                    \
  } while (0)

// fill the source set from the caller's arrays
int make_sources(const float* const* src_y, const int* src_hw, const int* src_preset, int n_src, RegionSrcSet& ss,
                 const char* fn) {
  if (n_src < 0 || n_src > RG_MAX_SRC || (n_src > 0 && (!src_y || !src_hw || !src_preset))) {
    set_error(std::string(fn) + ": between 0 and " + std::to_string(RG_MAX_SRC) + " sources");
    return NST_E_INVALID;
  }
  ss.n_src = n_src;
  for (int s = 0; s < n_src; ++s) {
    if (!src_y[s] || src_hw[2 * s] <= 0 || src_hw[2 * s + 1] <= 0 || !decode_consts_for_preset(src_preset[s], ss.s[s].d)) {
      set_error(std::string(fn) + ": bad source " + std::to_string(s));
      return NST_E_INVALID;
    }
    ss.s[s].y = src_y[s];
    ss.s[s].h = src_hw[2 * s];
    ss.s[s].w = src_hw[2 * s + 1];
  }
  return NST_OK;
}

}  // namespace

extern "C" {

int nst_region_masks(int kind, int count, int n_gen, const int* ivals, const double* dvals, const double* lo,
                     const double* hi, const int* rects, const double* points, const double* divisor, int h, int w,
                     float* masks, float* scratch, void* stream) {
  if (kind < NST_RG_RECTS || kind > NST_RG_CONCENTRIC || count <= 0 || count > RG_MAX || n_gen < 0 ||
      n_gen > count || h <= 0 || w <= 0 || !masks || !ivals || !dvals) {
    set_error("nst_region_masks: invalid arguments");
    return NST_E_INVALID;
  }
  if ((kind == NST_RG_RECTS && n_gen > 0 && !rects) || (kind == NST_RG_VORONOI && (!points || !divisor)) ||
      (kind != NST_RG_RECTS && kind != NST_RG_VORONOI && (!lo || !hi)) || (kind == NST_RG_WAVES && !scratch)) {
    set_error("nst_region_masks: missing geometry table for this kind");
    return NST_E_INVALID;
  }
  RegionGeomDev g = {};
  g.kind = kind; g.count = count; g.n_gen = n_gen;
  g.i0 = ivals[0]; g.i1 = ivals[1]; g.i2 = ivals[2];
  // double -> float casts round to nearest: torch's cast of a Python float scalar against a float32 tensor
  g.f0 = (float)dvals[0]; g.f1 = (float)dvals[1]; g.f2 = (float)dvals[2]; g.f3 = (float)dvals[3];
  for (int k = 0; k < n_gen; ++k) {
    if (lo && hi) { g.lo[k] = (float)lo[k]; g.hi[k] = (float)hi[k]; }
    if (kind == NST_RG_RECTS)
      for (int j = 0; j < 4; ++j) g.rect[k][j] = rects[4 * k + j];
    if (kind == NST_RG_VORONOI) {
      g.px[k] = (float)points[2 * k]; g.py[k] = (float)points[2 * k + 1]; g.pdiv[k] = (float)divisor[k];
    }
  }
  if ((kind == NST_RG_DIAGONAL || kind == NST_RG_CONCENTRIC) && !(g.f3 > 0.f)) {
    set_error("nst_region_masks: the normalising maximum must be positive");
    return NST_E_INVALID;
  }
  RG_LAUNCH(launch_region_masks(g, h, w, masks, scratch, (hipStream_t)stream), "region_masks");
  return NST_OK;
}

int nst_region_feather(float* masks, int k, int h, int w, const float* taps, int ks, float* scratch, void* stream) {
  if (!masks || !taps || !scratch || k <= 0 || h <= 0 || w <= 0 || ks < 1 || ks > RG_MAX_TAPS || (ks & 1) == 0) {
    set_error("nst_region_feather: invalid arguments (odd ks <= " + std::to_string(RG_MAX_TAPS) + ")");
    return NST_E_INVALID;
  }
  if (ks / 2 >= h || ks / 2 >= w) {  // F.pad(mode='reflect') needs pad < dim (torch raises too)
    set_error("nst_region_feather: padding " + std::to_string(ks / 2) + " must be smaller than the frame " +
              std::to_string(h) + "x" + std::to_string(w));
    return NST_E_SHAPE;
  }
  RG_LAUNCH(launch_region_feather(masks, k, h, w, taps, ks, scratch, (hipStream_t)stream), "region_feather");
  return NST_OK;
}

int nst_region_rotate(const float* in, int k, int h, int w, double angle_deg, float* out, void* stream) {
  if (!in || !out || in == out || k <= 0 || k > RG_MAX || h <= 0 || w <= 0) {
    set_error("nst_region_rotate: invalid arguments");
    return NST_E_INVALID;
  }
  // cv2.getRotationMatrix2D((W/2, H/2), angle, 1.0) then invertAffineTransform (warpAffine without
  // WARP_INVERSE_MAP maps destination pixels through the inverse)
  const double a = angle_deg * (M_PI / 180.0);
  const double al = cos(a), be = sin(a), cx = w / 2.0, cy = h / 2.0;
  const double M[6] = {al, be, (1 - al) * cx - be * cy, -be, al, be * cx + (1 - al) * cy};
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1.0 / D : 0.0;
  const double A11 = M[4] * D, A22 = M[0] * D, A12 = -M[1] * D, A21 = -M[3] * D;
  const double b1 = -A11 * M[2] - A12 * M[5], b2 = -A21 * M[2] - A22 * M[5];
  const double inv[6] = {A11, A12, b1, A21, A22, b2};
  RG_LAUNCH(launch_region_rotate(in, k, h, w, inv, out, (hipStream_t)stream), "region_rotate");
  return NST_OK;
}

int nst_region_morph_scratch_floats(int k, int h, int w, size_t* out) {
  if (k <= 0 || k > RG_MAX || h <= 0 || w <= 0 || !out) {
    set_error("nst_region_morph_scratch_floats: invalid arguments");
    return NST_E_INVALID;
  }
  *out = 3 * (size_t)k * h * w + (size_t)4 * k * 1024 + 4 * (size_t)k + 16;
  return NST_OK;
}

int nst_region_morph(const float* in, int k, int h, int w, int mode, double frequency, double time_offset,
                     double max_disp, const double* offsets, float* out, float* scratch, size_t scratch_floats,
                     void* stream) {
  size_t need = 0;
  if (!in || !out || in == out || !offsets || mode < 0 || mode > 3 || nst_region_morph_scratch_floats(k, h, w, &need) ||
      !scratch || scratch_floats < need) {
    set_error("nst_region_morph: invalid arguments (scratch: nst_region_morph_scratch_floats)");
    return NST_E_INVALID;
  }
  MorphDevHost m = {};
  m.mode = mode; m.k = k; m.freq = frequency; m.t = time_offset; m.max_disp = max_disp;
  for (int j = 0; j < k; ++j)
    for (int f = 0; f < 2; ++f)
      for (int o = 0; o < 2; ++o)
        for (int c = 0; c < 2; ++c) m.off[j][f][o][c] = offsets[((j * 2 + f) * 2 + o) * 2 + c];
  RG_LAUNCH(launch_region_morph(m, in, h, w, out, scratch, (hipStream_t)stream), "region_morph");
  return NST_OK;
}

int nst_region_bbox(const float* masks, int k, int h, int w, float threshold, int* bbox, void* stream) {
  if (!masks || !bbox || k <= 0 || k > 64 || h <= 0 || w <= 0) {
    set_error("nst_region_bbox: invalid arguments");
    return NST_E_INVALID;
  }
  RG_LAUNCH(launch_region_bbox(masks, k, h, w, threshold, bbox, (hipStream_t)stream), "region_bbox");
  return NST_OK;
}

int nst_region_scratch_floats(int n, int h, int w, int crops, int with_orig, size_t* out) {
  if (n <= 0 || h <= 0 || w <= 0 || !out) { set_error("nst_region_scratch_floats: invalid arguments"); return NST_E_INVALID; }
  const size_t plane = (size_t)n * 4 * h * w;
  *out = crops ? (with_orig ? plane : 3 * plane) : 0;
  return NST_OK;
}

int nst_region_composite_u8(const float* const* src_y, const int* src_hw, const int* src_preset, int n_src,
                            const int* n_terms, const int* term_src, const float* term_w, int n_regions,
                            const int* boxes, const uint8_t* orig, const float* masks, int n, int h, int w,
                            float* scratch, size_t scratch_floats, uint8_t* out, float* out_f32, void* stream) {
  if (!n_terms || !term_src || !term_w || !masks || n_regions <= 0 || n_regions > RG_MAX || n <= 0 || h <= 0 ||
      w <= 0 || (!out && !out_f32)) {
    set_error("nst_region_composite_u8: invalid arguments");
    return NST_E_INVALID;
  }
  RegionSrcSet ss = {};
  int rc = make_sources(src_y, src_hw, src_preset, n_src, ss, "nst_region_composite_u8");
  if (rc != NST_OK) return rc;
  RegionTermsDev t = {};
  t.n_regions = n_regions;
  for (int k = 0; k < n_regions; ++k) {
    if (n_terms[k] < 0 || n_terms[k] > RG_TERMS) {
      set_error("nst_region_composite_u8: region " + std::to_string(k) + " has more than 9 terms");
      return NST_E_INVALID;
    }
    t.n_terms[k] = (int8_t)n_terms[k];
    for (int j = 0; j < n_terms[k]; ++j) {
      const int s = term_src[k * RG_TERMS + j];
      if (s < -1 || s >= n_src || (s == -1 && !orig)) {
        set_error("nst_region_composite_u8: region " + std::to_string(k) + " term " + std::to_string(j) +
                  (s == -1 ? " uses the original frame but none was given" : " names a missing source"));
        return NST_E_INVALID;
      }
      t.src[k][j] = (int8_t)s;
      t.w[k][j] = term_w[k * RG_TERMS + j];
    }
    if (boxes) {
      const int* b = boxes + 4 * k;
      if (b[0] < 0 || b[1] < 0 || b[2] > w || b[3] > h || b[0] >= b[2] || b[1] >= b[3]) {
        set_error("nst_region_composite_u8: crop box " + std::to_string(k) + " outside the frame");
        return NST_E_SHAPE;
      }
      for (int j = 0; j < 4; ++j) t.box[k][j] = b[j];
    }
  }
  hipStream_t st = (hipStream_t)stream;
  if (!boxes) {
    RG_LAUNCH(launch_region_composite(ss, t, orig, masks, n, h, w, out, out_f32, st), "region_composite");
    return NST_OK;
  }
  size_t need = 0;
  nst_region_scratch_floats(n, h, w, 1, orig != nullptr, &need);
  if (!scratch || scratch_floats < need) {
    set_error("nst_region_composite_u8: crops need " + std::to_string(need) + " scratch floats");
    return NST_E_WORKSPACE;
  }
  const size_t plane = (size_t)n * 4 * h * w;
  RG_LAUNCH(launch_region_crops(ss, t, orig, masks, n, h, w, scratch, orig ? nullptr : scratch + plane, out, out_f32,
                                st),
            "region_crops");
  return NST_OK;
}

int nst_region_crop_input(const uint8_t* frames, int n, int h, int w, const int* box, int out_h, int out_w, float* out,
                          void* stream) {
  if (!frames || !box || !out || n <= 0 || h <= 0 || w <= 0 || out_h <= 0 || out_w <= 0 || box[0] < 0 || box[1] < 0 ||
      box[2] > w || box[3] > h || box[0] >= box[2] || box[1] >= box[3]) {
    set_error("nst_region_crop_input: invalid arguments");
    return NST_E_INVALID;
  }
  RG_LAUNCH(launch_region_crop_input(frames, n, h, w, box[0], box[1], box[2], box[3], out_h, out_w, out,
                                     (hipStream_t)stream),
            "region_crop_input");
  return NST_OK;
}

int nst_region_resize(const float* y, int n, int h, int w, int preset, int fit_h, int fit_w, int out_h, int out_w,
                      float* out, void* stream) {
  RegionSrcDev s = {};
  if (!y || !out || n <= 0 || h <= 0 || w <= 0 || fit_h <= 0 || fit_w <= 0 || out_h <= 0 || out_w <= 0 ||
      !decode_consts_for_preset(preset, s.d)) {
    set_error("nst_region_resize: invalid arguments");
    return NST_E_INVALID;
  }
  s.y = y; s.h = h; s.w = w;
  RG_LAUNCH(launch_region_resize_fit(s, n, fit_h, fit_w, out_h, out_w, out, (hipStream_t)stream), "region_resize");
  return NST_OK;
}

}  // extern "C"
