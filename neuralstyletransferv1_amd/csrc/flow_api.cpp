// flow_api.cpp — C ABI of the temporal stage (include/nst_hip.h "Temporal stage").
#include <string>

#include "flow_internal.h"
#include "nst_hip.h"
#include "nst_internal.h"

using namespace nst;

#define FL_LAUNCH(expr, what)                                                            \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      set_error(std::string(what) + " launch: " + hipGetErrorString(_e));                \
      return NST_E_HIP;                                                                  \
    }                                                                                    \
  } while (0)

extern "C" {

int nst_gray_u8(const uint8_t* rgb, int n, int h, int w, uint8_t* gray, void* stream) {
  if (!rgb || !gray || n <= 0 || h <= 0 || w <= 0) { set_error("nst_gray_u8: invalid arguments"); return NST_E_INVALID; }
  FL_LAUNCH(launch_gray(rgb, (size_t)n * h * w, gray, (hipStream_t)stream), "gray");
  return NST_OK;
}

int nst_flow_scratch_floats(int h, int w, size_t* out) {
  if (h <= 0 || w <= 0 || !out) { set_error("nst_flow_scratch_floats: invalid arguments"); return NST_E_INVALID; }
  *out = farneback_scratch_floats(h, w);
  return NST_OK;
}

int nst_flow_farneback(const uint8_t* prev, const uint8_t* next, int h, int w, double pyr_scale, int levels,
                       int winsize, int iterations, int poly_n, double poly_sigma, float* flow, float* scratch,
                       size_t scratch_floats, void* stream) {
  if (!prev || !next || !flow || !scratch || h < 2 || w < 2 || !(pyr_scale > 0 && pyr_scale < 1) || levels < 0 ||
      winsize < 1 || (winsize & 1) == 0 || iterations < 1 || poly_n < 1 || poly_n > 8 || scratch_floats < farneback_scratch_floats(h, w)) {
    set_error("nst_flow_farneback: invalid arguments (odd winsize, poly_n 1..8, scratch per nst_flow_scratch_floats)");
    return NST_E_INVALID;
  }
  FL_LAUNCH(launch_farneback(prev, next, h, w, pyr_scale, levels, winsize, iterations, poly_n, poly_sigma, flow, scratch,
                             (hipStream_t)stream),
            "farneback");
  return NST_OK;
}

int nst_flow_downscale_gray(const uint8_t* gray, int h, int w, int ds, uint8_t* out, void* stream) {
  if (!gray || !out || ds < 2) { set_error("nst_flow_downscale_gray: invalid arguments (ds >= 2)"); return NST_E_INVALID; }
  if (h / ds < 2 || w / ds < 2) {
    set_error("nst_flow_downscale_gray: frame " + std::to_string(w) + "x" + std::to_string(h) + " too small for factor " +
              std::to_string(ds));
    return NST_E_SHAPE;
  }
  FL_LAUNCH(launch_area_resize(gray, 1, h, w, 1, h / ds, w / ds, out, (hipStream_t)stream), "area_resize");
  return NST_OK;
}

int nst_flow_dis_scratch_bytes(int n, int h, int w, size_t* out) {
  if (n <= 0 || h <= 0 || w <= 0 || !out) { set_error("nst_flow_dis_scratch_bytes: invalid arguments"); return NST_E_INVALID; }
  const int rc = dis_check_shape(h, w);
  if (rc != 0) {
    set_error(std::string("nst_flow_dis: frame ") + std::to_string(w) + "x" + std::to_string(h) +
              (rc == -1 ? " is too small for DIS PRESET_FAST (its coarsest pyramid level would lie below the finest, 2)"
                        : " is too wide for the inverse search's stripe buffer"));
    return NST_E_SHAPE;
  }
  *out = dis_scratch_bytes(n, h, w);
  return NST_OK;
}

int nst_flow_dis(const uint8_t* prev, const uint8_t* next, int n, int h, int w, float* flow, void* scratch,
                 size_t scratch_bytes, void* stream) {
  size_t need = 0;
  if (!prev || !next || !flow || !scratch) { set_error("nst_flow_dis: invalid arguments"); return NST_E_INVALID; }
  const int rc = nst_flow_dis_scratch_bytes(n, h, w, &need);
  if (rc != NST_OK) return rc;
  if (scratch_bytes < need) { set_error("nst_flow_dis: scratch too small"); return NST_E_WORKSPACE; }
  FL_LAUNCH(launch_dis(prev, next, n, h, w, flow, scratch, (hipStream_t)stream), "dis");
  return NST_OK;
}

int nst_resize_area_u8(const uint8_t* in, int n, int h, int w, int c, uint8_t* out, int out_h, int out_w, void* stream) {
  if (!in || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || c > 4 || out_h <= 0 || out_w <= 0 || out_h > h || out_w > w) {
    set_error("nst_resize_area_u8: invalid arguments (downscaling only: 0 < out <= in, 1..4 channels)");
    return NST_E_INVALID;
  }
  FL_LAUNCH(launch_area_resize(in, n, h, w, c, out_h, out_w, out, (hipStream_t)stream), "area_resize");
  return NST_OK;
}

int nst_flow_upscale(const float* flow_small, int hs, int ws, int h, int w, float mul, float* flow, void* stream) {
  if (!flow_small || !flow || hs <= 0 || ws <= 0 || h <= 0 || w <= 0) {
    set_error("nst_flow_upscale: invalid arguments");
    return NST_E_INVALID;
  }
  FL_LAUNCH(launch_resize_lin(flow_small, 1, hs, ws, 2, h, w, mul, flow, (hipStream_t)stream), "flow_upscale");
  return NST_OK;
}

int nst_flow_fuse(const float* curr, const float* prev, const float* flow, int h, int w, float alpha,
                  float one_minus_alpha, float* out, void* stream) {
  if (!curr || !prev || !flow || !out || out == prev || h <= 0 || w <= 0) {
    set_error("nst_flow_fuse: invalid arguments");
    return NST_E_INVALID;
  }
  FL_LAUNCH(launch_flow_fuse(curr, prev, flow, h, w, alpha, one_minus_alpha, out, (hipStream_t)stream), "flow_fuse");
  return NST_OK;
}

int nst_motion_alpha(const float* flow, int h, int w, float motion_norm, double sigma, float max_alpha, float span,
                     float* alpha, float* scratch, void* stream) {
  if (!flow || !alpha || !scratch || h <= 0 || w <= 0 || !(motion_norm > 0) || !(sigma > 0) || sigma > 7.5) {
    set_error("nst_motion_alpha: invalid arguments");
    return NST_E_INVALID;
  }
  FL_LAUNCH(launch_motion_alpha(flow, h, w, motion_norm, sigma, max_alpha, span, alpha, scratch, (hipStream_t)stream),
            "motion_alpha");
  return NST_OK;
}

}  // extern "C"
