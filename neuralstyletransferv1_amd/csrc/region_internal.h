// region_internal.h — launchers of the region-blend compositor kernels (region_ops.hip), called by the
// C ABI in region_api.cpp.  Not part of the public ABI (include/nst_hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "post_common.h"

namespace nst {

constexpr int RG_MAX = 32;        // regions per composite (NST_REGION_MAX)
constexpr int RG_TERMS = 9;       // models A..H + the original per region
constexpr int RG_MAX_SRC = 16;    // model outputs (x scales) per composite
constexpr int RG_MAX_TAPS = 511;  // Gaussian feather taps (feather <= 255 px)

// geometry of one generate_region_masks call, fp32 constants already rounded as torch rounds them
struct RegionGeomDev {
  int kind, count, n_gen;
  int i0, i1, i2;      // diagonal: direction; radial/spiral/concentric: cx, cy; waves: direction
  float f0, f1, f2, f3;  // radial: rotation; spiral: tightness, rotation, max(H,W); waves: frequency, amplitude,
                         // phase; concentric: r.max(); diagonal: diagonal.max()
  float lo[RG_MAX], hi[RG_MAX];  // band thresholds i/count, (i+1)/count (or wedge bounds)
  int rect[RG_MAX][4];           // RECTS: y1, y2, x1, x2
  float px[RG_MAX], py[RG_MAX], pdiv[RG_MAX];  // VORONOI: seed points, distance divisor (0 = unweighted)
};

struct RegionSrcDev {
  const float* y;
  int h, w;
  DecodeConsts d;
};

// per-region terms of a composite: region k blends n_terms[k] sources (src -1 = the original frame)
struct RegionTermsDev {
  int n_regions;
  int8_t n_terms[RG_MAX];
  int8_t src[RG_MAX][RG_TERMS];
  float w[RG_MAX][RG_TERMS];
  int box[RG_MAX][4];  // crops: padded bbox x1, y1, x2, y2
};

struct RegionSrcSet {
  int n_src;
  RegionSrcDev s[RG_MAX_SRC];
};
// both tables travel as kernel arguments (4 KiB limit with the pointers and sizes beside them)
static_assert(sizeof(RegionSrcSet) + sizeof(RegionTermsDev) <= 3600, "region tables exceed the kernarg budget");

hipError_t launch_region_masks(const RegionGeomDev& g, int h, int w, float* masks, float* scratch, hipStream_t st);
hipError_t launch_region_feather(float* masks, int k, int h, int w, const float* taps, int ks, float* scratch,
                                 hipStream_t st);
hipError_t launch_region_rotate(const float* in, int k, int h, int w, const double* M, float* out, hipStream_t st);
hipError_t launch_region_bbox(const float* masks, int k, int h, int w, float thr, int* bbox, hipStream_t st);
hipError_t launch_region_composite(const RegionSrcSet& ss, const RegionTermsDev& t, const uint8_t* orig,
                                   const float* masks, int n, int h, int w, uint8_t* out, float* out_f32,
                                   hipStream_t st);
hipError_t launch_region_crops(const RegionSrcSet& ss, const RegionTermsDev& t, const uint8_t* orig,
                               const float* masks, int n, int h, int w, float* canvas, float* tmp, uint8_t* out,
                               float* out_f32, hipStream_t st);
hipError_t launch_region_crop_input(const uint8_t* frames, int n, int h, int w, int x1, int y1, int x2, int y2,
                                    int oh, int ow, float* out, hipStream_t st);
struct MorphDevHost {
  int mode, k;
  double freq, t, max_disp;
  double off[RG_MAX][2][2][2];
};
hipError_t launch_region_morph(const MorphDevHost& m, const float* in, int h, int w, float* out, float* scratch,
                               hipStream_t st);
hipError_t launch_region_resize_fit(const RegionSrcDev& s, int n, int fh, int fw, int oh, int ow, float* out,
                                    hipStream_t st);

}  // namespace nst
