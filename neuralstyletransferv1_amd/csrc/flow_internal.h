// flow_internal.h — launchers of the temporal-stage kernels (flow_ops.hip), called by flow_api.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace nst {

hipError_t launch_gray(const uint8_t* rgb, size_t npix, uint8_t* gray, hipStream_t st);
size_t farneback_scratch_floats(int h, int w);
hipError_t launch_farneback(const uint8_t* prev, const uint8_t* next, int h, int w, double pyr_scale, int levels,
                            int winsize, int iterations, int poly_n, double poly_sigma, float* flow, float* scratch,
                            hipStream_t st);
// cv2.resize INTER_AREA of n u8 images [h][w][ch] -> [oh][ow][ch] (downscaling: oh <= h, ow <= w)
// DIS optical flow (dis_ops.hip): scratch bytes for n pairs of h x w frames; 0 = ok, -1 frame too small for
// PRESET_FAST's pyramid, -2 too wide for the inverse search's LDS stripe
size_t dis_scratch_bytes(int n, int h, int w);
int dis_check_shape(int h, int w);
hipError_t launch_dis(const uint8_t* prev, const uint8_t* next, int n, int h, int w, float* flow, void* scratch,
                      hipStream_t st);
hipError_t launch_area_resize(const uint8_t* in, int n, int h, int w, int ch, int oh, int ow, uint8_t* out,
                              hipStream_t st);
hipError_t launch_resize_lin(const float* in, int k, int h, int w, int c, int oh, int ow, float mul, float* out,
                             hipStream_t st);
hipError_t launch_flow_fuse(const float* curr, const float* prev, const float* flow, int h, int w, float a, float oma,
                            float* out, hipStream_t st);
hipError_t launch_motion_alpha(const float* flow, int h, int w, float norm, double sigma, float max_alpha, float span,
                               float* alpha, float* tmp, hipStream_t st);

}  // namespace nst
