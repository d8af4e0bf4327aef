// seg_internal.h — shared declarations of the DeepLab v3+ mask program (configs[4]):
// the K-streaming implicit-GEMM conv (conv_gemm.hip), the segmentation / mask / resampling kernels
// (seg_ops.hip) and the C ABI that drives them (seg_deeplab.cpp).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "nst_hip.h"

namespace nst {

// One convolution as a GEMM: rows = output channels, columns = output pixels (n*ho*wo, NHWC order),
// K = taps x input channels streamed through LDS in stages of one tap x 128 bytes of channels
// (64 bf16 / 32 fp32).  Epilogue: y = acc * scale[c] + shift[c] (eval BatchNorm, or scale 1 + conv
// bias), + res (the bottleneck's identity / downsample branch), ReLU; stored at channel offset
// out_off of an NHWC buffer with channel stride out_cs (so concatenations are written in place).
struct GemmConvParams {
  const void* in;          // NHWC [n][hi][wi][cs] in the compute dtype
  int hi, wi, cs;          // source extent and channel stride (elements, multiple of the stage width)
  int cin;                 // channels per tap read (multiple of the stage width; weights zero past the real count)
  int kh, kw, stride, dil, pad;
  int ho, wo, npix;        // output extent, npix = n * ho * wo
  const void* wpk;         // packed weights [cout/64][stage][64 rows][128 B]
  const float* scale;      // [coutp]
  const float* shift;      // [coutp]
  const void* res;         // residual NHWC [npix][res_cs] (compute dtype) or nullptr
  int res_cs;
  int relu;
  void* out;               // NHWC [npix][out_cs] (compute dtype, or fp32 if out_f32)
  int out_cs, out_off;
  int cout_store;          // output channels written (multiple of 4; channels past the real count get 0)
  int out_f32;
  // taps that touch the image for some output pixel (the others only read zero padding and add exact zeros:
  // skipped — the ASPP's dilation-12/18 convs on a 9x16 map keep 3 and 1 of their 9 taps)
  int ntaps;
  unsigned char taps[64];  // ky * kw + kx
  // split-K (small GEMMs): blockIdx.z = K slice; slices write fp32 partials [ksplit][npix][cout_store] to
  // `partial` and gemm_splitk_reduce applies the epilogue, summing the slices in fixed order (deterministic)
  int ksplit;
  float* partial;
};

// dtype: NST_DT_F32 / NST_DT_BF16 / NST_DT_F16.  Picks the tile shape and the K split from the GEMM's size; p.taps /
// p.ntaps are filled here (gemm_live_taps).  partial: scratch of gemm_partial_bytes(...) bytes or nullptr
// (no split).
hipError_t launch_gemm_conv(int dtype, GemmConvParams& p, hipStream_t st);
// bytes of split-K scratch the launch of this conv would use (0: no split)
size_t gemm_partial_bytes(int dtype, const GemmConvParams& p);
// stage width in channels for a dtype (64 bf16 / fp16, 32 fp32)
inline int gemm_stage_channels(int dtype) { return (dtype == NST_DT_F32 || dtype == NST_DT_F32S) ? 32 : 64; }

// ---- seg_ops.hip ----
// Stem im2col for the 7x7/2 pad-3 first conv: source = frames u8 NHWC [n][h][w][3] normalised as
// sky_swap.py:179-183 preprocess_pil, or the module input f32 NCHW [n][3][h][w]; row k = (ky*7+kx)*3+c
// of output pixel (n,oy,ox) -> col [npix][kp] (zero padding, zero columns k >= 147).
hipError_t launch_seg_stem_im2col(int dtype, const void* x, int x_u8, int n, int h, int w, int ho, int wo, int kp,
                                  void* col, hipStream_t st);
// MaxPool2d(3, 2, 1) NHWC (channel stride c)
hipError_t launch_seg_maxpool(int dtype, const void* in, int n, int h, int w, int c, void* out, int ho, int wo,
                              hipStream_t st);
// AdaptiveAvgPool2d(1): [n][h][w][cs] -> [n][cs] (c channels averaged)
hipError_t launch_seg_avgpool(int dtype, const void* in, int n, int hw, int c, int cs, void* out, hipStream_t st);
// bilinear align_corners=True resize NHWC [n][h][w][cs_in] (c channels) -> channel offset off of
// [n][oh][ow][cs_out]; h == w == 1 broadcasts
hipError_t launch_seg_resize_ac(int dtype, const void* in, int n, int h, int w, int c, int cs_in, void* out, int oh,
                                int ow, int cs_out, int off, hipStream_t st);
// final logits [n][h4][w4][ncs] fp32 -> bilinear align_corners=True to [h][w], argmax over nc classes
// -> pred u8 [n][h][w]; logits_out (optional) f32 NCHW [n][nc][h][w]
hipError_t launch_seg_upsample_argmax(const float* logits, int n, int h4, int w4, int nc, int ncs, int h, int w,
                                      uint8_t* pred, float* logits_out, hipStream_t st);
// mask = 255 where pred is one of the ids (sky_swap.py:199-202); ids as a 256-bit set
struct SegIdSet {
  uint32_t bits[8];
};
hipError_t launch_seg_select(const uint8_t* pred, size_t npix, SegIdSet ids, uint8_t* mask, hipStream_t st);
// binary rectangle morphology (cv2.dilate / cv2.erode, kernel ones(k,k), default border): separable
// max / min over the window clipped to the image; op 0 dilate, 1 erode; tmp: n*h*w bytes
hipError_t launch_seg_morph(const uint8_t* in, int n, int h, int w, int k, int op, uint8_t* tmp, uint8_t* out,
                            hipStream_t st);
// cv2.GaussianBlur(m, (0,0), sigma) on u8 masks -> u8 (same restatement as the feather of nst_ops.hip)
hipError_t launch_seg_gauss_u8(const uint8_t* m, int n, int h, int w, float sigma, float* tmp, uint8_t* out,
                               hipStream_t st);
// cv2.resize(INTER_LINEAR) of u8 images [n][h][w][c] (fixed-point 11-bit taps)
hipError_t launch_resize_linear_cv_u8(const uint8_t* in, int n, int h, int w, int c, uint8_t* out, int oh, int ow,
                                      const int* xofs, const short* xalpha, const int* yofs, const short* ybeta,
                                      hipStream_t st);
// PIL Image.resize(LANCZOS) of RGB u8 frames: horizontal pass over rows [y0, y0+th) into tmp
// [n][th][ow][3], vertical pass into out [n][oh][ow][3]; integer taps (22 fractional bits)
hipError_t launch_resize_pil_u8(const uint8_t* in, int n, int h, int w, uint8_t* tmp, int y0, int th, uint8_t* out,
                                int oh, int ow, const int* xb, const int* xk, int kx, const int* yb, const int* yk,
                                int ky, int need_h, int need_v, hipStream_t st);

}  // namespace nst
