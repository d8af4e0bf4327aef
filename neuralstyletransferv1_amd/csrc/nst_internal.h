// nst_internal.h — shared declarations between the HIP translation units of libnst_hip.so.
// Not part of the public ABI (that is include/nst_hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <cmath>
#include <cstring>
#include <string>

#include "nst_hip.h"

namespace nst {

// IEEE binary16 of a host float, round to nearest even (values >= 65520 -> inf, as the device's
// v_cvt_pk_f16_f32): weight packing for NST_DT_F16
inline uint16_t f32_to_f16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
  uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return sign | 0x7e00u;   // NaN
  if (a >= 0x477ff000u) return sign | 0x7c00u;  // rounds past 65504
  if (a >= 0x38800000u) {                       // normal: rebias the exponent, RNE on the 13 dropped bits
    a -= 0x38000000u;
    a += 0xfffu + ((a >> 13) & 1u);
    return sign | (uint16_t)(a >> 13);
  }
  float af;  // subnormal or zero: units of 2^-24 (exact power-of-two scaling), nearbyint rounds to even
  std::memcpy(&af, &a, 4);
  return sign | (uint16_t)std::nearbyint(af * 16777216.0f);
}
// bfloat16 of a host float, round to nearest even (NaN stays NaN): weight packing for NST_DT_BF16
inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
// fp16 bits -> the value (exact)
inline float f16_to_f32(uint16_t h) {
  const int e = (h >> 10) & 31, m = h & 1023;
  float v = e == 0 ? std::ldexp((float)m, -24) : (e == 31 ? INFINITY : std::ldexp((float)(m | 1024), e - 25));
  return (h & 0x8000u) ? -v : v;
}
// Dtype of the HBM activations: 4-byte for fp32 and the split-fp16 mode, 2-byte for bf16 / fp16
inline bool f32_storage(int dtype) { return dtype == NST_DT_F32 || dtype == NST_DT_F32S; }
inline size_t act_elem_bytes(int dtype) { return f32_storage(dtype) ? 4 : 2; }

// ---- error plumbing (thread-local last error, see nst_last_error) ----
void set_error(const std::string& msg);
#define NST_HIP_CHECK(expr)                                                               \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      ::nst::set_error(std::string(#expr) + " failed: " + hipGetErrorString(_e));         \
      return NST_E_HIP;                                                                   \
    }                                                                                     \
  } while (0)

// ---- how a conv layer's input tile is sourced ----
enum InKind { IN_ACT = 0, IN_U8_NHWC = 1, IN_F32_NCHW = 2 };
// ---- what a conv layer's epilogue writes ----
enum OutKind { OUT_ACT = 0, OUT_U8_NHWC = 1, OUT_F32_NCHW = 2 };

// Virtual-coordinate -> source-pixel mapping of the conv input along one axis.
//   AX_REFLECT          ReflectionPad2d(pad)                       transformer_net.py:47-48, model.py:10
//   AX_REFLECT_UP2      interpolate(nearest, x2) then reflect pad  transformer_net.py:95-97, model.py:92-96
//   AX_ZERO             Conv2d(padding=pad)                        transformer_net_nst.py:19,32-34
//   AX_ZERO_PREREFLECT  ReflectionPad2d(pre) then Conv2d(padding)  transformer_net_nst.py:74,99,76
//   AX_ZINSERT          ConvTranspose2d(3, s2, p1, op1) as a conv over the zero-inserted grid
//                                                                  transformer_net_nst.py:50-53
//   AX_CLAMP            clamp to the source grid (phase-mode nearest-x2 convs: reflect-pad(1) of the
//                       upsampled grid == clamp on the source grid)
enum AxisMode { AX_REFLECT = 0, AX_REFLECT_UP2 = 1, AX_ZERO = 2, AX_ZERO_PREREFLECT = 3, AX_ZINSERT = 4, AX_CLAMP = 5 };

// conv_kernel mappings (see conv_impl.h)
enum ConvMode { MODE_STD = 0, MODE_PHASE = 1, MODE_XSHIFT = 2, MODE_KYROT = 3, MODE_WSTAT = 4, MODE_WPHASE = 5, MODE_WS2 = 6, MODE_WS9 = 7,
                MODE_WS1S = 8 };  // WS1S: conv_ws1s.hip (split-operand stride-1 trunk conv)  // KYROT: conv_out9.hip, WSTAT: conv_wstat.hip, WPHASE: conv_wphase.hip, WS2: conv_ws2.hip, WS9: conv_ws9.hip

struct ConvParams {
  // input
  const void* in;
  int hs, ws;   // source spatial dims
  int cs;       // source channel stride (elements) for IN_ACT
  int axis_mode, pad, pre;
  const float2* in_norm;  // [n][cs] {scale, shift} of the producer's InstanceNorm, or nullptr
  int in_relu;            // 1 whenever in_norm is set (the prologue always applies ReLU after the IN)
  // residual join fused into the fill (res_r != nullptr): the staged input is
  //   IN_in(in) + (res_rnorm ? ReLU(IN_r(res_r)) : res_r)  [+ ReLU if res_relu]
  // with in_norm = IN of `in` WITHOUT ReLU; res_out (optional, same layout as `in`) receives the
  // joined residual stream for the tile's own pixels (ResidualBlock / ResLayer output)
  const void* res_r;
  const float2* res_rnorm;
  void* res_out;
  int res_relu;
  // image-input preset encode: x_in[c] = ((x01[perm[c]] * a[c]) - b[c]) / d[c]
  float enc_a[3], enc_b[3], enc_d[3];
  int enc_perm[3];
  // pre-padded uint8 frames only (conv_prep.hip): stage x_in[c] = byte[perm[c]] / 256 (exact in bf16 / fp16) and
  // let the first layer's folded weights carry the encode (nst_api.cpp fold_first_layer)
  int enc_raw;
  // weights
  const void* wpk;     // packed fragments (see pack_conv_weights)
  const float* bias;   // [cout_pad]
  // output geometry
  int hconv, wconv;    // conv output extent (statistics count)
  int crop_y, crop_x;  // stored (oy,ox) -> conv coordinate (oy+crop_y, ox+crop_x)
  int oh, ow;          // stored output extent
  void* out;
  int cout_real;
  int cout_stride;     // channel stride of OUT_ACT buffers (= padded cout)
  float* partial;      // [n][tiles][cout_stride][2] InstanceNorm partial sums (OUT_ACT), or nullptr
  int tiles_x, tiles_y, n_cblk;
  int n_work;          // persistent form: work items (frames x channel blocks x tiles)
  // output decode: v[c] = (((y[perm[c]] + p[c]) * q[c]) / r[c]) + s[c]; clamp(0,1)
  float dec_p[3], dec_q[3], dec_r[3], dec_s[3];
  int dec_perm[3];
  int dec_tanh;  // apply tanh to the raw output first (ReCoNet ConvTanhLayer, model.py:77-80)
  int seg_len;    // MODE_KYROT: output rows per work item (set by the launcher)
  int ph_off[2];  // MODE_PHASE / MODE_WPHASE: LDS row/col offset of sub-pixel phase 0/1 ({0,1} nearest-up, {1,1} ConvTranspose)
};

// Kernel dtype codes of the split-precision layers (ConvKernelInfo::dtype only; not in the ABI):
//   SW:    fp16 operand (the first layer's exact raw bytes) x fp16 hi / lo weight pairs
//   SPLIT: fp32 input staged as an fp16 hi / lo operand pair x fp16 hi / lo weight pairs (Wh xh + Wh xl + Wl xh)
//   O32 / O16: fp32 / fp16 output storage
//   SPLITO: fp32 input staged as an fp16 hi / lo operand pair x fp16 weights (Wh xh + Wh xl), fp32 output
constexpr int NST_MAX_STREAM_SPLIT = 4;  // nst_set_stream_split
enum KernelDtype { NST_KDT_SW_O32 = 16, NST_KDT_SW_O16 = 17, NST_KDT_SPLIT_O32 = 18, NST_KDT_SPLIT_O16 = 19,
                   NST_KDT_SPLITO_O32 = 20 };

// Static description of one compiled conv kernel instantiation.
struct ConvKernelInfo {
  int dtype;  // NST_DT_* or NST_KDT_*
  int mode;   // ConvMode
  int ks, stride, cinp, bn, th, tw, wm, wn, in_kind, out_kind;
  // derived
  int pair, nch, cpc, kp, nchunk, nstep, nstep_pack, nsubt, nsub, lds_bytes;
  int persistent;  // resident workgroups walk the tiles (requires one channel block)
  int korder;      // packed K order: 0 tap-major, 1 chunk-group-major (persistent kernels)
  int part_rows;   // InstanceNorm partial rows per tile (persistent: one per channel-sharing wave)
  int wbytes;      // MODE_KYROT: bytes of the packed weight table
  int res;         // fill joins the residual stream (VAR_RES)
  int tanh_out;    // MODE_KYROT: tanh compiled into the output (ReCoNet); other kernels: p.dec_tanh
  int in_esz, out_esz;  // activation element bytes read / written (0: the dtype's own, act_elem_bytes)
  int split_w;          // packed weights are fp16 hi / lo pairs (pack functions place w and w - RNE16(w))
  int cinp_k, bn_k;     // compute widths where the stored channel stride (cinp / bn) is narrower (0: the same):
                        // the kernel zero-pads the staged input / drops the extra output channels
  void (*launch)(const ConvParams&, dim3 grid, hipStream_t);
};

// Look up a compiled instantiation; nullptr if the combination was not built.
const ConvKernelInfo* find_conv_kernel(int dtype, int mode, int ks, int stride, int cinp, int bn, int in_kind,
                                       int out_kind, int res = 0, bool no_persistent = false);

// ---- host helpers shared with the VGG program (nst_api.cpp) ----
int pack_upload_conv(const ConvKernelInfo& k, int cin, int cout, int ks, const float* W, int coutp, void** dev);
int upload_floats(const float* host, size_t n, float** dev);
void tile_grid_of(const ConvKernelInfo& k, int sh, int sw, int oh, int ow, int* tx, int* ty);
const ConvKernelInfo* conv_table_vgg(int* count);

// ---- VGG / Gatys kernels (vgg_ops.hip) ----
hipError_t launch_vgg_pool(const void* z, int h, int w, int c, void* out, hipStream_t st);
hipError_t launch_vgg_pool_bwd(const void* z, const void* gp, int h, int w, int c, void* gz, hipStream_t st);
hipError_t launch_vgg_relu_bwd(const void* z, const void* ga, const void* P, float cw, size_t elems, void* gz,
                               hipStream_t st);
hipError_t launch_vgg_gram_bwd(const void* z, const void* ga, const void* P, float cw, const void* Mb, int hw, int c,
                               void* gz, hipStream_t st);
int vgg_content_parts(size_t elems);
// spart (nullable): the 5 style layers' Gram-reduce block partials at stride sstride floats, snparts[l] each; their
// sums land in style_raw (else style_raw holds them already)
hipError_t launch_vgg_losses(const void* z, const void* P, size_t elems, float* part, float* style_raw,
                             float cscale, const float* sscale, float* losses, hipStream_t st,
                             const float* spart = nullptr, const int* snparts = nullptr, int sstride = 0);
hipError_t launch_adam(float* x, const float* g, float* m, float* v, int hw, int n, const float* inv_std, float lr,
                       float b1, float b2, float eps, float bc1, float bc2, int clamp01, hipStream_t st);

// ---- elementwise / reduction launchers (nst_ops.hip) ----
constexpr int IN_MAX_SEGMENTS = 128;
int in_finalize_segments(int tiles);
// seg_ws: n * IN_MAX_SEGMENTS * cstride * 16 bytes of scratch
hipError_t launch_check_finite(const float* v, size_t n, int* flag, hipStream_t st);
hipError_t launch_in_finalize(const float* partial, int n, int tiles, int cstride, double count,
                              const float* gamma, const float* beta, float eps, int frn, float2* out,
                              void* seg_ws, hipStream_t st);
hipError_t launch_residual(int dtype, const void* y, const float2* ys, const void* r,
                           const float2* rs, int r_relu, int relu_out, void* out, int n, int hw,
                           int c, hipStream_t st);
// NST_DT_F16M's first residual join: y, r fp32 (the split-precision block's output and the producer conv's raw
// output, normalised + ReLU'd as rs / r_relu say) -> the fp16 stream out = rr + (y * ys.x + ys.y) [+ ReLU]
hipError_t launch_residual_f32_to_f16(const void* y, const float2* ys, const void* r, const float2* rs, int r_relu,
                                      int relu_out, void* out, int n, int hw, int c, hipStream_t st);
hipError_t launch_decode_resize_u8(const float* y, int n, int h, int w, const float* p,
                                   const float* q, const float* r, const float* s, const int* perm,
                                   uint8_t* out, int oh, int ow, hipStream_t st);
constexpr int NST_MAX_MODELS = 8;  // slots A..H (pipeline.py model_b..model_h)
hipError_t launch_blend_models_u8(const float* const* ys, const float (*dp)[3], const float (*dq)[3],
                                  const float (*dr)[3], const float (*ds)[3], const int (*perm)[3], const float* wts,
                                  int m, int n, int h, int w, uint8_t* out, int oh, int ow, hipStream_t st);
// LAB tables on the device: 2^24 entries of {x, y, z, 0} bytes (one dword per lookup)
hipError_t launch_lab_ema(const uint32_t* rgb2lab, const uint32_t* lab2rgb, const uint8_t* in,
                          uint8_t* out, int n, int hw, int sl, float a, float oma, int sc, float ca,
                          float coma, float* state, int first, hipStream_t st);
// the EMA split for the sharded pipeline: owner extracts planes, rank 0 runs the ordered EMA on them, owner merges
hipError_t launch_lab_planes(const uint32_t* rgb2lab, const uint8_t* in, uint8_t* planes, int n, int hw, int sl, int sc,
                             hipStream_t st);
hipError_t launch_lab_ema_planes(const uint8_t* in, uint8_t* out, int n, int hw, int sl, float a, float oma, int sc,
                                 float ca, float coma, float* state, int first, hipStream_t st);
hipError_t launch_lab_merge(const uint32_t* rgb2lab, const uint32_t* lab2rgb, const uint8_t* in, const uint8_t* planes,
                            uint8_t* out, int n, int hw, int sl, int sc, hipStream_t st);
hipError_t launch_lab_blend(const uint32_t* rgb2lab, const uint32_t* lab2rgb, const uint8_t* const* frames,
                            const float* wrest, int nrest, float wL, float wab, size_t npix, uint8_t* out,
                            hipStream_t st);
hipError_t launch_mask_feather(const uint8_t* m, int n, int h, int w, float sigma, float* tmp, float* alpha,
                               hipStream_t st);
// rows of zeroed slack after the last frame of the pre-padded input: the 9x9 kernels' last tile rows read up
// to 16 halo rows past a frame's padded extent and a pair-chunk read wraps one pixel into the next row, so
// every byte such a read can reach after the last frame is written (zero) by the prepad launch — a stale
// NaN there would otherwise reach the MFMA through a zero weight (0 * NaN = NaN)
__host__ __device__ inline int prepad_slack_rows(int wp) { return 18 + (1024 + wp - 1) / wp; }
hipError_t launch_prepad_encode(int dtype, const ConvParams& p, int in_kind, int n, int hp, int wp, void* out,
                                hipStream_t st);
hipError_t launch_blend(const uint8_t* s, const uint8_t* o, const float* mask, int mode, float b,
                        float omb, uint8_t* out, int n, int hw, hipStream_t st, const uint8_t* mask8 = nullptr);
size_t gram_workspace_bytes(int n, int c, int hw);
// The Gatys style term fused into the Gram's reduce pass: Mb = bf16(k (G - A)) and loss_out = sum (G - A)^2
// (per-block partials in `parts`, <= GRAM_DELTA_MAX_PARTS = c*c/64 of them, summed in block order)
constexpr int GRAM_DELTA_MAX_PARTS = 512 * 512 / 64;
int gram_delta_parts(int n, int c, int hw);  // how many `parts` launch_gram's reduce writes
struct GramDelta {
  const float* A;
  float k;
  __bf16* Mb;
  float* parts;
  float* loss_out;  // nullptr: the caller sums `parts` itself (launch_vgg_losses' spart)
};
hipError_t launch_vgg_sum_parts(const float* parts, int n, float* out, hipStream_t st);
// relu: Gram of ReLU(F) (bf16 HWC only: the VGG program's stored pre-activations); delta: see GramDelta
hipError_t launch_gram(const void* F, int dtype, int layout_hwc, int n, int c, int hw, float* G, void* ws,
                       hipStream_t st, int relu = 0, const GramDelta* delta = nullptr);

}  // namespace nst
