// conv_prep.hip — first-layer input staging for the 16-bit (bf16 / fp16) paths.
//
// The 9x9 image conv (transformer_net.py:34 conv1 / transformer_net_nst.py:64 down1 / model.py:71)
// consumes the io_preset-encoded frame (pipeline.py:1445-1486).  Encoding inside that conv's LDS
// fill cost ~40 VALU per pixel (byte gathers, the reference's exact division, the padding map) and
// made it VALU-bound; here one streaming pass writes the encoded input ONCE, already padded
// (reflection / NST's pre-reflect + zero padding resolved), as bf16 or fp16 [n][hp][wp][4] (channel 3 = 0):
// 8 bytes per pixel, so the conv fill is plain 16-byte loads (two pixels per LDS entry) with an
// identity coordinate map.  Arithmetic per element is the reference's: x01 = byte / 255 (ToTensor),
// ((x01 * a) - b) / d, one RNE rounding to the 16-bit format — bit-identical to the fused encode it replaces
// (for uint8 frames through a per-block table of the 3 x 256 possible values).  With p.enc_raw the staged value
// is byte / 256 (exact in either format) and the first layer's weights carry the encode instead
// (nst_api.cpp fold_first_layer): the operand then adds no rounding at all.
#include <algorithm>

#include "conv_impl.h"

namespace nst {

// f32 NCHW input (tensor API): one thread per pixel, the encode formula per element
template <typename T>
__global__ __launch_bounds__(256) void prepad_encode_f32_kernel(ConvParams p, int hp, int wp, uint2* __restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y, n = blockIdx.z;
  if (x >= wp) return;
  if (n == (int)gridDim.z - 1) {  // the slice after the last frame: zeroed slack (prepad_slack_rows)
    if (y < prepad_slack_rows(wp)) out[((size_t)n * hp + y) * wp + x] = make_uint2(0u, 0u);
    return;
  }
  if (y >= hp) return;
  const int sy = map_axis(y - p.pad, p.hs, p.axis_mode, p.pre);
  const int sx = map_axis(x - p.pad, p.ws, p.axis_mode, p.pre);
  float v[3] = {0.f, 0.f, 0.f};
  if (sy >= 0 && sx >= 0) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float x01 = ((const float*)p.in)[(((size_t)n * 3 + p.enc_perm[ch]) * p.hs + sy) * p.ws + sx];
      v[ch] = ((x01 * p.enc_a[ch]) - p.enc_b[ch]) / p.enc_d[ch];
    }
  }
  out[((size_t)n * hp + y) * wp + x] = make_uint2(pack16<T>(v[0], v[1]), pack16<T>(v[2], 0.f));
}

// uint8 frames: the encoded bf16 value of a channel depends only on its byte, so each block first
// tabulates the 3 x 256 values with the exact per-element formula (768 evaluations, amortised
// over the block's 8 rows x 1024 pixels), then every pixel is 3 bytes (3 dword loads per 4 interior
// pixels) + 3 LDS lookups; 4 consecutive output pixels per thread (32-byte contiguous stores).
constexpr int PREP_PX = 4;
constexpr int PREP_ROWS = 8;  // padded rows per block: the 768-entry table is built once per 8 rows
template <typename T>
__global__ __launch_bounds__(256) void prepad_encode_u8_kernel(ConvParams p, int hp, int wp, uint4* __restrict__ out) {
  __shared__ uint16_t lut[3][256];
  for (int i = threadIdx.x; i < 3 * 256; i += blockDim.x) {
    const int ch = i >> 8, b = i & 255;
    const float x01 = (float)b / 255.0f;  // ToTensor: .float().div(255)
    // enc_raw: the byte itself, scaled by 2^-8 (exact); the encode is folded into the layer's weights and bias
    const float v = p.enc_raw ? (float)b * 0.00390625f : ((x01 * p.enc_a[ch]) - p.enc_b[ch]) / p.enc_d[ch];
    lut[ch][b] = (uint16_t)(pack16<T>(v, 0.f) & 0xffffu);
  }
  __syncthreads();
  const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * PREP_PX;
  const int n = blockIdx.z;
  if (x0 >= wp) return;
  if (n == (int)gridDim.z - 1) {  // the slice after the last frame: zeroed slack (prepad_slack_rows)
    const int ye = min(prepad_slack_rows(wp), (int)(blockIdx.y + 1) * PREP_ROWS);
    for (int y = blockIdx.y * PREP_ROWS; y < ye; ++y)
      for (int j = 0; j < PREP_PX && x0 + j < wp; ++j) ((uint2*)out)[((size_t)n * hp + y) * wp + x0 + j] = make_uint2(0u, 0u);
    return;
  }
  // the 4 source columns of this thread (same for every row): consecutive and dword-aligned in the
  // interior, so the 12 bytes come as 3 dword loads; reflected / padded edges take byte loads
  int sxs[PREP_PX];
#pragma unroll
  for (int j = 0; j < PREP_PX; ++j) sxs[j] = x0 + j < wp ? map_axis(x0 + j - p.pad, p.ws, p.axis_mode, p.pre) : -1;
  const bool run = sxs[0] >= 0 && sxs[PREP_PX - 1] == sxs[0] + PREP_PX - 1;
  const int pr0 = p.enc_perm[0], pr1 = p.enc_perm[1], pr2 = p.enc_perm[2];
  const int ybeg = blockIdx.y * PREP_ROWS;
  // interior column run of a whole block of rows with dword-aligned rows: every row's 3 dwords are requested before
  // the first is used (one HBM latency per block of rows instead of one per row: the pass ran at ~2.6 TB/s)
  if (run && ybeg + PREP_ROWS <= hp && (p.ws * 3) % 4 == 0 && ((uintptr_t)p.in & 3) == 0 && (sxs[0] * 3) % 4 == 0 &&
      x0 + PREP_PX <= wp && ((((size_t)n * hp + ybeg) * wp + x0) & 1) == 0 && (wp & 1) == 0) {
    uint32_t dw[PREP_ROWS][3];
    bool live[PREP_ROWS];
#pragma unroll
    for (int r = 0; r < PREP_ROWS; ++r) {
      const int sy = map_axis(ybeg + r - p.pad, p.hs, p.axis_mode, p.pre);
      live[r] = sy >= 0;
      const uint32_t* d = (const uint32_t*)((const uint8_t*)p.in + ((size_t)n * p.hs + (sy < 0 ? 0 : sy)) * p.ws * 3 +
                                            (size_t)sxs[0] * 3);
      dw[r][0] = d[0];
      dw[r][1] = d[1];
      dw[r][2] = d[2];
    }
#pragma unroll
    for (int r = 0; r < PREP_ROWS; ++r) {
      auto byte = [&](int k) { return (dw[r][k >> 2] >> (8 * (k & 3))) & 255u; };
      uint32_t w[2 * PREP_PX];
#pragma unroll
      for (int j = 0; j < PREP_PX; ++j) {
        w[2 * j] = live[r] ? ((uint32_t)lut[0][byte(3 * j + pr0)] | ((uint32_t)lut[1][byte(3 * j + pr1)] << 16)) : 0u;
        w[2 * j + 1] = live[r] ? ((uint32_t)lut[2][byte(3 * j + pr2)] | ((uint32_t)pack16<T>(0.f, 0.f) & 0xffff0000u)) : 0u;
      }
      uint4* o = (uint4*)((uint2*)out + ((size_t)n * hp + ybeg + r) * wp + x0);
      o[0] = make_uint4(w[0], w[1], w[2], w[3]);
      o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
    return;
  }
  for (int y = ybeg; y < min(hp, ybeg + PREP_ROWS); ++y) {
    const int sy = map_axis(y - p.pad, p.hs, p.axis_mode, p.pre);
    const uint8_t* row = (const uint8_t*)p.in + ((size_t)n * p.hs + (sy < 0 ? 0 : sy)) * p.ws * 3;
    uint32_t w[2 * PREP_PX];
    if (run && sy >= 0 && (((uintptr_t)row + (size_t)sxs[0] * 3) & 3) == 0) {
      const uint32_t* d = (const uint32_t*)(row + (size_t)sxs[0] * 3);
      const uint32_t dw[3] = {d[0], d[1], d[2]};
      auto byte = [&](int k) { return (dw[k >> 2] >> (8 * (k & 3))) & 255u; };
#pragma unroll
      for (int j = 0; j < PREP_PX; ++j) {
        w[2 * j] = (uint32_t)lut[0][byte(3 * j + pr0)] | ((uint32_t)lut[1][byte(3 * j + pr1)] << 16);
        w[2 * j + 1] = (uint32_t)lut[2][byte(3 * j + pr2)] | ((uint32_t)pack16<T>(0.f, 0.f) & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int j = 0; j < PREP_PX; ++j) {
        uint32_t lo = 0u, hi = 0u;
        if (sy >= 0 && sxs[j] >= 0) {
          const uint8_t* px = row + (size_t)sxs[j] * 3;
          lo = (uint32_t)lut[0][px[pr0]] | ((uint32_t)lut[1][px[pr1]] << 16);
          hi = (uint32_t)lut[2][px[pr2]] | ((uint32_t)pack16<T>(0.f, 0.f) & 0xffff0000u);
        }
        w[2 * j] = lo;
        w[2 * j + 1] = hi;
      }
    }
    uint2* o = (uint2*)out + ((size_t)n * hp + y) * wp + x0;
    if (x0 + PREP_PX <= wp && ((((size_t)n * hp + y) * wp + x0) & 1) == 0) {
      ((uint4*)o)[0] = make_uint4(w[0], w[1], w[2], w[3]);
      ((uint4*)o)[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
#pragma unroll
      for (int j = 0; j < PREP_PX; ++j)
        if (x0 + j < wp) o[j] = make_uint2(w[2 * j], w[2 * j + 1]);
    }
  }
}

template <typename T>
hipError_t launch_prepad(const ConvParams& p, int in_kind, int n, int hp, int wp, void* out, hipStream_t st) {
  if (in_kind == IN_U8_NHWC) {
    // z = n: the zeroed slack after the last frame
    const int rows = std::max(hp, prepad_slack_rows(wp));
    const dim3 grid((unsigned)((wp + 256 * PREP_PX - 1) / (256 * PREP_PX)), (unsigned)((rows + PREP_ROWS - 1) / PREP_ROWS),
                    (unsigned)n + 1);
    hipLaunchKernelGGL(prepad_encode_u8_kernel<T>, grid, dim3(256), 0, st, p, hp, wp, (uint4*)out);
  } else {
    const dim3 grid((unsigned)((wp + 255) / 256), (unsigned)std::max(hp, prepad_slack_rows(wp)), (unsigned)n + 1);
    hipLaunchKernelGGL(prepad_encode_f32_kernel<T>, grid, dim3(256), 0, st, p, hp, wp, (uint2*)out);
  }
  return hipGetLastError();
}

hipError_t launch_prepad_encode(int dtype, const ConvParams& p, int in_kind, int n, int hp, int wp, void* out,
                                hipStream_t st) {
  if (dtype == NST_DT_F16) return launch_prepad<_Float16>(p, in_kind, n, hp, wp, out, st);
  return launch_prepad<__bf16>(p, in_kind, n, hp, wp, out, st);
}

}  // namespace nst
