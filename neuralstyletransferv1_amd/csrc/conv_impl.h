// conv_impl.h — the one convolution kernel of the engine, templated per layer shape.
//
// Replaces every Conv2d / ConvTranspose2d of the three stylization nets
// (transformer_net.py:44-54,79-99; transformer_net_nst.py:12-59,76; model.py:5-11,69-80)
// together with what surrounds it in the reference graph:
//   * the padding (ReflectionPad2d / zero padding / NST's ReflectionPad2d(40)),
//   * nearest x2 upsampling (UpsampleConvLayer, Decoder nn.Upsample) and ConvTranspose2d,
//   * the PREVIOUS layer's InstanceNorm apply + ReLU (prologue, while filling LDS),
//   * this layer's InstanceNorm statistics (per-tile partial sums in the epilogue),
//   * for the first/last layer: the io_preset encode (pipeline.py:1445-1486) from uint8
//     frames and the decode + clamp(0,1) + ToPILImage truncation to uint8 frames.
//
// Shape of the computation (implicit GEMM, MI355X-first):
//   * one workgroup = 4 waves = one output tile x BN output channels of one frame; the whole
//     input halo, all input channels, is staged ONCE in LDS (NHWC, 16-byte chunks XOR-swizzled
//     so the 16 lanes of an MFMA operand read hit 16 distinct bank slots), then the K loop
//     (taps x channels) runs with no further barrier.
//   * MFMA operands: A = packed weights (rows = output channels) streamed from L2 as one
//     coalesced 1 KiB fragment per wave-instruction, prefetched one K-step ahead;
//     B = input pixels from LDS (cols = 16 output pixels).
//     bf16 / fp16: v_mfma_f32_16x16x32_{bf16,f16} (fp32 accumulate).  fp32: v_mfma_f32_16x16x4_f32
//     (exact fp32 FMA chain) — the parity mode.
//   * output-channel permutation: C row q of n-subtile t is output channel
//     4*NSUB*(q>>2) + 4*t + (q&3) of the wave's range, so each lane ends up owning
//     4*NSUB CONSECUTIVE channels of one pixel -> 16..64-byte contiguous NHWC stores.
//
// Three mappings of the same machinery (MODE):
//   MODE_STD    plain conv (any KS, stride 1/2; stride 2 uses a polyphase LDS column order so
//               stride-2 operand reads are unit-stride).
//   MODE_PHASE  x2 "up" convs — nearest-upsample + 3x3 conv, and ConvTranspose2d(3,s2,p1,op1) —
//               as four sub-pixel phases: wave w computes output phase (a,b) = (w>>1, w&1) as a
//               2x2 conv over the SOURCE grid with phase-summed weights (pack time).  2.25x
//               fewer MFMAs than the upsampled 3x3 conv, 4x fewer than the zero-inserted grid.
//   MODE_XSHIFT the 9x9 conv to 3 channels: the 16 MFMA rows carry 5 horizontal output shifts
//               x 3 channels (row q = 3*s + c) of a base pixel, K runs over 9 x 13 taps, bases
//               are 5 pixels apart (LDS columns in a polyphase-5 order): 3.46x fewer MFMAs than
//               padding N=3 to 16, and each base's 15 uint8 outputs are 15 consecutive bytes.
#pragma once
#include <type_traits>
#include "nst_internal.h"
#include "nst_hip.h"

// generic non-persistent fills with per-item channel chunks read the producer's IN constants from an LDS table
#ifndef NST_GEN_NTAB
#define NST_GEN_NTAB 1
#endif
#ifndef NST_GEN_RES_PASSES
#define NST_GEN_RES_PASSES 2
#endif
#ifndef NST_GEN_NTAB_RES
#define NST_GEN_NTAB_RES 1  // the residual-join fills too: ReCoNet 820 -> 828-835 frames/s (r05_ad)
#endif

namespace nst {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int reflect_idx(int v, int L) {
  v = v < 0 ? -v : v;
  v = v >= L ? 2 * L - 2 - v : v;
  return min(max(v, 0), L - 1);
}

// Virtual conv-input coordinate -> source index along one axis, -1 = zero padding.
__device__ __forceinline__ int map_axis(int v, int L, int mode, int pre) {
  switch (mode) {
    case AX_REFLECT:
      return reflect_idx(v, L);
    case AX_REFLECT_UP2:
      // reflect in the upsampled grid, then nearest: src = u >> 1  (== clamp in source space)
      return reflect_idx(v, 2 * L) >> 1;
    case AX_ZERO:
      return (v < 0 || v >= L) ? -1 : v;
    case AX_ZERO_PREREFLECT:
      return (v < 0 || v >= L + 2 * pre) ? -1 : reflect_idx(v - pre, L);
    case AX_CLAMP:
      return min(max(v, 0), L - 1);
    default:  // AX_ZINSERT: zero-inserted grid of length 2L-1
      return (v < 0 || v > 2 * L - 2 || (v & 1)) ? -1 : (v >> 1);
  }
}

// Bank-slot swizzle of the 16-B chunk index inside an LDS entry (one pixel, NCH chunks).
template <int NCH>
__device__ __forceinline__ int swz(int e) {
  if constexpr (NCH % 16 == 0) return e & 15;
  else if constexpr (NCH % 8 == 0) return (e >> 1) & 7;
  else if constexpr (NCH % 4 == 0) return (e >> 2) & 3;
  else return 0;
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef float f32x2v_t __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (round to nearest even): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  const f32x2v_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v_t));
}

// The two 16-bit activation formats of the MFMA paths, T = __bf16 or _Float16 (same layouts,
// same MFMA shapes and rates on gfx950):
//   bf16 (NST_DT_BF16)  the throughput mode: 8 significant bits;
//   fp16 (NST_DT_F16)   11 significant bits: the mode that holds the reference's +-1 LSB uint8 bar
//                       (stored conv outputs must stay inside the fp16 range, |v| <= 65504).
// lo16 / hi16 unpack one half of a packed pair exactly; pack16 rounds two floats to nearest even
// (one v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32).
template <typename T>
constexpr bool IS_F16 = std::is_same<T, _Float16>::value;
typedef _Float16 f16x2v_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ float lo16(uint32_t w) {
  if constexpr (IS_F16<T>) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
  else return bf16_lo(w);
}
template <typename T>
__device__ __forceinline__ float hi16(uint32_t w) {
  if constexpr (IS_F16<T>) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
  else return bf16_hi(w);
}
template <typename T>
__device__ __forceinline__ uint32_t pack16(float lo, float hi) {
  if constexpr (IS_F16<T>) {
    const f32x2v_t v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2v_t));
  } else {
    return pack_bf16(lo, hi);
  }
}
// pack16 of fp32 values rounded as they are (the generic kernel's fills and epilogue): without the opaque
// copies hipcc folds a producing fma / add into v_fma_mixlo_f16, which rounds the exact result to fp16 once,
// so a value whose fp32 rounding lands on an fp16 tie comes out one ulp off the documented
// fp32-then-fp16 arithmetic (and off the unfused residual kernel)
template <typename T>
__device__ __forceinline__ uint32_t pack16p(float lo, float hi) {
  if constexpr (IS_F16<T>) {
    asm("" : "+v"(lo));
    asm("" : "+v"(hi));
  }
  return pack16<T>(lo, hi);
}
// acc + A x B on v_mfma_f32_16x16x32_{bf16,f16} (builtin form: hipcc allocates the accumulator)
template <typename T>
__device__ __forceinline__ f32x4_t mfma16x16x32(const uint4& a, const uint4& b, const f32x4_t& c) {
  if constexpr (IS_F16<T>)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
typedef float f32x16_t __attribute__((ext_vector_type(16)));
template <typename T>
__device__ __forceinline__ f32x16_t mfma32x32x16(const uint4& a, const uint4& b, const f32x16_t& c) {
  if constexpr (IS_F16<T>)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
// The split-fp16 mode's activation type (NST_DT_F32S): fp32 in HBM, so every sizeof(T) == 4 path
// (fills, IN apply, joins, epilogue stores) is the fp32 one; only the LDS operand form and the
// MFMA differ.  A 16-B LDS chunk holds 4 channels as [hi0..hi3, lo0..lo3] (fp16, hi = RNE(v),
// lo = RNE(v - hi)); the packed weights carry two fragments per K step, [Wh0..3, Wh0..3] and
// [Wl0..3, 0 x 4], so two v_mfma_f32_16x16x32_f16 give Wh*(xh + xl) + Wl*xh (the dropped Wl*xl is
// ~2^-22 of the product).
struct F32Split {
  float v;
};
template <typename T>
constexpr bool IS_SPLIT = std::is_same<T, F32Split>::value;

template <typename T>
constexpr int dtype_code() {
  if constexpr (IS_SPLIT<T>) return NST_DT_F32S;
  return std::is_same<T, float>::value ? NST_DT_F32 : (IS_F16<T> ? NST_DT_F16 : NST_DT_BF16);
}

// 4 fp32 channels -> the split LDS chunk [hi0..hi3, lo0..lo3]
__device__ __forceinline__ uint4 split_chunk(uint4 raw) {
  float v[4] = {__uint_as_float(raw.x), __uint_as_float(raw.y), __uint_as_float(raw.z), __uint_as_float(raw.w)};
  _Float16 hi[4], lo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) asm("" : "+v"(v[j]));  // split the fp32 value itself (no v_fma_mixlo_f16 fold)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = (_Float16)v[j];
    lo[j] = (_Float16)(v[j] - (float)hi[j]);  // exact in fp32: v and hi share the exponent range
  }
  auto pk = [](_Float16 a, _Float16 b) {
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
  };
  return make_uint4(pk(hi[0], hi[1]), pk(hi[2], hi[3]), pk(lo[0], lo[1]), pk(lo[2], lo[3]));
}
// a staged chunk in the layer's LDS operand form
template <typename T>
__device__ __forceinline__ uint4 lds_form(uint4 v) {
  if constexpr (IS_SPLIT<T>) return split_chunk(v);
  else return v;
}

template <typename T, int MODE, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN>
struct ConvCfg {
  static constexpr int CPC = 16 / (int)sizeof(T);                                 // channels per 16-B chunk
  static constexpr bool PAIR = (MODE == MODE_STD) && (sizeof(T) == 2) && (CINP == 4);  // chunk = 2 px x 4 ch
  static constexpr int NCH = PAIR ? 1 : CINP / CPC;                               // chunks per LDS entry
  // LDS entry stride: channel-chunked entries (NCH % 4 == 0) are padded to NCH+2 chunks.  A stride
  // of 2*odd chunks puts the 16 lanes of every ds_read_b128 lane group ({0-3,12-15,20-27}, ...:
  // 8 pixels of lane group g and 8 of g^1) on 16 distinct bank slots with no XOR swizzle (pixel
  // parity alternates with g's chunk parity), so operand addresses are lane base + immediates.
  static constexpr int NXS_ = 5;
  // (a 4-byte x-shift halo that does not fit with 2 pad chunks takes one: NCH + 1 is odd, 2-way at worst)
  static constexpr int EB0 = ((NCH % 4) == 0 ? NCH + 2 : NCH) * 16;
  static constexpr int NENT0 = (MODE == MODE_PHASE ? TH + 2 : (TH - 1) * S + KS) *
                               (MODE == MODE_XSHIFT ? NXS_ * ((((TW - 1) * S + KS) + NXS_ - 1) / NXS_)
                                                    : ((S == 2) ? 2 * ((((TW - 1) * S + KS) + 1) / 2)
                                                                : (MODE == MODE_PHASE ? TW + 2 : (TW - 1) * S + KS)));
  static constexpr int EB = (NENT0 * EB0 > 150 * 1024 && (NCH % 4) == 0) ? (NCH + 1) * 16 : EB0;  // bytes per LDS entry
  static constexpr int NXS = 5;                                                   // x-shifts (XSHIFT)
  static constexpr int KP = PAIR ? (KS + 1) / 2 : (MODE == MODE_XSHIFT ? KS + NXS - 1 : KS);  // x-taps per row
  static constexpr int NTAP = MODE == MODE_PHASE ? 4 : KS * KP;
  static constexpr int NCHUNK = NTAP * NCH;                                       // 16-B chunks along K
  static constexpr int NSTEP = (NCHUNK + 3) / 4;                                  // one chunk per lane group
  static constexpr int LH = MODE == MODE_PHASE ? TH + 2 : (TH - 1) * S + KS;
  static constexpr int LW = MODE == MODE_PHASE ? TW + 2 : (TW - 1) * S + KS;
  static constexpr int HALF = (LW + 1) / 2;                                       // stride-2 polyphase split
  static constexpr int W5 = (LW + NXS - 1) / NXS;                                 // x-shift polyphase width
  static constexpr int LWP = MODE == MODE_XSHIFT ? NXS * W5 : ((S == 2) ? 2 * HALF : LW);
  static constexpr int NENT = LH * LWP;
  static constexpr int LDS_BYTES = NENT * EB;
  static constexpr int COLS = MODE == MODE_XSHIFT ? 16 * NXS : 16;                // output px per m-subtile row
  static constexpr int MSUBT = TH * (TW / COLS);
  static constexpr int MSUB = MSUBT / WM;
  static constexpr int NSUB = MODE == MODE_PHASE ? BN / 16 : (BN / 16) / WN;
  static constexpr int NSUBT = MODE == MODE_PHASE ? 4 * (BN / 16) : BN / 16;     // packed n-subtiles
  // K loop shape.  ROWED (NCH % 4 == 0): rows of the kernel window (runtime loop) x x-taps x
  // channel-chunk groups (both unrolled, so every LDS offset inside a row is a constant).
  // Otherwise (image layers, 1 chunk per pixel) a flat loop where each lane group reads its own tap.
  static constexpr bool ROWED = (NCH % 4) == 0;
  static constexpr int NCH4 = ROWED ? NCH / 4 : 1;                                // steps per tap
  static constexpr int ROWS = MODE == MODE_PHASE ? 2 : KS;                        // kernel rows
  static constexpr int KPR = MODE == MODE_PHASE ? 2 : KP;                         // x-taps per row
  static constexpr int RS = KPR * NCH4;                                           // steps per row
  // weight-fragment prefetch depth: enough K-steps in flight to cover ~512 cycles of L2 latency
  // with this tile's MFMA work per step (16 cycles per bf16 16x16x32, 4 x 32 per fp32 step);
  // in the rowed loop it must divide the steps per row so every ring slot index is static
  static constexpr int CYC_STEP = MSUB * NSUB * (sizeof(T) == 2 ? 16 : (IS_SPLIT<T> ? 32 : 128));
  static constexpr int AF = IS_SPLIT<T> ? 2 : 1;  // A fragments per (K step, n-subtile)
  static constexpr int PF_RAW0 = (512 + CYC_STEP - 1) / CYC_STEP;
  static constexpr int PF_RAW = PF_RAW0 < 2 ? 2 : (PF_RAW0 > 16 ? 16 : PF_RAW0);
  static constexpr int pf_div(int want, int n) {
    for (int d = want; d <= n; ++d)
      if (n % d == 0) return d;
    return n;
  }
  static constexpr int PF = ROWED ? pf_div(PF_RAW, RS) : PF_RAW;
  static constexpr int NSTEP_P = ROWED ? NSTEP : (NSTEP + PF - 1) / PF * PF;     // loop trip (zero-padded)
  static constexpr int NSTEP_PACK = NSTEP_P + PF;                                 // packed steps (prefetch tail)
  static constexpr int REDW = MODE == MODE_PHASE ? 4 * WM : WM;                   // waves sharing a channel
  static constexpr int RED_BYTES = REDW * BN * 2 * 4;
  static constexpr int MAP_OFF = (LDS_BYTES + 15) / 16 * 16;                      // per-block row/col source maps
  static constexpr int MAP_BYTES = (LH + LW) * 4;
  static constexpr int LDS_ALLOC0 = MAP_OFF + MAP_BYTES;
  static constexpr int LDS_ALLOC = LDS_ALLOC0 > RED_BYTES ? LDS_ALLOC0 : RED_BYTES;
  static_assert(!ROWED || NSTEP == ROWS * RS, "rowed K loop covers every step");
  static constexpr int NW = WM * WN;                                              // waves per workgroup
  static constexpr int NT = 64 * NW;                                              // threads per workgroup
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per workgroup");
  static_assert(TW % COLS == 0 && MSUBT % WM == 0, "m-subtiles must split over WM waves");
  static_assert(BN % 16 == 0, "n-subtiles of 16 channels");
  static_assert(MODE == MODE_PHASE || (BN / 16) % WN == 0, "n-subtiles must split over WN waves");
  static_assert(MODE != MODE_PHASE || ((WM == 1 || WM == 2) && WN == 4 && S == 1),
                "phase mode: one wave per phase (WM = 2: two, splitting the tile's pixel sub-tiles)");
  static_assert(MODE != MODE_XSHIFT || (BN == 16 && WN == 1 && S == 1), "x-shift mode: 16 rows = 5x3 + 1");
  static_assert(PAIR || (CINP % CPC) == 0, "channel padding");
  static_assert(PAIR || NCH == 1 || NCH % 4 == 0, "chunks per pixel must be 1 or a multiple of 4");
  static_assert(LDS_ALLOC <= 160 * 1024, "LDS budget");
  static_assert(S == 1 || CINP != 4, "image-input layers are stride 1");
};

// Producer InstanceNorm apply (+ReLU) on one 16-byte chunk: v = v*scale + shift.
// bf16: per channel pair, unpack (2 ops), one packed fp32 FMA (v_pk_fma_f32), one RNE pack
// (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32) and the ReLU as a packed int16 max with 0 on the 16-bit
// patterns (sign-magnitude: sign bit = int16 sign; rounding is monotone, so ReLU-after-round ==
// round-after-ReLU).
// Every producer IN the prologue applies is followed by a ReLU (ConvLayer -> IN -> ReLU in all
// three nets; the residual's second IN is applied by the residual add instead), so the ReLU is
// unconditional here.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ uint4 norm_chunk(uint4 raw, const float2* nm) {
  if constexpr (sizeof(T) == 2) {
    uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2_t x = {lo16<T>(w[j]), hi16<T>(w[j])};
      const f32x2_t sc = {nm[2 * j].x, nm[2 * j + 1].x};
      const f32x2_t sh = {nm[2 * j].y, nm[2 * j + 1].y};
      f32x2_t y; y.x = __builtin_fmaf(x.x, sc.x, sh.x); y.y = __builtin_fmaf(x.y, sc.y, sh.y);
      const i16x2_t r = __builtin_bit_cast(i16x2_t, pack16p<T>(y.x, y.y));
      w[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float v[4] = {__uint_as_float(raw.x), __uint_as_float(raw.y), __uint_as_float(raw.z), __uint_as_float(raw.w)};
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j] * nm[j].x + nm[j].y, 0.f);
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
  }
}

// Residual join, fused into the consumer conv's fill (ResidualBlock.forward transformer_net.py:71-76,
// transformer_net_nst.py:138-142; ReCoNet ResLayer model.py:55-60 adds the ReLU after the sum):
//   v = IN_y(y) + (rn ? ReLU(IN_r(r)) : r)  [then ReLU if relu_out]
// in the residual kernel's fp32 arithmetic (product, then sum: no contraction) with one rounding;
// ReLU(IN_r(r)) is the value a normalising fill would stage (bf16: rounded, as the stored x_0).
template <typename T>
__device__ __forceinline__ uint4 res_chunk(uint4 y, uint4 r, const float2* yn, const float2* rn, bool has_rn,
                                           bool relu_out) {
  constexpr int CPC = 16 / (int)sizeof(T);
  float fy[CPC], fr[CPC], o[CPC];
  const uint32_t wy[4] = {y.x, y.y, y.z, y.w}, wr[4] = {r.x, r.y, r.z, r.w};
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fy[2 * j] = lo16<T>(wy[j]); fy[2 * j + 1] = hi16<T>(wy[j]);
      fr[2 * j] = lo16<T>(wr[j]); fr[2 * j + 1] = hi16<T>(wr[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) { fy[j] = __uint_as_float(wy[j]); fr[j] = __uint_as_float(wr[j]); }
  }
#pragma unroll
  for (int j = 0; j < CPC; ++j) {
    float rr = fr[j];
    if (has_rn) {
      // r' = ReLU(IN_r(r)) exactly as a normalising fill stages it (norm_chunk): bf16 of one fma
      if constexpr (sizeof(T) == 2)
        rr = fmaxf(lo16<T>(pack16p<T>(__builtin_fmaf(rr, rn[j].x, rn[j].y), 0.f)), 0.f);
      else
        rr = fmaxf(rr * rn[j].x + rn[j].y, 0.f);
    }
    float v = fy[j] * yn[j].x + yn[j].y;
    v = rr + v;
    o[j] = relu_out ? fmaxf(v, 0.f) : v;
  }
  if constexpr (sizeof(T) == 2) {
    return make_uint4(pack16p<T>(o[0], o[1]), pack16p<T>(o[2], o[3]), pack16p<T>(o[4], o[5]), pack16p<T>(o[6], o[7]));
  } else {
    return make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3]));
  }
}

// One 16-byte LDS entry of an image-input layer (3 channels, preset encode fused):
// PAIR -> pixels vx, vx+1 (4 bf16 each); else one pixel (4 f32).
template <typename T, int INK, bool PAIR>
__device__ __forceinline__ uint4 load_image_entry(const ConvParams& p, int n, int vy, int vx) {
  float vals[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const int sy = map_axis(vy, p.hs, p.axis_mode, p.pre);
#pragma unroll
  for (int q = 0; q < (PAIR ? 2 : 1); ++q) {
    const int sx = map_axis(vx + q, p.ws, p.axis_mode, p.pre);
    if (sy < 0 || sx < 0) continue;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const int src_c = p.enc_perm[ch];
      float x01;
      if constexpr (INK == IN_U8_NHWC) {
        const uint8_t b = ((const uint8_t*)p.in)[(((size_t)n * p.hs + sy) * p.ws + sx) * 3 + src_c];
        x01 = (float)b / 255.0f;  // ToTensor: .float().div(255)
      } else {
        x01 = ((const float*)p.in)[(((size_t)n * 3 + src_c) * p.hs + sy) * p.ws + sx];
      }
      vals[q][ch] = ((x01 * p.enc_a[ch]) - p.enc_b[ch]) / p.enc_d[ch];
    }
  }
  if constexpr (PAIR) {
    return make_uint4(pack16<T>(vals[0][0], vals[0][1]), pack16<T>(vals[0][2], 0.f),
                      pack16<T>(vals[1][0], vals[1][1]), pack16<T>(vals[1][2], 0.f));
  } else {
    return make_uint4(__float_as_uint(vals[0][0]), __float_as_uint(vals[0][1]), __float_as_uint(vals[0][2]), 0u);
  }
}

// Sum over the 16 lanes of a DPP row (every lane gets the total): row_mirror pairs lane i with
// 15-i, row_half_mirror folds each half, then quad xor 2 and xor 1.
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xf, 0xf, false));  // row_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false));   // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad [1,0,3,2]
  return v;
}

// Reduce-scatter of 32 values over the 16 lanes of a DPP row (30 exchanges instead of 32 full
// row sums): partners 15-px (row_mirror), px^7 within 8 (row_half_mirror), px^3 and px^1 within
// a quad; at each step the lower partner keeps the lower half.  Afterwards lane px holds the row
// totals of values 2*px and 2*px+1.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int N, int CTRL>
__device__ __forceinline__ void rs_step(const float* in, float* out, bool upper) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float keep = upper ? in[i + N] : in[i];
    const float send = upper ? in[i] : in[i + N];
    out[i] = keep + dpp_f<CTRL>(send);
  }
}
__device__ __forceinline__ void row_reduce_scatter32(const float (&v)[32], int px, float& o0, float& o1) {
  float a[16], b[8], c[4], d[2];
  rs_step<16, 0x140>(v, a, px >= 8);
  rs_step<8, 0x141>(a, b, (px & 4) != 0);
  rs_step<4, 0x1b>(b, c, (px & 2) != 0);
  rs_step<2, 0xb1>(c, d, (px & 1) != 0);
  o0 = d[0];
  o1 = d[1];
}

__device__ __forceinline__ float decode_ch(float y, int ch, const ConvParams& p) {
  float v = (((y + p.dec_p[ch]) * p.dec_q[ch]) / p.dec_r[ch]) + p.dec_s[ch];
  return fminf(fmaxf(v, 0.f), 1.f);  // .clamp(0, 1)
}

// Kernel variants (VAR bits):
//  VAR_PERS  persistent form (activation-input layers with one channel block): a grid of resident
//            workgroups walks the tiles; each one issues the NEXT tile's halo loads into registers
//            before running the current tile's K loop, so the global-load latency of the fill hides
//            behind MFMAs and the weight-fragment ring rolls straight from one tile into the next.
//  VAR_WL    weights through LDS: the K loop's weight fragments are loaded ONCE per workgroup (each
//            wave loads 1/NW of every stage into registers, RR stages ahead) and shared by all waves
//            through a 3-stage LDS ring, instead of every wave streaming its own fragments from L2.
//            L2 weight traffic per output pixel drops by the number of waves sharing a channel range,
//            which is what bounds the register-streamed form on the wide (128-192 channel) layers.
//  VAR_RES   residual join fused into the fill (ConvParams::res_r): a second source per halo item.
enum { VAR_PERS = 1, VAR_WL = 2, VAR_RES = 4 };

// Weight-ring stage: SC K-steps (all NSUBT fragments of each), split evenly over the NW waves.
template <int NSTEP, int NSUBT, int NW>
constexpr int wl_stage_steps() {
  for (int sc = 2; sc <= 8; ++sc)
    if (NSTEP % sc == 0 && (sc * NSUBT) % NW == 0) return sc;
  return 0;
}

template <typename T, int MODE, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN, int INK, int OUTK,
          int VAR>
__global__ __launch_bounds__(64 * WM * WN) void conv_kernel(ConvParams p) {
  using C = ConvCfg<T, MODE, KS, S, CINP, BN, TH, TW, WM, WN>;
  constexpr bool PERS = (VAR & VAR_PERS) != 0;
  constexpr bool WL = (VAR & VAR_WL) != 0;
  constexpr int NT = C::NT;
  constexpr int NCH = C::NCH, EB = C::EB, LWP = C::LWP, HALF = C::HALF, LW = C::LW, W5 = C::W5;
  constexpr int MSUB = C::MSUB, NSUB = C::NSUB, NSUBT = C::NSUBT, COLS = C::COLS;
  constexpr bool PAIR = C::PAIR;
  static_assert(!PERS || (INK == IN_ACT && C::ROWED), "persistent form: activation-input rowed layers");
  static_assert(!WL || C::ROWED, "LDS weight ring: rowed K loop");
  static_assert(!PERS || WL, "the persistent form streams weights through the LDS ring");
  constexpr int AF = C::AF;
  static_assert(AF == 1 || !WL, "split-fp16 mode: register-streamed weights only");
  // weight ring geometry (WL)
  constexpr int SC = WL ? wl_stage_steps<C::NSTEP, NSUBT, C::NW>() : 1;  // K-steps per stage
  static_assert(!WL || SC >= 2, "weight-ring stage: >= 2 steps, split evenly over the waves");
  constexpr int NSTG = C::NSTEP / SC;                                      // stages per tile
  constexpr int FR_STG = SC * NSUBT;                                       // 1-KiB fragments per stage
  constexpr int FPW = FR_STG / C::NW;                                      // fragments each wave loads
  constexpr int RR = 3;                                                    // stages in flight in registers
  constexpr int STG_BYTES = FR_STG * 1024;
  // LDS: [halo][row/col maps x (PERS ? 2 : 1)][weight ring x 3 (WL)][bias (WL)][IN constants (PERS)]
  //      [reduction (PERS: own region; else aliases the halo)]
  constexpr int MAPB = (C::MAP_BYTES + 15) / 16 * 16;
  constexpr int RING_OFF = C::MAP_OFF + (PERS ? 2 : 1) * MAPB;
  constexpr int BIAS_OFF = RING_OFF + (WL ? 3 * STG_BYTES : 0);
  constexpr int NORM_OFF = BIAS_OFF + (WL ? BN * 4 : 0);       // PERS: next frame's IN {scale, shift}
  constexpr int RING_END = NORM_OFF + (PERS ? 2 * CINP * 8 : 0);
  constexpr int RED_OFF = PERS ? RING_END : 0;
  // non-persistent fill whose threads' chunks vary per item (NT % NCH != 0: ReCoNet's 96 / 192-channel layers): the
  // tile's frame's IN table {scale, shift} in LDS, read per item instead of from memory (e2 0.75 -> 0.61 ms, plain trunk
  // 0.64-0.73 -> 0.59-0.66 per batch of 8)
  constexpr bool NTAB = NST_GEN_NTAB && !PERS && INK == IN_ACT && (NT % NCH) != 0 && (NST_GEN_NTAB_RES || (VAR & VAR_RES) == 0);
  constexpr int NTAB_OFF = RING_END;
  constexpr int LDS_TOTAL0 = PERS ? RED_OFF + C::RED_BYTES : RING_END + (NTAB ? 2 * CINP * 8 : 0);
  constexpr int LDS_TOTAL = LDS_TOTAL0 > C::LDS_ALLOC ? LDS_TOTAL0 : C::LDS_ALLOC;
  static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[LDS_TOTAL];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, px = lane & 15;

  // work item w = (frame n, channel block cb, tile)
  struct Work {
    int n, cb, tile, ty0, tx0;  // PHASE: tile origin on the source grid
  };
  const int ntile = p.tiles_x * p.tiles_y;
  auto decode_work = [&](int wi) {
    Work r;
    r.tile = wi % ntile;
    const int ny = wi / ntile;
    r.n = ny / p.n_cblk;
    r.cb = ny - r.n * p.n_cblk;
    const int tyi = r.tile / p.tiles_x;
    r.ty0 = tyi * TH;
    r.tx0 = (r.tile - tyi * p.tiles_x) * TW;
    return r;
  };
  int w;
  if constexpr (PERS) {
    // workgroups b, b+8, ... run on one XCD (round-robin dispatch): give each XCD a contiguous run
    // of tiles per sweep so vertically/horizontally neighbouring halos meet in the same L2
    const int G = gridDim.x, b = blockIdx.x;
    w = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
    if (w >= p.n_work) return;
  } else {
    w = blockIdx.y * ntile + blockIdx.x;
  }
  Work cur = decode_work(w);

  // weights: fragment (step s, n-subtile t) of this wave lives at wp[(s*NSUBT + t)*64]; a ring of
  // PF steps is kept in flight (steps >= NSTEP are zero padding; PERS wraps to the next tile's step 0)
  constexpr int PF = C::PF;
  // (split mode: AF = 2 fragments per (step, n-subtile), fragment j of (s, t) at wp[((s*NSUBT + t)*2 + j)*64])
  const uint4* wp = (const uint4*)p.wpk + ((size_t)cur.cb * C::NSTEP_PACK * NSUBT + wn * NSUB) * AF * 64 + lane;
  uint4 a_ring[WL ? 1 : PF][NSUB * AF];
  auto a_load = [&](uint4 (&dst)[NSUB * AF], int s) {
#pragma unroll
    for (int f = 0; f < NSUB * AF; ++f) dst[f] = wp[(s * NSUBT * AF + f) * 64];
  };
  if constexpr (!WL) {
#pragma unroll
    for (int d = 0; d < PF; ++d) a_load(a_ring[d], d);
  }
  // WL: stage j's fragments are contiguous in the packed weights; this wave loads fragments
  // [wave*FPW, wave*FPW+FPW) of each stage and stores them to the same place in the LDS ring
  // (buffer loads: the stage offset rides in an SGPR, so every stage shares one lane-offset VGPR)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.wpk + (size_t)cur.cb * C::NSTEP_PACK * NSUBT * 1024), (short)0,
      C::NSTEP_PACK * NSUBT * 1024, 0x00020000);
  const uint32_t wvoff = (uint32_t)((wave * FPW * 64 + lane) * 16);
  auto wld = [&](int j, int f) -> uint4 {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoff, (j * FR_STG + f) * 1024, 0));
  };
  char* ring = smem + RING_OFF;
  // in-flight stages form a shift register (oldest in wreg[0]) so every register index is static
  constexpr int RRA = WL ? RR : 1;
  uint4 wreg[RRA][FPW > 0 ? FPW : 1];
  auto wl_issue = [&](int j) {  // load stage j into the youngest slot
#pragma unroll
    for (int f = 0; f < FPW; ++f) wreg[RRA - 1][f] = wld(j, f);
  };
  auto wl_store = [&](int slot_off) {  // store the oldest stage to a ring slot, shift the rest down
#pragma unroll
    for (int f = 0; f < FPW; ++f)
      *(uint4*)(ring + slot_off + ((wave * FPW + f) * 64 + lane) * 16) = wreg[0][f];
#pragma unroll
    for (int r = 0; r + 1 < RRA; ++r)
#pragma unroll
      for (int f = 0; f < FPW; ++f) wreg[r][f] = wreg[r + 1][f];
  };
  if constexpr (WL) {
    if constexpr (OUTK == OUT_ACT) {
      float* bias_l = (float*)(smem + BIAS_OFF);
      for (int t = tid; t < BN; t += NT) bias_l[t] = p.bias[cur.cb * BN + t];
    }
    // stages 0..RR-1 in flight while the halo is staged
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      if (PERS || j < NSTG) {
#pragma unroll
        for (int f = 0; f < FPW; ++f) wreg[j][f] = wld(j % NSTG, f);
      }
    }
  }

  // ---- stage the input halo (prologue transform applied) ----
  // The padding / reflection / upsample / crop mapping of halo row ly and column lx to a source
  // row/column (or -1 = zero) is evaluated once per tile into two small LDS maps.  Then all of
  // a thread's loads are issued before any is consumed (IPT independent 16-B loads in flight per
  // lane), transformed (producer IN + ReLU) and written to LDS: the fill costs ~one latency.
  constexpr int NITEMS = C::NENT * NCH;
  constexpr int IPT = (NITEMS + NT - 1) / NT;
  // entry e -> logical (ly, lx) of the halo, false for the padding entries of a polyphase order
  auto entry_xy = [&](int e, int& ly, int& lx) -> bool {
    ly = e / LWP;
    const int pc = e - ly * LWP;
    if constexpr (MODE == MODE_XSHIFT) {
      const int ph = pc / W5;
      lx = C::NXS * (pc - ph * W5) + ph;
      return lx < LW;
    } else if constexpr (S == 2) {
      lx = pc < HALF ? 2 * pc : 2 * (pc - HALF) + 1;
      return lx < LW;
    } else {
      lx = pc;
      return true;
    }
  };
  // when NT % NCH == 0 a thread always stages the same channel chunk, so it applies the same
  // CPC channels' IN constants to every item
  constexpr bool FIXED_CHUNK = (NT % NCH) == 0;
  const int c_fixed = tid % NCH;
  auto build_maps = [&](const Work& wk, int slot) {
    // byte offsets within the frame (host guarantees a frame is < 2 GiB), -1 = zero padding
    int* rowmap = (int*)(smem + C::MAP_OFF + slot * MAPB);
    int* colmap = rowmap + C::LH;
    const int vy0 = (wk.ty0 + p.crop_y) * S - p.pad;
    const int vx0 = (wk.tx0 + p.crop_x) * S - p.pad;
    const int pix_bytes = p.cs * (int)sizeof(T);
    for (int t = tid; t < C::LH + LW; t += NT) {
      if (t < C::LH) {
        const int sy = map_axis(vy0 + t, p.hs, p.axis_mode, p.pre);
        rowmap[t] = sy < 0 ? -1 : sy * p.ws * pix_bytes;
      } else {
        const int sx = map_axis(vx0 + t - C::LH, p.ws, p.axis_mode, p.pre);
        colmap[t - C::LH] = sx < 0 ? -1 : sx * pix_bytes;
      }
    }
  };
  // item k of this thread -> LDS entry e, chunk c; returns the source byte offset in the frame,
  // -1 for zero padding (evaluated from the maps in slot, at load time and again at store time)
  auto item_src = [&](int slot, int k, int& e, int& c) -> int {
    const int* rowmap = (const int*)(smem + C::MAP_OFF + slot * MAPB);
    const int* colmap = rowmap + C::LH;
    const int it = tid + k * NT;
    e = it / NCH;
    c = FIXED_CHUNK ? c_fixed : it - e * NCH;
    int ly, lx;
    const bool ok = entry_xy(e, ly, lx) && it < NITEMS;
    const int ro = ok ? rowmap[ly] : -1;
    const int co = ok ? colmap[lx] : -1;
    return (ro >= 0 && co >= 0) ? ro + co + c * 16 : -1;
  };
  // residual join fused into the fill (p.res_r): second source, optional residual-stream write of
  // the tile's own pixels (plain stride-1 convs: those halo entries are the pixels themselves); without a
  // join, p.res_out receives the normalised input of those pixels (x_0 = ReLU(IN(C)) of block 1's conv1)
  constexpr bool CAN_RESOUT = MODE == MODE_STD && S == 1 && INK == IN_ACT;
  constexpr bool resf = INK == IN_ACT && (VAR & VAR_RES) != 0;
  const bool has_rn = p.res_rnorm != nullptr;
  const size_t frame_bytes = (size_t)p.hs * p.ws * p.cs * sizeof(T);
  // halo entry (ly, lx) of tile wk is one of the tile's own output pixels
  auto interior = [&](const Work& wk, int ly, int lx) -> bool {
    return ly >= p.pad && ly < p.pad + TH && lx >= p.pad && lx < p.pad + TW && wk.ty0 + ly - p.pad < p.oh &&
           wk.tx0 + lx - p.pad < p.ow;
  };
  // srcs[k] keeps each item's source offset (-1 = zero padding) for the store pass
  // items kbase .. kbase + N - 1 of this thread (N = the arrays' extent: the whole fill, or one pass of it)
  auto issue_loads = [&](const Work& wk, int slot, auto& raw, auto& raw2, auto& srcs, int kbase) {
    constexpr int N = std::extent_v<std::remove_reference_t<decltype(srcs)>>;
    const char* img = (const char*)p.in + (size_t)wk.n * frame_bytes;
    const char* img2 = (const char*)p.res_r + (size_t)wk.n * frame_bytes;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      int e, c;
      const int src = item_src(slot, k + kbase, e, c);
      srcs[k] = src;
      raw[k] = make_uint4(0u, 0u, 0u, 0u);
      raw2[k] = make_uint4(0u, 0u, 0u, 0u);
      if (src >= 0) {
        raw[k] = *(const uint4*)(img + (unsigned)src);
        if (resf) raw2[k] = *(const uint4*)(img2 + (unsigned)src);
      }
    }
  };
  auto load_norm = [&](int n, float2 (&nmc)[C::CPC], float2 (&rnmc)[C::CPC]) {
    if (FIXED_CHUNK && p.in_norm != nullptr) {
#pragma unroll
      for (int j = 0; j < C::CPC; ++j) nmc[j] = p.in_norm[(size_t)n * p.cs + c_fixed * C::CPC + j];
    }
    if (FIXED_CHUNK && resf && has_rn) {
#pragma unroll
      for (int j = 0; j < C::CPC; ++j) rnmc[j] = p.res_rnorm[(size_t)n * p.cs + c_fixed * C::CPC + j];
    }
  };
  auto stage = [&](const Work& wk, const auto& raw, const auto& raw2, const auto& srcs, const float2 (&nmc)[C::CPC],
                   const float2 (&rnmc)[C::CPC], int kbase) {
    constexpr int N = std::extent_v<std::remove_reference_t<decltype(srcs)>>;
    char* rout = (char*)p.res_out + (size_t)wk.n * frame_bytes;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const int it = tid + (k + kbase) * NT;
      if (it < NITEMS) {
        const int e = it / NCH, c = FIXED_CHUNK ? c_fixed : it - e * NCH;
        uint4 v = raw[k];
        if (srcs[k] >= 0 && (resf || p.in_norm != nullptr)) {
          float2 nmv[C::CPC], rnv[C::CPC];
          if constexpr (FIXED_CHUNK) {
#pragma unroll
            for (int j = 0; j < C::CPC; ++j) { nmv[j] = nmc[j]; rnv[j] = rnmc[j]; }
          } else if constexpr (NTAB) {
            const float2* nt = (const float2*)(smem + NTAB_OFF);
#pragma unroll
            for (int j = 0; j < C::CPC; ++j) {
              nmv[j] = nt[c * C::CPC + j];
              rnv[j] = has_rn && resf ? nt[CINP + c * C::CPC + j] : make_float2(1.f, 0.f);
            }
          } else {
#pragma unroll
            for (int j = 0; j < C::CPC; ++j) {
              nmv[j] = p.in_norm[(size_t)wk.n * p.cs + c * C::CPC + j];
              rnv[j] = has_rn && resf ? p.res_rnorm[(size_t)wk.n * p.cs + c * C::CPC + j] : make_float2(1.f, 0.f);
            }
          }
          if (resf) {
            v = res_chunk<T>(v, raw2[k], nmv, rnv, has_rn, p.res_relu != 0);
            if constexpr (CAN_RESOUT) {
              int ly, lx;
              if (p.res_out != nullptr && entry_xy(e, ly, lx) && interior(wk, ly, lx))
                *(uint4*)(rout + (unsigned)srcs[k]) = v;
            }
          } else {
            v = norm_chunk<T>(v, nmv);
            if constexpr (CAN_RESOUT) {  // x_0 export (block 1's conv1): the normalised input of its own pixels
              int ly, lx;
              if (p.res_out != nullptr && entry_xy(e, ly, lx) && interior(wk, ly, lx))
                *(uint4*)(rout + (unsigned)srcs[k]) = v;
            }
          }
        }
        *(uint4*)(smem + e * EB + 16 * c) = lds_form<T>(v);
      }
    }
  };
  // PERS streams the next tile's halo in NCH4 parts, part q = channel chunks 4q..4q+3 of every
  // entry (the K loop runs chunk group q's taps before q+1's, so part q's LDS is free once they
  // are done); item i of a part -> entry i/4, chunk 4q + i%4 (a thread keeps its chunk i%4)
  constexpr int NPART = C::NCH4;
  constexpr int PITEMS = C::NENT * 4;
  constexpr int IPP = (PITEMS + NT - 1) / NT;
  // The next tile's item sources are resolved ONCE per tile (psrc: part-0 byte offset in the frame,
  // -1 = zero padding / no item; part q adds 64*q), with the interior flags of the residual-stream
  // write in pint.  Loads are raw buffer loads (frame base in SGPRs, one VGPR offset, no branch),
  // so the wait counter stays countable across the K loop; an invalid item loads offset 0 and is
  // replaced by zero at write time.
  int psrc[IPP];
  unsigned pint = 0;
  int tid_p = tid;  // laundered per use: LDS item addresses are recomputed, not held across the K loop
  auto part_items = [&](const Work& wk, int slot) {
    const int* rowmap = (const int*)(smem + C::MAP_OFF + slot * MAPB);
    const int* colmap = rowmap + C::LH;
    pint = 0;
#pragma unroll
    for (int k = 0; k < IPP; ++k) {
      const int it = tid + k * NT;
      int ly, lx;
      const bool ok = entry_xy(it >> 2, ly, lx) && it < PITEMS;
      const int ro = ok ? rowmap[ly] : -1;
      const int co = ok ? colmap[lx] : -1;
      psrc[k] = (ro >= 0 && co >= 0) ? ro + co + (it & 3) * 16 : -1;
      if (CAN_RESOUT && ok && interior(wk, ly, lx)) pint |= 1u << k;
    }
  };
  auto frame_rsrc = [&](const void* base, int n) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (size_t)n * frame_bytes), (short)0,
                                             (int)frame_bytes, 0x00020000);
  };
  auto issue_part = [&](const Work& wk, int q, uint4 (&praw)[IPP], uint4 (&praw2)[IPP]) {
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc(p.in, wk.n);
#pragma unroll
    for (int k = 0; k < IPP; ++k) {
      const uint32_t off = psrc[k] >= 0 ? (uint32_t)(psrc[k] + 64 * q) : 0u;
      praw[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
    if (resf) {
      const __amdgpu_buffer_rsrc_t rs2 = frame_rsrc(p.res_r, wk.n);
#pragma unroll
      for (int k = 0; k < IPP; ++k) {
        const uint32_t off = psrc[k] >= 0 ? (uint32_t)(psrc[k] + 64 * q) : 0u;
        praw2[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs2, off, 0, 0));
      }
    }
  };
  // the IN constants of the part's frame come from the LDS tables (norm_l: producer / residual y,
  // rnorm_l: residual r)
  auto write_part = [&](const Work& wk, int q, const uint4 (&praw)[IPP], const uint4 (&praw2)[IPP],
                        const float2* norm_l, const float2* rnorm_l) {
    float2 nm[C::CPC], rnm[C::CPC];
    const int cq = (4 * q + (tid & 3)) * C::CPC;
#pragma unroll
    for (int j = 0; j < C::CPC; ++j) {
      nm[j] = p.in_norm != nullptr ? norm_l[cq + j] : make_float2(1.f, 0.f);
      rnm[j] = resf && has_rn ? rnorm_l[cq + j] : make_float2(1.f, 0.f);
    }
    char* rout = (char*)p.res_out + (size_t)wk.n * frame_bytes;
    asm volatile("" : "+v"(tid_p));
#pragma unroll
    for (int k = 0; k < IPP; ++k) {
      const int it = tid_p + k * NT;
      if (it < PITEMS) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);  // zero padding stays zero (pad after IN + ReLU)
        if (psrc[k] >= 0) {
          if (resf) {
            v = res_chunk<T>(praw[k], praw2[k], nm, rnm, has_rn, p.res_relu != 0);
            if (CAN_RESOUT && ((pint >> k) & 1u) && p.res_out != nullptr)
              *(uint4*)(rout + (unsigned)(psrc[k] + 64 * q)) = v;
          } else {
            v = p.in_norm != nullptr ? norm_chunk<T>(praw[k], nm) : praw[k];
            if (CAN_RESOUT && ((pint >> k) & 1u) && p.res_out != nullptr)  // x_0 export, as above
              *(uint4*)(rout + (unsigned)(psrc[k] + 64 * q)) = v;
          }
        }
        *(uint4*)(smem + (it >> 2) * EB + (it & 3) * 16 + 64 * q) = lds_form<T>(v);
      }
    }
  };
  auto stage_image = [&](const Work& wk) {
    static_assert(INK == IN_ACT || MODE == MODE_STD, "image input only on plain convs");
    const int vy0 = (wk.ty0 + p.crop_y) * S - p.pad;
    const int vx0 = (wk.tx0 + p.crop_x) * S - p.pad;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int it = tid + k * NT;
      if (it < NITEMS) {
        const int e = it / NCH;
        const int ly = e / LWP, lx = e - ly * LWP;
        const uint4 v = load_image_entry<T, INK, PAIR>(p, wk.n, vy0 + ly, vx0 + lx);
        *(uint4*)(smem + e * EB) = lds_form<T>(v);
      }
    }
  };

  // ---- K loop: taps x channel chunks ----
  int base[MSUB];
#pragma unroll
  for (int m = 0; m < MSUB; ++m) {
    const int ms = wm * MSUB + m;
    const int r = ms / (TW / COLS), cbk = ms - r * (TW / COLS);
    if constexpr (MODE == MODE_XSHIFT) base[m] = r * LWP + px;  // base pixel 5*px of row r
    else base[m] = (S == 2 ? 2 * r : r) * LWP + cbk * 16 + px;
  }
  int phy = 0, phx = 0;  // PHASE: LDS row/col offset of this wave's sub-pixel phase
  if constexpr (MODE == MODE_PHASE) {
    phy = p.ph_off[wn >> 1];
    phx = p.ph_off[wn & 1];
  }
  typedef f32x4_t AccT[MSUB][NSUB];

  auto mfma_step = [&](AccT& acc, const uint4 (&a)[NSUB * AF], const uint4 (&b)[MSUB]) {
#pragma unroll
    for (int m = 0; m < MSUB; ++m) {
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        if constexpr (IS_SPLIT<T>) {
          acc[m][t] = mfma16x16x32<_Float16>(a[2 * t], b[m], acc[m][t]);      // Wh * (xh + xl)
          acc[m][t] = mfma16x16x32<_Float16>(a[2 * t + 1], b[m], acc[m][t]);  // Wl * xh
        } else if constexpr (sizeof(T) == 2) {
          acc[m][t] = mfma16x16x32<T>(a[t], b[m], acc[m][t]);
        } else {
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].x), __uint_as_float(b[m].x), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].y), __uint_as_float(b[m].y), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].z), __uint_as_float(b[m].z), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].w), __uint_as_float(b[m].w), acc[m][t], 0, 0, 0);
        }
      }
    }
    // the step's operand fragments stay live past its MFMAs: hipcc (ROCm 7.2) otherwise may place an MFMA's
    // destination partially over a source register that dies there (tools/check_mfma_overlap.py)
#pragma unroll
    for (int t = 0; t < NSUB * AF; ++t) asm volatile("" ::"v"(__builtin_bit_cast(u32x4_t, a[t])));
#pragma unroll
    for (int m = 0; m < MSUB; ++m) asm volatile("" ::"v"(__builtin_bit_cast(u32x4_t, b[m])));
  };

  // kloop(acc, rot, hook): rot = ring slot of this tile's stage 0 (PERS: the ring runs on across
  // tiles); hook(k) runs after stage k's barrier (PERS: the next tile's maps / halo loads)
  auto kloop = [&](AccT& acc, int rot, auto&& hook) {
#pragma unroll
    for (int m = 0; m < MSUB; ++m)
#pragma unroll
      for (int t = 0; t < NSUB; ++t) acc[m][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    if constexpr (WL) {
      // fully unrolled steps; stage k = steps [k*SC, k*SC+SC) reads ring slot k%3.  After the first
      // step of stage k a barrier retires every wave's reads of slot (k+2)%3 (stage k-1), so stage
      // k+2 (loaded RR stages ago) is stored there and stage k+2+RR is issued into the freed registers;
      // the next stage's barrier publishes the store before stage k+2's first read (SC >= 2).
      constexpr int NCH4 = C::NCH4, RS = C::RS;
      int lbase[MSUB];
#pragma unroll
      for (int m = 0; m < MSUB; ++m) lbase[m] = base[m] * EB + 16 * g;
      const char* abase = ring + ((wn * NSUB) * 64 + lane) * 16;
      // byte offset of the ring slot holding stage k (+3 for the wrap): so[k % 3]
      int so[3];
      if constexpr (NSTG % 3 == 0) rot = 0;
#pragma unroll
      for (int i = 0; i < 3; ++i) so[i] = ((rot + i) % 3) * STG_BYTES;
      // operands of step s (double-buffered by parity: step s+1's reads are issued before step s's
      // barrier, so no LDS latency is exposed after it)
      uint4 a[2][NSUB], b[2][MSUB];
      auto load_step = [&](int s, uint4 (&av)[NSUB], uint4 (&bv)[MSUB]) {
        // K order: tap-major (s = tap*NCH4 + cg) or, PERS, chunk-group-major (s = cg*taps + tap)
        int row, dx, cg;
        if constexpr (PERS) {
          cg = s / (C::ROWS * C::KPR);
          const int tap = s - cg * (C::ROWS * C::KPR);
          row = tap / C::KPR;
          dx = tap - row * C::KPR;
        } else {
          row = s / RS;
          const int pos = s - row * RS;
          dx = pos / NCH4;
          cg = pos - dx * NCH4;
        }
        const int rowoff = (MODE == MODE_PHASE ? (phy + row) * LWP + phx : row * LWP) * EB;
        const int xo = MODE == MODE_XSHIFT ? (dx % C::NXS) * W5 + dx / C::NXS
                                           : (S == 2 ? (dx & 1) * HALF + (dx >> 1) : dx);
        const int k = s / SC, ss = s - k * SC;
#pragma unroll
        for (int t = 0; t < NSUB; ++t) av[t] = *(const uint4*)(abase + so[k % 3] + (ss * NSUBT + t) * 1024);
#pragma unroll
        for (int m = 0; m < MSUB; ++m) bv[m] = *(const uint4*)(smem + lbase[m] + rowoff + xo * EB + 64 * cg);
      };
      load_step(0, a[0], b[0]);
#pragma unroll
      for (int s = 0; s < C::NSTEP; ++s) {
        // one scheduling region per step: step s+1's operand reads interleaved with step s's MFMAs
        if (s + 1 < C::NSTEP) load_step(s + 1, a[(s + 1) & 1], b[(s + 1) & 1]);
        // the work hooked to stage k's barrier (step k*SC) runs in the next step's region, so the
        // scheduler interleaves it with MFMAs instead of every wave stalling on it together
        if (s >= 1 && (s - 1) % SC == 0) hook((s - 1) / SC);
        mfma_step(acc, a[s & 1], b[s & 1]);
#pragma unroll
        for (int i = 0; i < NSUB + MSUB; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        }
        __builtin_amdgcn_sched_group_barrier(0x008, MSUB * NSUB - (NSUB + MSUB), 0);
        __builtin_amdgcn_sched_barrier(0);
        const int k = s / SC;
        if (s - k * SC == 0) {
          // every wave is past its stage k-1 reads: refill slot (k+2)%3
          __syncthreads();
          if constexpr (PERS) {
            // the ring runs on into the next tile (same channel block, so the same weights)
            wl_store(so[(k + 2) % 3]);
            wl_issue((k + 2 + RR) % NSTG);
          } else if (k + 2 < NSTG) {
            wl_store(so[(k + 2) % 3]);
            if (k + 2 + RR < NSTG) wl_issue(k + 2 + RR);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else if constexpr (C::ROWED) {
      // rows (runtime) x x-taps x chunk groups (unrolled): step s = row*RS + dx*NCH4 + cg reads
      // chunk 4*cg + g of tap (row, dx); PF divides RS, so the ring slot of each position is static
      constexpr int NCH4 = C::NCH4, KPR = C::KPR, RS = C::RS;
      // per-lane LDS byte base of each m-subtile (lane group g's chunk folded in); per row one add,
      // per tap / chunk group only immediate offsets
      int lbase[MSUB];
#pragma unroll
      for (int m = 0; m < MSUB; ++m) lbase[m] = base[m] * EB + 16 * g;
      for (int row = 0; row < C::ROWS; ++row) {
        const int rowoff = (MODE == MODE_PHASE ? (phy + row) * LWP + phx : row * LWP) * EB;
        const char* rp[MSUB];
#pragma unroll
        for (int m = 0; m < MSUB; ++m) rp[m] = smem + lbase[m] + rowoff;
#pragma unroll
        for (int dx = 0; dx < KPR; ++dx) {
          // constant column offset of x-tap dx in this mode's LDS column order
          const int xo = MODE == MODE_XSHIFT ? (dx % C::NXS) * W5 + dx / C::NXS
                                             : (S == 2 ? (dx & 1) * HALF + (dx >> 1) : dx);
#pragma unroll
          for (int cg = 0; cg < NCH4; ++cg) {
            const int pos = dx * NCH4 + cg;  // position within the row (compile-time after unrolling)
            const int slot = pos % PF;
            uint4 b[MSUB];
#pragma unroll
            for (int m = 0; m < MSUB; ++m) b[m] = *(const uint4*)(rp[m] + xo * EB + 64 * cg);
            mfma_step(acc, a_ring[slot], b);
            a_load(a_ring[slot], row * RS + pos + PF);
          }
        }
      }
    } else {
      for (int s0 = 0; s0 < C::NSTEP_P; s0 += PF) {
#pragma unroll
        for (int d = 0; d < PF; ++d) {
          const int s = s0 + d;
          const int i = 4 * s + g;
          int tap = 0, c = 0;
          if (i < C::NCHUNK) {
            tap = i / NCH;
            c = i - tap * NCH;
          }
          const int dy = tap / C::KP, dxp = tap - dy * C::KP;
          const int dx = PAIR ? 2 * dxp : dxp;
          const int toff = dy * LWP + dx;
          uint4 b[MSUB];
#pragma unroll
          for (int m = 0; m < MSUB; ++m) {
            const int e = base[m] + toff;
            b[m] = *(const uint4*)(smem + e * EB + 16 * (c ^ swz<NCH>(e)));
          }
          mfma_step(acc, a_ring[d], b);
          a_load(a_ring[d], s + PF);
        }
      }
    }
  };

  // ---- epilogue ----
  auto epilogue = [&](const Work& wk, const AccT& acc) {
    const int n = wk.n, cb = wk.cb, ty0 = wk.ty0, tx0 = wk.tx0;
    // output pixel of m-subtile m for this lane (STD / PHASE)
    auto out_px = [&](int m, int& oy, int& ox) {
      const int ms = wm * MSUB + m;
      const int r = ms / (TW / COLS), cbk = ms - r * (TW / COLS);
      if constexpr (MODE == MODE_PHASE) {
        oy = 2 * (ty0 + r) + (wn >> 1);
        ox = 2 * (tx0 + cbk * 16 + px) + (wn & 1);
      } else {
        oy = ty0 + r;
        ox = tx0 + cbk * 16 + px;
      }
    };
    if constexpr (OUTK == OUT_ACT) {
      const int cwave = cb * BN + (MODE == MODE_PHASE ? 0 : wn * NSUB * 16);  // first channel of this wave
      const int cbase = cwave + 4 * NSUB * g;                                 // this lane's 4*NSUB channels
      float bias_v[4 * NSUB];
      if constexpr (WL) {
        const float* bias_l = (const float*)(smem + BIAS_OFF) + (cbase - cb * BN);
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) bias_v[j] = bias_l[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) bias_v[j] = p.bias[cbase + j];
      }
      // bias add and statistics as 4-wide vectors: the per-element arithmetic (add, fma) is the same,
      // issued as packed v_pk_add_f32 / v_pk_fma_f32 pairs
      f32x4_t bias4[NSUB], s1v[NSUB], s2v[NSUB];
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        bias4[t] = (f32x4_t){bias_v[4 * t], bias_v[4 * t + 1], bias_v[4 * t + 2], bias_v[4 * t + 3]};
        s1v[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        s2v[t] = s1v[t];
      }
      // 32-bit offsets inside the frame (host guarantees a frame is < 2 GiB); a wave whose pixels
      // are all inside the image (every wave but the edge tiles') takes the branch-free copy
      char* fout = (char*)p.out + (size_t)n * p.oh * p.ow * p.cout_stride * sizeof(T);
      bool lane_ok = true;
#pragma unroll
      for (int m = 0; m < MSUB; ++m) {
        int oy, ox;
        out_px(m, oy, ox);
        lane_ok = lane_ok && (oy < p.oh) && (ox < p.ow);
      }
      auto store_tile = [&](auto all_valid) {
#pragma unroll
        for (int m = 0; m < MSUB; ++m) {
          int oy, ox;
          out_px(m, oy, ox);
          const bool valid = decltype(all_valid)::value || ((oy < p.oh) && (ox < p.ow));
          f32x4_t v4[NSUB];
          float v[4 * NSUB];
#pragma unroll
          for (int t = 0; t < NSUB; ++t) {
            v4[t] = acc[m][t] + bias4[t];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[4 * t + q] = v4[t][q];
          }
          if (valid) {
            char* dst = fout + (unsigned)(((oy * p.ow + ox) * p.cout_stride + cbase) * (int)sizeof(T));
            if constexpr (sizeof(T) == 2) {
#pragma unroll
              for (int h = 0; h < NSUB; h += 2) {
                if (h + 1 < NSUB) {
                  *(uint4*)(dst + h * 8) = make_uint4(pack16p<T>(v[4 * h], v[4 * h + 1]), pack16p<T>(v[4 * h + 2], v[4 * h + 3]),
                                                      pack16p<T>(v[4 * h + 4], v[4 * h + 5]), pack16p<T>(v[4 * h + 6], v[4 * h + 7]));
                } else {
                  *(uint2*)(dst + h * 8) = make_uint2(pack16p<T>(v[4 * h], v[4 * h + 1]), pack16p<T>(v[4 * h + 2], v[4 * h + 3]));
                }
              }
            } else {
#pragma unroll
              for (int t = 0; t < NSUB; ++t)
                *(float4*)(dst + t * 16) = make_float4(v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]);
            }
#pragma unroll
            for (int t = 0; t < NSUB; ++t) {
              s1v[t] += v4[t];
              s2v[t] = __builtin_elementwise_fma(v4[t], v4[t], s2v[t]);
            }
          }
        }
      };
      if (__builtin_amdgcn_ballot_w64(!lane_ok) == 0) {
        store_tile(std::true_type{});
      } else {
        store_tile(std::false_type{});
      }
      float s1[4 * NSUB], s2[4 * NSUB];
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) { s1[4 * t + q] = s1v[t][q]; s2[4 * t + q] = s2v[t][q]; }
      if constexpr (PERS && 4 * NSUB == 16) {
        // one partial row per channel-sharing wave (tile*REDW + rw): no barrier, no LDS; the 16
        // pixel lanes of a lane group reduce-scatter so lane px ends with channel cbase + px
        if (p.partial != nullptr) {
          float v[32];
#pragma unroll
          for (int j = 0; j < 16; ++j) { v[2 * j] = s1[j]; v[2 * j + 1] = s2[j]; }
          float t1, t2;
          row_reduce_scatter32(v, px, t1, t2);
          const int rw = MODE == MODE_PHASE ? wave : wm;
          float* dst = p.partial + ((((size_t)n * ntile + wk.tile) * C::REDW + rw) * p.cout_stride + cbase + px) * 2;
          *(float2*)dst = make_float2(t1, t2);
        }
        return;
      }
      constexpr bool RS_STATS = !PERS && (NSUB == 1 || NSUB == 2 || NSUB == 4);
      if (RS_STATS && p.partial != nullptr) {
        // reduce-scatter the 2 x 4*NSUB statistics over the 16 pixel lanes of each lane group (one
        // DPP row; log2(16) exchange steps instead of a full row sum per value), then combine the
        // channel-sharing waves in LDS
        const int rw = MODE == MODE_PHASE ? wave : wm;
        const int cl0 = cwave - cb * BN + 4 * NSUB * g;
        __syncthreads();  // LDS tile no longer read (the reduction aliases it)
        float* red = (float*)(smem + RED_OFF);  // [REDW][BN][2]
        constexpr int NV = 8 * NSUB;
        float v[NV];
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) { v[2 * j] = s1[j]; v[2 * j + 1] = s2[j]; }
        if constexpr (NV == 32) {
          float t1, t2;
          row_reduce_scatter32(v, px, t1, t2);  // lane px: channel cl0 + px
          *(float2*)(red + (rw * BN + cl0 + px) * 2) = make_float2(t1, t2);
        } else if constexpr (NV == 16) {
          float a8[8], a4[4], a2[2], a1[1];
          rs_step<8, 0x140>(v, a8, px >= 8);
          rs_step<4, 0x141>(a8, a4, (px & 4) != 0);
          rs_step<2, 0x1b>(a4, a2, (px & 2) != 0);
          rs_step<1, 0xb1>(a2, a1, (px & 1) != 0);  // lane px: statistic px & 1 of channel cl0 + px / 2
          red[(rw * BN + cl0 + (px >> 1)) * 2 + (px & 1)] = a1[0];
        } else if constexpr (NV == 8) {
          float a4[4], a2[2], a1[1];
          rs_step<4, 0x140>(v, a4, px >= 8);
          rs_step<2, 0x141>(a4, a2, (px & 4) != 0);
          rs_step<1, 0x1b>(a2, a1, (px & 2) != 0);
          const float t = a1[0] + dpp_f<0xb1>(a1[0]);
          const int idx = (px >= 8 ? 4 : 0) + ((px & 4) ? 2 : 0) + ((px & 2) ? 1 : 0);
          if ((px & 1) == 0) red[(rw * BN + cl0 + (idx >> 1)) * 2 + (idx & 1)] = t;
        }
        __syncthreads();
        for (int cl = tid; cl < BN; cl += NT) {
          float a = 0.f, b2 = 0.f;
#pragma unroll
          for (int rr = 0; rr < C::REDW; ++rr) { a += red[(rr * BN + cl) * 2]; b2 += red[(rr * BN + cl) * 2 + 1]; }
          float* dst = p.partial + (((size_t)n * ntile + wk.tile) * p.cout_stride + cb * BN + cl) * 2;
          dst[0] = a;
          dst[1] = b2;
        }
      } else if (p.partial != nullptr) {
        // reduce over the 16 pixel lanes of each lane group (one DPP row)
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) {
          s1[j] = row_sum16(s1[j]);
          s2[j] = row_sum16(s2[j]);
        }
        const int rw = MODE == MODE_PHASE ? wave : wm;
        if constexpr (PERS) {
          // one partial row per channel-sharing wave (tile*REDW + rw): no barrier, no LDS
          if (px == 0) {
            float* dst = p.partial + ((((size_t)n * ntile + wk.tile) * C::REDW + rw) * p.cout_stride +
                                      cwave + 4 * NSUB * g) * 2;
#pragma unroll
            for (int j = 0; j < 4 * NSUB; j += 2)
              *(float4*)(dst + 2 * j) = make_float4(s1[j], s2[j], s1[j + 1], s2[j + 1]);
          }
          return;
        }
        __syncthreads();  // LDS tile no longer read (the reduction aliases it)
        float* red = (float*)(smem + RED_OFF);  // [REDW][BN][2]
        if (px == 0) {
#pragma unroll
          for (int j = 0; j < 4 * NSUB; ++j) {
            const int cl = cwave - cb * BN + 4 * NSUB * g + j;
            red[(rw * BN + cl) * 2 + 0] = s1[j];
            red[(rw * BN + cl) * 2 + 1] = s2[j];
          }
        }
        __syncthreads();
        for (int cl = tid; cl < BN; cl += NT) {
          float a = 0.f, b2 = 0.f;
#pragma unroll
          for (int rr = 0; rr < C::REDW; ++rr) { a += red[(rr * BN + cl) * 2]; b2 += red[(rr * BN + cl) * 2 + 1]; }
          float* dst = p.partial + (((size_t)n * ntile + wk.tile) * p.cout_stride + cb * BN + cl) * 2;
          dst[0] = a;
          dst[1] = b2;
        }
      }
    } else if constexpr (MODE == MODE_XSHIFT) {
      // lane (base px, group g) holds rows q = 4g+j = 3*shift + channel (channel order baked
      // into the packed weights and bias); base px's 15 outputs are bytes 15*px .. 15*px+14
#pragma unroll
      for (int m = 0; m < MSUB; ++m) {
        const int oy = ty0 + wm * MSUB + m;
        if (oy >= p.oh) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = 4 * g + j;
          if (q >= 15) continue;
          const int sft = q / 3, ch = q - 3 * sft;
          const int ox = tx0 + C::NXS * px + sft;
          if (ox >= p.ow) continue;
          float y = acc[m][0][j] + p.bias[q];
          if (p.dec_tanh) y = tanhf(y);
          if constexpr (OUTK == OUT_F32_NCHW) {
            ((float*)p.out)[(((size_t)n * 3 + ch) * p.oh + oy) * p.ow + ox] = y;
          } else {
            ((uint8_t*)p.out)[(((size_t)n * p.oh + oy) * p.ow + ox) * 3 + ch] =
                (uint8_t)(decode_ch(y, ch, p) * 255.0f);  // ToPILImage: pic.mul(255).byte()
          }
        }
      }
    } else {
      // STD final layer: 3 output channels live in lane group 0 (channels 0..3 of n-subtile 0)
      if (g == 0) {
        const float b0 = p.bias[0], b1 = p.bias[1], b2v = p.bias[2];
#pragma unroll
        for (int m = 0; m < MSUB; ++m) {
          int oy, ox;
          out_px(m, oy, ox);
          if (oy >= p.oh || ox >= p.ow) continue;
          float y[3] = {acc[m][0][0] + b0, acc[m][0][1] + b1, acc[m][0][2] + b2v};
          if (p.dec_tanh) { y[0] = tanhf(y[0]); y[1] = tanhf(y[1]); y[2] = tanhf(y[2]); }
          if constexpr (OUTK == OUT_F32_NCHW) {
            float* o = (float*)p.out;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) o[(((size_t)n * 3 + ch) * p.oh + oy) * p.ow + ox] = y[ch];
          } else {
            uint8_t* o = (uint8_t*)p.out + (((size_t)n * p.oh + oy) * p.ow + ox) * 3;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) o[ch] = (uint8_t)(decode_ch(y[p.dec_perm[ch]], ch, p) * 255.0f);
          }
        }
      }
    }
  };

  AccT acc;
  auto no_hook = [](int) {};
  if constexpr (PERS) {
    // part q of the next tile is stored at the first stage barrier after which no read of chunk
    // group q remains (the barrier after step s follows the reads of steps <= s+1)
    constexpr int TAPS = C::ROWS * C::KPR;
    auto part_stage = [](int q) { return ((q + 1) * TAPS - 2 + SC - 1) / SC; };  // ceil((.)/SC)
    static_assert(part_stage(0) >= 2, "part 0 is issued after stage 1's barrier");
    float2* norm_l = (float2*)(smem + NORM_OFF);
    float2* rnorm_l = norm_l + CINP;
    auto load_norm_table = [&](int n) {
      if (p.in_norm != nullptr)
        for (int t = tid; t < CINP; t += NT) norm_l[t] = p.in_norm[(size_t)n * p.cs + t];
      if (resf && has_rn)
        for (int t = tid; t < CINP; t += NT) rnorm_l[t] = p.res_rnorm[(size_t)n * p.cs + t];
    };
    uint4 praw[IPP], praw2[IPP];
    // prologue: tile w staged part by part, weight stages 0/1 in ring slots 0/1, RR stages in flight
    build_maps(cur, 0);
    load_norm_table(cur.n);
    __syncthreads();
    part_items(cur, 0);
#pragma unroll
    for (int q = 0; q < NPART; ++q) {
      issue_part(cur, q, praw, praw2);
      write_part(cur, q, praw, praw2, norm_l, rnorm_l);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wl_store(j * STG_BYTES);
      wl_issue((j + RR) % NSTG);
    }
    __syncthreads();
    int wnext = w + (int)gridDim.x;
    int rot = 0;  // ring slot of the current tile's stage 0
    for (int it = 0;; ++it) {
      const bool more = wnext < p.n_work;
      const Work nxt = more ? decode_work(wnext) : cur;
      const int ns = (it + 1) & 1;  // map slot of the next tile
      kloop(acc, rot, [&](int k) {
        if (!more) return;
        if (k == 0) {  // the current tile's halo is complete: reuse the tables and the other map slot
          build_maps(nxt, ns);
          load_norm_table(nxt.n);
        }
        if (k == 1) {
          part_items(nxt, ns);
          issue_part(nxt, 0, praw, praw2);
        }
#pragma unroll
        for (int q = 0; q < NPART; ++q) {
          if (k == part_stage(q) && k < NSTG) {
            write_part(nxt, q, praw, praw2, norm_l, rnorm_l);
            if (q + 1 < NPART) issue_part(nxt, q + 1, praw, praw2);
          }
        }
      });
      if constexpr (part_stage(NPART - 1) >= NSTG) {
        // the last part(s) have no stage barrier after their reads: store after the K loop
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NPART; ++q) {
          if (more && part_stage(q) >= NSTG) {
            write_part(nxt, q, praw, praw2, norm_l, rnorm_l);
            if (q + 1 < NPART) issue_part(nxt, q + 1, praw, praw2);
          }
        }
      }
      epilogue(cur, acc);
      if (!more) break;
      __syncthreads();  // publishes the next tile's halo parts
      cur = nxt;
      wnext += (int)gridDim.x;
      rot = (rot + NSTG) % 3;
    }
  } else {
    if constexpr (INK == IN_ACT) {
      // the residual join holds two staged tensors per item: with many items per thread (ReCoNet's 192-channel
      // halos: 16-17) the fill runs in two passes, so its registers do not spill (the joined trunk conv: 92 B/lane of
      // scratch in one pass, 0.89-0.94 -> 0.77-0.78 ms in two; the 192-channel phase up-conv keeps 12 B either way and
      // measured slower in three)
      constexpr int NPASS = (resf && IPT > 8) ? NST_GEN_RES_PASSES : 1;
      constexpr int IPP = (IPT + NPASS - 1) / NPASS;
      uint4 raw[IPP], raw2[IPP];
      int srcs[IPP];
      float2 nmc[C::CPC], rnmc[C::CPC];
      build_maps(cur, 0);
      if constexpr (NTAB) {
        float2* nt = (float2*)(smem + NTAB_OFF);
        for (int t = tid; t < CINP; t += NT) {
          if (p.in_norm != nullptr) nt[t] = p.in_norm[(size_t)cur.n * p.cs + t];
          if (resf && has_rn) nt[CINP + t] = p.res_rnorm[(size_t)cur.n * p.cs + t];
        }
      }
      __syncthreads();
      load_norm(cur.n, nmc, rnmc);
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        issue_loads(cur, 0, raw, raw2, srcs, ps * IPP);
        stage(cur, raw, raw2, srcs, nmc, rnmc, ps * IPP);
      }
    } else {
      stage_image(cur);
    }
    if constexpr (WL) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j < NSTG) {
          wl_store(j * STG_BYTES);
          if (j + RR < NSTG) wl_issue(j + RR);
        }
      }
    }
    __syncthreads();
    kloop(acc, 0, no_hook);
    epilogue(cur, acc);
  }
}

// Instantiation helper: a launcher + a registry entry.
template <typename T, int MODE, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN, int INK, int OUTK,
          int VAR = 0>
struct ConvInst {
  using C = ConvCfg<T, MODE, KS, S, CINP, BN, TH, TW, WM, WN>;
  static constexpr bool PERS = (VAR & VAR_PERS) != 0;
  static constexpr auto kernel = conv_kernel<T, MODE, KS, S, CINP, BN, TH, TW, WM, WN, INK, OUTK, VAR>;
  // resident workgroups of the persistent form on this device (CUs x occupancy)
  static int resident_blocks() {
    static const int slots = [] {
      int dev = 0, cus = 0, occ = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, C::NT, 0) != hipSuccess || occ < 1) occ = 1;
      return cus * occ;
    }();
    return slots;
  }
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    if constexpr (PERS) {
      ConvParams p = p0;
      p.n_work = (int)(grid.x * grid.y);
      const int nb = p.n_work < resident_blocks() ? p.n_work : resident_blocks();
      hipLaunchKernelGGL(kernel, dim3(nb), dim3(C::NT), 0, st, p);
    } else {
      hipLaunchKernelGGL(kernel, grid, dim3(C::NT), 0, st, p0);
    }
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));  // fields this mapping does not set (wbytes, tanh_out, in/out_esz, ...) are 0
    k.dtype = dtype_code<T>();
    k.mode = MODE;
    k.ks = KS; k.stride = S; k.cinp = CINP; k.bn = BN; k.th = TH; k.tw = TW; k.wm = WM; k.wn = WN;
    k.in_kind = INK; k.out_kind = OUTK;
    k.pair = C::PAIR ? 1 : 0; k.nch = C::NCH; k.cpc = C::CPC; k.kp = C::KP; k.nchunk = C::NCHUNK;
    k.nstep = C::NSTEP; k.nstep_pack = C::NSTEP_PACK; k.nsubt = C::NSUBT; k.nsub = C::NSUB; k.lds_bytes = C::LDS_ALLOC;
    k.persistent = PERS ? 1 : 0;
    k.korder = PERS ? 1 : 0;
    k.part_rows = PERS ? C::REDW : 1;
    k.res = (VAR & VAR_RES) != 0 ? 1 : 0;
    k.launch = &launch;
    return k;
  }
};

}  // namespace nst
