// conv_impl.h — the one convolution kernel of the engine, templated per layer shape.
//
// Replaces every Conv2d / ConvTranspose2d of the three stylization nets
// (transformer_net.py:44-54,79-99; transformer_net_nst.py:12-59,76; model.py:5-11,69-80)
// together with what surrounds it in the reference graph:
//   * the padding (ReflectionPad2d / zero padding / NST's ReflectionPad2d(40)),
//   * nearest x2 upsampling (UpsampleConvLayer, Decoder nn.Upsample) and ConvTranspose2d
//     (as a conv over the zero-inserted grid),
//   * the PREVIOUS layer's InstanceNorm apply + ReLU (prologue, while filling LDS),
//   * this layer's InstanceNorm statistics (per-tile partial sums in the epilogue),
//   * for the first/last layer: the io_preset encode (pipeline.py:1445-1486) from uint8
//     frames and the decode + clamp(0,1) + ToPILImage truncation to uint8 frames.
//
// Shape of the computation (implicit GEMM, MI355X-first):
//   * one workgroup = 4 waves = one TH x TW tile of output pixels x BN output channels
//     of one frame; the whole (TH-1)*S+KS x (TW-1)*S+KS input halo, all input channels,
//     is staged ONCE in LDS (NHWC, 16-byte chunks XOR-swizzled so the 16 lanes of an
//     MFMA operand read hit 16 distinct bank slots), then the K loop (taps x channels)
//     runs with no further barrier.
//   * MFMA operands: A = packed weights (rows = output channels) streamed from L2 as one
//     coalesced 1 KiB fragment per wave-instruction, prefetched one K-step ahead;
//     B = input pixels from LDS (cols = 16 consecutive output pixels of one row).
//     bf16: v_mfma_f32_16x16x32_bf16 (fp32 accumulate).  fp32: v_mfma_f32_16x16x4_f32
//     (exact fp32 FMA chain) — the parity mode.
//   * output-channel permutation: C row q of n-subtile t is output channel
//     4*NSUB*(q>>2) + 4*t + (q&3) of the wave's range, so each lane ends up owning
//     4*NSUB CONSECUTIVE channels of one pixel -> 16..64-byte contiguous NHWC stores.
//   * stride 2 uses a polyphase LDS column order (even columns, then odd) so stride-2
//     operand reads are unit-stride in LDS.
#pragma once
#include "nst_internal.h"
#include "nst_hip.h"

namespace nst {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

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
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

template <typename T, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN>
struct ConvCfg {
  static constexpr int CPC = 16 / (int)sizeof(T);                 // channels per 16-B chunk
  static constexpr bool PAIR = (sizeof(T) == 2) && (CINP == 4);   // bf16 image layer: chunk = 2 pixels x 4 ch
  static constexpr int NCH = PAIR ? 1 : CINP / CPC;               // chunks per LDS entry
  static constexpr int EB = 16 * NCH;                             // bytes per LDS entry
  static constexpr int KP = PAIR ? (KS + 1) / 2 : KS;             // x-taps per kernel row
  static constexpr int NTAP = KS * KP;
  static constexpr int NCHUNK = NTAP * NCH;                       // 16-B chunks along K
  static constexpr int NSTEP = (NCHUNK + 3) / 4;                  // 4 chunks (one per lane group) per step
  static constexpr int LH = (TH - 1) * S + KS;
  static constexpr int LW = (TW - 1) * S + KS;
  static constexpr int HALF = (LW + 1) / 2;
  static constexpr int LWP = (S == 2) ? 2 * HALF : LW;
  static constexpr int NENT = LH * LWP;
  static constexpr int LDS_BYTES = NENT * EB;
  static constexpr int MSUBT = TH * TW / 16;
  static constexpr int MSUB = MSUBT / WM;
  static constexpr int NSUBT = BN / 16;
  static constexpr int NSUB = NSUBT / WN;
  static constexpr int RED_BYTES = WM * BN * 2 * 4;
  static constexpr int LDS_ALLOC = LDS_BYTES > RED_BYTES ? LDS_BYTES : RED_BYTES;
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(TW % 16 == 0 && MSUBT % WM == 0, "m-subtiles must split over WM waves");
  static_assert(BN % 16 == 0 && NSUBT % WN == 0, "n-subtiles must split over WN waves");
  static_assert(PAIR || (CINP % CPC) == 0, "channel padding");
  static_assert(PAIR || NCH == 1 || NCH % 4 == 0, "chunks per pixel must be 1 or a multiple of 4");
  static_assert(LDS_ALLOC <= 160 * 1024, "LDS budget");
};

// Load one 16-byte LDS entry chunk (after prologue transform) for virtual coords (vy, vx).
template <typename T, int CINP, int INK, bool PAIR, int CPC>
__device__ __forceinline__ uint4 load_entry(const ConvParams& p, int n, int vy, int vx, int c) {
  uint4 zero = {0u, 0u, 0u, 0u};
  if constexpr (INK == IN_ACT) {
    const int sy = map_axis(vy, p.hs, p.axis_mode, p.pre);
    const int sx = map_axis(vx, p.ws, p.axis_mode, p.pre);
    if (sy < 0 || sx < 0) return zero;
    const size_t off = ((((size_t)n * p.hs + sy) * p.ws + sx) * p.cs + (size_t)c * CPC) * sizeof(T);
    uint4 raw = *(const uint4*)((const char*)p.in + off);
    if (p.in_norm == nullptr) return raw;
    const float2* nm = p.in_norm + (size_t)n * p.cs + c * CPC;
    if constexpr (sizeof(T) == 2) {
      uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 s0 = nm[2 * j], s1 = nm[2 * j + 1];
        float lo = bf16_lo(w[j]) * s0.x + s0.y;
        float hi = bf16_hi(w[j]) * s1.x + s1.y;
        if (p.in_relu) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
        w[j] = pack_bf16(lo, hi);
      }
      return make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      float v[4] = {__uint_as_float(raw.x), __uint_as_float(raw.y), __uint_as_float(raw.z),
                    __uint_as_float(raw.w)};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = v[j] * nm[j].x + nm[j].y;
        if (p.in_relu) v[j] = fmaxf(v[j], 0.f);
      }
      return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                        __float_as_uint(v[3]));
    }
  } else {
    // image input (3 channels): PAIR -> pixels vx, vx+1 (4 bf16 each); else one pixel (4 f32)
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
      return make_uint4(pack_bf16(vals[0][0], vals[0][1]), pack_bf16(vals[0][2], 0.f),
                        pack_bf16(vals[1][0], vals[1][1]), pack_bf16(vals[1][2], 0.f));
    } else {
      return make_uint4(__float_as_uint(vals[0][0]), __float_as_uint(vals[0][1]),
                        __float_as_uint(vals[0][2]), 0u);
    }
  }
}

template <typename T, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN, int INK,
          int OUTK>
__global__ __launch_bounds__(256) void conv_kernel(ConvParams p) {
  using C = ConvCfg<T, KS, S, CINP, BN, TH, TW, WM, WN>;
  constexpr int NCH = C::NCH, EB = C::EB, LWP = C::LWP, HALF = C::HALF, LW = C::LW;
  constexpr int MSUB = C::MSUB, NSUB = C::NSUB, NSUBT = C::NSUBT, NSTEP = C::NSTEP;
  constexpr bool PAIR = C::PAIR;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS_ALLOC];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, px = lane & 15;
  const int tile = blockIdx.x;
  const int tyi = tile / p.tiles_x, txi = tile - tyi * p.tiles_x;
  const int n = blockIdx.y / p.n_cblk, cb = blockIdx.y - n * p.n_cblk;
  const int ty0 = tyi * TH, tx0 = txi * TW;

  // weights: fragment (step s, n-subtile t) of this wave lives at wp[(s*NSUBT + t)*64]
  const uint4* wp = (const uint4*)p.wpk + ((size_t)cb * (NSTEP + 1) * NSUBT + wn * NSUB) * 64 + lane;
  uint4 a_cur[NSUB];
#pragma unroll
  for (int t = 0; t < NSUB; ++t) a_cur[t] = wp[t * 64];

  // ---- stage the input halo (prologue transform applied) ----
  const int vy0 = (ty0 + p.crop_y) * S - p.pad;
  const int vx0 = (tx0 + p.crop_x) * S - p.pad;
  for (int it = tid; it < C::NENT * NCH; it += 256) {
    const int e = it / NCH, c = it - e * NCH;
    const int ly = e / LWP, pc = e - ly * LWP;
    int lx = pc;
    bool pad_entry = false;
    if constexpr (S == 2) {
      lx = pc < HALF ? 2 * pc : 2 * (pc - HALF) + 1;
      pad_entry = lx >= LW;
    }
    uint4 v = {0u, 0u, 0u, 0u};
    if (!pad_entry) v = load_entry<T, CINP, INK, PAIR, C::CPC>(p, n, vy0 + ly, vx0 + lx, c);
    *(uint4*)(smem + e * EB + 16 * (c ^ swz<NCH>(e))) = v;
  }
  __syncthreads();

  // ---- K loop: taps x channel chunks ----
  int base[MSUB];
#pragma unroll
  for (int m = 0; m < MSUB; ++m) {
    const int ms = wm * MSUB + m;
    const int r = ms / (TW / 16), cbk = ms - r * (TW / 16);
    const int oxl = cbk * 16 + px;
    base[m] = (S == 2 ? 2 * r : r) * LWP + oxl;
  }
  f32x4_t acc[MSUB][NSUB];
#pragma unroll
  for (int m = 0; m < MSUB; ++m)
#pragma unroll
    for (int t = 0; t < NSUB; ++t) acc[m][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

#pragma unroll 2
  for (int s = 0; s < NSTEP; ++s) {
    uint4 a_nxt[NSUB];
#pragma unroll
    for (int t = 0; t < NSUB; ++t) a_nxt[t] = wp[((s + 1) * NSUBT + t) * 64];  // step NSTEP is zero padding
    const int i = 4 * s + g;
    int tap = 0, c = 0;
    if (i < C::NCHUNK) {
      tap = i / NCH;
      c = i - tap * NCH;
    }
    const int dy = tap / C::KP, dxp = tap - dy * C::KP;
    const int dx = PAIR ? 2 * dxp : dxp;
    const int toff = dy * LWP + (S == 2 ? ((dx & 1) * HALF + (dx >> 1)) : dx);
    uint4 b[MSUB];
#pragma unroll
    for (int m = 0; m < MSUB; ++m) {
      const int e = base[m] + toff;
      b[m] = *(const uint4*)(smem + e * EB + 16 * (c ^ swz<NCH>(e)));
    }
#pragma unroll
    for (int m = 0; m < MSUB; ++m) {
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        if constexpr (sizeof(T) == 2) {
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, a_cur[t]), __builtin_bit_cast(bf16x8_t, b[m]), acc[m][t], 0, 0, 0);
        } else {
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a_cur[t].x), __uint_as_float(b[m].x), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a_cur[t].y), __uint_as_float(b[m].y), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a_cur[t].z), __uint_as_float(b[m].z), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a_cur[t].w), __uint_as_float(b[m].w), acc[m][t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NSUB; ++t) a_cur[t] = a_nxt[t];
  }

  // ---- epilogue ----
  const int cwave = cb * BN + wn * NSUB * 16;  // first channel of this wave
  const int cbase = cwave + 4 * NSUB * g;      // this lane's 4*NSUB consecutive channels
  if constexpr (OUTK == OUT_ACT) {
    float bias_v[4 * NSUB];
#pragma unroll
    for (int j = 0; j < 4 * NSUB; ++j) bias_v[j] = p.bias[cbase + j];
    float s1[4 * NSUB], s2[4 * NSUB];
#pragma unroll
    for (int j = 0; j < 4 * NSUB; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
#pragma unroll
    for (int m = 0; m < MSUB; ++m) {
      const int ms = wm * MSUB + m;
      const int r = ms / (TW / 16), cbk = ms - r * (TW / 16);
      const int oy = ty0 + r, ox = tx0 + cbk * 16 + px;
      const bool valid = (oy < p.oh) && (ox < p.ow);
      float v[4 * NSUB];
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[4 * t + q] = acc[m][t][q] + bias_v[4 * t + q];
      if (valid) {
        char* dst = (char*)p.out + ((((size_t)n * p.oh + oy) * p.ow + ox) * p.cout_stride + cbase) * sizeof(T);
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int h = 0; h < NSUB; h += 2) {
            if (h + 1 < NSUB) {
              *(uint4*)(dst + h * 8) = make_uint4(pack_bf16(v[4 * h], v[4 * h + 1]), pack_bf16(v[4 * h + 2], v[4 * h + 3]),
                                                  pack_bf16(v[4 * h + 4], v[4 * h + 5]), pack_bf16(v[4 * h + 6], v[4 * h + 7]));
            } else {
              *(uint2*)(dst + h * 8) = make_uint2(pack_bf16(v[4 * h], v[4 * h + 1]), pack_bf16(v[4 * h + 2], v[4 * h + 3]));
            }
          }
        } else {
#pragma unroll
          for (int t = 0; t < NSUB; ++t)
            *(float4*)(dst + t * 16) = make_float4(v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]);
        }
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) { s1[j] += v[j]; s2[j] += v[j] * v[j]; }
      }
    }
    if (p.partial != nullptr) {
      // reduce over the 16 pixel lanes of each lane group
#pragma unroll
      for (int j = 0; j < 4 * NSUB; ++j) {
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) {
          s1[j] += __shfl_xor(s1[j], off);
          s2[j] += __shfl_xor(s2[j], off);
        }
      }
      __syncthreads();  // LDS tile no longer read
      float* red = (float*)smem;  // [WM][BN][2]
      if (px == 0) {
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) {
          const int cl = wn * NSUB * 16 + 4 * NSUB * g + j;
          red[(wm * BN + cl) * 2 + 0] = s1[j];
          red[(wm * BN + cl) * 2 + 1] = s2[j];
        }
      }
      __syncthreads();
      const int ntiles = p.tiles_x * p.tiles_y;
      for (int cl = tid; cl < BN; cl += 256) {
        float a = 0.f, b2 = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { a += red[(w * BN + cl) * 2]; b2 += red[(w * BN + cl) * 2 + 1]; }
        float* dst = p.partial + (((size_t)n * ntiles + tile) * p.cout_stride + cb * BN + cl) * 2;
        dst[0] = a;
        dst[1] = b2;
      }
    }
  } else {
    // final layer: 3 output channels live in lane group 0 (channels 0..3 of n-subtile 0)
    if (g == 0) {
      const float b0 = p.bias[0], b1 = p.bias[1], b2v = p.bias[2];
#pragma unroll
      for (int m = 0; m < MSUB; ++m) {
        const int ms = wm * MSUB + m;
        const int r = ms / (TW / 16), cbk = ms - r * (TW / 16);
        const int oy = ty0 + r, ox = tx0 + cbk * 16 + px;
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
          for (int ch = 0; ch < 3; ++ch) {
            float v = (((y[p.dec_perm[ch]] + p.dec_p[ch]) * p.dec_q[ch]) / p.dec_r[ch]) + p.dec_s[ch];
            v = fminf(fmaxf(v, 0.f), 1.f);  // .clamp(0, 1)
            o[ch] = (uint8_t)(v * 255.0f);   // ToPILImage: pic.mul(255).byte() (truncation)
          }
        }
      }
    }
  }
}

// Instantiation helper: a launcher + a registry entry.
template <typename T, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN, int INK, int OUTK>
struct ConvInst {
  using C = ConvCfg<T, KS, S, CINP, BN, TH, TW, WM, WN>;
  static void launch(const ConvParams& p, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((conv_kernel<T, KS, S, CINP, BN, TH, TW, WM, WN, INK, OUTK>), grid, dim3(256), 0, st, p);
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    k.dtype = sizeof(T) == 2 ? NST_DT_BF16 : NST_DT_F32;
    k.ks = KS; k.stride = S; k.cinp = CINP; k.bn = BN; k.th = TH; k.tw = TW; k.wm = WM; k.wn = WN;
    k.in_kind = INK; k.out_kind = OUTK;
    k.pair = C::PAIR ? 1 : 0; k.nch = C::NCH; k.cpc = C::CPC; k.kp = C::KP; k.nchunk = C::NCHUNK;
    k.nstep = C::NSTEP; k.nsubt = C::NSUBT; k.nsub = C::NSUB; k.lds_bytes = C::LDS_ALLOC;
    k.launch = &launch;
    return k;
  }
};

}  // namespace nst
