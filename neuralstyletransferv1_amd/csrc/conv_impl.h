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
//     bf16: v_mfma_f32_16x16x32_bf16 (fp32 accumulate).  fp32: v_mfma_f32_16x16x4_f32
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
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
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
  static constexpr int EB = ((NCH % 4) == 0 ? NCH + 2 : NCH) * 16;               // bytes per LDS entry
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
  static constexpr int CYC_STEP = MSUB * NSUB * (sizeof(T) == 2 ? 16 : 128);
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
  static constexpr int REDW = MODE == MODE_PHASE ? 4 : WM;                        // waves sharing a channel
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
  static_assert(MODE != MODE_PHASE || (WM == 1 && WN == 4 && S == 1), "phase mode: one wave per phase");
  static_assert(MODE != MODE_XSHIFT || (BN == 16 && WN == 1 && S == 1), "x-shift mode: 16 rows = 5x3 + 1");
  static_assert(PAIR || (CINP % CPC) == 0, "channel padding");
  static_assert(PAIR || NCH == 1 || NCH % 4 == 0, "chunks per pixel must be 1 or a multiple of 4");
  static_assert(LDS_ALLOC <= 160 * 1024, "LDS budget");
  static_assert(S == 1 || CINP != 4, "image-input layers are stride 1");
};

// Producer InstanceNorm apply (+ReLU) on one 16-byte chunk: v = v*scale + shift.
template <typename T>
__device__ __forceinline__ uint4 norm_chunk(uint4 raw, const float2* nm, int relu) {
  if constexpr (sizeof(T) == 2) {
    uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float2 s0 = nm[2 * j], s1 = nm[2 * j + 1];
      float lo = bf16_lo(w[j]) * s0.x + s0.y;
      float hi = bf16_hi(w[j]) * s1.x + s1.y;
      if (relu) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
      w[j] = pack_bf16(lo, hi);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float v[4] = {__uint_as_float(raw.x), __uint_as_float(raw.y), __uint_as_float(raw.z), __uint_as_float(raw.w)};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = v[j] * nm[j].x + nm[j].y;
      if (relu) v[j] = fmaxf(v[j], 0.f);
    }
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
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
    return make_uint4(pack_bf16(vals[0][0], vals[0][1]), pack_bf16(vals[0][2], 0.f),
                      pack_bf16(vals[1][0], vals[1][1]), pack_bf16(vals[1][2], 0.f));
  } else {
    return make_uint4(__float_as_uint(vals[0][0]), __float_as_uint(vals[0][1]), __float_as_uint(vals[0][2]), 0u);
  }
}

__device__ __forceinline__ float decode_ch(float y, int ch, const ConvParams& p) {
  float v = (((y + p.dec_p[ch]) * p.dec_q[ch]) / p.dec_r[ch]) + p.dec_s[ch];
  return fminf(fmaxf(v, 0.f), 1.f);  // .clamp(0, 1)
}

template <typename T, int MODE, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN, int INK, int OUTK>
__global__ __launch_bounds__(64 * WM * WN) void conv_kernel(ConvParams p) {
  using C = ConvCfg<T, MODE, KS, S, CINP, BN, TH, TW, WM, WN>;
  constexpr int NT = C::NT;
  constexpr int NCH = C::NCH, EB = C::EB, LWP = C::LWP, HALF = C::HALF, LW = C::LW, W5 = C::W5;
  constexpr int MSUB = C::MSUB, NSUB = C::NSUB, NSUBT = C::NSUBT, COLS = C::COLS;
  constexpr bool PAIR = C::PAIR;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS_ALLOC];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, px = lane & 15;
  const int tile = blockIdx.x;
  const int tyi = tile / p.tiles_x, txi = tile - tyi * p.tiles_x;
  const int n = blockIdx.y / p.n_cblk, cb = blockIdx.y - n * p.n_cblk;
  const int ty0 = tyi * TH, tx0 = txi * TW;  // PHASE: tile origin on the source grid

  // weights: fragment (step s, n-subtile t) of this wave lives at wp[(s*NSUBT + t)*64]; a ring of
  // PF steps is kept in flight (steps >= NSTEP are zero padding)
  constexpr int PF = C::PF;
  const uint4* wp = (const uint4*)p.wpk + ((size_t)cb * C::NSTEP_PACK * NSUBT + wn * NSUB) * 64 + lane;
  uint4 a_ring[PF][NSUB];
#pragma unroll
  for (int d = 0; d < PF; ++d)
#pragma unroll
    for (int t = 0; t < NSUB; ++t) a_ring[d][t] = wp[(d * NSUBT + t) * 64];

  // ---- stage the input halo (prologue transform applied) ----
  // The padding / reflection / upsample / crop mapping of halo row ly and column lx to a source
  // row/column (or -1 = zero) is evaluated once per block into two small LDS maps.  Then all of
  // a thread's loads are issued before any is consumed (IPT independent 16-B loads in flight per
  // lane), transformed (producer IN + ReLU) and written to LDS: the fill costs ~one latency.
  const int vy0 = (ty0 + p.crop_y) * S - p.pad;
  const int vx0 = (tx0 + p.crop_x) * S - p.pad;
  int* rowmap = (int*)(smem + C::MAP_OFF);
  int* colmap = rowmap + C::LH;
  if constexpr (INK == IN_ACT) {
    // byte offsets within the frame (host guarantees a frame is < 2 GiB), -1 = zero padding
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
    __syncthreads();
  }
  {
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
    if constexpr (INK == IN_ACT) {
      uint4 raw[IPT];
      bool live[IPT];
      // when NT % NCH == 0 a thread always stages the same channel chunk
      constexpr bool FIXED_CHUNK = (NT % NCH) == 0;
      const int c_fixed = tid % NCH;
      const char* img = (const char*)p.in + (size_t)n * p.hs * p.ws * p.cs * sizeof(T);
      // a FIXED_CHUNK thread applies the same CPC channels' IN constants to every item
      float2 nmc[C::CPC];
      if (FIXED_CHUNK && p.in_norm != nullptr) {
#pragma unroll
        for (int j = 0; j < C::CPC; ++j) nmc[j] = p.in_norm[(size_t)n * p.cs + c_fixed * C::CPC + j];
      }
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const int it = tid + k * NT;
        const int e = it / NCH, c = FIXED_CHUNK ? c_fixed : it - e * NCH;
        int ly, lx;
        bool ok = entry_xy(e, ly, lx) && it < NITEMS;
        const int ro = ok ? rowmap[ly] : -1;
        const int co = ok ? colmap[lx] : -1;
        ok = ok && ro >= 0 && co >= 0;
        live[k] = ok;
        raw[k] = make_uint4(0u, 0u, 0u, 0u);
        if (ok) raw[k] = *(const uint4*)(img + (unsigned)(ro + co + c * 16));
      }
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const int it = tid + k * NT;
        if (it < NITEMS) {
          const int e = it / NCH, c = FIXED_CHUNK ? c_fixed : it - e * NCH;
          uint4 v = raw[k];
          if (live[k] && p.in_norm != nullptr)
            v = norm_chunk<T>(v, FIXED_CHUNK ? nmc : p.in_norm + (size_t)n * p.cs + c * C::CPC, p.in_relu);
          *(uint4*)(smem + e * EB + 16 * c) = v;
        }
      }
    } else {
      static_assert(MODE == MODE_STD, "image input only on plain convs");
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const int it = tid + k * NT;
        if (it < NITEMS) {
          const int e = it / NCH;
          const int ly = e / LWP, lx = e - ly * LWP;
          const uint4 v = load_image_entry<T, INK, PAIR>(p, n, vy0 + ly, vx0 + lx);
          *(uint4*)(smem + e * EB) = v;
        }
      }
    }
  }
  __syncthreads();

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
  f32x4_t acc[MSUB][NSUB];
#pragma unroll
  for (int m = 0; m < MSUB; ++m)
#pragma unroll
    for (int t = 0; t < NSUB; ++t) acc[m][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto mfma_step = [&](const uint4 (&a)[NSUB], const uint4 (&b)[MSUB]) {
#pragma unroll
    for (int m = 0; m < MSUB; ++m) {
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        if constexpr (sizeof(T) == 2) {
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, a[t]), __builtin_bit_cast(bf16x8_t, b[m]), acc[m][t], 0, 0, 0);
        } else {
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].x), __uint_as_float(b[m].x), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].y), __uint_as_float(b[m].y), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].z), __uint_as_float(b[m].z), acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[t].w), __uint_as_float(b[m].w), acc[m][t], 0, 0, 0);
        }
      }
    }
  };

  if constexpr (C::ROWED) {
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
          mfma_step(a_ring[slot], b);
          const int s = row * RS + pos;
#pragma unroll
          for (int t = 0; t < NSUB; ++t) a_ring[slot][t] = wp[((s + PF) * NSUBT + t) * 64];
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
        mfma_step(a_ring[d], b);
#pragma unroll
        for (int t = 0; t < NSUB; ++t) a_ring[d][t] = wp[((s + PF) * NSUBT + t) * 64];
      }
    }
  }

  // ---- epilogue ----
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
#pragma unroll
    for (int j = 0; j < 4 * NSUB; ++j) bias_v[j] = p.bias[cbase + j];
    float s1[4 * NSUB], s2[4 * NSUB];
#pragma unroll
    for (int j = 0; j < 4 * NSUB; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
#pragma unroll
    for (int m = 0; m < MSUB; ++m) {
      int oy, ox;
      out_px(m, oy, ox);
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
      float* red = (float*)smem;  // [REDW][BN][2]
      const int rw = MODE == MODE_PHASE ? wave : wm;
      if (px == 0) {
#pragma unroll
        for (int j = 0; j < 4 * NSUB; ++j) {
          const int cl = cwave - cb * BN + 4 * NSUB * g + j;
          red[(rw * BN + cl) * 2 + 0] = s1[j];
          red[(rw * BN + cl) * 2 + 1] = s2[j];
        }
      }
      __syncthreads();
      const int ntiles = p.tiles_x * p.tiles_y;
      for (int cl = tid; cl < BN; cl += NT) {
        float a = 0.f, b2 = 0.f;
#pragma unroll
        for (int w = 0; w < C::REDW; ++w) { a += red[(w * BN + cl) * 2]; b2 += red[(w * BN + cl) * 2 + 1]; }
        float* dst = p.partial + (((size_t)n * ntiles + tile) * p.cout_stride + cb * BN + cl) * 2;
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
}

// Instantiation helper: a launcher + a registry entry.
template <typename T, int MODE, int KS, int S, int CINP, int BN, int TH, int TW, int WM, int WN, int INK, int OUTK>
struct ConvInst {
  using C = ConvCfg<T, MODE, KS, S, CINP, BN, TH, TW, WM, WN>;
  static void launch(const ConvParams& p, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((conv_kernel<T, MODE, KS, S, CINP, BN, TH, TW, WM, WN, INK, OUTK>), grid, dim3(C::NT), 0, st, p);
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    k.dtype = sizeof(T) == 2 ? NST_DT_BF16 : NST_DT_F32;
    k.mode = MODE;
    k.ks = KS; k.stride = S; k.cinp = CINP; k.bn = BN; k.th = TH; k.tw = TW; k.wm = WM; k.wn = WN;
    k.in_kind = INK; k.out_kind = OUTK;
    k.pair = C::PAIR ? 1 : 0; k.nch = C::NCH; k.cpc = C::CPC; k.kp = C::KP; k.nchunk = C::NCHUNK;
    k.nstep = C::NSTEP; k.nstep_pack = C::NSTEP_PACK; k.nsubt = C::NSUBT; k.nsub = C::NSUB; k.lds_bytes = C::LDS_ALLOC;
    k.launch = &launch;
    return k;
  }
};

}  // namespace nst
