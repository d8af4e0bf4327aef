// conv_ws9.hip — weight-stationary persistent first layer: the 9x9 image conv, 3 -> 32 channels.
//
// Replaces ConvLayer(3, 32, kernel 9, stride 1) = ReflectionPad2d(4) + Conv2d
// (transformer_net.py:8 conv1, transformer_net.py:46-54) and NST's down1 (transformer_net_nst.py:64,
// zero padding after the 40-pixel pre-reflect), reading the pre-padded encoded frame of
// conv_prep.hip (bf16 [n][hp][wp][4], channel 3 = 0, padding already resolved) with an identity
// coordinate map; this layer's InstanceNorm partial sums in the epilogue.
//
// The generic implicit-GEMM kernel ran this layer at ~0.5 ms per batch of 8 1080p frames, VALU-
// and wait-bound (5 VALU per MFMA).  Here the whole weight tensor (32 x 9 x 9 x 4 bf16) lives in
// every wave's registers (84 VGPRs) and the K loop is LDS reads + MFMAs only:
//   * K = (ky, kx, c).  For kx 0..7 one 16x16x32 MFMA covers a whole kernel row ky: lane (px, g)
//     holds the 16 contiguous bytes of padded pixels x + 2g, x + 2g + 1 (4 channels each) of input
//     row y + ky, so the B operand of input row r serves output rows r - ky for all nine ky.
//     Column kx = 8 is a 16x16x16 MFMA over 4 kernel rows (lane group g = kernel row 4j + g, one
//     8-byte pixel): operand K(s) = rows s..s+3 serves output rows s, s - 4, s - 8 (j = 0, 1, 2).
//     Issued K = 9 x 32 + 3 x 16 = 336 for 324 useful (96 %), at the MFMA cost of 9 + 1.5 steps.
//   * workgroup = NW waves (4), tile = 8 output rows x 16 NW columns, wave w = 8 rows x columns
//     16w..16w+15 and all 32 output channels (two M tiles): 16 input-row operands + 16 column-8
//     operands feed 192 MFMAs per wave and tile;
//   * persistent over (frame, tile) items, XCD-aware order, two 4-wave workgroups per CU (register
//     allocation bounded to two waves per SIMD): their barriers are independent, so one's epilogue
//     and stores overlap the other's MFMAs.  Unbounded, hipcc spilled the accumulators to AGPRs at
//     one wave per SIMD and only one workgroup per CU was resident (0.465 vs 0.367 ms);
//   * the next item's 16-row halo (RCH 16-byte chunks per row, contiguous in the padded frame)
//     travels by LDS-DMA into the second of two halo buffers while the current item computes;
//   * output tile staged in LDS (8-byte slots XOR-swizzled by pixel) and stored as whole 64-byte
//     pixels, 16 B per lane (half-pixel stores from the accumulators measured ~3 % slower);
//     per-wave IN partials (DPP reduce-scatter) combined in fixed order into one partial row per
//     tile.  Measured (bench, 8 x 1080p): 0.367 ms vs 0.51 for the generic kernel.
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "conv_ws_common.h"

namespace nst {

#ifndef NST_WS9_TH
#define NST_WS9_TH 8
#endif
constexpr int WS9_TH = NST_WS9_TH;    // output rows per tile (each wave's rows)
#ifndef NST_WS9_OCC
#define NST_WS9_OCC 2
#endif
constexpr int WS9_OCC = NST_WS9_OCC;   // waves per SIMD the register allocation must allow (two 4-wave workgroups per CU)
#ifndef NST_WS9_NW
#define NST_WS9_NW 4
#endif
constexpr int WS9_NW = NST_WS9_NW;    // waves per workgroup: 4 = two workgroups per CU drifting out of phase
#ifndef NST_WS9_RING
#define NST_WS9_RING 2
#endif
constexpr int WS9_RING = NST_WS9_RING;  // input-row operands in flight ahead of the MFMAs

// SW (split weights, the split-precision modes' first layer): the exact raw-byte operand of conv_prep.hip's
// enc_raw staging against fp16 hi / lo weight pairs (Wh = RNE(w), Wl = RNE(w - Wh)): the two MFMAs the plain
// kernel spends on the two 16-channel M tiles go to Wh and Wl of ONE M tile, into separate accumulators added in
// the epilogue, so a wave covers 16 output channels (wave w: channel half w / (NW/2), 16-column strip w % (NW/2))
// and a tile is half as wide.  O32: fp32 output (the next layer reads it as a split hi / lo operand).
// CO (plain weights only): output channels, 32 or 64.  64 (ReCoNet's 48 -> 64 padded first layer): two channel
// halves of 32 (each wave: one half's two M tiles and weight set, the same registers as 32 channels), so a tile
// has half as many 16-column strips.
template <int NW_, bool SW = false, bool O32 = false, int CO = 32>
struct W9Cfg {
  static constexpr int NW = NW_, NT = 64 * NW, TH = WS9_TH, COUT = CO;
  static constexpr int MH = SW ? 2 : CO / 32;      // channel halves (SW: hi / lo weight halves of 16 channels)
  static constexpr int NSTRIP = NW / MH;           // 16-column strips per tile
  static_assert(!SW || CO == 32, "split weights: 32 channels");
  static_assert(CO == 32 || CO == 64, "32 or 64 output channels");
  static constexpr int TW = 16 * NSTRIP;
  static constexpr int HR = TH + 8;                 // halo rows
  // 16-B chunks per halo row: TW + 8 px used, rounded up so the row stride is == 32 mod 64 dwords
  // (the column-8 operand's four rows land in disjoint bank halves)
  static constexpr int RCH = ((TW + 8) / 2 + 7) / 16 * 16 + 8;
  static constexpr int RS = RCH * 16;
  static constexpr int HALO = HR * RS;
  static constexpr int NCHK = HR * RCH;
  static constexpr int NREQ = (NCHK + NT - 1) / NT; // request slots per thread (the last partial)
  static constexpr int PIXB = COUT * (O32 ? 4 : 2);  // bytes per output pixel
  static constexpr int OUT_OFF = 2 * HALO;
  static constexpr int OUTB = TH * TW * PIXB;       // the LDS output tile
  static constexpr int NST = TH * TW * PIXB / (NT * 16);  // 16-B stores per thread
  static constexpr int PXS = NT * 16 / PIXB;        // output pixels per store instruction
  static constexpr int PART_OFF = OUT_OFF + OUTB;
  static constexpr int BIAS_OFF = PART_OFF + NW * 64 * 4;
  static constexpr int LDS = BIAS_OFF + COUT * 4;
  static constexpr int NWM = 9 * 2;                 // 16x16x32 weight fragments (ky, m)
  static constexpr int NWK = 3 * 2;                 // 16x16x16 weight fragments (j, m)
  static constexpr int WHALF = NWM * 64 * 16 + NWK * 64 * 8;  // one weight set (SW: one channel half)
  static constexpr int WBYTES = MH * WHALF;
  static_assert(NCHK % 64 == 0, "whole-wave DMA requests");
  static_assert(2 * RCH >= TW + 8 && (RS / 4) % 64 == 32, "halo row");
  static_assert(NST * NT * 16 == TH * TW * PIXB, "whole 16-B stores per thread");
  static_assert(PXS % TW == 0, "a store instruction covers whole tile rows (a thread's column is fixed)");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint64_t lds_u64;

// CST: output channels stored (<= CO; ReCoNet's 48-channel first layer computes 64 and stores 48 unpadded).  Stores of
// the padding chunks / statistics go to the out-of-range offset, still issued (the waits count store_out's stores)
template <typename T, int NW, bool SW, bool O32, int CO, int CST = CO>
__global__ __launch_bounds__(64 * NW, WS9_OCC) void ws9_kernel(ConvParams p) {
  using C = W9Cfg<NW, SW, O32, CO>;
  static_assert(!SW || IS_F16<T>, "split weights are fp16 pairs");
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, px = lane & 15;
  const int strip = wv % C::NSTRIP;  // the wave's 16 output columns
  const int mh = wv / C::NSTRIP;     // SW: the wave's 16 output channels 16 mh ..; CO = 64: its 32 channels 32 mh ..

  struct Work {
    int n, tile, oy0, ox0;
  };
  const int ntile = p.tiles_x * p.tiles_y;
  auto decode = [&](int wi) {
    Work r;
    r.n = wi / ntile;
    r.tile = wi - r.n * ntile;
    const int ty = r.tile / p.tiles_x;
    r.oy0 = ty * C::TH;
    r.ox0 = (r.tile - ty * p.tiles_x) * C::TW;
    return r;
  };
  // workgroups b, b+8, ... share an XCD: each XCD takes a contiguous run of tiles per sweep
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int w0 = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  if (w0 >= p.n_work) return;

  // ---- the whole weight tensor (SW: the wave's channel half, hi and lo), resident for the launch ----
  // wm[2 ky + m]: M tile m (plain) or weight part m = hi / lo of channel half mh (SW); wk likewise
  uint4 wm[C::NWM];
  uint2 wk[C::NWK];
  {
    const char* wbase = (const char*)p.wpk + (size_t)mh * C::WHALF;
    const uint4* src = (const uint4*)wbase + lane;
#pragma unroll
    for (int s = 0; s < C::NWM; ++s) wm[s] = src[s * 64];
    const uint2* srck = (const uint2*)(wbase + C::NWM * 64 * 16) + lane;
#pragma unroll
    for (int s = 0; s < C::NWK; ++s) wk[s] = srck[s * 64];
  }
  if (tid < C::COUT) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];

  // ---- halo requests: chunk j = k NT + tid -> halo row j / RCH, chunk j % RCH; LDS j * 16 ----
  const size_t frame_bytes = (size_t)p.hs * p.ws * 8;
  const uint32_t smem_u = (uint32_t)(uintptr_t)smem;
  // the tile moves the frame offset only (soffset); a thread's chunk offsets are launch constants.
  // The last tile row's halo and the columns past a row's end read finite data of the next rows or
  // frame, or the workspace's tail slack behind the last frame (make_plan sizes it for the 16 halo
  // rows), whether or not the range check covers soffset; such reads only feed outputs past the
  // frame edge, which are masked
  uint32_t roff[C::NREQ];
#pragma unroll
  for (int k = 0; k < C::NREQ; ++k) {
    const int j = k * C::NT + tid;
    const int row = j / C::RCH, c = j - row * C::RCH;
    roff[k] = (uint32_t)((row * p.ws + 2 * c) * 8);
  }
  auto request = [&](const Work& wk_, int buf) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.in + (size_t)wk_.n * frame_bytes), (short)0, (int)frame_bytes, 0x00020000);
    const int soff = (wk_.oy0 * p.ws + wk_.ox0) * 8;
#pragma unroll
    for (int k = 0; k < C::NREQ; ++k) {
      if (k * C::NT + wv * 64 >= C::NCHK) continue;  // wave-uniform
      dma16(rs, roff[k], smem_u + buf * C::HALO + (k * C::NT + wv * 64) * 16, soff);
    }
  };

  typedef f32x4_t Acc[C::TH][2];
  // SW: asm MFMAs (accumulators tied in place: the builtins let hipcc allocate a destination over an operand,
  // mfma16x16x16_tied); the epilogue then drains the MFMA pipe before its VALU reads
  auto mfma32 = [&](f32x4_t& c, const uint4& a, const uint4& bop, bool first) {
    if constexpr (SW) {
      mfma_tied<T>(c, a, bop, first);
      return;
    }
    const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
    c = mfma16x16x32<T>(a, bop, first ? z : c);
  };
  auto mfma16 = [&](f32x4_t& c, const uint2& a, const uint2& bop) {
    if constexpr (SW)
      mfma16x16x16_tied<T>(c, a, bop);
    else if constexpr (IS_F16<T>)
      c = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4_t, a), __builtin_bit_cast(f16x4_t, bop), c, 0, 0, 0);
    else
      c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4_t, a), __builtin_bit_cast(s16x4_t, bop), c,
                                                    0, 0, 0);
  };
  // ---- K loop over the wave's 16 halo rows ----
  auto kloop = [&](Acc& acc, int buf) {
    int fb = buf * C::HALO + (16 * strip + px + 2 * g) * 8;  // row-r operand: + r * RS
    int kb = buf * C::HALO + (16 * strip + px + 8) * 8;      // column-8 operand rows r + g (clamped)
    asm volatile("" : "+v"(fb), "+v"(kb));
    // the row operand of lane (px, g) starts at pixel 16 wv + px + 2g: 8-byte aligned, not 16.  A ds_read_b128 off
    // its 16-byte alignment is replayed at ~64 cycles per wave-instruction (cdna_hip_programming.md Guideline
    // 17), which made this kernel LDS-bound (SQ_LDS_IDX_ACTIVE ~0.8 of its cycles): two naturally aligned
    // ds_read_b64 instead (volatile: never merged into a ds_read2_b64)
    auto fread = [&](int r) {
      const char* a = smem + fb + r * C::RS;
      const uint64_t lo = *(const volatile lds_u64*)a, hi = *(const volatile lds_u64*)(a + 8);
      return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    };
    // rows past the halo only meet zero weights (kernel rows 9..11): read row HR - 1 instead
    typedef uint2 KOp;
    auto kread = [&](int r) {
      const int kr = (r + 3 < C::HR) ? (r + g) * C::RS : min(r + g, C::HR - 1) * C::RS;
      return *(const uint2*)(smem + kb + kr);
    };
    // operands of row r + D are read while row r's MFMAs issue (register ring, explicit order)
    constexpr int D = WS9_RING;
    uint4 fr[D];
    KOp kf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      fr[i] = fread(i);
      kf[i] = kread(i);
    }
#pragma unroll
    for (int r = 0; r < C::HR; ++r) {
      const uint4 f = fr[r % D];
      const KOp k8 = kf[r % D];
      if (r + D < C::HR) {
        fr[r % D] = fread(r + D);
        kf[r % D] = kread(r + D);
      }
#pragma unroll
      for (int y = 0; y < C::TH; ++y) {
        const int ky = r - y;
        if (ky < 0 || ky > 8) continue;
        mfma32(acc[y][0], wm[2 * ky + 0], f, ky == 0);
        mfma32(acc[y][1], wm[2 * ky + 1], f, ky == 0);
      }
#pragma unroll
      for (int y = 0; y < C::TH; ++y) {
        const int d = r - y;
        if (d < 0 || d > 8 || (d & 3)) continue;
        mfma16(acc[y][0], wk[2 * (d >> 2) + 0], k8);
        mfma16(acc[y][1], wk[2 * (d >> 2) + 1], k8);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: bias, 16-bit values into the LDS output tile, IN partials from the fp32 values ----
  auto epilogue = [&](const Work& wk_, Acc& acc) {
    if constexpr (!SW) {
      const f32x4_t bias0 = *(const f32x4_t*)(smem + C::BIAS_OFF + (32 * mh + 4 * g) * 4);
      const f32x4_t bias1 = *(const f32x4_t*)(smem + C::BIAS_OFF + (32 * mh + 16 + 4 * g) * 4);
      const int e = 2 * ((px >> 2) & 3);  // slot swizzle of this lane's pixel
      int obase = C::OUT_OFF + (16 * strip + px) * C::PIXB;
      asm volatile("" : "+v"(obase));
      const int o0 = ((8 * mh + 0 + g) ^ e) * 8, o1 = ((8 * mh + 4 + g) ^ e) * 8;
      f32x4_t s1a = {0.f, 0.f, 0.f, 0.f}, s2a = s1a, s1b = s1a, s2b = s1a;
      // interior tiles (all but the frame's last row / column of tiles) take the select-free copy
      auto rows = [&](auto masked) {
#pragma unroll
        for (int y = 0; y < C::TH; ++y) {
          const f32x4_t va = add4(acc[y][0], bias0), vb = add4(acc[y][1], bias1);
          const u32x2_t pa = {pack16<T>(va[0], va[1]), pack16<T>(va[2], va[3])};
          const u32x2_t pb = {pack16<T>(vb[0], vb[1]), pack16<T>(vb[2], vb[3])};
          *(u32x2_t*)(smem + obase + y * C::TW * C::PIXB + o0) = pa;
          *(u32x2_t*)(smem + obase + y * C::TW * C::PIXB + o1) = pb;
          f32x4_t xa = va, xb = vb;
          if constexpr (decltype(masked)::value) {
            const bool valid = wk_.oy0 + y < p.oh && wk_.ox0 + 16 * strip + px < p.ow;
            const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
            xa = valid ? va : z;
            xb = valid ? vb : z;
          }
          stat4(s1a, s2a, xa);
          stat4(s1b, s2b, xb);
        }
      };
      if (wk_.oy0 + C::TH <= p.oh && wk_.ox0 + C::TW <= p.ow)
        rows(std::false_type{});
      else
        rows(std::true_type{});
      // value v = 8 m + 2 c + k (channel 16 m + 4 g + c, k = sum / sum of squares); after the
      // reduce-scatter over the 16 pixel lanes lane px holds the row total of value px
      const float vv[16] = {s1a[0], s2a[0], s1a[1], s2a[1], s1a[2], s2a[2], s1a[3], s2a[3],
                            s1b[0], s2b[0], s1b[1], s2b[1], s1b[2], s2b[2], s1b[3], s2b[3]};
      float a8[8], a4[4], a2[2], a1[1];
      rs_step<8, 0x140>(vv, a8, px >= 8);
      rs_step<4, 0x141>(a8, a4, (px & 4) != 0);
      rs_step<2, 0x1b>(a4, a2, (px & 2) != 0);
      rs_step<1, 0xb1>(a2, a1, (px & 1) != 0);
      const int ch = 16 * (px >> 3) + 4 * g + ((px >> 1) & 3);
      ((float*)(smem + C::PART_OFF))[wv * 64 + ch * 2 + (px & 1)] = a1[0];
    } else {
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // asm MFMA results -> VALU reads
      // hi + lo partial sums of channels 16 mh + 4 g .. + 3, + bias (fp32), into the staged tile
      const f32x4_t bias = *(const f32x4_t*)(smem + C::BIAS_OFF + (16 * mh + 4 * g) * 4);
      int obase = C::OUT_OFF + (16 * strip + px) * C::PIXB;
      asm volatile("" : "+v"(obase));
      // O32: 16-B chunk 4 mh + g of the 8-chunk pixel, XOR-swizzled by pixel (2-way at most); 16-bit: 8-B slot
      const int oo = O32 ? (((4 * mh + g) ^ (px & 7)) * 16) : (((4 * mh + g) ^ (2 * ((px >> 2) & 3))) * 8);
      f32x4_t s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
      auto rows = [&](auto masked) {
#pragma unroll
        for (int y = 0; y < C::TH; ++y) {
          const f32x4_t v = add4(add4(acc[y][0], acc[y][1]), bias);
          if constexpr (O32) {
            *(f32x4_t*)(smem + obase + y * C::TW * C::PIXB + oo) = v;
          } else {
            const u32x2_t pv = {pack16<T>(v[0], v[1]), pack16<T>(v[2], v[3])};
            *(u32x2_t*)(smem + obase + y * C::TW * C::PIXB + oo) = pv;
          }
          f32x4_t x = v;
          if constexpr (decltype(masked)::value) {
            const bool valid = wk_.oy0 + y < p.oh && wk_.ox0 + 16 * strip + px < p.ow;
            x = valid ? v : (f32x4_t){0.f, 0.f, 0.f, 0.f};
          }
          stat4(s1, s2, x);
        }
      };
      if (wk_.oy0 + C::TH <= p.oh && wk_.ox0 + C::TW <= p.ow)
        rows(std::false_type{});
      else
        rows(std::true_type{});
      // reduce-scatter of the 8 statistics over the 16 pixel lanes, then the xor-1 partner: lane px (even)
      // ends with statistic idx & 1 of channel 4 g + (idx >> 1) of the half, idx = 4 (px >= 8) + 2 (px & 4) + (px & 2) / 2
      const float vv[8] = {s1[0], s2[0], s1[1], s2[1], s1[2], s2[2], s1[3], s2[3]};
      float a4[4], a2[2], a1[1];
      rs_step<4, 0x140>(vv, a4, px >= 8);
      rs_step<2, 0x141>(a4, a2, (px & 4) != 0);
      rs_step<1, 0x1b>(a2, a1, (px & 2) != 0);
      const float t = a1[0] + dpp_f<0xb1>(a1[0]);
      const int idx = (px >= 8 ? 4 : 0) + ((px & 4) ? 2 : 0) + ((px & 2) ? 1 : 0);
      if ((px & 1) == 0) ((float*)(smem + C::PART_OFF))[wv * 64 + (4 * g + (idx >> 1)) * 2 + (idx & 1)] = t;
    }
  };
  // wave 0: the tile's partial row (fixed-order sum over the waves of a channel half); all: whole-pixel stores.
  // store k of thread t covers tile bytes (k NT + t) 16 .. + 15: pixel (k NT + t) / (PIXB / 16), chunk (t % (PIXB / 16))
  constexpr int CPP = C::PIXB / 16;  // 16-B chunks per pixel
  const int sq = tid / CPP, scb = (tid % CPP) * 16;  // pixel (within a store's PXS) and byte of this thread
  auto lds_chunk = [&](int pp) {  // LDS address of this thread's chunk of tile pixel pp (row-major, TW per row)
    const int x = pp % C::TW;
    if constexpr (SW && O32) return C::OUT_OFF + pp * C::PIXB + (((scb >> 4) ^ (x & 7)) << 4);
    return C::OUT_OFF + pp * C::PIXB + (((scb >> 3) ^ (2 * ((x >> 2) & 3))) << 3);
  };
  const int sx = sq % C::TW;  // this thread's tile column in every store
  int srd = lds_chunk(sq);
  asm volatile("" : "+v"(srd));
  auto store_out = [&](const Work& wk_) {
    if (wv == 0) {
      const float* pp = (const float*)(smem + C::PART_OFF);
      float t;
      if constexpr (!SW && CO == 64) {
        // 64 channels x 2 statistics: lane l sums value l of half 0 and of half 1 over the half's strips
        const __amdgpu_buffer_rsrc_t prs2 = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.partial + ((size_t)wk_.n * ntile + wk_.tile) * (2 * CST)), (short)0, 2 * CST * 4, 0x00020000);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float u = pp[(h * C::NSTRIP) * 64 + lane];
#pragma unroll
          for (int s2 = 1; s2 < C::NSTRIP; ++s2) u += pp[(h * C::NSTRIP + s2) * 64 + lane];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(u), prs2,
                                                64 * h + lane < 2 * CST ? (uint32_t)((64 * h + lane) * 4) : 0x80000000u, 0, 0);
        }
      } else if constexpr (!SW) {
        t = pp[lane];
#pragma unroll
        for (int w = 1; w < C::NW; ++w) t += pp[w * 64 + lane];
      } else {
        const int ch = lane >> 1, h = ch >> 4, e = (ch & 15) * 2 + (lane & 1);
        t = pp[(h * C::NSTRIP) * 64 + e];
#pragma unroll
        for (int s2 = 1; s2 < C::NSTRIP; ++s2) t += pp[(h * C::NSTRIP + s2) * 64 + e];
      }
      if constexpr (SW || CO == 32) {
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.partial + ((size_t)wk_.n * ntile + wk_.tile) * 64), (short)0, 256, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t), prs, (uint32_t)(lane * 4), 0, 0);
      }
    }
    constexpr int OPB = C::PIXB / CO * CST;  // stored bytes per output pixel
    const size_t obytes = (size_t)p.oh * p.ow * OPB;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((char*)p.out + (size_t)wk_.n * obytes), (short)0, (int)obytes, 0x00020000);
    const uint32_t voff = (wk_.ox0 + sx < p.ow && scb < OPB) ? (uint32_t)((wk_.ox0 + sx) * OPB + scb) : 0x80000000u;
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {  // store k: tile rows (k PXS + sq) / TW
      const int row = (k * C::PXS + sq) / C::TW;
      const u32x4_t v = *(const u32x4_t*)(smem + srd + k * C::PXS * C::PIXB);
      if (wk_.oy0 + row < p.oh)
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, voff, (wk_.oy0 + row) * p.ow * OPB, ST_AUX);
    }
  };

  // ---- persistent walk: [wait own DMA | B1] request next | MFMAs | epilogue | B2 | stores ----
  // vmcnt: after the next item's requests a wave issues only the stores of store_out (NST, plus
  // the partial row on wave 0, issued first), so vmcnt(NST) at the top of the next iteration
  // covers its requests; each wave waits for its own requests, the barrier for everyone's.
  Work cur = decode(w0);
  int buf = 0;
  request(cur, 0);
  for (int wn = w0 + G;; wn += G) {
    vm_wait<C::NST>();
    __syncthreads();
    const bool more = wn < p.n_work;
    Work nxt = cur;
    if (more) {
      nxt = decode(wn);
      request(nxt, buf ^ 1);
    }
    Acc acc;
    kloop(acc, buf);
    epilogue(cur, acc);
    __syncthreads();
    store_out(cur);
    if (!more) break;
    cur = nxt;
    buf ^= 1;
  }
  vm_wait<0>();
}

template <typename T, int NW, bool SW = false, bool O32 = false, int CO = 32, int CST = CO>
struct Ws9Inst {
  using C = W9Cfg<NW, SW, O32, CO>;
  static int cus() {
    static const int v = [] {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        c = 256;
      return c;
    }();
    return v;
  }
  // grid.x = output tiles per frame, grid.y = frames
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    ConvParams p = p0;
    p.n_work = (int)grid.x * (int)grid.y;
    const int nb = std::min(p.n_work, cus() * (8 / NW));  // 8 waves per CU (VGPRs)
    hipLaunchKernelGGL((ws9_kernel<T, NW, SW, O32, CO, CST>), dim3(nb), dim3(C::NT), 0, st, p);
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = SW ? (O32 ? NST_KDT_SW_O32 : NST_KDT_SW_O16) : dtype_code<T>();
    k.mode = MODE_WS9;
    k.ks = 9; k.stride = 1; k.cinp = 4; k.bn = CST; k.th = C::TH; k.tw = C::TW; k.wm = 1; k.wn = C::NW;
    k.bn_k = CST != CO ? CO : 0;
    k.in_esz = 2;
    k.out_esz = O32 ? 4 : 2;
    k.split_w = SW ? 1 : 0;
    k.in_kind = IN_ACT; k.out_kind = OUT_ACT;
    k.cpc = 4; k.nch = 1; k.lds_bytes = C::LDS;
    k.wbytes = C::WBYTES;
    k.persistent = 1;
    k.part_rows = 1;
    k.korder = 0;  // column-8 packing: 16x16x16 fragments over kernel-row quads (pack_ws9_weights)
    k.launch = &launch;
    return k;
  }
};

const ConvKernelInfo* conv_table_ws9(int* count) {
  static const ConvKernelInfo table[] = {Ws9Inst<__bf16, WS9_NW>::info(), Ws9Inst<_Float16, WS9_NW>::info(),
                                         Ws9Inst<_Float16, WS9_NW, true, true>::info(),
                                         Ws9Inst<_Float16, WS9_NW, true, false>::info(),
                                         // ReCoNet's 9x9 first layer (48 channels padded to 64)
                                         Ws9Inst<__bf16, WS9_NW, false, false, 64>::info(),
                                         Ws9Inst<_Float16, WS9_NW, false, false, 64>::info(),
                                         // ... storing its 48 channels unpadded
                                         Ws9Inst<__bf16, WS9_NW, false, false, 64, 48>::info(),
                                         Ws9Inst<_Float16, WS9_NW, false, false, 64, 48>::info()};
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}

}  // namespace nst
