// conv_ws2.hip — weight-stationary persistent stride-2 3x3 convs (the encoder's down-convs).
//
// Replaces ConvLayer(k3, stride 2) = ReflectionPad2d(1) + Conv2d (transformer_net.py:57-66, used at
// transformer_net.py:11-14 for conv2 32->64 and conv3 64->128) and the zero-padded ConvBlock form
// of transformer_net_nst.py, with the producer's InstanceNorm + ReLU applied in the fill and this
// layer's InstanceNorm partial sums in the epilogue.
//
// The generic implicit-GEMM kernel re-reads the whole weight tensor from L2 for every 4x16 tile
// (147 KB per tile for conv3, ~2.4 GB of L2 traffic per launch); here each wave keeps its 16
// output channels' 3x3xCIN weights in registers for the launch (72 VGPRs for conv3, 36 for conv2):
//   * workgroup = 8 waves; wave w: channel group w % (COUT/16), output row group w / (COUT/16);
//   * persistent over (frame, TH x 16 output tiles), XCD-aware tile order; conv2 (8-row tiles, 126
//     VGPRs, 72 KB LDS) runs two workgroups per CU, so one's fill / epilogue / stores overlap the
//     other's MFMAs and loads (16-row tiles at one per CU: 0.447 vs 0.393 ms); conv3 one per CU;
//   * the input halo (2TH+1) x 33 in LDS in column-polyphase order ([row][x & 1][x >> 1], entry
//     stride 2 x odd chunks), so lane px of x-tap dx reads entry px + (dx >> 1) of phase dx & 1 —
//     consecutive entries, conflict-free ds_read_b128; input row y is the B operand of output rows
//     (y - dy) / 2 for the y-taps of y's parity;
//   * the next tile's halo is loaded into registers (16 B per lane and slot, coalesced 33-pixel
//     row runs) before the current tile's MFMAs and written to LDS after them (IN + ReLU applied),
//     so its HBM latency hides behind the compute; three barriers per tile.  Its source offsets
//     come from per-tile row / column maps in LDS (built a tile ahead) and its IN constants from
//     an LDS table (loaded with the halo, written after the MFMAs), so no address or padding math
//     and no dependent global load sits in the fill;
//   * output tile staged in LDS (8-byte slots XOR-swizzled by pixel: epilogue writes 2-way, store
//     reads conflict-free; a 32-byte wave-slot swizzle was 4-way on the writes) and stored as whole pixels,
//     16 B per lane; one InstanceNorm partial row per tile and row group.
#include <algorithm>
#include <cstring>

#include "conv_ws_common.h"

namespace nst {

constexpr int W2_RING = 3;  // operand reads in flight ahead of the MFMAs
// !PF fill: halo slots loaded per round (each round's HBM latency is exposed: the K loop is over)
#ifndef NST_W2_FD_B
#define NST_W2_FD_B 16  // all of them (NPF <= 16): conv3 SPL 0.64 -> 0.56 ms over 4 per round (r05_k)
#endif

// SPL (the split-precision modes' down-convs): fp32 input; the fill stages each normalised value v as an fp16
// pair xh = RNE(v), xl = RNE(v - xh) in two planes of the LDS entry ([xh: CINP x 2 B][xl: CINP x 2 B]); the
// weights are fp16 pairs too (Wh, Wl in registers), and each K step is three MFMAs, Wh xh into one accumulator
// and Wh xl + Wl xh into a second (Wl xl, ~2^-22 of the product, is dropped): ~22-bit products, fp32 sums.
// O32: fp32 output.  PF: prefetch the next tile's halo into registers during the MFMAs (off: loaded after
// the epilogue, for the shapes whose split weights leave no registers for it).
// 8 waves; 12 (three per SIMD) for 96 output channels (ReCoNet's unpadded encoder.layers.1): 6 groups x 2 row groups
constexpr int w2_threads(int cout) { return cout == 96 ? 768 : 512; }
template <int CINP, int COUT, int TH, bool SPL = false, bool O32 = false>
struct W2Cfg {
  static constexpr int NCG = COUT / 16;             // 16-channel groups
  static constexpr int NW = w2_threads(COUT) / 64, NT = NW * 64, TW = 16;
  static constexpr int NRG = NW / NCG;              // output row groups
  static constexpr int THW = TH / NRG;              // output rows per wave
  static constexpr int IESZ = SPL ? 4 : 2;          // input element bytes
  static constexpr int NCH = CINP * IESZ / 16;      // 16-B chunks per input pixel (and per LDS entry)
  static constexpr int LO_OFF = CINP * 2;           // SPL: byte offset of the xl plane in an entry
  static constexpr int NPART = CINP / 32;           // 32-channel K steps per tap
  static constexpr int NSTEP = 9 * NPART;           // weight registers (uint4) per wave
  static constexpr int LH = 2 * TH + 1, LW = 2 * TW + 1;
  static constexpr int LWE = TW + 1;                // entries per column phase
  static constexpr int EB = (NCH + 2) * 16;         // entry stride: 2 x odd chunks
  static constexpr int RS = 2 * LWE * EB;           // bytes per halo row
  static constexpr int HALO = LH * RS;
  static constexpr int NCHK = LH * LW * NCH;        // 16-B chunks per halo
  static constexpr int NPF = (NCHK + NT - 1) / NT;  // fill slots per thread
  static constexpr int PIXB = COUT * (O32 ? 4 : 2);
  // 16-bit output staging: 8-byte slot s of pixel px at slot s ^ 2 (px & 7), or (s + 2 (px & 7)) mod NSL when the
  // pixel's slot count is not a power of two (96 channels: 24 slots), so a slot never leaves its pixel
  static constexpr int NSL = PIXB / 8;
  static constexpr bool SWZ_XOR = (NSL & (NSL - 1)) == 0;
  static __device__ __forceinline__ int oslot(int s, int px) {
    return SWZ_XOR ? (s ^ (2 * (px & 7))) : (s + 2 * (px & 7)) % NSL;
  }
  static constexpr int OUT_OFF = HALO;
  static constexpr int OUTB = TH * TW * PIXB;
  static constexpr int NST = OUTB / (NT * 16);      // 16-B output stores per thread
  static constexpr int BIAS_OFF = OUT_OFF + OUTB;
  static constexpr int NORM_OFF = BIAS_OFF + COUT * 4;     // the landing tile's IN {scale, shift} per channel
  static constexpr int MAPB = ((LH + LW) * 4 + 15) / 16 * 16;
  static constexpr int MAP_OFF = NORM_OFF + CINP * 8;       // 2 slots: halo row / column source offsets
  static constexpr int LDS = MAP_OFF + 2 * MAPB;
  static constexpr int WBYTES = NCG * NSTEP * 64 * 16 * (SPL ? 2 : 1);
  static_assert(CINP % 32 == 0 && COUT % 16 == 0, "channel shapes");
  static_assert(NT % NCH == 0, "a thread's chunk is the same in every fill slot");
  static_assert(NW % NCG == 0 && TH % NRG == 0, "waves split channel groups x row groups");
  static_assert(NST * NT * 16 == OUTB, "whole 16-B stores per thread");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(!O32 || (PIXB & (PIXB - 1)) == 0, "fp32 staging: XOR swizzle over a power-of-two pixel");
};

// OCC = waves per SIMD the register allocation must allow (12-wave form: 3 = one workgroup per CU): 4 = two
// workgroups per CU (conv2's
// 8-row tiles fit 126 VGPRs and 72 KB of LDS), 2 = one
// CLD: input channels stored (<= CINP; ReCoNet's unpadded 48-channel first-layer output): the chunks past them stage
// zeros (IN constants 0 -> ReLU(0))
template <typename T, int CINP, int COUT, int TH, bool ZPAD, int OCC, bool SPL, bool O32, bool PF, int CLD = CINP>
__global__ __launch_bounds__(w2_threads(COUT), OCC) void ws2_kernel(ConvParams p) {
  using C = W2Cfg<CINP, COUT, TH, SPL, O32>;
  static_assert(!SPL || IS_F16<T>, "split operands / weights are fp16 pairs");
  static_assert(PF || SPL, "the 16-bit kernels always prefetch");
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wv % C::NCG, rg = wv / C::NCG;
  const int g = lane >> 4, px = lane & 15;

  struct Work {
    int n, tile, oy0, ox0;
  };
  const int ntile = p.tiles_x * p.tiles_y;
  auto decode = [&](int wi) {
    Work r;
    r.n = wi / ntile;
    r.tile = wi - r.n * ntile;
    const int ty = r.tile / p.tiles_x;
    r.oy0 = ty * TH;
    r.ox0 = (r.tile - ty * p.tiles_x) * C::TW;
    return r;
  };
  // workgroups b, b+8, ... share an XCD: each XCD takes a contiguous run of tiles per sweep
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int w0 = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  if (w0 >= p.n_work) return;

  // ---- this wave's 16 output channels x 9 x CINP weights (SPL: Wh and Wl), resident for the launch ----
  uint4 wr[C::NSTEP];
  uint4 wl[SPL ? C::NSTEP : 1];
  {
    const uint4* wsrc = (const uint4*)p.wpk + (size_t)cg * (SPL ? 2 : 1) * C::NSTEP * 64 + lane;
#pragma unroll
    for (int s = 0; s < C::NSTEP; ++s) wr[s] = wsrc[s * 64];
    if constexpr (SPL) {
#pragma unroll
      for (int s = 0; s < C::NSTEP; ++s) wl[s] = wsrc[(C::NSTEP + s) * 64];
    }
  }
  if (tid < COUT) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];

  // ---- halo fill: slot k of this thread = chunk j = k NT + tid (entry j / NCH, chunk fc) ----
  const size_t frame_bytes = (size_t)p.hs * p.ws * p.cs * C::IESZ;
  const int fc = tid % C::NCH;
  auto build_maps = [&](const Work& wk, int slot) {  // source byte offsets of the halo rows / columns, -1 = pad
    int* map = (int*)(smem + C::MAP_OFF + slot * C::MAPB);
    for (int t = tid; t < C::LH + C::LW; t += C::NT) {
      if (t < C::LH) {
        const int sy = map_axis(2 * wk.oy0 - p.pad + t, p.hs, p.axis_mode, p.pre);
        map[t] = sy < 0 ? -1 : sy * p.ws * p.cs * C::IESZ;
      } else {
        const int sx = map_axis(2 * wk.ox0 - p.pad + t - C::LH, p.ws, p.axis_mode, p.pre);
        map[t] = sx < 0 ? -1 : sx * p.cs * C::IESZ;
      }
    }
  };
  auto entry_of = [&](int k, int& ly, int& lx) {
    const int e = (k * C::NT + tid) / C::NCH;
    ly = e / C::LW;
    lx = e - ly * C::LW;
  };
  float2 nv = make_float2(0.f, 0.f);  // this thread's channel of the landing tile's IN constants (tid < CINP)
  float2 nsp[SPL ? 4 : 1];             // SPL: the IN constants of this thread's 4 channels (chunk fc)
  uint32_t padm = 0;                   // bit k: slot k is zero padding
  auto issue = [&](const Work& wk, int slot, uint4 (&pf)[C::NPF]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.in + (size_t)wk.n * frame_bytes), (short)0, (int)frame_bytes, 0x00020000);
    const int* map = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    padm = 0;
#pragma unroll
    for (int k = 0; k < C::NPF; ++k) {
      int ly, lx;
      entry_of(k, ly, lx);
      const bool ok = (k + 1) * C::NT <= C::NCHK || k * C::NT + tid < C::NCHK;
      const int ro = map[ok ? ly : 0], co = map[C::LH + (ok ? lx : 0)];
      const bool pad = ro < 0 || co < 0;
      padm |= pad ? 1u << k : 0u;
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(
          rs, (ok && !pad && fc * (16 / C::IESZ) < CLD) ? (uint32_t)(ro + co + fc * 16) : 0x80000000u, 0, 0);
      pf[k] = __builtin_bit_cast(uint4, v);
    }
    if constexpr (SPL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) nsp[j] = p.in_norm[(size_t)wk.n * p.cs + 4 * fc + j];
    } else if (tid < CINP) {
      nv = tid < CLD ? p.in_norm[(size_t)wk.n * p.cs + tid] : make_float2(0.f, 0.f);
    }
  };
  auto put_norm = [&]() {  // after the MFMAs: the landing tile's IN constants into LDS
    if (tid < CINP) *(float2*)(smem + C::NORM_OFF + tid * 8) = nv;
  };
  // SPL: one staged fp32 chunk (4 channels) -> IN + ReLU in fp32 -> fp16 hi / lo halves of the entry
  auto land_split = [&](const uint4& raw, bool pad, int ly, int lx) {
    float v[4] = {__uint_as_float(raw.x), __uint_as_float(raw.y), __uint_as_float(raw.z), __uint_as_float(raw.w)};
    _Float16 hi[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x = fmaxf(__builtin_fmaf(v[j], nsp[j].x, nsp[j].y), 0.f);  // fma: as the 16-bit fill's IN apply
      if (ZPAD && pad) x = 0.f;
      asm("" : "+v"(x));  // split the fp32 value itself
      hi[j] = (_Float16)x;
      lo[j] = (_Float16)(x - (float)hi[j]);  // exact in fp32
    }
    auto pk = [](_Float16 a, _Float16 b) {
      return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
    };
    char* e = smem + ly * C::RS + (lx & 1) * C::LWE * C::EB + (lx >> 1) * C::EB + fc * 8;
    *(u32x2_t*)e = (u32x2_t){pk(hi[0], hi[1]), pk(hi[2], hi[3])};
    *(u32x2_t*)(e + C::LO_OFF) = (u32x2_t){pk(lo[0], lo[1]), pk(lo[2], lo[3])};
  };
  auto land = [&](const uint4 (&pf)[C::NPF]) {
    if constexpr (SPL) {
#pragma unroll
      for (int k = 0; k < C::NPF; ++k) {
        if ((k + 1) * C::NT > C::NCHK && k * C::NT + tid >= C::NCHK) continue;
        int ly, lx;
        entry_of(k, ly, lx);
        land_split(pf[k], ((padm >> k) & 1u) != 0, ly, lx);
      }
      return;
    }
    float2 nm[8];  // the producer's IN {scale, shift} of this thread's 8 channels
    const float4* nl = (const float4*)(smem + C::NORM_OFF + fc * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 v = nl[i];
      nm[2 * i] = make_float2(v.x, v.y);
      nm[2 * i + 1] = make_float2(v.z, v.w);
    }
#pragma unroll
    for (int k = 0; k < C::NPF; ++k) {
      if ((k + 1) * C::NT > C::NCHK && k * C::NT + tid >= C::NCHK) continue;
      int ly, lx;
      entry_of(k, ly, lx);
      uint4 v = norm_chunk<T>(pf[k], nm);  // IN + ReLU (as the generic kernel's fill)
      if (ZPAD && ((padm >> k) & 1u)) v = make_uint4(0u, 0u, 0u, 0u);  // zero padding stays zero after IN + ReLU
      *(uint4*)(smem + ly * C::RS + (lx & 1) * C::LWE * C::EB + (lx >> 1) * C::EB + fc * 16) = v;
    }
  };

  // !PF: the next tile's halo straight through a few registers after the epilogue (no overlap with the MFMAs)
  auto fill_direct = [&](const Work& wk, int slot) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.in + (size_t)wk.n * frame_bytes), (short)0, (int)frame_bytes, 0x00020000);
    const int* map = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    if constexpr (SPL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) nsp[j] = p.in_norm[(size_t)wk.n * p.cs + 4 * fc + j];
    }
    constexpr int B = NST_W2_FD_B < C::NPF ? NST_W2_FD_B : C::NPF;  // slots in flight
#pragma unroll
    for (int k0 = 0; k0 < C::NPF; k0 += B) {
      uint4 v[B];
      bool pd[B];
#pragma unroll
      for (int k = k0; k < k0 + B && k < C::NPF; ++k) {
        int ly, lx;
        entry_of(k, ly, lx);
        const bool ok = (k + 1) * C::NT <= C::NCHK || k * C::NT + tid < C::NCHK;
        const int ro = map[ok ? ly : 0], co = map[C::LH + (ok ? lx : 0)];
        pd[k - k0] = ro < 0 || co < 0;
        v[k - k0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
            rs, (ok && !pd[k - k0]) ? (uint32_t)(ro + co + fc * 16) : 0x80000000u, 0, 0));
      }
#pragma unroll
      for (int k = k0; k < k0 + B && k < C::NPF; ++k) {
        if ((k + 1) * C::NT > C::NCHK && k * C::NT + tid >= C::NCHK) continue;
        int ly, lx;
        entry_of(k, ly, lx);
        land_split(v[k - k0], pd[k - k0], ly, lx);
      }
    }
  };

  // ---- K loop: part q, x-tap dx, halo row y (the wave's 2 THW + 1 rows) ----
  typedef f32x4_t Acc[C::THW];
  const int r0 = rg * C::THW;
  constexpr int NRD = 2 * C::THW + 1;  // reads per (part, dx)
  constexpr int PRD = 3 * NRD;         // reads per part
  auto bread = [&](int i) -> uint4 {
    const int q = i / PRD, rem = i - q * PRD;
    const int dx = rem / NRD, y = rem % NRD;
    int base = (2 * r0) * C::RS + px * C::EB + g * 16;
    asm volatile("" : "+v"(base));
    return *(const uint4*)(smem + base + y * C::RS + (dx & 1) * C::LWE * C::EB + (dx >> 1) * C::EB + 64 * q);
  };
  auto mfma = [&](f32x4_t& c, const uint4& a, const uint4& bop, bool first) { mfma_tied<T>(c, a, bop, first); };
  auto bread_lo = [&](int i) -> uint4 {  // SPL: the xl plane of read i
    const int q = i / PRD, rem = i - q * PRD;
    const int dx = rem / NRD, y = rem % NRD;
    int base = (2 * r0) * C::RS + px * C::EB + g * 16 + C::LO_OFF;
    asm volatile("" : "+v"(base));
    return *(const uint4*)(smem + base + y * C::RS + (dx & 1) * C::LWE * C::EB + (dx >> 1) * C::EB + 64 * q);
  };
  auto kloop = [&](Acc& acc, Acc& acc2) {
    constexpr int NI = C::NPART * PRD, D = W2_RING;
    uint4 ring[D], ringl[SPL ? D : 1];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      ring[i] = bread(i);
      if constexpr (SPL) ringl[i] = bread_lo(i);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = i / PRD, rem = i - q * PRD;
      const int dx = rem / NRD, y = rem % NRD;
      const uint4 bcur = ring[i % D];
      const uint4 bl = SPL ? ringl[i % D] : bcur;
      if (i + D < NI) {
        ring[i % D] = bread(i + D);
        if constexpr (SPL) ringl[i % D] = bread_lo(i + D);
      }
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        if ((y - dy) & 1) continue;
        const int r = (y - dy) / 2;
        if (y - dy < 0 || r >= C::THW) continue;
        // row r's first MFMA: q = 0, dx = 0, y = 2r (dy = 0)
        const int s = q * 9 + 3 * dy + dx;
        const bool first = q == 0 && dx == 0 && dy == 0;
        mfma(acc[r], wr[s], bcur, first);
        if constexpr (SPL) {
          mfma(acc2[r], wr[s], bl, first);
          mfma(acc2[r], wl[s], bcur, false);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: bias, 16-bit values into the LDS output tile, IN partials from the fp32 values ----
  auto epilogue = [&](const Work& wk, Acc& acc, Acc& acc2) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // MFMA results -> VALU reads
    const int c0 = 16 * cg + 4 * g;
    const f32x4_t bias = *(const f32x4_t*)(smem + C::BIAS_OFF + c0 * 4);
    // 16-bit: 8-B slots swizzled by pixel; O32: 16-B chunk 4 cg + g of the pixel, XOR (px & 15): conflict-free
    int obase = C::OUT_OFF + px * C::PIXB + (O32 ? (((4 * cg + g) ^ (px & 15)) * 16) : (C::oslot(4 * cg + g, px) * 8));
    asm volatile("" : "+v"(obase));
    f32x4_t s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
    const bool full = wk.oy0 + TH <= p.oh && wk.ox0 + C::TW <= p.ow;
#pragma unroll
    for (int r = 0; r < C::THW; ++r) {
      const int row = r0 + r;
      const bool valid = full || (wk.oy0 + row < p.oh && wk.ox0 + px < p.ow);
      const f32x4_t v = SPL ? add4(add4(acc[r], acc2[r]), bias) : add4(acc[r], bias);
      if constexpr (O32) {
        *(f32x4_t*)(smem + obase + row * C::TW * C::PIXB) = v;
      } else {
        const u32x2_t pk = {pack16<T>(v[0], v[1]), pack16<T>(v[2], v[3])};
        *(u32x2_t*)(smem + obase + row * C::TW * C::PIXB) = pk;
      }
      const f32x4_t x = valid ? v : (f32x4_t){0.f, 0.f, 0.f, 0.f};
      stat4(s1, s2, x);
    }
    const float vv[8] = {s1[0], s2[0], s1[1], s2[1], s1[2], s2[2], s1[3], s2[3]};
    float a4[4], a2[2], a1[1];
    rs_step<4, 0x140>(vv, a4, px >= 8);
    rs_step<2, 0x141>(a4, a2, (px & 4) != 0);
    rs_step<1, 0x1b>(a2, a1, (px & 2) != 0);
    const float t = a1[0] + dpp_f<0xb1>(a1[0]);
    const int idx = (px >= 8 ? 4 : 0) + ((px & 4) ? 2 : 0) + ((px & 2) ? 1 : 0);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.partial + (((size_t)wk.n * ntile + wk.tile) * C::NRG + rg) * p.cout_stride * 2), (short)0,
        p.cout_stride * 8, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t), prs,
                                          (px & 1) ? 0x80000000u : (uint32_t)(((c0 + (idx >> 1)) * 2 + (idx & 1)) * 4), 0, 0);
  };
  // the staged tile as whole pixels: 16 B per lane, TW * PIXB contiguous bytes per tile row
  auto store_out = [&](const Work& wk) {
    const size_t obytes = (size_t)p.oh * p.ow * C::PIXB;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((char*)p.out + (size_t)wk.n * obytes), (short)0, (int)obytes, 0x00020000);
    int t0 = tid;
    asm volatile("" : "+v"(t0));
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int off = (k * C::NT + t0) * 16;
      const int pp = off / C::PIXB, cb = off - pp * C::PIXB;
      const int x = pp % C::TW, oy = wk.oy0 + pp / C::TW, ox = wk.ox0 + x;
      const int la = O32 ? (((cb >> 4) ^ (x & 15)) << 4) : (C::oslot(cb >> 3, x) << 3);
      const u32x4_t v = *(const u32x4_t*)(smem + C::OUT_OFF + pp * C::PIXB + la);
      const bool ok = oy < p.oh && ox < p.ow;
      __builtin_amdgcn_raw_buffer_store_b128(v, ors, ok ? (uint32_t)((oy * p.ow + ox) * C::PIXB + cb) : 0x80000000u, 0, ST_AUX);
    }
  };

  // ---- persistent walk: B1 halo ready | MFMAs | B2 halo free | epilogue + next halo | B3 | stores ----
  // map slot of the tile being issued: it & 1 (the maps of the tile after it are built before B3)
  Work cur = decode(w0);
  uint4 pf[PF ? C::NPF : 1];
  build_maps(cur, 0);
  build_maps(decode(min(w0 + G, p.n_work - 1)), 1);
  __syncthreads();
  if constexpr (PF) {
    issue(cur, 0, pf);
    if (!SPL) put_norm();
    __syncthreads();
    land(pf);
  } else {
    fill_direct(cur, 0);
  }
  for (int wn = w0 + G, it = 1;; wn += G, ++it) {
    __syncthreads();
    const bool more = wn < p.n_work;
    const Work nxt = decode(more ? wn : w0);
    if constexpr (PF) {
      if (more) issue(nxt, it & 1, pf);
    }
    Acc acc, acc2;
    kloop(acc, acc2);
    if (!SPL) put_norm();
    __syncthreads();
    epilogue(cur, acc, acc2);
    if (more) {
      if constexpr (PF) land(pf);
      else fill_direct(nxt, it & 1);
    }
    build_maps(decode(min(wn + G, p.n_work - 1)), (it + 1) & 1);
    __syncthreads();
    store_out(cur);
    if (!more) break;
    cur = nxt;
  }
}

template <typename T, int CINP, int COUT, int TH, int OCC, bool SPL = false, bool O32 = false, bool PF = true,
          int CLD = CINP>
struct Ws2Inst {
  using C = W2Cfg<CINP, COUT, TH, SPL, O32>;
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
    const int nb = std::min(p.n_work, cus() * (OCC * 4 / C::NW));  // workgroups resident per CU
    // the narrow-input form serves ReCoNet's reflection-padded layer only (its zero-padded instantiation spills at
    // three waves per SIMD): nst_api selects it for that net alone
    if constexpr (CLD == CINP) {
      if (p.axis_mode == AX_ZERO || p.axis_mode == AX_ZERO_PREREFLECT) {
        hipLaunchKernelGGL((ws2_kernel<T, CINP, COUT, TH, true, OCC, SPL, O32, PF, CLD>), dim3(nb), dim3(C::NT), 0, st, p);
        return;
      }
    }
    hipLaunchKernelGGL((ws2_kernel<T, CINP, COUT, TH, false, OCC, SPL, O32, PF, CLD>), dim3(nb), dim3(C::NT), 0, st, p);
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = SPL ? (O32 ? NST_KDT_SPLIT_O32 : NST_KDT_SPLIT_O16) : dtype_code<T>();
    k.in_esz = C::IESZ;
    k.out_esz = O32 ? 4 : 2;
    k.split_w = SPL ? 1 : 0;
    k.mode = MODE_WS2;
    k.ks = 3; k.stride = 2; k.cinp = CLD; k.bn = COUT;
    k.cinp_k = CLD != CINP ? CINP : 0; k.th = TH; k.tw = C::TW; k.wm = C::NRG; k.wn = C::NCG;
    k.in_kind = IN_ACT; k.out_kind = OUT_ACT;
    k.cpc = SPL ? 4 : 8; k.nch = C::NCH; k.lds_bytes = C::LDS;
    k.wbytes = C::WBYTES;
    k.persistent = 1;
    k.part_rows = C::NRG;
    k.launch = &launch;
    return k;
  }
};

constexpr int W2_C2_TH = 8;  // 8 rows: two workgroups per CU (16 rows, one per CU: 0.447 vs 0.393 ms)
constexpr int W2_C3_TH = 8;
#define E(...) Ws2Inst<__VA_ARGS__>::info()
const ConvKernelInfo* conv_table_ws2(int* count) {
  static const ConvKernelInfo table[] = {
      //  T     CINP COUT TH OCC
      E(__bf16, 32, 64, W2_C2_TH, W2_C2_TH <= 8 ? 4 : 2),    // conv2 / down2
      E(__bf16, 64, 128, W2_C3_TH, W2_C3_TH <= 4 ? 4 : 2),   // conv3 / down3 / ReCoNet 48 -> 96 (padded 64 -> 128)
      E(_Float16, 32, 64, W2_C2_TH, W2_C2_TH <= 8 ? 4 : 2),  // fp16 mode
      E(_Float16, 64, 128, W2_C3_TH, W2_C3_TH <= 4 ? 4 : 2),
      // ReCoNet encoder.layers.1 48 -> 96 with its 96 output channels unpadded (48 in, padded to 64): 12 waves
      E(__bf16, 64, 96, 8, 3),
      E(_Float16, 64, 96, 8, 3),
      // ... reading the first layer's 48 channels unpadded
      E(__bf16, 64, 96, 8, 3, false, false, true, 48),
      E(_Float16, 64, 96, 8, 3, false, false, true, 48),
      // split-precision head (NST_DT_F16M): conv2 with fp32 output, conv3 with fp32 or fp16 output
      //  T        CINP COUT TH OCC SPL   O32    PF
      E(_Float16, 32, 64, 8, 2, true, true, true),
      E(_Float16, 64, 128, 4, 2, true, true, false),
      E(_Float16, 64, 128, 4, 2, true, false, false),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E

}  // namespace nst
