// conv_ws1s.hip — weight-stationary stride-1 3x3 conv with split-fp16 operands (NST_DT_F16M's first residual
// blocks, 128 -> 128 channels).
//
// Replaces ConvLayer(128, 128, 3, 1) of the first two residual blocks (transformer_net.py:57-76 res1, res2;
// transformer_net_nst.py:28-43) in the split-precision head: fp32 activations in HBM, each staged operand value v
// kept as the fp16 pair xh = RNE(v), xl = RNE(v - xh) (two planes of the LDS entry), the weights fp16 in registers
// (128 x 1152 = 144 VGPRs per wave, as conv_wstat.hip), and two MFMAs per K step, Wh xh and Wh xl, accumulated
// in one chain: the operand keeps ~22 bits (its rounding is what reaches the frame most, tests/precision_study.py:
// "o" and "s" of these layers; their fp16 weights add little).  Fill: the producer's InstanceNorm + ReLU in fp32
// (or the residual stream as stored: RAW), the layer's InstanceNorm partial sums in the epilogue, fp32 output.
//
//   * workgroup = 8 waves, wave w = output channels 16w..16w+15, persistent over (frame, 4 x 16 tile) items,
//     XCD-aware order, one workgroup per CU (weights + two accumulator sets + the fill's registers);
//   * halo 6 x 18 entries of [xh: 128 x 2 B][xl: 128 x 2 B] + 2 pad chunks (34 chunks = 2 x odd: the 16 lanes of a
//     ds_read_b128 lane group hit distinct bank slots); halo row y of x-tap dx is the B operand of tile row
//     y - dy for every y-tap dy, so each pair of reads feeds up to six MFMAs;
//   * the next tile's halo is loaded into registers (16 B = 4 fp32 channels per slot) before the MFMAs and
//     written (normalised, split) after them, as conv_ws2.hip's fill; output tile staged in LDS (16-B chunks
//     XOR-swizzled by pixel) and stored as whole 512-B pixels.
#include <algorithm>
#include <cstring>

#include "conv_ws_common.h"

namespace nst {

template <int TH>
struct W1sCfg {
  static constexpr int NW = 8, NT = 512, TW = 16, CINP = 128, COUT = 128;
  static constexpr int LH = TH + 2, LW = TW + 2, NENT = LH * LW;
  static constexpr int NCH = CINP * 4 / 16;         // 16-B fp32 chunks per input pixel (4 channels each)
  static constexpr int LO_OFF = CINP * 2;           // byte offset of the xl plane in an entry
  static constexpr int EB = (2 * CINP * 2 / 16 + 2) * 16;  // 544 B per LDS entry
  static constexpr int HALO = NENT * EB;
  static constexpr int NCHK = NENT * NCH;
  static constexpr int NPF = (NCHK + NT - 1) / NT;  // fill slots per thread
  static constexpr int NSTEP = 36;                  // 4 parts x 9 taps (K = 32 per step)
  static constexpr int PIXB = COUT * 4;             // fp32 output pixel
  static constexpr int OUT_OFF = HALO;
  static constexpr int OUTB = TH * TW * PIXB;
  static constexpr int NST = OUTB / (NT * 16);      // 16-B output stores per thread
  static constexpr int BIAS_OFF = OUT_OFF + OUTB;
  static constexpr int MAPB = ((LH + LW) * 4 + 15) / 16 * 16;
  static constexpr int MAP_OFF = BIAS_OFF + COUT * 4;  // 2 slots: halo row / column source offsets
  static constexpr int LDS = MAP_OFF + 2 * MAPB;
  static constexpr int WBYTES = NW * NSTEP * 64 * 16;
  static_assert(NT % NCH == 0, "a thread's chunk is the same in every fill slot");
  static_assert(NST * NT * 16 == OUTB, "whole 16-B stores per thread");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// NRM: the fill applies the producer's InstanceNorm + ReLU; else it stages the (residual-stream) input as is
template <int TH, bool ZPAD, bool NRM>
__global__ __launch_bounds__(512, 1) void ws1s_kernel(ConvParams p) {
  using C = W1sCfg<TH>;
  using T = _Float16;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  // ---- this wave's 16 output channels x 1152 K of fp16 weights, resident for the launch ----
  uint4 wr[C::NSTEP];
  {
    const uint4* wsrc = (const uint4*)p.wpk + (size_t)wv * C::NSTEP * 64 + lane;
#pragma unroll
    for (int s = 0; s < C::NSTEP; ++s) wr[s] = wsrc[s * 64];
  }
  if (tid < C::COUT) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];

  // ---- halo fill: slot k of this thread = chunk j = k NT + tid (entry j / NCH, chunk fc = 4 channels) ----
  const size_t frame_bytes = (size_t)p.hs * p.ws * p.cs * 4;
  const int fc = tid % C::NCH;
  auto build_maps = [&](const Work& wk, int slot) {  // source byte offsets of the halo rows / columns, -1 = pad
    int* map = (int*)(smem + C::MAP_OFF + slot * C::MAPB);
    for (int t = tid; t < C::LH + C::LW; t += C::NT) {
      if (t < C::LH) {
        const int sy = map_axis(wk.oy0 - p.pad + t, p.hs, p.axis_mode, p.pre);
        map[t] = sy < 0 ? -1 : sy * p.ws * p.cs * 4;
      } else {
        const int sx = map_axis(wk.ox0 - p.pad + t - C::LH, p.ws, p.axis_mode, p.pre);
        map[t] = sx < 0 ? -1 : sx * p.cs * 4;
      }
    }
  };
  float2 nsp[4];   // the landing tile's IN constants of this thread's 4 channels (NRM)
  uint32_t padm = 0;
  auto issue = [&](const Work& wk, int slot, uint4 (&pf)[C::NPF]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.in + (size_t)wk.n * frame_bytes), (short)0, (int)frame_bytes, 0x00020000);
    const int* map = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    padm = 0;
#pragma unroll
    for (int k = 0; k < C::NPF; ++k) {
      const int e = (k * C::NT + tid) / C::NCH;
      const bool ok = (k + 1) * C::NT <= C::NCHK || k * C::NT + tid < C::NCHK;
      const int ly = ok ? e / C::LW : 0, lx = ok ? e - (e / C::LW) * C::LW : 0;
      const int ro = map[ly], co = map[C::LH + lx];
      const bool pad = ro < 0 || co < 0;
      padm |= pad ? 1u << k : 0u;
      pf[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
          rs, (ok && !pad) ? (uint32_t)(ro + co + fc * 16) : 0x80000000u, 0, 0));
    }
    if constexpr (NRM) {
#pragma unroll
      for (int j = 0; j < 4; ++j) nsp[j] = p.in_norm[(size_t)wk.n * p.cs + 4 * fc + j];
    }
  };
  auto land = [&](const uint4 (&pf)[C::NPF]) {
#pragma unroll
    for (int k = 0; k < C::NPF; ++k) {
      if ((k + 1) * C::NT > C::NCHK && k * C::NT + tid >= C::NCHK) continue;
      const int e = (k * C::NT + tid) / C::NCH;
      const float v[4] = {__uint_as_float(pf[k].x), __uint_as_float(pf[k].y), __uint_as_float(pf[k].z),
                          __uint_as_float(pf[k].w)};
      _Float16 hi[4], lo[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = NRM ? fmaxf(__builtin_fmaf(v[j], nsp[j].x, nsp[j].y), 0.f) : v[j];
        if (ZPAD && ((padm >> k) & 1u)) x = 0.f;  // zero padding stays zero after IN + ReLU
        asm("" : "+v"(x));  // split the fp32 value itself
        hi[j] = (_Float16)x;
        lo[j] = (_Float16)(x - (float)hi[j]);  // exact in fp32
      }
      auto pk = [](_Float16 a, _Float16 bb) {
        return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, bb) << 16);
      };
      char* ep = smem + e * C::EB + fc * 8;
      *(u32x2_t*)ep = (u32x2_t){pk(hi[0], hi[1]), pk(hi[2], hi[3])};
      *(u32x2_t*)(ep + C::LO_OFF) = (u32x2_t){pk(lo[0], lo[1]), pk(lo[2], lo[3])};
    }
  };

  // ---- K loop: part q, x-tap dx, halo row y; reads of the xh and xl planes ----
  typedef f32x4_t Acc[TH];
  constexpr int NRD = TH + 2, PRD = 3 * NRD;
  auto bread = [&](int i, int plane) -> uint4 {
    const int q = i / PRD, rem = i - q * PRD;
    const int dx = rem / NRD, y = rem % NRD;
    int base = px * C::EB + g * 16 + plane;
    asm volatile("" : "+v"(base));
    return *(const uint4*)(smem + base + (y * C::LW + dx) * C::EB + 64 * q);
  };
  auto kloop = [&](Acc& acc) {
    constexpr int NI = 4 * PRD, D = 2;
    uint4 rh[D], rl[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      rh[i] = bread(i, 0);
      rl[i] = bread(i, C::LO_OFF);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = i / PRD, rem = i - q * PRD;
      const int dx = rem / NRD, y = rem % NRD;
      const uint4 bh = rh[i % D], bl = rl[i % D];
      if (i + D < NI) {
        rh[i % D] = bread(i + D, 0);
        rl[i % D] = bread(i + D, C::LO_OFF);
      }
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int r = y - dy;
        if (r < 0 || r >= TH) continue;
        const int s = q * 9 + 3 * dy + dx;
        mfma_tied<T>(acc[r], wr[s], bh, q == 0 && dx == 0 && dy == 0);  // row r's first: y = r, dx = dy = 0
      }
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {  // the xl terms into the same accumulators (an accumulation chain)
        const int r = y - dy;
        if (r < 0 || r >= TH) continue;
        mfma_tied<T>(acc[r], wr[q * 9 + 3 * dy + dx], bl, false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: Wh xh + Wh xl + bias (fp32) into the staged tile, InstanceNorm partial sums ----
  auto epilogue = [&](const Work& wk, Acc& acc) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // MFMA results -> VALU reads
    const int c0 = 16 * wv + 4 * g;
    const f32x4_t bias = *(const f32x4_t*)(smem + C::BIAS_OFF + c0 * 4);
    // 16-B chunk 4 wv + g of the 32-chunk pixel, XOR (px & 15): conflict-free
    int obase = C::OUT_OFF + px * C::PIXB + (((4 * wv + g) ^ (px & 15)) * 16);
    asm volatile("" : "+v"(obase));
    f32x4_t s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
    const bool full = wk.oy0 + TH <= p.oh && wk.ox0 + C::TW <= p.ow;
#pragma unroll
    for (int r = 0; r < TH; ++r) {
      const bool valid = full || (wk.oy0 + r < p.oh && wk.ox0 + px < p.ow);
      const f32x4_t v = add4(acc[r], bias);
      *(f32x4_t*)(smem + obase + r * C::TW * C::PIXB) = v;
      stat4(s1, s2, valid ? v : (f32x4_t){0.f, 0.f, 0.f, 0.f});
    }
    const float vv[8] = {s1[0], s2[0], s1[1], s2[1], s1[2], s2[2], s1[3], s2[3]};
    float a4[4], a2[2], a1[1];
    rs_step<4, 0x140>(vv, a4, px >= 8);
    rs_step<2, 0x141>(a4, a2, (px & 4) != 0);
    rs_step<1, 0x1b>(a2, a1, (px & 2) != 0);
    const float t = a1[0] + dpp_f<0xb1>(a1[0]);
    const int idx = (px >= 8 ? 4 : 0) + ((px & 4) ? 2 : 0) + ((px & 2) ? 1 : 0);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.partial + ((size_t)wk.n * ntile + wk.tile) * p.cout_stride * 2), (short)0, p.cout_stride * 8,
        0x00020000);
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
      const u32x4_t v = *(const u32x4_t*)(smem + C::OUT_OFF + pp * C::PIXB + (((cb >> 4) ^ (x & 15)) << 4));
      const bool ok = oy < p.oh && ox < p.ow;
      __builtin_amdgcn_raw_buffer_store_b128(v, ors, ok ? (uint32_t)((oy * p.ow + ox) * C::PIXB + cb) : 0x80000000u, 0,
                                             ST_AUX);
    }
  };

  // ---- persistent walk: B1 halo ready | MFMAs | B2 halo free | epilogue + next halo | B3 | stores ----
  Work cur = decode(w0);
  uint4 pf[C::NPF];
  build_maps(cur, 0);
  build_maps(decode(min(w0 + G, p.n_work - 1)), 1);
  __syncthreads();
  issue(cur, 0, pf);
  land(pf);
  for (int wn = w0 + G, it = 1;; wn += G, ++it) {
    __syncthreads();
    const bool more = wn < p.n_work;
    const Work nxt = decode(more ? wn : w0);
    if (more) issue(nxt, it & 1, pf);
    Acc acc;
    kloop(acc);
    __syncthreads();
    epilogue(cur, acc);
    if (more) land(pf);
    build_maps(decode(min(wn + G, p.n_work - 1)), (it + 1) & 1);
    __syncthreads();
    store_out(cur);
    if (!more) break;
    cur = nxt;
  }
}

template <int TH>
struct Ws1sInst {
  using C = W1sCfg<TH>;
  static int cus() {
    static const int v = [] {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        c = 256;
      return c;
    }();
    return v;
  }
  template <bool ZPAD, bool NRM>
  static void go(const ConvParams& p, int nb, hipStream_t st) {
    hipLaunchKernelGGL((ws1s_kernel<TH, ZPAD, NRM>), dim3(nb), dim3(C::NT), 0, st, p);
  }
  // grid.x = output tiles per frame, grid.y = frames
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    ConvParams p = p0;
    p.n_work = (int)grid.x * (int)grid.y;
    const int nb = std::min(p.n_work, cus());  // one workgroup per CU
    const bool zp = p.axis_mode == AX_ZERO || p.axis_mode == AX_ZERO_PREREFLECT;
    if (p.in_norm != nullptr)
      zp ? go<true, true>(p, nb, st) : go<false, true>(p, nb, st);
    else
      zp ? go<true, false>(p, nb, st) : go<false, false>(p, nb, st);
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = NST_KDT_SPLITO_O32;
    k.mode = MODE_WS1S;
    k.ks = 3; k.stride = 1; k.cinp = C::CINP; k.bn = C::COUT; k.th = TH; k.tw = C::TW; k.wm = 1; k.wn = C::NW;
    k.in_kind = IN_ACT; k.out_kind = OUT_ACT;
    k.cpc = 8; k.nch = C::NCH; k.lds_bytes = C::LDS;
    k.wbytes = C::WBYTES;
    k.persistent = 1;
    k.part_rows = 1;
    k.in_esz = 4;
    k.out_esz = 4;
    k.launch = &launch;
    return k;
  }
};

const ConvKernelInfo* conv_table_ws1s(int* count) {
  static const ConvKernelInfo table[] = {Ws1sInst<4>::info()};
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}

}  // namespace nst
