// conv_wst16.hip — weight-stationary residual-trunk conv on 16x16x32 MFMAs, one wave per SIMD.
//
// conv_wst32.hip's design (4 waves, each holding 32 output channels x 1152 K of weights for the whole launch in 256
// AGPRs + 32 VGPRs; tiles of TH rows x 32 pixels; LDS-DMA staged fill cut into per-MFMA micro-steps) on the MFMA
// shape that costs less energy per FLOP: the residual trunk runs at the board's power limit, and
// bare bf16 loops deliver ~1.12-1.15x the FLOP/s on v_mfma_f32_16x16x32 than on 32x32x16 at equal cycles per FLOP
// (MI355X_MICROARCH 'DVFS give-back' (7)).  Same layer and fusions (transformer_net.py:57-76 res1..res5,
// transformer_net_nst.py:28-43): the producer's InstanceNorm apply + ReLU or the residual join in the fill, this
// layer's InstanceNorm partial sums in the epilogue.
//
//   * each wave's 32 channels are two 16-row A blocks; a B read is 32 K x 16 pixels (half a tile row) and feeds both
//     blocks for every y-tap (up to six MFMAs), so LDS reads per FLOP stay half of conv_wstat.hip's.
//   * an MFMA holds the SIMD's issue for 8 of its 16 cycles: the fill's micro-steps are one to three instructions
//     each, one after each MFMA (288 MFMAs per part).
//   * halo entry stride 288 B (18 x 16 B): the 16 pixels x 4 K-groups of a B read land on 16 distinct 4-bank slots
//     in each ds_read_b128 lane group (stride 2 slots per pixel, K-groups of a lane group on odd offsets).
//   * epilogue: bias, packing, v_permlane16_swap pairs (pixel halves) into 16-byte stores, the IN partial sums
//     reduced over each 16-lane row.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "conv_ws_common.h"

namespace nst {

constexpr uint32_t OOB = 0xFFFFFF00u;  // buffer offset past every launch's records: loads 0, stores dropped
// cache policy of the output and residual-stream stores (32- / 64-byte pieces at the pixel stride, not whole lines):
// default.  The streaming (nt) policy that suits conv_wstat.hip's whole-line stores made this kernel's epilogue
// 3.6x slower (4.8k -> 17.5k cycles per tile, tools/w32_stamps.py)
#ifndef NST_W32_ST
#define NST_W32_ST 0
#endif

// diagnostic build (-DNST_WST32_STAMP=1, a separate library): s_memtime intervals summed per wave in scalar registers
// (the loop's counted vmcnt waits see no extra memory instruction) and written once at the end into a buffer of its
// own (nst_debug_w16_stamps): [0..3] parts, [4] epilogue, [5] loop head, [6] tiles
#ifndef NST_WST32_STAMP
#define NST_WST32_STAMP 0
#endif
// experiment builds (tools/gpu_stamps.sh): only the bf16 reflection-padded Johnson trunk variants (a third of the compile)
#ifndef NST_W32_MIN
#define NST_W32_MIN 0
#endif
#if NST_WST32_STAMP
constexpr int STAMP_IT = 1, STAMP_PT = 16;
__device__ long long g_w16_stamp[256 * 4 * STAMP_IT * STAMP_PT];
#endif

template <int TH, int FILL>
struct W16Cfg {
  static constexpr bool RES = FILL == WF_RES;
  static constexpr int NW = 4, NT = 256;            // one wave per SIMD, wave w: channels 32w..32w+31
  static constexpr int TW = 32;                     // tile width = two MFMA column blocks
  static constexpr int CINP = 128;
  static constexpr int LH = TH + 2, LW = TW + 2;
  static constexpr int NENT = LH * LW;
  static constexpr int EB = 288;                    // 16 chunks + 2 pad chunks
  static constexpr int NKS = 72;                    // 4 parts x 9 taps x 2 channel blocks (K = 32 per MFMA)
  static constexpr int NA = 64;                     // weight steps held in AGPRs (all 256 of them)
  static constexpr int NV = NKS - NA;               // ... and in VGPRs
  static constexpr int NIT = (NENT + 63) / 64;      // items per wave and region (one chunk per wave)
  static constexpr int LASTN = NENT - 64 * (NIT - 1);  // lanes with an entry in the last item
  static constexpr int NFMAX = RES ? 8 : 16;        // frames per launch (IN tables resident in LDS)
  static constexpr int DPU = RES ? 2 : 1;           // LDS-DMA requests per item
  static constexpr int SLOTB = DPU * 1024;          // a staging slot: [y | r] x lane x 16 B
  static constexpr int MAPB = ((LH + LW) * 4 + 15) / 16 * 16;
  static constexpr int MAP_OFF = NENT * EB;
  static constexpr int NORM_OFF = MAP_OFF + 2 * MAPB;
  static constexpr int NORM_TAB = NFMAX * CINP * 8;
  static constexpr int BIAS_OFF = NORM_OFF + NORM_TAB;
  static constexpr int DUMMY_OFF = BIAS_OFF + CINP * 4;  // sink of the lanes without an entry
  static constexpr int STG_OFF = DUMMY_OFF + 64 * 16;
  static constexpr int LDS = STG_OFF + NIT * NW * SLOTB;
  static constexpr int SST = TH * TW * 4 / NT;      // residual-stream stores per lane and part
  static constexpr int EPI = 2 * TH + 1;            // epilogue vector-memory instructions per wave
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(TH * TW * 4 % NT == 0 && TW == 32, "pixel-quarter stores");
};

template <typename T>
__device__ __forceinline__ void mfma16_a(f32x4_t& c, const u32x4_t& a, const u32x4_t& b, bool first) {
  if constexpr (IS_F16<T>) {
    if (first) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(c) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
  } else {
    if (first) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(c) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
  }
}
template <typename T>
__device__ __forceinline__ void mfma16_v(f32x4_t& c, const u32x4_t& a, const u32x4_t& b, bool first) {
  if constexpr (IS_F16<T>) {
    if (first) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  } else {
    if (first) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  }
}

template <typename T, int TH, int FILL, bool ZPAD, bool XO>
__global__ __launch_bounds__(256) void wst16_kernel(ConvParams p) {
  using C = W16Cfg<TH, FILL>;
  constexpr bool RES = C::RES;
  static_assert(!XO || FILL == WF_NORM, "x_0 export is a normalising fill");
  constexpr bool SOUT = RES || XO;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, p16 = lane & 15;  // MFMA K-group / output-row group, pixel within a 16-pixel half

  struct Work {
    int n, tile, ty0, tx0;
  };
  const int ntile = p.tiles_x * p.tiles_y;
  const int nfr = p.n_work / ntile;
  auto decode = [&](int wi) {
    Work r;
    r.n = wi / ntile;
    r.tile = wi - r.n * ntile;
    const int ty = r.tile / p.tiles_x;
    r.ty0 = ty * TH;
    r.tx0 = (r.tile - ty * p.tiles_x) * C::TW;
    return r;
  };
  // workgroups b, b+8, ... share an XCD (round-robin dispatch): a contiguous run of tiles per XCD and sweep
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int w0 = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  if (w0 >= p.n_work) return;

  // ---- this wave's 32 output channels x 1152 K: steps 0..NA-1 in AGPRs, the rest in VGPRs ----
  // packed [wave][step][lane][8 x 16 bit], step s = 2 (9 q + 3 dy + dx) + block
  u32x4_t wa[C::NA];
  u32x4_t wvr[C::NV];
  {
    const u32x4_t* wsrc = (const u32x4_t*)p.wpk + (size_t)wv * C::NKS * 64 + lane;
#pragma unroll
    for (int s = 0; s < C::NA; ++s) asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(wa[s]) : "v"(wsrc + s * 64) : "memory");
#pragma unroll
    for (int s = 0; s < C::NV; ++s) wvr[s] = wsrc[(C::NA + s) * 64];
  }
  // ---- the launch's IN constants and bias, resident in LDS (per frame and chunk: 4 x {scale lo, hi, shift lo, hi}) ----
  float* norm_y = (float*)(smem + C::NORM_OFF);
  if (FILL != WF_RAW) {
    for (int t = tid; t < nfr * C::CINP; t += C::NT) {
      const int f = t / C::CINP, c = t - f * C::CINP;
      const int o = (f * 16 + (c >> 3)) * 16 + 4 * ((c & 7) >> 1) + (c & 1);
      const float2 v = p.in_norm[(size_t)f * p.cs + c];
      norm_y[o] = v.x;
      norm_y[o + 2] = v.y;
    }
  }
  if (tid < C::CINP) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];

  const uint32_t fb = (uint32_t)p.hs * p.ws * p.cs * 2;          // bytes per frame: in, res_r, res_out
  const uint32_t ob = (uint32_t)p.oh * p.ow * p.cout_stride * 2;  // ... out
  auto launch_rsrc = [&](const void* base, uint32_t frame) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(frame * (uint32_t)nfr), 0x00020000);
  };
  auto build_maps = [&](const Work& wk, int slot) {
    int* rowmap = (int*)(smem + C::MAP_OFF + slot * C::MAPB);
    int* colmap = rowmap + C::LH;
    const int vy0 = wk.ty0 - p.pad, vx0 = wk.tx0 - p.pad;
    const int pix = p.cs * 2;
    // the launcher picks ZPAD = (axis_mode != AX_REFLECT): the reflection-padded trunk needs only reflect_idx
    auto axis = [&](int v, int L) { return ZPAD ? map_axis(v, L, p.axis_mode, p.pre) : reflect_idx(v, L); };
    static_assert(C::LH + C::LW <= 64, "one wave builds the maps");
    const int t = tid;
    if (t < C::LH) {
      const int sy = axis(vy0 + t, p.hs);
      rowmap[t] = sy < 0 ? -1 : sy * p.ws * pix;
    } else if (t < C::LH + C::LW) {
      const int sx = axis(vx0 + t - C::LH, p.ws);
      colmap[t - C::LH] = sx < 0 ? -1 : sx * pix;
    }
  };
  // item k of a region: entry 64 k + lane, chunk 4 R + wv (wave-uniform: its IN constants are one broadcast LDS
  // row).  Items of 16 entries x the region's 4 chunks (64 contiguous bytes per entry and lane quad, 16 pixels per
  // DMA instead of 64) measured the same (plain trunk conv 0.261 vs 0.262 ms) with more registers
  constexpr int IT_STRIDE = 64;  // entries per item
  auto item_entry = [&](int k) { return 64 * k + lane; };
  auto item_chunk = [&](int R) { return 4 * R + wv; };
  // the tile's item sources: entry 64 k + lane of every region, OOB = zero padding / no entry; bit k of pad:
  // a zero-padding entry (ZPAD keeps it zero after the IN apply)
  struct Src {
    uint32_t voff[C::NIT];
    uint32_t pad;
  };
  auto sources = [&](const Work& wk, int slot) {
    const int* rowmap = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    const int* colmap = rowmap + C::LH;
    Src s;
    s.pad = 0;
#pragma unroll
    for (int k = 0; k < C::NIT; ++k) {
      const int e0 = item_entry(k);
      const bool valid = k < C::NIT - 1 || lane < C::LASTN;
      const int e = valid ? e0 : 0;
      const int ly = e / C::LW, lx = e - ly * C::LW;
      const int ro = rowmap[ly], co = colmap[lx];
      const bool in = valid && ro >= 0 && co >= 0;
      s.voff[k] = in ? (uint32_t)(ro + co) + (uint32_t)wk.n * fb : OOB;
      if (valid && !in) s.pad |= 1u << k;
    }
    return s;
  };
  const uint32_t stg = (uint32_t)(uintptr_t)(smem + C::STG_OFF) + wv * C::SLOTB;
  const __amdgpu_buffer_rsrc_t rs_in = launch_rsrc(p.in, fb);
  const __amdgpu_buffer_rsrc_t rs_r = launch_rsrc(RES ? p.res_r : p.in, fb);
  // item k of region R: chunk 4R + wv of entry 64 k + lane, into staging slot k of this wave
  auto request = [&](int k, int R, uint32_t voff) {
    const uint32_t lds = stg + k * C::NW * C::SLOTB;
    const int soff = (4 * R + wv) * 16;
    dma16(rs_in, voff, lds, soff);
    if constexpr (RES) dma16(rs_r, voff, lds + 1024, soff);
  };
  struct Staged {
    uint4 y, r;
  };
  auto stage_read = [&](int k) {
    const char* sp = smem + C::STG_OFF + (k * C::NW + wv) * C::SLOTB + lane * 16;
    Staged st;
    st.y = *(const uint4*)sp;
    st.r = RES ? *(const uint4*)(sp + 1024) : make_uint4(0u, 0u, 0u, 0u);
    return st;
  };
  // IN + ReLU / residual join of a staged item into its halo entry
  auto consume = [&](int n, int k, int R, uint32_t padbits, const Staged& st) {
    const int ch = item_chunk(R);
    const uint4 y = st.y, rr = st.r;
    const float4* ny = (const float4*)(norm_y + (n * 16 + ch) * 16);
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint32_t o[4];
    if constexpr (RES) {
      // ResidualBlock join (transformer_net.py:71-76): IN_y(y) + r in fp32, product then sum, one rounding
      const uint32_t w2[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 nn = ny[j];
        const float a = lo16<T>(w[j]) * nn.x + nn.z;
        const float bb = hi16<T>(w[j]) * nn.y + nn.w;
        o[j] = pack16<T>(lo16<T>(w2[j]) + a, hi16<T>(w2[j]) + bb);
      }
    } else if constexpr (FILL == WF_RAW) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = w[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 nn = ny[j];
        const float a = __builtin_fmaf(lo16<T>(w[j]), nn.x, nn.z);
        const float bb = __builtin_fmaf(hi16<T>(w[j]), nn.y, nn.w);
        const i16x2_t r = __builtin_bit_cast(i16x2_t, pack16<T>(a, bb));
        o[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
      }
    }
    const bool pad = ZPAD && ((padbits >> k) & 1u);
    const u32x4_t v = {pad ? 0u : o[0], pad ? 0u : o[1], pad ? 0u : o[2], pad ? 0u : o[3]};
    const bool valid = k < C::NIT - 1 || lane < C::LASTN;
    int eb = item_entry(0) * C::EB + ch * 16;
    asm volatile("" : "+v"(eb));
    *(u32x4_t*)(smem + (valid ? eb + k * IT_STRIDE * C::EB : C::DUMMY_OFF + lane * 16)) = v;
  };
  // vmcnt before consuming item k: the NIT - 1 items' requests issued after its own, SST residual-stream stores
  // (RES / XO: piece i at slot 24 i + 23 of every part), and (part 0) the epilogue's stores
  constexpr int KIN = (C::NIT - 1) * C::DPU + (SOUT ? C::SST : 0);
  constexpr int KEP = KIN + C::EPI;

  // ---- K loop ----
  typedef f32x4_t Acc[TH][2][2];  // [tile row][channel block][pixel half]
  const int lbase = p16 * C::EB + g4 * 16;
  // K order inside part q: x-tap dx, halo row y, pixel half hx.  LDS row y of x-tap dx is the B operand of tile row
  // y - dy for every y-tap dy and of both channel blocks: up to six MFMAs per ds_read_b128.
  constexpr int NRD = 2 * C::LH;  // reads per dx (halo row, pixel half)
  constexpr int PRD = 3 * NRD;    // reads per part
  auto bread = [&](int i) -> u32x4_t {
    const int q = i / PRD, rem = i - q * PRD;
    const int dx = rem / NRD, y = (rem % NRD) >> 1, hx = rem & 1;
    return *(const u32x4_t*)(smem + lbase + (y * C::LW + dx + 16 * hx) * C::EB + 4 * q * 16);
  };
  // One wave per SIMD: nothing hides this wave's non-MFMA work but its own MFMAs' shadow (a 16x16x32 MFMA holds the
  // issue for 8 of its 16 cycles), so the fill is cut into micro-steps of one to three instructions, one after each
  // MFMA (`slot`: the MFMA's index in its part), instead of lumps that leave the MFMA pipe idle.
  auto kloop = [&](Acc& acc, auto&& filler, auto&& bound) {
    // B reads in flight ahead of their MFMAs: 3, or 2 where the residual-stream pieces need the registers
    constexpr int NI = 4 * PRD, D = SOUT ? 2 : 3;
    u32x4_t ring[D];
#pragma unroll
    for (int i = 0; i < D; ++i) ring[i] = bread(i);
    int slot = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = i / PRD, rem = i - q * PRD;
      const int dx = rem / NRD, y = (rem % NRD) >> 1, hx = rem & 1;
      if (rem == 0) slot = 0;
      const u32x4_t bcur = ring[i % D];
      if (i + D < NI) ring[i % D] = bread(i + D);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int r = y - dy;
        if (r < 0 || r >= TH) continue;
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int s = 2 * (q * 9 + 3 * dy + dx) + bb;
          const bool first = q == 0 && dx == 0 && dy == 0;
          if (s < C::NA) mfma16_a<T>(acc[r][bb][hx], wa[s], bcur, first);
          else mfma16_v<T>(acc[r][bb][hx], wvr[s - C::NA], bcur, first);
          filler(q, slot);
          ++slot;
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (rem == PRD - 1) {
        lds_barrier();
        bound(q);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: lane (g4, p16) holds channels 32 wv + 16 bb + 4 g4 + i of pixels p16 / 16 + p16 of every row ----
  const float* biasl = (const float*)(smem + C::BIAS_OFF) + 32 * wv + 4 * g4;
  auto epilogue = [&](const Work& wk, Acc& acc) {
    // the last MFMAs' results: XDL write -> VALU read wait states
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    const __amdgpu_buffer_rsrc_t ors = launch_rsrc(p.out, ob);
    const uint32_t row_bytes = (uint32_t)p.ow * p.cout_stride * 2;
    // after the swaps lane l stores 8 channels (32 wv + 16 bb + 8 (g4 >> 1) + 0..7) of pixel p16 (g4 even) or
    // 16 + p16 (g4 odd): each store covers the 32 pixels x 32 bytes of one channel block
    const int spx = wk.tx0 + ((g4 & 1) ? 16 : 0) + p16;
    const uint32_t soff = (uint32_t)wk.n * ob + (uint32_t)(((wk.ty0 * p.ow + spx) * p.cout_stride + 32 * wv + 8 * (g4 >> 1)) * 2);
    const bool sok = spx < p.ow;
    const bool ok0 = wk.tx0 + p16 < p.ow, ok1 = wk.tx0 + 16 + p16 < p.ow;
    const f32x4_t bias0 = *(const f32x4_t*)(biasl), bias1 = *(const f32x4_t*)(biasl + 16);
    f32x4_t s1[2], s2[2];
    auto rows = [&](auto all_valid) {
#pragma unroll
      for (int r = 0; r < TH; ++r) {
        const bool rv = decltype(all_valid)::value || wk.ty0 + r < p.oh;
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const f32x4_t v0 = acc[r][bb][0] + (bb ? bias1 : bias0), v1 = acc[r][bb][1] + (bb ? bias1 : bias0);
          // rows of 16 lanes 1 / 3 of the pixel-half-0 pair swap with rows 0 / 2 of the half-1 pair: lanes of even
          // rows then hold 8 channels of pixel p16, of odd rows 8 channels of pixel 16 + p16
          const auto sx = __builtin_amdgcn_permlane16_swap(pack16<T>(v0[0], v0[1]), pack16<T>(v1[0], v1[1]), false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(pack16<T>(v0[2], v0[3]), pack16<T>(v1[2], v1[3]), false, false);
          const u32x4_t pk = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(pk, ors, (rv && sok) ? soff + r * row_bytes + 32 * bb : OOB, 0, NST_W32_ST);
          const f32x4_t x0 = (decltype(all_valid)::value || (rv && ok0)) ? v0 : (f32x4_t){0.f, 0.f, 0.f, 0.f};
          const f32x4_t x1 = (decltype(all_valid)::value || (rv && ok1)) ? v1 : (f32x4_t){0.f, 0.f, 0.f, 0.f};
          if (r == 0) {
            s1[bb] = x0 + x1;
            s2[bb] = __builtin_elementwise_fma(x1, x1, x0 * x0);
          } else {
            s1[bb] = (s1[bb] + x0) + x1;
            s2[bb] = __builtin_elementwise_fma(x1, x1, __builtin_elementwise_fma(x0, x0, s2[bb]));
          }
        }
      }
    };
    if (wk.ty0 + TH <= p.oh && wk.tx0 + C::TW <= p.ow) rows(std::true_type{});
    else rows(std::false_type{});
    // 16 statistics per lane, v[(4 bb + i) 2 + st], reduce-scattered over the 16 pixel lanes of the row: lane p16 ends
    // with value 8 (p16 >= 8) + 4 (p16 & 4) + 2 (p16 & 2) + (p16 & 1)
    const float v[16] = {s1[0][0], s2[0][0], s1[0][1], s2[0][1], s1[0][2], s2[0][2], s1[0][3], s2[0][3],
                         s1[1][0], s2[1][0], s1[1][1], s2[1][1], s1[1][2], s2[1][2], s1[1][3], s2[1][3]};
    float a8[8], a4[4], a2[2], a1[1];
    rs_step<8, 0x140>(v, a8, p16 >= 8);
    rs_step<4, 0x141>(a8, a4, (p16 & 4) != 0);
    rs_step<2, 0x1b>(a4, a2, (p16 & 2) != 0);
    rs_step<1, 0xb1>(a2, a1, (p16 & 1) != 0);
    const int idx = (p16 >= 8 ? 8 : 0) + ((p16 & 4) ? 4 : 0) + ((p16 & 2) ? 2 : 0) + (p16 & 1);
    const int co = 32 * wv + 16 * (idx >> 3) + 4 * g4 + ((idx >> 1) & 3);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.partial + ((size_t)wk.n * ntile + wk.tile) * p.cout_stride * 2), (short)0, p.cout_stride * 8, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a1[0]), prs, (uint32_t)((co * 2 + (idx & 1)) * 4), 0, 0);
  };

  // ---- persistent walk ----
  Work cur = decode(w0);
  int wn = w0 + G;
  const int last = p.n_work - 1;
  build_maps(cur, 0);
  build_maps(decode(min(wn, last)), 1);
  // the AGPR weight loads (asm) and the tables above: complete before anything reads them
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // prologue: regions 0..2 of the first tile into the halo, region 3 in flight (the loop's part 0 consumes it
  // and requests region 0 of the next tile); drained once so every later wait counts steady-state instructions
  uint32_t pad3;  // ZPAD: bit k = cur's region-3 item k is zero padding (consumed in part 0)
  {
    const Src s0 = sources(cur, 0);
    pad3 = s0.pad;  // the loop's first part 0 consumes the first tile's region 3
#pragma unroll
    for (int k = 0; k < C::NIT; ++k) request(k, 0, s0.voff[k]);
#pragma unroll
    for (int R = 0; R < 3; ++R) {
      vm_wait<0>();
#pragma unroll
      for (int k = 0; k < C::NIT; ++k) {
        consume(cur.n, k, R, s0.pad, stage_read(k));
        request(k, R + 1, s0.voff[k]);
      }
    }
  }
  vm_wait<0>();
  __syncthreads();
  // Micro-step schedule of item k (MFMA slots 48 k + o of a part; a part has 288 MFMAs), at most ~2 instructions
  // each (the 8 free issue cycles of a 16x16x32 MFMA):
  //   o = 0: wait for the item's LDS-DMA, staging read | 2: map reads of the next region's item k (the next tile's
  //   entry) | 4 + 8 j: IN constants of channel pair j | 8 + 8 j .. 11 + 8 j: pair j's value steps | 36, 37: the
  //   request's source offset | 38: halo write | 40: the next region's request of item k (not held across parts).
  //   RES / XO store residual-stream piece k < SST (42: halo read, 47: store, after the part's k-th request: SST
  //   stores lie between any item's request and its wait).
  constexpr int SLOTS_PER_ITEM = 48;
  static_assert(SLOTS_PER_ITEM * C::NIT <= 9 * TH * 4 && C::SST <= C::NIT, "micro-step slots");
  Acc acc;
  Staged sy;                 // the staged chunk(s) of the item in flight
  float4 n0;                 // IN constants of one channel pair
  float tl, th;              // a pair's lo / hi value between its micro-steps
  uint32_t o4[4];            // the item's packed output
  int mro = 0, mco = 0;      // map entries of the next tile's item k
  bool padk = false;         // ZPAD: the consumed item k is zero padding (parts 1..3)
  bool mok = false;          // the next tile's item k has a source (not padding, an entry)
  uint32_t rvoff = OOB;      // ... its source offset
  u32x4_t sv;                // residual-stream piece between its halo read and its store
#if NST_WST32_STAMP
  unsigned st_acc[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned st_prev = (unsigned)__builtin_amdgcn_s_memtime();
#endif
  auto stamp = [&](int it, int pt) {  // pt: interval ending here (0 = loop head)
#if NST_WST32_STAMP
    const unsigned t = (unsigned)__builtin_amdgcn_s_memtime();
    st_acc[pt == 0 ? 5 : pt - 1] += t - st_prev;
    st_prev = t;
    if (pt == 0) st_acc[6] += 1;
#endif
  };
  for (int it = 0;; ++it) {
    stamp(it, 0);
    const bool more = wn < p.n_work;
    const Work nxt = more ? decode(wn) : cur;
    const Work nxt2 = decode(min(wn + G, last));
    const int cs = it & 1, ns = cs ^ 1;
    kloop(
        acc,
        [&](int q, int slot) {
          const int k = slot / SLOTS_PER_ITEM, o = slot - k * SLOTS_PER_ITEM;
          if (k >= C::NIT) return;
          // part 0: region 3 of cur; part q > 0: region q - 1 of nxt
          const int R = q == 0 ? 3 : q - 1;
          const int n = q == 0 ? cur.n : nxt.n;
          const int ch = item_chunk(R);
          const float4* ny = (const float4*)(norm_y + (n * 16 + ch) * 16);
          // pair j's value steps: NORM IN + ReLU (fma lo | fma hi | pack + max); RES join (lo: y scale | + shift,
          // + r | hi: the same | pack; product then sum, one rounding per op, as the unfused residual kernel)
          auto pair_step = [&](int j, int st) {
            const uint32_t wy = j == 0 ? sy.y.x : j == 1 ? sy.y.y : j == 2 ? sy.y.z : sy.y.w;
            if constexpr (RES) {
              const uint32_t wr = j == 0 ? sy.r.x : j == 1 ? sy.r.y : j == 2 ? sy.r.z : sy.r.w;
              // ResidualBlock join (transformer_net.py:71-76): IN_y(y) + r in fp32
              if (st == 0) tl = lo16<T>(wy) * n0.x;
              else if (st == 1) tl = lo16<T>(wr) + (tl + n0.z);
              else if (st == 2) th = hi16<T>(wy) * n0.y;
              else o4[j] = pack16<T>(tl, hi16<T>(wr) + (th + n0.w));
            } else if constexpr (FILL == WF_RAW) {
              if (st == 3) o4[j] = wy;
            } else {
              if (st == 0) tl = __builtin_fmaf(lo16<T>(wy), n0.x, n0.z);
              else if (st == 1) th = __builtin_fmaf(hi16<T>(wy), n0.y, n0.w);
              else if (st == 3) {
                const i16x2_t r = __builtin_bit_cast(i16x2_t, pack16<T>(tl, th));
                o4[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
              }
            }
          };
          if (o == 0) {
            if (q == 0) vm_wait<KEP>(); else vm_wait<KIN>();
            sy = stage_read(k);
          } else if (o >= 4 && o < 36 && (o - 4) % 8 == 0) {
            if (FILL != WF_RAW) n0 = ny[(o - 4) / 8];  // pair j's IN constants, four MFMAs before its first step
          } else if (o >= 8 && o < 36 && (o - 4) % 8 >= 4) {
            pair_step((o - 4) / 8, (o - 4) % 8 - 4);
          } else if (o == 2) {
            const int* rowmap = (const int*)(smem + C::MAP_OFF + ns * C::MAPB);
            const bool valid = k < C::NIT - 1 || lane < C::LASTN;
            const int e = valid ? item_entry(k) : 0;
            const int ly = e / C::LW, lx = e - ly * C::LW;
            mro = rowmap[ly];
            mco = rowmap[C::LH + lx];
          } else if (o == 36) {
            const bool valid = k < C::NIT - 1 || lane < C::LASTN;
            mok = valid && mro >= 0 && mco >= 0;
            // ZPAD: a zero-padding entry.  Parts 1..3 consume the item they request (nxt's item k); part 3 keeps
            // the flags for the next iteration's part 0, which consumes this tile's region 3
            if (ZPAD) {
              padk = valid && !mok;
              if (q == 3) pad3 = (pad3 & ~(1u << k)) | (padk ? 1u << k : 0u);
            }
          } else if (o == 37) {
            rvoff = mok ? (uint32_t)(mro + mco) + (uint32_t)nxt.n * fb : OOB;
          } else if (o == 38) {
            const bool pad = ZPAD && (q == 0 ? ((pad3 >> k) & 1u) != 0 : padk);
            const u32x4_t v = {pad ? 0u : o4[0], pad ? 0u : o4[1], pad ? 0u : o4[2], pad ? 0u : o4[3]};
            const bool valid = k < C::NIT - 1 || lane < C::LASTN;
            int eb = item_entry(0) * C::EB + ch * 16;
            asm volatile("" : "+v"(eb));
            *(u32x4_t*)(smem + (valid ? eb + k * IT_STRIDE * C::EB : C::DUMMY_OFF + lane * 16)) = v;
          } else if (o == 40) {
            request(k, q, rvoff);  // region q of nxt
          }
          // the tile after nxt into cur's map slot (cur's sources were resolved in the previous iteration; the
          // barriers ending parts 1..3 publish it before the next iteration's part 0 reads it)
          if (q == 1 && k == 0 && o == 44) build_maps(nxt2, cs);
          if (SOUT && k < C::SST && o == 42) {
            const int cl = lane >> 4, x16 = ((lane & 15) - cl) & 15;
            const int P = 16 * (C::SST * wv + k) + x16;
            sv = *(const u32x4_t*)(smem + (((P >> 5) + 1) * C::LW + (P & 31) + 1) * C::EB + (4 * q + cl) * 16);
          }
          if (SOUT && k < C::SST && o == 47) {
            const int cl = lane >> 4, x16 = ((lane & 15) - cl) & 15;
            const int P = 16 * (C::SST * wv + k) + x16;
            const int c = 4 * q + cl, oy = cur.ty0 + (P >> 5), ox = cur.tx0 + (P & 31);
            const bool ok = oy < p.oh && ox < p.ow;
            __builtin_amdgcn_raw_buffer_store_b128(sv, launch_rsrc(p.res_out, fb),
                                                   ok ? (uint32_t)cur.n * fb + (uint32_t)(((oy * p.ws + ox) * p.cs + c * 8) * 2) : OOB,
                                                   0, NST_W32_ST);
          }
        },
        [&](int q) { stamp(it, 1 + q); });
    epilogue(cur, acc);
    stamp(it, 5);
    if (!more) break;
    cur = nxt;
    wn += G;
  }
  vm_wait<0>();  // no LDS-DMA may land after the workgroup has released its LDS
#if NST_WST32_STAMP
  if (lane == 0 && b < 256)
    for (int i = 0; i < 7; ++i) g_w16_stamp[(b * 4 + wv) * STAMP_PT + i] = st_acc[i];
#endif
}

template <typename T, int TH, bool RES>
struct Wst16Inst {
  using C = W16Cfg<TH, RES ? WF_RES : WF_NORM>;
  static int cus() {
    static const int v = [] {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        c = 256;
      return c;
    }();
    return v;
  }
  template <int FILL, bool ZPAD, bool XO = false>
  static void go(const ConvParams& p, int nb, hipStream_t st) {
    hipLaunchKernelGGL((wst16_kernel<T, TH, FILL, ZPAD, XO>), dim3(nb), dim3(C::NT), 0, st, p);
  }
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    const int ntile = (int)grid.x, n = (int)grid.y;
    const size_t fin = (size_t)p0.hs * p0.ws * p0.cs * 2, fout = (size_t)p0.oh * p0.ow * p0.cout_stride * 2;
    const int fmax = (int)std::min<size_t>(C::NFMAX, (size_t)OOB / std::max(fin, fout));
    if (fmax < 1) return;
    for (int f0 = 0; f0 < n; f0 += fmax) {
      const int nf = std::min(fmax, n - f0);
      ConvParams p = p0;
      p.in = (const char*)p0.in + f0 * fin;
      p.out = (char*)p0.out + f0 * fout;
      if (p0.res_r) p.res_r = (const char*)p0.res_r + f0 * fin;
      if (p0.res_out) p.res_out = (char*)p0.res_out + f0 * fin;
      if (p0.in_norm) p.in_norm = p0.in_norm + (size_t)f0 * p0.cs;
      p.partial = p0.partial + (size_t)f0 * ntile * p0.cout_stride * 2;
      p.n_work = nf * ntile;
      const int nb = std::min(p.n_work, cus());
      const bool zp = p.axis_mode != AX_REFLECT;
#if NST_W32_MIN
      // experiment build: the Johnson trunk's three variants only (reflection padding)
      if (zp) return;
      if constexpr (RES) go<WF_RES, false>(p, nb, st);
      else if (p.res_out != nullptr) go<WF_NORM, false, true>(p, nb, st);
      else go<WF_NORM, false>(p, nb, st);
#else
      if constexpr (RES) {
        zp ? go<WF_RES, true>(p, nb, st) : go<WF_RES, false>(p, nb, st);
      } else {
        if (p.in_norm != nullptr && p.res_out != nullptr)
          zp ? go<WF_NORM, true, true>(p, nb, st) : go<WF_NORM, false, true>(p, nb, st);
        else if (p.in_norm != nullptr)
          zp ? go<WF_NORM, true>(p, nb, st) : go<WF_NORM, false>(p, nb, st);
        else
          zp ? go<WF_RAW, true>(p, nb, st) : go<WF_RAW, false>(p, nb, st);
      }
#endif
    }
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = dtype_code<T>();
    k.mode = MODE_WSTAT;
    k.ks = 3; k.stride = 1; k.cinp = C::CINP; k.bn = 128; k.th = TH; k.tw = C::TW; k.wm = C::NW; k.wn = 2;  // wn = 2: two 16-channel blocks per wave (pack_wst16_weights)
    k.in_kind = IN_ACT; k.out_kind = OUT_ACT;
    k.cpc = 8; k.nch = 16; k.lds_bytes = C::LDS;
    k.wbytes = C::NW * C::NKS * 1024;
    k.persistent = 1;
    k.part_rows = 1;
    k.res = RES ? 1 : 0;
    k.launch = &launch;
    return k;
  }
};

#ifndef NST_WST16_TH
#define NST_WST16_TH 8
#endif
// Build split: one kernel instantiation compiles for ~2-3 min (fully unrolled 1,152-MFMA tiles), so the library
// compiles this file nine times in parallel.  NST_W16_PART = 0..7 explicitly instantiate two kernels each (dtype
// bf16 for 0..3, fp16 for 4..7; p % 4 = 0: normalising fill without / with the x_0 export, 1: the same zero-padded,
// 2: identity fill, reflect / zero-padded, 3: residual join, reflect / zero-padded); 8 holds the launchers, infos and
// the table, with every kernel an extern template; -1 (experiment builds): all in one object, instantiated by use.
#ifndef NST_W16_PART
#define NST_W16_PART -1
#endif
#define W16_KERNELS(X, T)                                                                                     \
  X(T, WF_NORM, false, false) X(T, WF_NORM, false, true) X(T, WF_NORM, true, false) X(T, WF_NORM, true, true) \
  X(T, WF_RAW, false, false) X(T, WF_RAW, true, false) X(T, WF_RES, false, false) X(T, WF_RES, true, false)
#define W16_EXTERN(T, F, Z, X_) extern template __global__ void wst16_kernel<T, NST_WST16_TH, F, Z, X_>(ConvParams);
#define W16_INST(T, F, Z, X_) template __global__ void wst16_kernel<T, NST_WST16_TH, F, Z, X_>(ConvParams);
#if NST_W16_PART >= 0 && NST_W16_PART < 8
#define W16_T_ __bf16
#if NST_W16_PART >= 4
#undef W16_T_
#define W16_T_ _Float16
#endif
#if NST_W16_PART % 4 == 0
W16_INST(W16_T_, WF_NORM, false, false)
W16_INST(W16_T_, WF_NORM, false, true)
#elif NST_W16_PART % 4 == 1
W16_INST(W16_T_, WF_NORM, true, false)
W16_INST(W16_T_, WF_NORM, true, true)
#elif NST_W16_PART % 4 == 2
W16_INST(W16_T_, WF_RAW, false, false)
W16_INST(W16_T_, WF_RAW, true, false)
#else
W16_INST(W16_T_, WF_RES, false, false)
W16_INST(W16_T_, WF_RES, true, false)
#endif
#else
#if NST_W16_PART == 8
W16_KERNELS(W16_EXTERN, __bf16)
W16_KERNELS(W16_EXTERN, _Float16)
#endif
// searched before conv_table_wstat (first match wins); NST_WST16=0 in the environment hides it (A/B runs)
const ConvKernelInfo* conv_table_wst16(int* count) {
  static const ConvKernelInfo table[] = {
      Wst16Inst<__bf16, NST_WST16_TH, false>::info(),  // residual trunk
      Wst16Inst<__bf16, NST_WST16_TH, true>::info(),   // + residual join in the fill
#if !NST_W32_MIN
      Wst16Inst<_Float16, NST_WST16_TH, false>::info(),  // fp16 mode
      Wst16Inst<_Float16, NST_WST16_TH, true>::info(),
#endif
  };
  const char* env = std::getenv("NST_WST16");
  *count = (env != nullptr && env[0] == '0') ? 0 : (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#endif

}  // namespace nst

#if NST_WST32_STAMP
extern "C" int nst_debug_w16_stamps(long long* host, int n) {
  const int cap = 256 * 4 * nst::STAMP_IT * nst::STAMP_PT;
  if (n > cap) n = cap;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(nst::g_w16_stamp), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif
