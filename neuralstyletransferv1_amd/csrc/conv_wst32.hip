// conv_wst32.hip — weight-stationary residual-trunk conv on 32x32x16 MFMAs, one wave per SIMD.
//
// Same layer and fusions as conv_wstat.hip (the residual blocks' ConvLayer(128, 128, 3, 1) of
// transformer_net.py:57-76 / transformer_net_nst.py:28-43 with the producer's InstanceNorm apply + ReLU or the
// residual join in the fill and this layer's InstanceNorm partial sums in the epilogue), re-tiled for the
// measured bound of that kernel: vector-instruction issue, not MFMA (VALU/MFMA 2.37, MFMA busy 0.55;
// ≈10.6k issue cycles per tile and SIMD against 9.2k of MFMA).
//
//   * 4 waves, one per SIMD, each holding 32 output channels x 1152 K of weights for the whole launch:
//     288 registers per lane, 256 of them AGPRs (MFMA A operands may be AGPRs) and 32 VGPRs.
//   * v_mfma_f32_32x32x16: one MFMA is 32 channels x 32 pixels x 16 K and holds the SIMD's issue for 8 of its
//     32 cycles, where two 16x16x32 MFMAs hold it for 16 (MI355X_MICROARCH 'vector-instruction ISSUE cost');
//     each B operand read (32 pixels x 16 K from LDS) feeds 32 output channels instead of 16, so LDS reads per
//     MFMA cycle halve too.
//   * tile = TH rows x 32 pixels (a tile row is one MFMA column block), TH accumulators of 16 fp32 per lane;
//     halo (TH+2) x 34 entries x 128 channels in LDS, entry stride 272 B (17 x 16 B: the 32 pixels of a B read
//     land on 16 distinct 4-bank slots in each ds_read_b128 lane group).
//   * K order: part q (input channels 32q..32q+31), x-tap dx, halo row y, K half kk; LDS row y of x-tap dx is
//     the B operand of tile row y - dy for every y-tap dy (up to three MFMAs per read).
//   * fill: region q (chunks 4q..4q+3 of every halo entry) of the NEXT tile streams in while part q+1 of this
//     tile computes (region 3 of this tile during its own part 0); wave w stages chunk 4q + w of every entry,
//     NIT items of 64 entries, by LDS-DMA into a ring of NIT slots one region ahead.
//   * epilogue: bias, bf16 / fp16 packing, v_permlane32_swap pairs into 16-byte stores straight to HBM (no LDS
//     staging: the 32-pixel halo leaves no room for it), InstanceNorm partial sums reduced over the 32 pixel lanes.
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
// own (nst_debug_w32_stamps): [0..3] parts, [4] epilogue, [5] loop head, [6] tiles
#ifndef NST_WST32_STAMP
#define NST_WST32_STAMP 0
#endif
// experiment builds (tools/gpu_stamps.sh): only the bf16 reflection-padded Johnson trunk variants (a third of the compile)
#ifndef NST_W32_COAL
#define NST_W32_COAL 0
#endif
#ifndef NST_W32_MIN
#define NST_W32_MIN 0
#endif
#if NST_WST32_STAMP
constexpr int STAMP_IT = 1, STAMP_PT = 16;
__device__ long long g_w32_stamp[256 * 4 * STAMP_IT * STAMP_PT];
#endif

template <int TH, int FILL>
struct W32Cfg {
  static constexpr bool RES = FILL == WF_RES;
  static constexpr int NW = 4, NT = 256;            // one wave per SIMD, wave w: channels 32w..32w+31
  static constexpr int TW = 32;                     // tile width = MFMA column block
  static constexpr int CINP = 128;
  static constexpr int LH = TH + 2, LW = TW + 2;
  static constexpr int NENT = LH * LW;
  static constexpr int EB = 272;                    // 16 chunks + 1 pad chunk
  static constexpr int NKS = 72;                    // 4 parts x 9 taps x 2 K halves (K = 16 per MFMA)
  static constexpr int NA = 64;                     // weight steps held in AGPRs (all 256 of them)
  static constexpr int NV = NKS - NA;               // ... and in VGPRs
#if NST_W32_COAL
  // an item is 16 entries x the region's 4 chunks (64 contiguous bytes per entry: one DMA touches 16 pixels'
  // half-lines instead of 64 pixels' 16-byte pieces); wave w stages entries EW w .. EW w + EW - 1
  static constexpr int EW = (NENT + 3) / 4;
  static constexpr int NIT = (EW + 15) / 16;
  static constexpr int LASTN = (EW - 16 * (NIT - 1)) * 4;  // lanes with an entry in the last item
  static_assert(NENT % 4 == 0, "four waves split the entries evenly");
#else
  static constexpr int NIT = (NENT + 63) / 64;      // items per wave and region (one chunk per wave)
  static constexpr int LASTN = NENT - 64 * (NIT - 1);  // lanes with an entry in the last item
#endif
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
  static constexpr int EPI = 2 * TH + 2;            // epilogue vector-memory instructions per wave
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(TH * TW * 4 % NT == 0 && TW == 32, "pixel-quarter stores");
};

template <typename T>
__device__ __forceinline__ void mfma32_a(f32x16_t& c, const u32x4_t& a, const u32x4_t& b, bool first) {
  if constexpr (IS_F16<T>) {
    if (first) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
  } else {
    if (first) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "a"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
  }
}
template <typename T>
__device__ __forceinline__ void mfma32_v(f32x16_t& c, const u32x4_t& a, const u32x4_t& b, bool first) {
  if constexpr (IS_F16<T>) {
    if (first) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  } else {
    if (first) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  }
}

template <typename T, int TH, int FILL, bool ZPAD, bool XO>
__global__ __launch_bounds__(256) void wst32_kernel(ConvParams p) {
  using C = W32Cfg<TH, FILL>;
  constexpr bool RES = C::RES;
  static_assert(!XO || FILL == WF_NORM, "x_0 export is a normalising fill");
  constexpr bool SOUT = RES || XO;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, px = lane & 31;

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
  // packed [wave][step][lane][8 x 16 bit], step s = 2 (9 q + 3 dy + dx) + kk
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
  // item k of a region: this lane's halo entry and chunk (item_chunk(R)); lane_coff: the chunk's byte offset
  // within the region's 64 bytes of a pixel when it varies per lane (the DMA's scalar offset carries the rest)
  constexpr int IT_STRIDE = NST_W32_COAL ? 16 : 64;  // entries per item
  auto item_entry = [&](int k) { return NST_W32_COAL ? ((C::NENT + 3) / 4) * wv + 16 * k + (lane >> 2) : 64 * k + lane; };
  auto item_chunk = [&](int R) { return NST_W32_COAL ? 4 * R + (lane & 3) : 4 * R + wv; };
  const uint32_t lane_coff = NST_W32_COAL ? (uint32_t)(lane & 3) * 16 : 0u;
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
      s.voff[k] = in ? (uint32_t)(ro + co) + (uint32_t)wk.n * fb + lane_coff : OOB;
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
    const int soff = (NST_W32_COAL ? 4 * R : 4 * R + wv) * 16;
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
  typedef f32x16_t Acc[TH];
  const int lbase = px * C::EB + h * 16;
  constexpr int NRD = 2 * C::LH;  // reads per dx (halo row, K half)
  constexpr int PRD = 3 * NRD;    // reads per part
  auto bread = [&](int i) -> u32x4_t {
    const int q = i / PRD, rem = i - q * PRD;
    const int dx = rem / NRD, y = (rem % NRD) >> 1, kk = rem & 1;
    return *(const u32x4_t*)(smem + lbase + (y * C::LW + dx) * C::EB + (4 * q + 2 * kk) * 16);
  };
  // One wave per SIMD: nothing hides this wave's non-MFMA work but its own MFMAs' shadow (an MFMA holds the issue
  // for 8 of its 32 cycles), so the fill is cut into micro-steps of a few instructions, one after each MFMA
  // (`slot`: the MFMA's index in its part), instead of lumps that leave the MFMA pipe idle.
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
      const int dx = rem / NRD, y = (rem % NRD) >> 1, kk = rem & 1;
      if (rem == 0) slot = 0;
      const u32x4_t bcur = ring[i % D];
      if (i + D < NI) ring[i % D] = bread(i + D);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int r = y - dy;
        if (r < 0 || r >= TH) continue;
        const int s = 2 * (q * 9 + 3 * dy + dx) + kk;
        const bool first = q == 0 && dx == 0 && dy == 0 && kk == 0;
        if (s < C::NA) mfma32_a<T>(acc[r], wa[s], bcur, first);
        else mfma32_v<T>(acc[r], wvr[s - C::NA], bcur, first);
        filler(q, slot);
        ++slot;
        __builtin_amdgcn_sched_barrier(0);
      }
      if (rem == PRD - 1) {
        lds_barrier();
        bound(q);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: lane (h, px) holds channels 32 wv + 8 j + 4 h + i (reg 4 j + i) of pixel px of every row ----
  const float* biasl = (const float*)(smem + C::BIAS_OFF) + 32 * wv + 4 * h;
  auto epilogue = [&](const Work& wk, Acc& acc) {
    // the last MFMAs' results: 16-pass XDL write -> VALU read needs >= 18 wait states
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    const __amdgpu_buffer_rsrc_t ors = launch_rsrc(p.out, ob);
    const int ox = wk.tx0 + px;
    const uint32_t row_bytes = (uint32_t)p.ow * p.cout_stride * 2;
    const uint32_t off0 = (uint32_t)wk.n * ob + (uint32_t)(((wk.ty0 * p.ow + ox) * p.cout_stride + 32 * wv) * 2) + 16 * h;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.partial + ((size_t)wk.n * ntile + wk.tile) * p.cout_stride * 2), (short)0, p.cout_stride * 8, 0x00020000);
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      // channel groups g = 2 jp + e (regs 4 g .. 4 g + 3): channels 32 wv + 8 g + 4 h + i
      const f32x4_t b0 = *(const f32x4_t*)(biasl + 16 * jp), b1 = *(const f32x4_t*)(biasl + 16 * jp + 8);
      f32x4_t s1a, s2a, s1b, s2b;
      auto rows = [&](auto all_valid) {
#pragma unroll
        for (int r = 0; r < TH; ++r) {
          const bool valid = decltype(all_valid)::value || (wk.ty0 + r < p.oh && ox < p.ow);
          const f32x4_t va = (f32x4_t){acc[r][8 * jp], acc[r][8 * jp + 1], acc[r][8 * jp + 2], acc[r][8 * jp + 3]} + b0;
          const f32x4_t vb = (f32x4_t){acc[r][8 * jp + 4], acc[r][8 * jp + 5], acc[r][8 * jp + 6], acc[r][8 * jp + 7]} + b1;
          // lanes 32-63 of group 2jp swap with lanes 0-31 of group 2jp+1: lanes 0-31 then hold channels
          // 16 jp + 0..7 (16 contiguous bytes), lanes 32-63 channels 16 jp + 8..15
          const auto sx = __builtin_amdgcn_permlane32_swap(pack16<T>(va[0], va[1]), pack16<T>(vb[0], vb[1]), false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(pack16<T>(va[2], va[3]), pack16<T>(vb[2], vb[3]), false, false);
          const u32x4_t pk = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(pk, ors, valid ? off0 + r * row_bytes + 32 * jp : OOB, 0, NST_W32_ST);
          const f32x4_t xa = valid ? va : (f32x4_t){0.f, 0.f, 0.f, 0.f};
          const f32x4_t xb = valid ? vb : (f32x4_t){0.f, 0.f, 0.f, 0.f};
          if (r == 0) {
            s1a = xa; s2a = xa * xa; s1b = xb; s2b = xb * xb;
          } else {
            s1a = s1a + xa; s2a = __builtin_elementwise_fma(xa, xa, s2a);
            s1b = s1b + xb; s2b = __builtin_elementwise_fma(xb, xb, s2b);
          }
        }
      };
      if (wk.ty0 + TH <= p.oh && wk.tx0 + C::TW <= p.ow) rows(std::true_type{});
      else rows(std::false_type{});
      // 16 statistics {s1, s2} x 8 channels, summed over the 32 pixel lanes of each half: v[2 ci + st]
      const float v[16] = {s1a[0], s2a[0], s1a[1], s2a[1], s1a[2], s2a[2], s1a[3], s2a[3],
                           s1b[0], s2b[0], s1b[1], s2b[1], s1b[2], s2b[2], s1b[3], s2b[3]};
      // rows of 16 lanes: the lower row keeps values 0..7, the upper 8..15, each summed over both rows
      float a8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
        a8[i] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
      }
      const int pr = px & 15, upper = (px >> 4) & 1;
      float a4[4], a2[2], a1[1];
      rs_step<4, 0x140>(a8, a4, pr >= 8);
      rs_step<2, 0x141>(a4, a2, (pr & 4) != 0);
      rs_step<1, 0x1b>(a2, a1, (pr & 2) != 0);
      const float t = a1[0] + dpp_f<0xb1>(a1[0]);
      // even lane pr of row `upper` holds value 8 upper + idx: channel ci = value >> 1, statistic value & 1
      const int idx = 8 * upper + (pr >= 8 ? 4 : 0) + ((pr & 4) ? 2 : 0) + ((pr & 2) ? 1 : 0);
      const int ci = idx >> 1;
      const int co = 32 * wv + 16 * jp + (ci < 4 ? 4 * h + ci : 8 + 4 * h + ci - 4);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t), prs, (pr & 1) ? 0x80000000u : (uint32_t)((co * 2 + (idx & 1)) * 4),
                                            0, 0);
    }
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
  // Micro-step schedule of item k (MFMA slots 24 k + o of a part; a part has 144 MFMAs):
  //   o = 0: wait for the item's LDS-DMA, staging read | 2 + 5 j: IN constants of channel pair j (one pair's
  //   registers at a time) | 5 + 5 j / 6 + 5 j: pair j's lo / hi value | 22: halo write, then the next region's
  //   request of item k, whose source is resolved at 3 / 8 (map reads, offset; not held across parts: registers).
  //   RES / XO store residual-stream piece k < SST (19: halo read, 23: store, after the part's k-th request: SST
  //   stores lie between any item's request and its wait).
  constexpr int SLOTS_PER_ITEM = 24;
  static_assert(SLOTS_PER_ITEM * C::NIT <= 9 * TH * 2 && C::SST <= C::NIT, "micro-step slots");
  Acc acc;
  Staged sy;                 // the staged chunk(s) of the item in flight
  float4 n0;                 // IN constants of one channel pair
  float tl;                  // a pair's lo value between its two micro-steps
  uint32_t o4[4];            // the item's packed output
  int mro = 0, mco = 0;      // map entries of the next tile's item k
  bool padk = false;         // ZPAD: the consumed item k is zero padding (parts 1..3)
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
          auto half = [&](int j, int hi) {  // pair j of the staged chunk, lo (hi = 0) or hi value
            const uint32_t wy = j == 0 ? sy.y.x : j == 1 ? sy.y.y : j == 2 ? sy.y.z : sy.y.w;
            const float4 nn = n0;
            if constexpr (RES) {
              const uint32_t wr = j == 0 ? sy.r.x : j == 1 ? sy.r.y : j == 2 ? sy.r.z : sy.r.w;
              // ResidualBlock join (transformer_net.py:71-76): IN_y(y) + r in fp32, product then sum, one rounding
              if (!hi) {
                tl = lo16<T>(wr) + (lo16<T>(wy) * nn.x + nn.z);
              } else {
                o4[j] = pack16<T>(tl, hi16<T>(wr) + (hi16<T>(wy) * nn.y + nn.w));
              }
            } else if constexpr (FILL == WF_RAW) {
              if (hi) o4[j] = wy;
            } else {
              if (!hi) {
                tl = __builtin_fmaf(lo16<T>(wy), nn.x, nn.z);
              } else {
                const i16x2_t r = __builtin_bit_cast(i16x2_t, pack16<T>(tl, __builtin_fmaf(hi16<T>(wy), nn.y, nn.w)));
                o4[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
              }
            }
          };
          if (o == 0) {
            if (q == 0) vm_wait<KEP>(); else vm_wait<KIN>();
            sy = stage_read(k);
          } else if (o == 2 || o == 7 || o == 12 || o == 17) {
            if (FILL != WF_RAW) n0 = ny[(o - 2) / 5];  // pair j's IN constants, read three MFMAs before its use
          } else if (o == 5 || o == 10 || o == 15 || o == 20) {
            half((o - 5) / 5, 0);
          } else if (o == 6 || o == 11 || o == 16 || o == 21) {
            half((o - 6) / 5, 1);
          } else if (o == 22) {
            const bool pad = ZPAD && (q == 0 ? ((pad3 >> k) & 1u) != 0 : padk);
            const u32x4_t v = {pad ? 0u : o4[0], pad ? 0u : o4[1], pad ? 0u : o4[2], pad ? 0u : o4[3]};
            const bool valid = k < C::NIT - 1 || lane < C::LASTN;
            int eb = item_entry(0) * C::EB + ch * 16;
            asm volatile("" : "+v"(eb));
            *(u32x4_t*)(smem + (valid ? eb + k * IT_STRIDE * C::EB : C::DUMMY_OFF + lane * 16)) = v;
            request(k, q, rvoff);  // region q of nxt
          } else if (o == 3) {
            const int* rowmap = (const int*)(smem + C::MAP_OFF + ns * C::MAPB);
            const bool valid = k < C::NIT - 1 || lane < C::LASTN;
            const int e = valid ? item_entry(k) : 0;
            const int ly = e / C::LW, lx = e - ly * C::LW;
            mro = rowmap[ly];
            mco = rowmap[C::LH + lx];
          } else if (o == 8) {
            const bool valid = k < C::NIT - 1 || lane < C::LASTN;
            const bool in = valid && mro >= 0 && mco >= 0;
            rvoff = in ? (uint32_t)(mro + mco) + (uint32_t)nxt.n * fb + lane_coff : OOB;
            // ZPAD: a zero-padding entry.  Parts 1..3 consume the item they request (nxt's item k: !in); part 3
            // keeps the flags for the next iteration's part 0, which consumes this tile's region 3
            if (ZPAD) {
              padk = valid && !in;
              if (q == 3) pad3 = (pad3 & ~(1u << k)) | (padk ? 1u << k : 0u);
            }
          }
          // the tile after nxt into cur's map slot (cur's sources were resolved in the previous iteration; the
          // barriers ending parts 1..3 publish it before the next iteration's part 0 reads it)
          if (q == 1 && k == 0 && o == 18) build_maps(nxt2, cs);
          if (SOUT && k < C::SST && o == 19) {
            const int cl = lane >> 4, x16 = ((lane & 15) - cl) & 15;
            const int P = 16 * (C::SST * wv + k) + x16;
            sv = *(const u32x4_t*)(smem + (((P >> 5) + 1) * C::LW + (P & 31) + 1) * C::EB + (4 * q + cl) * 16);
          }
          if (SOUT && k < C::SST && o == 23) {
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
    for (int i = 0; i < 7; ++i) g_w32_stamp[(b * 4 + wv) * STAMP_PT + i] = st_acc[i];
#endif
}

template <typename T, int TH, bool RES>
struct Wst32Inst {
  using C = W32Cfg<TH, RES ? WF_RES : WF_NORM>;
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
    hipLaunchKernelGGL((wst32_kernel<T, TH, FILL, ZPAD, XO>), dim3(nb), dim3(C::NT), 0, st, p);
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
    k.ks = 3; k.stride = 1; k.cinp = C::CINP; k.bn = 128; k.th = TH; k.tw = C::TW; k.wm = C::NW; k.wn = 1;
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

#ifndef NST_WST32_TH
#define NST_WST32_TH 8
#endif
// The four instantiations compile ~1.5 min each (fully unrolled 576-MFMA tiles), so the library builds this file
// four times in parallel, NST_W32_PART = 0..3 one (dtype, join) pair each; -1 (experiment builds): all in one object.
#ifndef NST_W32_PART
#define NST_W32_PART -1
#endif
ConvKernelInfo wst32_info_0();
ConvKernelInfo wst32_info_1();
ConvKernelInfo wst32_info_2();
ConvKernelInfo wst32_info_3();
#if NST_W32_PART < 0 || NST_W32_PART == 0
ConvKernelInfo wst32_info_0() { return Wst32Inst<__bf16, NST_WST32_TH, false>::info(); }  // residual trunk
#endif
#if NST_W32_PART < 0 || NST_W32_PART == 1
ConvKernelInfo wst32_info_1() { return Wst32Inst<__bf16, NST_WST32_TH, true>::info(); }   // + residual join in the fill
#endif
#if !NST_W32_MIN && (NST_W32_PART < 0 || NST_W32_PART == 2)
ConvKernelInfo wst32_info_2() { return Wst32Inst<_Float16, NST_WST32_TH, false>::info(); }  // fp16 mode
#endif
#if !NST_W32_MIN && (NST_W32_PART < 0 || NST_W32_PART == 3)
ConvKernelInfo wst32_info_3() { return Wst32Inst<_Float16, NST_WST32_TH, true>::info(); }
#endif
#if NST_W32_PART <= 0
// searched before conv_table_wstat (first match wins); NST_WST32=0 in the environment hides it (A/B runs)
const ConvKernelInfo* conv_table_wst32(int* count) {
  static const ConvKernelInfo table[] = {
      wst32_info_0(),
      wst32_info_1(),
#if !NST_W32_MIN
      wst32_info_2(),
      wst32_info_3(),
#endif
  };
  const char* env = std::getenv("NST_WST32");
  *count = (env != nullptr && env[0] == '0') ? 0 : (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#endif

}  // namespace nst

#if NST_WST32_STAMP
extern "C" int nst_debug_w32_stamps(long long* host, int n) {
  const int cap = 256 * 4 * nst::STAMP_IT * nst::STAMP_PT;
  if (n > cap) n = cap;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(nst::g_w32_stamp), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif
