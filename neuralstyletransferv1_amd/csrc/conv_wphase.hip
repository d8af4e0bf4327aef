// conv_wphase.hip — weight-stationary persistent x2 up-convs as four sub-pixel phases.
//
// Replaces UpsampleConvLayer (transformer_net.py:79-99: nearest x2 + ReflectionPad(1) + 3x3) and
// ConvTranspose2d(3, s2, p1, op1) (transformer_net_nst.py:46-59) for the 128->64 and 64->32
// layers, with the producer's InstanceNorm + ReLU (or the last residual join) in the fill and this
// layer's InstanceNorm partial sums in the epilogue — the conv_wstat.hip machinery applied to the
// phase decomposition of conv_impl.h's MODE_PHASE: output pixel (2y + a, 2x + b) is a 2x2 conv
// over the SOURCE grid with phase-summed weights.
//
//   * workgroup = 8 waves: wave w computes phase (a, b) = ((w & 3) >> 1, w & 1) for output channels
//     half w >> 2 (COUT / 2 channels); its 4 taps x CINP weights stay in registers for the launch.
//   * persistent over (frame, TH x 16 source tiles); the halo (TH+2) x 18 x CINP in LDS (entry stride
//     2 x odd chunks, conflict-free ds_read_b128); halo row y of x-tap tx is the B operand of rows
//     y - ty for both y-taps, so each read feeds two MFMAs per 16-channel subtile.
//   * K order part-major (part q = input channels 32q..32q+31 = one K step per tap); the next tile's
//     halo streams in by LDS-DMA into a 4-slot staging ring (conv_wstat.hip's schedule, generalised
//     to 2, 3 or 4 parts) and is consumed (IN + ReLU / residual join) into each region once freed.
//   * one InstanceNorm partial row per phase and tile (part_rows = 4).
#include <algorithm>
#include <cstring>

#include "conv_ws_common.h"

namespace nst {

constexpr int WP_RING = 3;  // operand reads in flight ahead of the MFMAs
// the conv bias as the C operand of each (row, subtile)'s first MFMA and the epilogue's InstanceNorm sums as packed
// f32 pairs (after the MFMA drain): conv_wstat.hip's epilogue, for the phase kernels whose epilogue is half their VALU
#ifndef NST_WP_BIAS_C
#define NST_WP_BIAS_C 1
#endif
#ifndef NST_WP_PK_STATS
#define NST_WP_PK_STATS 1
#endif
#ifndef NST_WP_PAIR
#define NST_WP_PAIR 1
#endif

template <int CINP, int COUT, int TH, int NF, int SW = 2>
struct WpCfg {  // SW: staged tensors per unit (2: the residual join's y and r, 1: y)
  static constexpr int NW = 8, NT = 512;          // wave w: phase w & 3, channel half w >> 2
  static constexpr int TW = 16;                   // source columns per tile = MFMA column block
  static constexpr int NCH = CINP / 8;            // 16-B chunks per pixel
  static constexpr int NPART = CINP / 32;         // parts: one 32-channel K step per tap
  static constexpr int NUNIT = 2 * NPART;         // half parts: unit u = chunks 2u (team 0), 2u+1 (team 1)
  static constexpr int NSUBW = COUT / 32;         // 16-channel subtiles per wave
  static constexpr int NSTEP = 4 * NPART;         // weight steps per wave: part x tap (2x2)
  static constexpr int LH = TH + 2, LW = TW + 2;  // source halo
  static constexpr int NENT = LH * LW;
  static constexpr int EB = (NCH + 2) * 16;       // 2 x odd chunks
  static constexpr int QENT = NENT / 4;           // entries per wave and unit (four waves per chunk)
  static constexpr int NFMAX = NF;                // frames per launch (IN tables resident in LDS)
  // staging slots: unit u lands in slot u % NSLOT and unit u + 4 is requested once u is consumed, so the ring must
  // divide a tile's units (three parts: one slot per unit)
  static constexpr int NSLOT = NUNIT % 4 == 0 ? 4 : NUNIT;
  static constexpr int SLOTB = SW * NW * 1024;    // [y | r] x wave x lane x 16 B
  static constexpr int MAPB = ((LH + LW) * 4 + 15) / 16 * 16;
  static constexpr int MAP_OFF = NENT * EB;
  static constexpr int NORM_OFF = MAP_OFF + 2 * MAPB;        // [y | r][frame][chunk]{scale[8], shift[8]}
  static constexpr int NORM_TAB = NFMAX * CINP * 8;
  static constexpr int BIAS_OFF = NORM_OFF + 2 * NORM_TAB;
  static constexpr int DUMMY_OFF = BIAS_OFF + COUT * 4;
  static constexpr int STG_OFF = DUMMY_OFF + 64 * 16;
  // output tile staged in LDS for contiguous 16-B stores (when it fits): [row 2TH][pixel 32][COUT
  // channels (+ 32 B pad at 32 channels)], 8-byte slots XOR-swizzled by pixel (swz below): the
  // epilogue's ds_write_b64 and the store pass's ds_read_b128 at most 2-way bank-conflicted (a
  // 16-B pad without swizzle was 4-way / 3-way); NST = 16-B stores per thread
  static constexpr int OUT_OFF = STG_OFF + NSLOT * SLOTB;
  static constexpr int PIXB = COUT * 2, PIXP = COUT == 32 ? PIXB + 32 : PIXB, ROWB = 2 * TW * PIXB;
  static constexpr int SWZ_SH = COUT == 32 ? 2 : 1;
  // even slot offset (keeps 16-B slot pairs together) of staged pixel q (0 .. 2TW-1 within a row)
  static __device__ __forceinline__ int swz(int q) { return 2 * ((q ^ (q >> SWZ_SH)) & (PIXB / 16 - 1)); }
  static constexpr int OUTB = 2 * TH * 2 * TW * PIXP;
  static constexpr bool OST = OUT_OFF + OUTB <= 160 * 1024;
  static constexpr int NST = 2 * TH * ROWB / (NT * 16);
  static constexpr int LDS = OST ? OUT_OFF + OUTB : OUT_OFF;
  static_assert(!OST || NST * NT * 16 == 2 * TH * ROWB, "whole 16-B stores per thread");
  static constexpr int WBYTES = NW * NSTEP * NSUBW * 64 * 16;
  static_assert(CINP % 32 == 0 && COUT % 32 == 0 && NPART >= 2 && NPART <= 4, "channel shapes");
  static_assert(NENT % 4 == 0 && QENT <= 64, "four waves per unit chunk, one item per lane");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// CST: output channels stored (<= COUT; ReCoNet's 96 -> 48 up-conv computes 64 and stores its 48 unpadded)
template <typename T, int CINP, int COUT, int TH, int NF, int FILL, bool ZPAD, int CST = COUT>
__global__ __launch_bounds__(512) void wphase_kernel(ConvParams p) {
  using C = WpCfg<CINP, COUT, TH, NF, (FILL >= WF_RES) ? 2 : 1>;
  constexpr bool RES = FILL >= WF_RES, RN = FILL == WF_RESRN;
  constexpr int U = C::NUNIT, NS = C::NSUBW;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wv >> 2, ph = wv & 3;
  const int g = lane >> 4, px = lane & 15;

  struct Work {
    int n, tile, ty0, tx0;
  };
  const int ntile = p.tiles_x * p.tiles_y;
  auto decode = [&](int wi) {
    Work r;
    r.n = wi / ntile;
    r.tile = wi - r.n * ntile;
    const int ty = r.tile / p.tiles_x;
    r.ty0 = ty * TH;
    r.tx0 = (r.tile - ty * p.tiles_x) * C::TW;
    return r;
  };
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int w0 = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  if (w0 >= p.n_work) return;

  // ---- this wave's phase weights (4 taps x CINP x COUT/2), resident for the launch ----
  uint4 wr[C::NSTEP][NS];
  {
    const uint4* wsrc = (const uint4*)p.wpk + (size_t)wv * C::NSTEP * NS * 64 + lane;
#pragma unroll
    for (int s = 0; s < C::NSTEP; ++s)
#pragma unroll
      for (int t = 0; t < NS; ++t) wr[s][t] = wsrc[(s * NS + t) * 64];
  }
  float* norm_y = (float*)(smem + C::NORM_OFF);
  float* norm_r = norm_y + C::NFMAX * CINP * 2;
  if (FILL != WF_RAW) {
    const int nfr = p.n_work / ntile;
    for (int t = tid; t < nfr * CINP; t += C::NT) {
      const int f = t / CINP, c = t - f * CINP;
      const int o = (f * C::NCH + (c >> 3)) * 16 + (c & 7);
      const float2 v = p.in_norm[(size_t)f * p.cs + c];
      norm_y[o] = v.x;
      norm_y[o + 8] = v.y;
      if (RN) {
        const float2 r = p.res_rnorm[(size_t)f * p.cs + c];
        norm_r[o] = r.x;
        norm_r[o + 8] = r.y;
      }
    }
  }
  if (tid < COUT) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];

  // ---- halo staging (conv_wstat.hip) ----
  // one buffer resource per tensor for the whole launch (the launcher keeps a launch's frames below
  // 2^31 bytes): a frame is a 32-bit offset, no 64-bit scalar math per request
  const uint32_t fb = (uint32_t)p.hs * p.ws * p.cs * 2;
  const uint32_t launch_bytes = fb * (uint32_t)(p.n_work / ntile);
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc((void*)p.in, (short)0, (int)launch_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_r =
      __builtin_amdgcn_make_buffer_rsrc((void*)(RES ? p.res_r : p.in), (short)0, (int)launch_bytes, 0x00020000);
  auto build_maps = [&](const Work& wk, int slot) {
    int* rowmap = (int*)(smem + C::MAP_OFF + slot * C::MAPB);
    int* colmap = rowmap + C::LH;
    const int vy0 = wk.ty0 - p.pad, vx0 = wk.tx0 - p.pad;
    const int pix = p.cs * 2;
    for (int t = tid; t < C::LH + C::LW; t += C::NT) {
      if (t < C::LH) {
        const int sy = map_axis(vy0 + t, p.hs, p.axis_mode, p.pre);
        rowmap[t] = sy < 0 ? -1 : sy * p.ws * pix;
      } else {
        const int sx = map_axis(vx0 + t - C::LH, p.ws, p.axis_mode, p.pre);
        colmap[t - C::LH] = sx < 0 ? -1 : sx * pix;
      }
    }
  };
  // paired units (four parts, at most 32 halo entries per wave and unit): lanes 0-31 stage / consume unit 2p and
  // lanes 32-63 unit 2p + 1, i.e. both 16-channel halves of part p in one request and one consume pass (54 of
  // 64 lanes busy at QENT = 27 instead of 27 of 64: deconv1's fill was VALU-issue-bound on the idle lanes)
  constexpr bool PR = NST_WP_PAIR && C::NPART == 4 && C::QENT <= 32;
  const int plane = PR ? (lane & 31) : lane, phalf = PR ? (lane >> 5) : 0;
  const int ebase = (wv & 3) * C::QENT + plane;
  struct Item {
    int src;
    bool valid;
  };
  auto items = [&](int slot) {
    const int* rowmap = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    const int* colmap = rowmap + C::LH;
    Item it;
    it.valid = plane < C::QENT;
    const int e = it.valid ? ebase : 0;
    const int ly = e / C::LW, lx = e - ly * C::LW;
    const int ro = rowmap[ly], co = colmap[lx];
    it.src = (ro >= 0 && co >= 0) ? ro + co : -1;
    return it;
  };
  const uint32_t stg = (uint32_t)(uintptr_t)(smem + C::STG_OFF) + wv * 1024;
  auto request = [&](int n, int u, const Item& it) {
    const uint32_t voff = (it.valid && it.src >= 0) ? (uint32_t)it.src + (uint32_t)n * fb : 0x80000000u;
    const int soff = (2 * u + team) * 16;
    const uint32_t lds = stg + (u % C::NSLOT) * C::SLOTB;
    dma16(rs_in, voff, lds, soff);
    if constexpr (RES) dma16(rs_r, voff, lds + C::NW * 1024, soff);
  };
  // part pp of the paired form: units 2pp (lanes 0-31) and 2pp + 1 (lanes 32-63), staging slot pp % 2
  auto request_p = [&](int n, int pp, const Item& it) {
    const uint32_t voff =
        (it.valid && it.src >= 0) ? (uint32_t)it.src + (uint32_t)n * fb + 32u * (uint32_t)phalf : 0x80000000u;
    const int soff = (4 * pp + team) * 16;
    const uint32_t lds = stg + (pp % 2) * C::SLOTB;
    dma16(rs_in, voff, lds, soff);
    if constexpr (RES) dma16(rs_r, voff, lds + C::NW * 1024, soff);
  };
  // unit u (this lane's; chunk 2u + team) from staging slot `slot`
  auto consume_s = [&](const Work& wk, int u, int slot, const Item& it) {
    const int ch = 2 * u + team;
    const char* sp = smem + C::STG_OFF + slot * C::SLOTB + (wv * 64 + lane) * 16;
    const uint4 y = *(const uint4*)sp;
    const uint4 rr = RES ? *(const uint4*)(sp + C::NW * 1024) : make_uint4(0u, 0u, 0u, 0u);
    const float* ny = norm_y + (wk.n * C::NCH + ch) * 16;
    const float* nr = norm_r + (wk.n * C::NCH + ch) * 16;
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint32_t o[4];
    if constexpr (RES) {
      // the last residual join IN_y(y) + r (ResidualBlock.forward): product then sum, one rounding
      const uint32_t w2[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float r0 = lo16<T>(w2[j]), r1 = hi16<T>(w2[j]);
        if (RN) {  // ReLU(IN_r(r)) as a normalising fill stages it: one fma, rounded to T
          const uint32_t rn = pack16<T>(__builtin_fmaf(r0, nr[2 * j], nr[8 + 2 * j]),
                                        __builtin_fmaf(r1, nr[2 * j + 1], nr[8 + 2 * j + 1]));
          r0 = fmaxf(lo16<T>(rn), 0.f);
          r1 = fmaxf(hi16<T>(rn), 0.f);
        }
        const float a = lo16<T>(w[j]) * ny[2 * j] + ny[8 + 2 * j];
        const float bb = hi16<T>(w[j]) * ny[2 * j + 1] + ny[8 + 2 * j + 1];
        o[j] = pack16<T>(r0 + a, r1 + bb);
      }
    } else if constexpr (FILL == WF_RAW) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = w[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = __builtin_fmaf(lo16<T>(w[j]), ny[2 * j], ny[8 + 2 * j]);
        const float bb = __builtin_fmaf(hi16<T>(w[j]), ny[2 * j + 1], ny[8 + 2 * j + 1]);
        const i16x2_t r = __builtin_bit_cast(i16x2_t, pack16<T>(a, bb));
        o[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
      }
    }
    const bool pad = ZPAD && it.src < 0;
    const u32x4_t v = {pad ? 0u : o[0], pad ? 0u : o[1], pad ? 0u : o[2], pad ? 0u : o[3]};
    int eb = ebase * C::EB + ch * 16;
    asm volatile("" : "+v"(eb));
    *(u32x4_t*)(smem + (it.valid ? eb : C::DUMMY_OFF + lane * 16)) = v;
  };
  auto consume = [&](const Work& wk, int u, const Item& it) { consume_s(wk, u, u % C::NSLOT, it); };
  auto consume_p = [&](const Work& wk, int pp, const Item& it) { consume_s(wk, 2 * pp + phalf, pp % 2, it); };
  // vmcnt accounting as in conv_wstat.hip: 3 units' requests after unit g's, plus the epilogue's
  // TH * NS output stores and NS partial stores when one lies in between
  constexpr int DPU = RES ? 2 : 1;
  // paired: one part's requests (DPU) after the consumed part's, two parts in flight
  constexpr int KIN = (PR ? 1 : 3) * DPU;
  constexpr int KEP = KIN + (C::OST ? C::NST : TH * NS) + NS;

  // ---- K loop ----
  typedef f32x4_t Acc[TH][NS];
  const int phy = p.ph_off[ph >> 1], phx = p.ph_off[ph & 1];
  const int lbase = (phy * C::LW + phx + px) * C::EB + g * 16;
  constexpr int NRD = TH + 1;   // reads per x-tap
  constexpr int PRD = 2 * NRD;  // reads per part
  auto bread = [&](int i) -> uint4 {  // read i of the tile: (q, tx, y)
    const int q = i / PRD, rem = i - q * PRD;
    const int tx = rem / NRD, y = rem % NRD;
    return *(const uint4*)(smem + lbase + (y * C::LW + tx) * C::EB + 64 * q);
  };
  auto kloop = [&](Acc& acc, auto&& hook, auto&& bound) {
    constexpr int NI = C::NPART * PRD, D = WP_RING;
    f32x4_t bias0[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t)
      bias0[t] = NST_WP_BIAS_C ? *(const f32x4_t*)(smem + C::BIAS_OFF + (team * (COUT / 2) + t * 16 + 4 * g) * 4)
                               : (f32x4_t){0.f, 0.f, 0.f, 0.f};
    auto mfma = [&](f32x4_t& c, const uint4& a, const uint4& bop, bool first, int t) {
      if constexpr (NST_WP_BIAS_C) mfma_tied_c<T>(c, a, bop, first, bias0[t]);
      else mfma_tied<T>(c, a, bop, first);
    };
    uint4 ring[D];
#pragma unroll
    for (int i = 0; i < D; ++i) ring[i] = bread(i);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = i / PRD, rem = i - q * PRD;
      const int tx = rem / NRD, y = rem % NRD;
      const uint4 bcur = ring[i % D];
      // two parts: part 1's region is consumed during part 0, so its reads wait for the part barrier
      const bool defer = C::NPART == 2 && q == 0 && i + D >= PRD;
      if (i + D < NI && !defer) ring[i % D] = bread(i + D);
#pragma unroll
      for (int ty = 0; ty < 2; ++ty) {
        const int r = y - ty;
        if (r < 0 || r >= TH) continue;
#pragma unroll
        for (int t = 0; t < NS; ++t) mfma(acc[r][t], wr[q * 4 + 2 * ty + tx][t], bcur, q == 0 && tx == 0 && ty == 0, t);
      }
      hook(q, rem);
      if (rem == PRD - 1) {
        lds_barrier();
        bound(q);
        if (C::NPART == 2 && q == 0) {
#pragma unroll
          for (int j = 0; j < D; ++j) ring[(i + 1 + j) % D] = bread(i + 1 + j);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: bias, 16-bit NHWC stores of this phase's pixels, one partial row per phase ----
  auto epilogue = [&](const Work& wk, Acc& acc) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // MFMA results -> VALU reads
    const size_t obytes = (size_t)p.oh * p.ow * p.cout_stride * 2;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((char*)p.out + (size_t)wk.n * obytes), (short)0, (int)obytes, 0x00020000);
    const int ox = 2 * (wk.tx0 + px) + (ph & 1);
    const int oy0 = 2 * wk.ty0 + (ph >> 1);
    const uint32_t row2 = (uint32_t)p.ow * p.cout_stride * 2 * 2;  // two output rows
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.partial + (((size_t)wk.n * ntile + wk.tile) * 4 + ph) * p.cout_stride * 2), (short)0,
        p.cout_stride * 8, 0x00020000);
    const bool full = 2 * (wk.ty0 + TH) <= p.oh && 2 * (wk.tx0 + C::TW) <= p.ow;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int c0 = team * (COUT / 2) + t * 16 + 4 * g;
      // a subtile of padding channels (c0 >= CST): its stores and statistics go to the out-of-range offset, still
      // issued (the unit waits count this epilogue's vector-memory instructions)
      const bool live = team * (COUT / 2) + t * 16 < CST;
      const f32x4_t bias = NST_WP_BIAS_C ? (f32x4_t){0.f, 0.f, 0.f, 0.f} : *(const f32x4_t*)(smem + C::BIAS_OFF + c0 * 4);
      const uint32_t off0 = (uint32_t)(((oy0 * p.ow + ox) * p.cout_stride + c0) * 2);
      f32x4_t s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
      auto rows = [&](auto all_valid) {
#pragma unroll
        for (int r = 0; r < TH; ++r) {
          const bool valid = decltype(all_valid)::value || (oy0 + 2 * r < p.oh && ox < p.ow);
          const f32x4_t v = NST_WP_BIAS_C ? acc[r][t] : add4(acc[r][t], bias);
          const u32x2_t pk = {pack16<T>(v[0], v[1]), pack16<T>(v[2], v[3])};
          if constexpr (C::OST) {  // into the LDS output tile: row 2r + a, pixel 2 px + b
            *(u32x2_t*)(smem + C::OUT_OFF + ((2 * r + (ph >> 1)) * 2 * C::TW + 2 * px + (ph & 1)) * C::PIXP +
                        (((c0 >> 2) ^ C::swz(2 * px + (ph & 1))) << 3)) = pk;
          } else {
            __builtin_amdgcn_raw_buffer_store_b64(pk, ors, valid && live ? off0 + r * row2 : 0x80000000u, 0, ST_AUX);
          }
          const f32x4_t x = valid ? v : (f32x4_t){0.f, 0.f, 0.f, 0.f};
          if constexpr (NST_WP_PK_STATS) {
            if (r == 0) {
              s1 = x;
              s2 = x * x;
            } else {
              s1 = s1 + x;
              s2 = __builtin_elementwise_fma(x, x, s2);
            }
          } else {
            stat4(s1, s2, x);
          }
        }
      };
      if (full)
        rows(std::true_type{});
      else
        rows(std::false_type{});
      const float vv[8] = {s1[0], s2[0], s1[1], s2[1], s1[2], s2[2], s1[3], s2[3]};
      float a4[4], a2[2], a1[1];
      rs_step<4, 0x140>(vv, a4, px >= 8);
      rs_step<2, 0x141>(a4, a2, (px & 4) != 0);
      rs_step<1, 0x1b>(a2, a1, (px & 2) != 0);
      const float sv = a1[0] + dpp_f<0xb1>(a1[0]);
      const int idx = (px >= 8 ? 4 : 0) + ((px & 4) ? 2 : 0) + ((px & 2) ? 1 : 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sv), prs,
                                            ((px & 1) || !live) ? 0x80000000u : (uint32_t)(((c0 + (idx >> 1)) * 2 + (idx & 1)) * 4), 0, 0);
    }
    if constexpr (C::OST) {
      // the staged tile as whole rows: 2 TW pixels x COUT channels contiguous in HBM (NHWC,
      // cout_stride == COUT), 16 B per lane
      lds_barrier();
      const int ox0 = 2 * wk.tx0, oyb = 2 * wk.ty0;
#pragma unroll
      for (int k = 0; k < C::NST; ++k) {
        const int off = (k * C::NT + tid) * 16;
        const int row = off / C::ROWB, rem = off - row * C::ROWB;
        const int pix = rem / C::PIXB, cb = rem - pix * C::PIXB;
        const u32x4_t v =
            *(const u32x4_t*)(smem + C::OUT_OFF + (row * 2 * C::TW + pix) * C::PIXP + (((cb >> 3) ^ C::swz(pix)) << 3));
        const int oy = oyb + row, ox = ox0 + pix;
        const bool ok = oy < p.oh && ox < p.ow && cb < CST * 2;
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, ok ? (uint32_t)((oy * p.ow + ox) * CST * 2 + cb) : 0x80000000u, 0, ST_AUX);
      }
    }
  };

  // ---- persistent walk (conv_wstat.hip's, with NPART parts) ----
  Work cur = decode(w0);
  int wn = w0 + G;
  const int last = p.n_work - 1;
  build_maps(cur, 0);
  build_maps(decode(min(wn, last)), 1);
  __syncthreads();
  Item xx = items(0);
  Item xd = xx;
  if constexpr (PR) {
    // parts 0 and 1 in flight; consume parts 0..2, each freeing its slot for the part after next
    request_p(cur.n, 0, xd);
    request_p(cur.n, 1, xd);
    const Work n1 = decode(min(wn, last));
#pragma unroll
    for (int pp = 0; pp < C::NPART - 1; ++pp) {
      vm_wait<0>();
      consume_p(cur, pp, xx);
      if (pp + 2 < C::NPART) {
        request_p(cur.n, pp + 2, xd);
      } else {
        if (pp + 2 == C::NPART) xd = items(1);
        request_p(n1.n, pp + 2 - C::NPART, xd);
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) request(cur.n, u, xd);
    const Work n1 = decode(min(wn, last));
#pragma unroll
    for (int u = 0; u < U - 2; ++u) {
      vm_wait<0>();
      consume(cur, u, xx);
      if (u + 4 < U) {
        request(cur.n, u + 4, xd);
      } else {
        if (u + 4 == U) xd = items(1);
        request(n1.n, u + 4 - U, xd);
      }
    }
  }
  if constexpr (C::NPART == 2) {
    // two parts: the tile after next resolves its sources in part 1 of the first iteration
    __syncthreads();  // every wave is past items(cur) (slot 0)
    build_maps(decode(min(wn + G, last)), 0);
  }
  vm_wait<0>();
  __syncthreads();
  constexpr int POS_A = 0, POS_B = PRD / 2, DT = PRD / 4;
  Acc acc;
  for (int it = 0;; ++it) {
    const bool more = wn < p.n_work;
    const Work nxt = more ? decode(wn) : cur;
    const Work nxt2 = decode(min(wn + G, last));
    const int cs = it & 1, ns = cs ^ 1;
    kloop(
        acc,
        [&](int q, int rem) {
          const int pa = POS_A + (team ? DT : 0), pb = POS_B + (team ? DT : 0);
          if constexpr (PR) {
            // one pass per part: the current tile's last part at part 0 (requesting the next tile's part 1), else
            // the next tile's part q - 1 (requesting part q + 1, or the tile after next's part q - 3)
            if (rem != pa) return;
            if (q == 0) {
              vm_wait<KEP>();
              consume_p(cur, C::NPART - 1, xx);
              request_p(nxt.n, 1, xd);
            } else {
              const int pp = q - 1;
              if (pp == 0) xx = items(ns);
              if (q == 1) vm_wait<KEP>(); else vm_wait<KIN>();
              consume_p(nxt, pp, xx);
              if (pp + 2 < C::NPART) {
                request_p(nxt.n, pp + 2, xd);
              } else {
                if (pp + 2 == C::NPART) xd = items(cs);
                request_p(nxt2.n, pp + 2 - C::NPART, xd);
              }
            }
            return;
          }
          if (rem != pa && rem != pb) return;
          const int half = rem == pa ? 0 : 1;
          if (q == 0) {  // the current tile's last region: units U-2, U-1; request 2, 3 of nxt
            vm_wait<KEP>();
            consume(cur, U - 2 + half, xx);
            request(nxt.n, 2 + half, xd);
          } else {
            const int u = 2 * (q - 1) + half;
            if (u == 0) xx = items(ns);
            if (2 * q + half < 4) vm_wait<KEP>(); else vm_wait<KIN>();
            consume(nxt, u, xx);
            if (u + 4 < U) {
              request(nxt.n, u + 4, xd);
            } else {
              if (u == U - 4) xd = items(cs);
              request(nxt2.n, u + 4 - U, xd);
            }
          }
        },
        [&](int q) {
          if constexpr (C::NPART >= 3) {
            if (q == 0) build_maps(nxt2, cs);  // published by the barrier ending part 1 (read in part 2)
          } else {
            // two parts: the tile after nxt2 into nxt's slot (nxt's sources were resolved in
            // part 1); published by the next iteration's first barrier
            if (q == 1) build_maps(decode(min(wn + 2 * G, last)), ns);
          }
        });
    epilogue(cur, acc);
    if (!more) break;
    cur = nxt;
    wn += G;
  }
  vm_wait<0>();  // no LDS-DMA may land after the workgroup has released its LDS
}

template <typename T, int CINP, int COUT, int TH, int NF, bool RES, int CST = COUT>
struct WphaseInst {
  using C = WpCfg<CINP, COUT, TH, NF, RES ? 2 : 1>;
  static int cus() {
    static const int v = [] {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        c = 256;
      return c;
    }();
    return v;
  }
  template <int FILL, bool ZPAD>
  static void go(const ConvParams& p, int nb, hipStream_t st) {
    hipLaunchKernelGGL((wphase_kernel<T, CINP, COUT, TH, NF, FILL, ZPAD, CST>), dim3(nb), dim3(C::NT), 0, st, p);
  }
  // grid.x = source tiles per frame, grid.y = frames; chunks of <= NFMAX frames per launch
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    const int ntile = (int)grid.x, n = (int)grid.y;
    const size_t fin = (size_t)p0.hs * p0.ws * p0.cs * 2, fout = (size_t)p0.oh * p0.ow * p0.cout_stride * 2;
    // frames per launch: the LDS IN tables' capacity, and a launch's input below 2^31 bytes (32-bit
    // request offsets; 0x80000000 is the out-of-range offset)
    const int fmax = (int)std::min<size_t>(C::NFMAX, (size_t)0x7FFFFF00u / std::max<size_t>(fin, 1));
    if (fmax < 1) return;  // nst_api validates sizes before launching
    for (int f0 = 0; f0 < n; f0 += fmax) {
      const int nf = std::min(fmax, n - f0);
      ConvParams p = p0;
      p.in = (const char*)p0.in + f0 * fin;
      p.out = (char*)p0.out + f0 * fout;
      if (p0.res_r) p.res_r = (const char*)p0.res_r + f0 * fin;
      if (p0.in_norm) p.in_norm = p0.in_norm + (size_t)f0 * p0.cs;
      if (p0.res_rnorm) p.res_rnorm = p0.res_rnorm + (size_t)f0 * p0.cs;
      p.partial = p0.partial + (size_t)f0 * ntile * 4 * p0.cout_stride * 2;
      p.n_work = nf * ntile;
      const int nb = std::min(p.n_work, cus());
      const bool zp = p.axis_mode == AX_ZERO;  // ConvTranspose: zeros past the edge
      if constexpr (RES) {
        // the join of a normalised stream (WF_RESRN) is not instantiated: it spilled (12-16 B of scratch per lane
        // in a counted-vmcnt kernel) and no program reaches it (the up-conv joins the stored x_5; nst_api rejects
        // a normalised residual for this kernel before launching)
        if (p.res_rnorm == nullptr) zp ? go<WF_RES, true>(p, nb, st) : go<WF_RES, false>(p, nb, st);
      } else {
        if (p.in_norm != nullptr)
          zp ? go<WF_NORM, true>(p, nb, st) : go<WF_NORM, false>(p, nb, st);
        else
          zp ? go<WF_RAW, true>(p, nb, st) : go<WF_RAW, false>(p, nb, st);
      }
    }
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = dtype_code<T>();
    k.mode = MODE_WPHASE;
    k.ks = 3; k.stride = 1; k.cinp = CINP; k.bn = CST; k.th = TH; k.tw = C::TW; k.wm = 1; k.wn = C::NW;
    k.bn_k = CST != COUT ? COUT : 0;
    k.in_kind = IN_ACT; k.out_kind = OUT_ACT;
    k.cpc = 8; k.nch = C::NCH; k.lds_bytes = C::LDS;
    k.wbytes = C::WBYTES;
    k.persistent = 1;
    k.part_rows = 4;
    k.res = RES ? 1 : 0;
    k.launch = &launch;
    return k;
  }
};

#ifndef NST_WP1_TH
#define NST_WP1_TH 4
#endif
constexpr int WP1_TH = NST_WP1_TH;  // 128 -> 64: 8 rows spill (6 rows too: 40-52 B of scratch per lane, r04) (128 weight + 64 accumulator VGPRs); 4 leaves LDS room for the staged output tile
constexpr int WP1_NF = 8;  // frames per launch (IN tables in LDS)
#ifndef NST_WPR_TH
#define NST_WPR_TH 6
#endif
constexpr int WPR_TH = NST_WPR_TH;  // ReCoNet 96 -> 64 tile rows: 6 (0.81-0.87 ms per batch of 8) over 4 (0.92-0.97) and 2 (1.38); 8 leaves no LDS for the staged output tile (2.9)
#ifndef NST_WP2_TH
#define NST_WP2_TH 12
#endif
constexpr int WP2_TH = NST_WP2_TH;  // 64 -> 32 tile rows: 12 (540 = 45 tiles) fit with one-tensor slots
#define E(...) WphaseInst<__VA_ARGS__>::info()
const ConvKernelInfo* conv_table_wphase(int* count) {
  static const ConvKernelInfo table[] = {
      //  T     CINP COUT TH NF RES
      E(__bf16, 128, 64, WP1_TH, WP1_NF, false),    // deconv1 / up1
      E(__bf16, 128, 64, WP1_TH, WP1_NF, true),     // deconv1 joining the last residual block (fused join)
      E(__bf16, 64, 32, WP2_TH, 8, false),          // deconv2 / up2
      E(__bf16, 96, 64, WPR_TH, 8, false),          // ReCoNet decoder 96 -> 48 (padded to 64; three parts)
      E(__bf16, 96, 64, WPR_TH, 8, false, 48),      // ... storing its 48 channels unpadded
      E(_Float16, 128, 64, WP1_TH, WP1_NF, false),  // fp16 mode
      E(_Float16, 128, 64, WP1_TH, WP1_NF, true),
      E(_Float16, 64, 32, WP2_TH, 8, false),
      E(_Float16, 96, 64, WPR_TH, 8, false),
      E(_Float16, 96, 64, WPR_TH, 8, false, 48),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E

}  // namespace nst
