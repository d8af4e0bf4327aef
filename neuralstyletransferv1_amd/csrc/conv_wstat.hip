// conv_wstat.hip — weight-stationary residual-trunk conv (3x3, 128 -> 128 channels, stride 1).
//
// Replaces the residual blocks' ConvLayer(128, 128, 3, 1) (transformer_net.py:57-76 res1..res5,
// transformer_net_nst.py:28-43) together with what the generic conv kernel fuses around it: the
// producer's InstanceNorm apply + ReLU (or the residual join, RES) in the fill, this layer's
// InstanceNorm partial sums in the epilogue.
//
// Why a separate kernel: 128 x 1152 bf16 weights are 144 VGPRs per wave when eight waves split the
// output channels 16 each — the whole weight tensor fits in one CU's register file.  So each wave
// loads its 16 channels' weights ONCE per launch and keeps them in registers; the K loop reads only
// pixel operands from LDS, has no weight stream, no weight ring and no per-stage barrier.  The
// generic kernel (conv_impl.h, VAR_WL) spends a barrier every two K steps and half its LDS
// bandwidth on weights.
//
//   * workgroup = 8 waves, two per SIMD, persistent over (frame, tile) work items; tiles of TH rows
//     x 16 pixels: one 16x16x32 MFMA column block per tile row, TH accumulators of 4 fp32 per lane.
//     (v_mfma_f32_16x16x32_bf16 holds a ~13 % higher clock than 32x32x16 under load, MI355X_MICROARCH
//     'DVFS give-back' (7); two waves per SIMD let one wave's fill work run beside its partner's MFMAs.)
//   * halo (TH+2) x 18 entries x 128 channels in LDS, entry stride 288 B (18 chunks, 2 x odd) so the
//     16 lanes of each ds_read_b128 lane group hit 16 distinct bank slots.  Halo row y of x-tap dx is
//     the B operand of tile row y - dy for every y-tap dy: each read feeds up to three MFMAs.
//   * K order part-major: part q = input channels 32q..32q+31 = one K step per tap.  The NEXT tile's
//     halo streams in 8 half-part units while this tile computes: a unit is loaded into registers
//     and written (IN + ReLU / residual join applied) into its region once the barrier ending that
//     part has freed it; team 0 (waves 0-3, even chunks) and team 1 (waves 4-7, odd chunks) do their
//     unit work a quarter part apart, so the two waves of a SIMD never stage at the same time.
//   * a unit chunk is wave-uniform, so its 8 channels' IN constants are one broadcast LDS row.
#include <algorithm>
#include <cstring>

#include "conv_impl.h"

#ifndef WS_RING
#define WS_RING 3  // operand reads in flight ahead of the MFMAs
#endif

namespace nst {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <int TH>
struct WsCfg {
  static constexpr int NW = 8, NT = 512;           // two waves per SIMD, wave w: channels 16w..16w+15
  static constexpr int TW = 16;                    // tile width = MFMA column block
  static constexpr int CINP = 128;
  static constexpr int LH = TH + 2, LW = TW + 2;   // 3x3 halo
  static constexpr int NENT = LH * LW;
  static constexpr int EB = 288;                   // bytes per LDS entry: 16 chunks + 2 pad chunks
  static constexpr int NSTEP = 36;                 // 4 parts x 9 taps (K = 32 per step)
  static constexpr int NUNIT = 8;                  // half parts: unit u = chunks 2u (team 0), 2u+1 (team 1)
  static constexpr int QENT = NENT / 4;            // entries per wave and unit (four waves per chunk)
  static constexpr int IPL = (QENT + 63) / 64;     // items per lane and unit
  static constexpr int MAPB = ((LH + LW) * 4 + 15) / 16 * 16;
  static constexpr int MAP_OFF = NENT * EB;
  static constexpr int NORM_OFF = MAP_OFF + 2 * MAPB;  // 2 slots x {y, r} x 16 chunks x {scale[8], shift[8]}
  static constexpr int NORM_SLOT = 2 * CINP * 8;
  static constexpr int BIAS_OFF = NORM_OFF + 2 * NORM_SLOT;  // 128 fp32
  static constexpr int DUMMY_OFF = BIAS_OFF + CINP * 4;      // sink of the lanes without an item
  static constexpr int LDS = DUMMY_OFF + 64 * 16;
  static constexpr int WBYTES = NW * NSTEP * 64 * 16;  // packed weights
  static_assert(NENT % 4 == 0, "four waves per unit chunk");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// what the fill applies to a staged input chunk
enum WsFill { WF_NORM = 0, WF_RAW = 1, WF_RES = 2, WF_RESRN = 3 };  // IN+ReLU / identity / join / join of ReLU(IN(r))

template <int TH, int FILL>
__global__ __launch_bounds__(512) void wstat_kernel(ConvParams p) {
  using C = WsCfg<TH>;
  constexpr bool RES = FILL >= WF_RES, RN = FILL == WF_RESRN;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wv >> 2;
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
  // workgroups b, b+8, ... share an XCD (round-robin dispatch): each XCD gets a contiguous run of
  // tiles per sweep so neighbouring halos meet in its L2
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int w0 = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  if (w0 >= p.n_work) return;

  // ---- this wave's 16 output channels x 1152 K of weights, resident for the whole launch ----
  uint4 wr[C::NSTEP];
  {
    const uint4* wsrc = (const uint4*)p.wpk + (size_t)wv * C::NSTEP * 64 + lane;
#pragma unroll
    for (int s = 0; s < C::NSTEP; ++s) wr[s] = wsrc[s * 64];
  }

  // ---- halo staging ----
  const size_t frame_bytes = (size_t)p.hs * p.ws * p.cs * 2;
  auto frame_rsrc = [&](const void* base, int n) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (size_t)n * frame_bytes), (short)0,
                                             (int)frame_bytes, 0x00020000);
  };
  auto build_maps = [&](const Work& wk, int slot) {
    int* rowmap = (int*)(smem + C::MAP_OFF + slot * C::MAPB);
    int* colmap = rowmap + C::LH;
    const int vy0 = wk.ty0 - p.pad, vx0 = wk.tx0 - p.pad;
    const int pix = p.cs * 2;
    // the tile's frame's IN constants (producer, or residual y), per chunk as scale[8], shift[8]
    float* norm_l = (float*)(smem + C::NORM_OFF + slot * C::NORM_SLOT);
    if (FILL != WF_RAW && tid < C::CINP) {
      const float2 v = p.in_norm[(size_t)wk.n * p.cs + tid];
      norm_l[(tid >> 3) * 16 + (tid & 7)] = v.x;
      norm_l[(tid >> 3) * 16 + 8 + (tid & 7)] = v.y;
      if (RN) {  // the residual's own IN (+ReLU): block 1's x_0 = ReLU(IN(conv3)) is not materialised
        const float2 r = p.res_rnorm[(size_t)wk.n * p.cs + tid];
        norm_l[2 * C::CINP + (tid >> 3) * 16 + (tid & 7)] = r.x;
        norm_l[2 * C::CINP + (tid >> 3) * 16 + 8 + (tid & 7)] = r.y;
      }
    }
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
  // item k of this lane in every unit: entry ebase + 64k of chunk 2u + team; psrc = its byte offset
  // in the frame (chunk 0), -1 = zero padding; pvalid / pint bit k: the item exists / is one of the
  // tile's own pixels (RES: residual-stream write).  Branch-free, so it can sit between MFMAs.
  const int ebase = (wv & 3) * C::QENT + lane;
  int psrc[C::IPL];
  unsigned pvalid = 0, pint = 0;
  auto items = [&](const Work& wk, int slot) {
    const int* rowmap = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    const int* colmap = rowmap + C::LH;
    pvalid = 0;
    pint = 0;
#pragma unroll
    for (int k = 0; k < C::IPL; ++k) {
      const bool ok = lane + 64 * k < C::QENT;
      const int e = ok ? ebase + 64 * k : 0;
      const int ly = e / C::LW, lx = e - ly * C::LW;
      const int ro = rowmap[ly], co = colmap[lx];
      psrc[k] = (ro >= 0 && co >= 0) ? ro + co : -1;
      pvalid |= (ok ? 1u : 0u) << k;
      const bool in = ok && ly >= p.pad && ly < p.pad + TH && lx >= p.pad && lx < p.pad + C::TW &&
                      wk.ty0 + ly - p.pad < p.oh && wk.tx0 + lx - p.pad < p.ow;
      pint |= (in ? 1u : 0u) << k;
    }
  };
  uint4 praw[C::IPL], praw2[C::IPL];
  auto issue_unit = [&](int n, int u) {
#ifdef WS_NOLOAD  // experiment: no fill loads (measures the rest of the pipeline)
    for (int k = 0; k < C::IPL; ++k) { praw[k] = make_uint4(0u, 0u, 0u, 0u); praw2[k] = praw[k]; }
    return;
#endif
    const int soff = (2 * u + team) * 16;  // the unit's chunk for this wave
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc(p.in, n);
#pragma unroll
    for (int k = 0; k < C::IPL; ++k)
      praw[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, psrc[k] > 0 ? psrc[k] : 0, soff, 0));
    if constexpr (RES) {
      const __amdgpu_buffer_rsrc_t rs2 = frame_rsrc(p.res_r, n);
#pragma unroll
      for (int k = 0; k < C::IPL; ++k)
        praw2[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs2, psrc[k] > 0 ? psrc[k] : 0, soff, 0));
    }
  };
  // live = false: a restaging pass past the last work item (LDS only, no residual-stream stores)
  auto write_unit = [&](const Work& wk, int slot, int u, bool live) {
    const int ch = 2 * u + team;
    // the chunk's 8 scales and 8 shifts: one wave-uniform (broadcast) LDS row
    const float* nl = (const float*)(smem + C::NORM_OFF + slot * C::NORM_SLOT) + ch * 16;
    float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = nl[j];
      sh[j] = nl[8 + j];
      rsc[j] = RN ? nl[2 * C::CINP + j] : 1.f;
      rsh[j] = RN ? nl[2 * C::CINP + 8 + j] : 0.f;
    }
    const __amdgpu_buffer_rsrc_t ro = frame_rsrc(p.res_out, wk.n);
    int eb = ebase * C::EB + ch * 16;  // recomputed per unit, not held across the loop
    asm volatile("" : "+v"(eb));
#pragma unroll
    for (int k = 0; k < C::IPL; ++k) {
      const uint32_t w[4] = {praw[k].x, praw[k].y, praw[k].z, praw[k].w};
      uint32_t o[4];
      if constexpr (RES) {
        // ResidualBlock join (transformer_net.py:71-76): IN_y(y) + r in fp32, product then sum
        // (the file is built with -ffp-contract=off), one rounding — as res_chunk / residual_kernel
        const uint32_t wr2[4] = {praw2[k].x, praw2[k].y, praw2[k].z, praw2[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float r0 = bf16_lo(wr2[j]), r1 = bf16_hi(wr2[j]);
          if (RN) {
            r0 = fmaxf(r0 * rsc[2 * j] + rsh[2 * j], 0.f);
            r1 = fmaxf(r1 * rsc[2 * j + 1] + rsh[2 * j + 1], 0.f);
          }
          const float a = bf16_lo(w[j]) * sc[2 * j] + sh[2 * j];
          const float bb = bf16_hi(w[j]) * sc[2 * j + 1] + sh[2 * j + 1];
          o[j] = pack_bf16(r0 + a, r1 + bb);
        }
      } else if constexpr (FILL == WF_RAW) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = w[j];
      } else {
        // producer IN apply + ReLU, as norm_chunk
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = __builtin_fmaf(bf16_lo(w[j]), sc[2 * j], sh[2 * j]);
          const float bb = __builtin_fmaf(bf16_hi(w[j]), sc[2 * j + 1], sh[2 * j + 1]);
          const i16x2_t r = __builtin_bit_cast(i16x2_t, pack_bf16(a, bb));
          o[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
        }
      }
      const bool pad = psrc[k] < 0;  // zero padding stays zero (pad after IN + ReLU)
      const u32x4_t v = {pad ? 0u : o[0], pad ? 0u : o[1], pad ? 0u : o[2], pad ? 0u : o[3]};
      if constexpr (RES) {
        const bool own = live && ((pint >> k) & 1u);
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, own ? (uint32_t)(psrc[k] + ch * 16) : 0x80000000u, 0, 0);
      }
      const bool valid = (pvalid >> k) & 1u;
      const int dst = valid ? eb + 64 * k * C::EB : C::DUMMY_OFF + lane * 16;
      *(u32x4_t*)(smem + dst) = v;
    }
  };

  // ---- K loop ----
  typedef f32x4_t Acc[TH];
  const int lbase = px * C::EB + g * 16;
  // K order inside part q: x-tap dx, then halo row y.  LDS row y of x-tap dx is the B operand of
  // tile row r = y - dy for every y-tap dy, so each ds_read_b128 feeds up to three MFMAs.
  constexpr int NRD = TH + 2;   // reads per dx
  constexpr int PRD = 3 * NRD;  // reads per part
  auto bread = [&](int i) -> uint4 {  // read i of the tile: (q, dx, y)
    const int q = i / PRD, rem = i - q * PRD;
    const int dx = rem / NRD, y = rem % NRD;
    return *(const uint4*)(smem + lbase + (y * C::LW + dx) * C::EB + 64 * q);
  };
  auto kloop = [&](Acc& acc, auto&& hook, auto&& bound) {
    {  // accumulators start at the bias of this lane's 4 channels
      const f32x4_t bv = *(const f32x4_t*)(smem + C::BIAS_OFF + (16 * wv + 4 * g) * 4);
#pragma unroll
      for (int r = 0; r < TH; ++r) acc[r] = bv;
    }
    constexpr int NI = 4 * PRD, D = WS_RING;
    uint4 ring[D];
#pragma unroll
    for (int i = 0; i < D; ++i) ring[i] = bread(i);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = i / PRD, rem = i - q * PRD;
      const int dx = rem / NRD, y = rem % NRD;
      const uint4 bcur = ring[i % D];
      if (i + D < NI) ring[i % D] = bread(i + D);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int r = y - dy;
        if (r < 0 || r >= TH) continue;
        const int s = q * 9 + 3 * dy + dx;  // packed weight step
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wr[s]),
                                                         __builtin_bit_cast(bf16x8_t, bcur), acc[r], 0, 0, 0);
      }
#ifndef WS_NOHOOK  // experiment: K loop + epilogue only
#ifndef WS_NOUNIT  // experiment: barriers but no unit work
      hook(q, rem);
#endif
      if (rem == PRD - 1) {
#ifndef WS_NOBAR  // experiment: unit work without barriers (racy: timing only)
        __syncthreads();  // every wave is past its reads of part q
#endif
        bound(q);
      }
#endif
      // pin the order: read i + D with read i's MFMAs (the scheduler otherwise pulls every read
      // down next to its consumers, exposing the LDS latency on each one)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: bf16 NHWC store (bias is the accumulators' initial value), InstanceNorm partial
  // sums: lane (px, g) holds channels 16 wv + 4g .. +3 of pixel px of every tile row ----
  auto epilogue = [&](const Work& wk, Acc& acc) {
    const int c0 = 16 * wv + 4 * g;
    const size_t obytes = (size_t)p.oh * p.ow * p.cout_stride * 2;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((char*)p.out + (size_t)wk.n * obytes), (short)0, (int)obytes, 0x00020000);
    const int ox = wk.tx0 + px;
    float vv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] = 0.f;
#pragma unroll
    for (int r = 0; r < TH; ++r) {
      const int oy = wk.ty0 + r;
      const bool valid = oy < p.oh && ox < p.ow;
      const f32x4_t v = acc[r];
      const uint32_t off = valid ? (uint32_t)(((oy * p.ow + ox) * p.cout_stride + c0) * 2) : 0x80000000u;
      const u32x2_t pk = {pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3])};
      __builtin_amdgcn_raw_buffer_store_b64(pk, ors, off, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = valid ? v[e] : 0.f;
        vv[2 * e] += x;
        vv[2 * e + 1] = __builtin_fmaf(x, x, vv[2 * e + 1]);
      }
    }
    if (p.partial != nullptr) {
      // reduce-scatter of the 8 statistics over the 16 pixel lanes of the DPP row, then the xor-1
      // partner: lane px (even) ends with statistic idx & 1 of channel c0 + (idx >> 1),
      // idx = 4 (px >= 8) + 2 (px & 4) + (px & 2) / 2
      float a4[4], a2[2], a1[1];
      rs_step<4, 0x140>(vv, a4, px >= 8);
      rs_step<2, 0x141>(a4, a2, (px & 4) != 0);
      rs_step<1, 0x1b>(a2, a1, (px & 2) != 0);
      const float t = a1[0] + dpp_f<0xb1>(a1[0]);
      const int idx = (px >= 8 ? 4 : 0) + ((px & 4) ? 2 : 0) + ((px & 2) ? 1 : 0);
      if ((px & 1) == 0)
        p.partial[(((size_t)wk.n * ntile + wk.tile) * p.cout_stride + c0 + (idx >> 1)) * 2 + (idx & 1)] = t;
    }
  };

  // ---- persistent walk ----
  if (tid < C::CINP) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];
  Work cur = decode(w0);
  int wn = w0 + G;
  const int last = p.n_work - 1;
  build_maps(cur, 0);
  build_maps(decode(min(wn, last)), 1);
  __syncthreads();
  items(cur, 0);
  // units 0..5 now; unit 6 stays in flight and is written in part 0 like every later tile's
#pragma unroll
  for (int u = 0; u < C::NUNIT - 1; ++u) {
    issue_unit(cur.n, u);
    if (u + 2 < C::NUNIT) write_unit(cur, 0, u, true);
    __builtin_amdgcn_sched_barrier(0);  // one unit's loads in flight at a time
  }
  __syncthreads();
  // Unit schedule (u = 2q + half; region q is free once the barrier ending part q has passed):
  //   part 0: A: write 6 of cur, load 7 | B: write 7 of cur, next tile's item sources, load 0
  //   part q = 1..3: A: write 2q-2, load 2q-1 | B: write 2q-1, load 2q      (of the next tile)
  // so every unit's loads have half a part of MFMAs to land.  A is right after the part's first
  // reads, B half a part later; team 1 runs a quarter part behind team 0.
  constexpr int POS_A = 0, POS_B = PRD / 2, DT = PRD / 4;
  Acc acc;
  for (int it = 0;; ++it) {
    // past the last work item the hooks restage LDS with whatever the next-tile slots hold (never
    // read again) and store nothing, so they need no branch
    const bool more = wn < p.n_work;
    const Work nxt = more ? decode(wn) : cur;
    const int cs = it & 1, ns = cs ^ 1;  // map / IN-table slots of cur and nxt
    kloop(
        acc,
        [&](int q, int rem) {  // after read rem of part q
          const int pa = POS_A + (team ? DT : 0), pb = POS_B + (team ? DT : 0);
          if (q == 0) {
            if (rem == pa) {
              write_unit(cur, cs, 6, true);
              issue_unit(cur.n, 7);
            }
            if (rem == pb) {
              write_unit(cur, cs, 7, true);
              items(nxt, ns);
              issue_unit(nxt.n, 0);
            }
          } else {
            if (rem == pa) {
              write_unit(nxt, ns, 2 * q - 2, more);
              issue_unit(nxt.n, 2 * q - 1);
            }
            if (rem == pb) {
              write_unit(nxt, ns, 2 * q - 1, more);
              issue_unit(nxt.n, 2 * q);
            }
          }
        },
        [&](int q) {  // after the barrier that ends part q
          // the tile after nxt into cur's slot: its last reader (cur's units 6/7) ran in part 0, and
          // the barriers ending parts 2 and 3 publish it before nxt's part 0 reads it (items)
          if (q == 1) build_maps(decode(min(wn + G, last)), cs);
        });
    epilogue(cur, acc);
    if (!more) break;
    cur = nxt;
    wn += G;
  }
}

template <int TH, bool RES>
struct WstatInst {
  using C = WsCfg<TH>;
  static int cus() {
    static const int v = [] {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        c = 256;
      return c;
    }();
    return v;
  }
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    ConvParams p = p0;
    p.n_work = (int)(grid.x * grid.y);
    const int nb = std::min(p.n_work, cus());  // one workgroup per CU (registers)
    if constexpr (RES) {
      if (p.res_rnorm != nullptr)  // block 1's join: the residual is ReLU(IN(conv3)), applied here
        hipLaunchKernelGGL((wstat_kernel<TH, WF_RESRN>), dim3(nb), dim3(C::NT), 0, st, p);
      else
        hipLaunchKernelGGL((wstat_kernel<TH, WF_RES>), dim3(nb), dim3(C::NT), 0, st, p);
    } else {
      if (p.in_norm != nullptr)
        hipLaunchKernelGGL((wstat_kernel<TH, WF_NORM>), dim3(nb), dim3(C::NT), 0, st, p);
      else  // the residual stream itself (unfused joins)
        hipLaunchKernelGGL((wstat_kernel<TH, WF_RAW>), dim3(nb), dim3(C::NT), 0, st, p);
    }
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = NST_DT_BF16;
    k.mode = MODE_WSTAT;
    k.ks = 3; k.stride = 1; k.cinp = C::CINP; k.bn = 128; k.th = TH; k.tw = C::TW; k.wm = C::NW; k.wn = 1;
    k.in_kind = IN_ACT; k.out_kind = OUT_ACT;
    k.cpc = 8; k.nch = 16; k.lds_bytes = C::LDS;
    k.wbytes = C::WBYTES;
    k.persistent = 1;
    k.part_rows = 1;
    k.res = RES ? 1 : 0;
    k.launch = &launch;
    return k;
  }
};

#ifndef NST_WSTAT_TH
#define NST_WSTAT_TH 8
#endif
#define E(...) WstatInst<__VA_ARGS__>::info()
const ConvKernelInfo* conv_table_wstat(int* count) {
  static const ConvKernelInfo table[] = {
      E(NST_WSTAT_TH, false),  // residual trunk
      E(NST_WSTAT_TH, true),   // + residual join in the fill
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E

}  // namespace nst
