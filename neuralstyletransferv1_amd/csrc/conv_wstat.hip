// conv_wstat.hip — weight-stationary residual-trunk conv (3x3, 128 -> 128 channels, stride 1).
//
// Replaces the residual blocks' ConvLayer(128, 128, 3, 1) (transformer_net.py:57-76 res1..res5,
// transformer_net_nst.py:28-43) together with what the generic conv kernel fuses around it: the
// producer's InstanceNorm apply + ReLU (or the residual join, RES) in the fill, this layer's
// InstanceNorm partial sums in the epilogue.
//
// Why a separate kernel: 128 x 1152 16-bit (bf16 / fp16) weights are 144 VGPRs per wave when eight waves split the
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

#include "conv_ws_common.h"

namespace nst {

#ifndef NST_WS_RING
#define NST_WS_RING 3
#endif
constexpr int WS_RING = NST_WS_RING;  // operand reads in flight ahead of the MFMAs
constexpr int WS_SPLIT = 1;  // read steps between a unit's staging read and its transform (0: back to back)
constexpr uint32_t OOB = 0xFFFFFF00u;  // buffer offset past every launch's records: loads 0, stores dropped
// the conv bias enters as the C operand of each tile row's first MFMA (bias + the K sum in the accumulator, one
// rounding per MFMA as before) instead of 32 epilogue adds per wave and tile
#ifndef NST_WS_BIAS_C
#define NST_WS_BIAS_C 1
#endif
// the epilogue's InstanceNorm sums as packed f32 pairs (v_pk_add_f32 / v_pk_fma_f32, no MFMA of this wave in flight)
#ifndef NST_WS_PK_STATS
#define NST_WS_PK_STATS 1
#endif
// experiment switches (tools/build_variants.sh): the join's IN apply as one fma per value (NOT the unfused residual
// kernel's product-then-sum arithmetic: off in the product), and s_setprio 1 for team 1 (waves 4-7, the second
// half of the workgroup: MI355X_MICROARCH.md 'Two waves per SIMD' item 4)
#ifndef NST_WS_JOIN_FMA
#define NST_WS_JOIN_FMA 0
#endif
#ifndef NST_WS_PRIO
#define NST_WS_PRIO 0
#endif

template <int TH, int FILL>
struct WsCfg {
  static constexpr bool RES = FILL == WF_RES;
  static constexpr int NW = 8, NT = 512;           // two waves per SIMD, wave w: channels 16w..16w+15
  static constexpr int TW = 16;                    // tile width = MFMA column block
  static constexpr int CINP = 128;
  static constexpr int LH = TH + 2, LW = TW + 2;   // 3x3 halo
  static constexpr int NENT = LH * LW;
  static constexpr int EB = 288;                   // bytes per LDS entry: 16 chunks + 2 pad chunks
  static constexpr int NSTEP = 36;                 // 4 parts x 9 taps (K = 32 per step)
  static constexpr int NUNIT = 8;                  // half parts: unit u = chunks 2u (team 0), 2u+1 (team 1)
  static constexpr int QENT = NENT / 4;            // entries per wave and unit (four waves per chunk)
  static constexpr int NFMAX = RES ? 8 : 16;       // frames per launch (IN tables resident in LDS)
  static constexpr int NSLOT = 4;                  // staging slots: units in flight
  static constexpr int SLOTB = (RES ? 2 : 1) * NW * 1024;  // a slot: [y | r] x wave x lane x 16 B
  static constexpr int MAPB = ((LH + LW) * 4 + 15) / 16 * 16;
  static constexpr int MAP_OFF = NENT * EB;
  static constexpr int NORM_OFF = MAP_OFF + 2 * MAPB;        // [y | r][frame][channel] float2
  static constexpr int NORM_TAB = NFMAX * CINP * 8;
  static constexpr int BIAS_OFF = NORM_OFF + NORM_TAB;  // 128 fp32
  static constexpr int DUMMY_OFF = BIAS_OFF + CINP * 4;      // sink of the lanes without an item
  static constexpr int STG_OFF = DUMMY_OFF + 64 * 16;
  // output tile staged in LDS (when it fits: not the ReLU(IN(r)) join) for whole-pixel 16-B
  // stores: [row][px][256 B], 8-byte slot s (wave w, lane group g: s = 4w + g) at s ^ 2 (px & 7): the
  // epilogue's ds_write_b64 2-way bank-conflicted (the former 32-byte wave-slot swizzle: 4-way)
  static constexpr int OUT_OFF = STG_OFF + NSLOT * SLOTB;
  static constexpr int OUTB = TH * TW * 256;
  static constexpr bool OST = OUT_OFF + OUTB <= 160 * 1024;
  static constexpr int NST = OUTB / (NT * 16);  // 16-B stores per thread
  static constexpr int LDS = OST ? OUT_OFF + OUTB : OUT_OFF;
  static constexpr int WBYTES = NW * NSTEP * 64 * 16;  // packed weights
  static_assert(NENT % 4 == 0 && QENT <= 64, "four waves per unit chunk, one item per lane");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// XO: a WF_NORM fill also writes what it staged for the tile's own pixels (ReLU(IN(y)), the first
// residual block's input x_0) to res_out, so the next join reads x_0 instead of re-normalising
template <typename T, int TH, int FILL, bool ZPAD, bool XO>
__global__ __launch_bounds__(512) void wstat_kernel(ConvParams p) {
  using C = WsCfg<TH, FILL>;
  constexpr bool RES = C::RES;
  static_assert(!XO || FILL == WF_NORM, "x_0 export is a normalising fill");
  constexpr bool SOUT = RES || XO;  // residual-stream stores from the halo
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wv >> 2;
  const int g = lane >> 4, px = lane & 15;

  struct Work {
    int n, tile, ty0, tx0;
  };
  const int ntile = p.tiles_x * p.tiles_y;
  const int nfr = p.n_work / ntile;  // frames in this launch
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
  // ---- the launch's IN constants (<= NFMAX frames) and bias, resident in LDS ----
  // per frame and 8-channel chunk: 4 x {scale lo, scale hi, shift lo, shift hi} (one ds_read_b128 per
  // channel pair, read right before its use: few registers live in the fill)
  float* norm_y = (float*)(smem + C::NORM_OFF);
  if (FILL != WF_RAW) {
    for (int t = tid; t < nfr * C::CINP; t += C::NT) {
      const int f = t / C::CINP, c = t - f * C::CINP;
      // chunk layout: per channel pair j = (c & 7) >> 1: {scale lo, scale hi, shift lo, shift hi}
      const int o = (f * 16 + (c >> 3)) * 16 + 4 * ((c & 7) >> 1) + (c & 1);
      const float2 v = p.in_norm[(size_t)f * p.cs + c];
      norm_y[o] = v.x;
      norm_y[o + 2] = v.y;
    }
  }
  if (tid < C::CINP) ((float*)(smem + C::BIAS_OFF))[tid] = p.bias[tid];

  // ---- halo staging ----
  // one buffer resource per tensor for the whole launch (the launcher keeps a launch's frames within
  // 32-bit offsets): a frame is a 32-bit offset, nothing per request is 64-bit scalar math
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
  // this lane's item in every unit of a tile: entry ebase of chunk 2u + team.  voff = its byte offset
  // in the launch's input (chunk 0), OOB = zero padding (reads 0); valid: the entry exists
  const int ebase = (wv & 3) * C::QENT + lane;
  struct Item {
    uint32_t voff;
    bool valid;
  };
  auto items = [&](const Work& wk, int slot) {
    const int* rowmap = (const int*)(smem + C::MAP_OFF + slot * C::MAPB);
    const int* colmap = rowmap + C::LH;
    Item it;
    it.valid = lane < C::QENT;
    const int e = it.valid ? ebase : 0;
    const int ly = e / C::LW, lx = e - ly * C::LW;
    const int ro = rowmap[ly], co = colmap[lx];
    it.voff = (it.valid && ro >= 0 && co >= 0) ? (uint32_t)(ro + co) + (uint32_t)wk.n * fb : OOB;
    return it;
  };
  // Units travel by LDS-DMA (buffer_load ... lds: no VGPR destination) into a 4-slot staging ring:
  // unit g + 4 is requested right after unit g is consumed, so every unit has two parts of MFMAs to
  // land.  Each lane reads back only its own 16 bytes, so only this wave's vmcnt orders them.  The
  // loads are asm, invisible to hipcc's wait counting, and every vector-memory instruction issues in
  // order: before unit g is consumed, vmcnt(K) with K = the instructions this wave issued after
  // unit g's requests — 3 units' requests, 2 residual-stream region stores (RES), and the
  // epilogue's TH + 1 stores when one lies in between (units 0, 1, 6, 7).  Any extra instruction
  // hipcc adds only makes such a wait stricter.
  const uint32_t stg = (uint32_t)(uintptr_t)(smem + C::STG_OFF) + wv * 1024;
  const __amdgpu_buffer_rsrc_t rs_in = launch_rsrc(p.in, fb);
  const __amdgpu_buffer_rsrc_t rs_r = launch_rsrc(RES ? p.res_r : p.in, fb);
  auto request = [&](int u, const Item& it) {
    const int soff = (2 * u + team) * 16;  // the unit's chunk
    const uint32_t lds = stg + (u % C::NSLOT) * C::SLOTB;
    dma16(rs_in, it.voff, lds, soff);
    if constexpr (RES) dma16(rs_r, it.voff, lds + C::NW * 1024, soff);
  };
  // unit u's staged chunk (this lane's 16 B of the input, and of the residual stream for RES), read
  // WS_SPLIT read steps before its transform so the LDS latency runs under MFMAs
  struct Staged {
    uint4 y, r;
  };
  auto stage_read = [&](int u) {
    const char* sp = smem + C::STG_OFF + (u % C::NSLOT) * C::SLOTB + (wv * 64 + lane) * 16;
    Staged st;
    st.y = *(const uint4*)sp;
    st.r = RES ? *(const uint4*)(sp + C::NW * 1024) : make_uint4(0u, 0u, 0u, 0u);
    return st;
  };
  // consume unit u of tile wk: IN + ReLU / residual join of the staged chunk into the halo.
  auto consume = [&](const Work& wk, int u, const Item& it, const Staged& st) {
    const int ch = 2 * u + team;
    const uint4 y = st.y, rr = st.r;
    const float4* ny = (const float4*)(norm_y + (wk.n * 16 + ch) * 16);  // per pair: {scale lo, hi, shift lo, hi}
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint32_t o[4];
    if constexpr (RES) {
      // ResidualBlock join (transformer_net.py:71-76): IN_y(y) + r in fp32, product then sum (the
      // file is built with -ffp-contract=off), one rounding — as res_chunk / residual_kernel
      const uint32_t w2[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float r0 = lo16<T>(w2[j]), r1 = hi16<T>(w2[j]);
        const float4 n = ny[j];
        const float a = NST_WS_JOIN_FMA ? __builtin_fmaf(lo16<T>(w[j]), n.x, n.z) : lo16<T>(w[j]) * n.x + n.z;
        const float bb = NST_WS_JOIN_FMA ? __builtin_fmaf(hi16<T>(w[j]), n.y, n.w) : hi16<T>(w[j]) * n.y + n.w;
        o[j] = pack16<T>(r0 + a, r1 + bb);
      }
    } else if constexpr (FILL == WF_RAW) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = w[j];
    } else {
      // producer IN apply + ReLU, as norm_chunk
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 n = ny[j];
        const float a = __builtin_fmaf(lo16<T>(w[j]), n.x, n.z);
        const float bb = __builtin_fmaf(hi16<T>(w[j]), n.y, n.w);
        const i16x2_t r = __builtin_bit_cast(i16x2_t, pack16<T>(a, bb));
        o[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(r, (i16x2_t){0, 0}));
      }
    }
    const bool pad = ZPAD && it.voff == OOB;  // zero padding stays zero (pad after IN + ReLU); reflection never pads
    const u32x4_t v = {pad ? 0u : o[0], pad ? 0u : o[1], pad ? 0u : o[2], pad ? 0u : o[3]};
    int eb = ebase * C::EB + ch * 16;  // recomputed per unit, not held across the loop
    asm volatile("" : "+v"(eb));
    *(u32x4_t*)(smem + (it.valid ? eb : C::DUMMY_OFF + lane * 16)) = v;
  };
  // RES / XO: the joined residual stream x_{k+1} (x_0) of the tile's own pixels goes to res_out from the halo,
  // region by region (region q during part q: complete since unit 2q+1 was consumed, overwritten
  // only in part q+1), as 64-byte pixel quarters — one store per lane and part, instead of 16-byte
  // pieces per unit (which cost as much as the rest of the join)
  auto store_region = [&](const Work& wk, int q) {
    const int pix = tid >> 2, c = 4 * q + (tid & 3);  // 128 pixels x 4 chunks
    const int r = pix >> 4, x = pix & 15;
    const int oy = wk.ty0 + r, ox = wk.tx0 + x;
    const u32x4_t v = *(const u32x4_t*)(smem + ((r + 1) * C::LW + x + 1) * C::EB + c * 16);
    const bool ok = oy < p.oh && ox < p.ow;
    __builtin_amdgcn_raw_buffer_store_b128(v, launch_rsrc(p.res_out, fb),
                                           ok ? (uint32_t)wk.n * fb + (uint32_t)(((oy * p.ws + ox) * p.cs + c * 8) * 2) : OOB, 0, ST_AUX);
  };
  constexpr int DPU = RES ? 2 : 1;                // requests per unit
  constexpr int KIN = 3 * DPU + (SOUT ? 2 : 0);   // vmcnt before a unit whose wait spans no epilogue
  constexpr int KEP = KIN + (C::OST ? C::NST : TH) + 1;  // ... one that spans the epilogue's stores

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
  // The MFMAs are asm with the accumulator tied in place: hipcc's VGPR-form selection otherwise
  // moves every accumulator into fresh registers and pads the reuse of the old ones with s_nops.
  // The hazards hipcc cannot see are covered by construction: each tile's first MFMA of a row
  // takes C = 0 (no VALU write feeds an MFMA), operands come from loads it waits for, an
  // accumulation chain needs no wait states, and mfma_drain() pads before the epilogue reads.
  auto kloop = [&](Acc& acc, auto&& hook, auto&& bound) {
    // the zero-padded join (NST_Train's trunk) keeps one operand read fewer in flight: at three it spilled 8 B
    // per lane in this counted-vmcnt kernel (ring depth 2 / 3 / 4 measured within noise on the reflect trunk)
    constexpr int NI = 4 * PRD, D = (RES && ZPAD) ? 2 : WS_RING;
    f32x4_t bias0;
    if constexpr (NST_WS_BIAS_C) bias0 = *(const f32x4_t*)(smem + C::BIAS_OFF + (16 * wv + 4 * g) * 4);
    auto mfma = [&](f32x4_t& c, const uint4& a, const uint4& bop, bool first) {
      if constexpr (NST_WS_BIAS_C) mfma_tied_c<T>(c, a, bop, first, bias0);
      else mfma_tied<T>(c, a, bop, first);
    };
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
        mfma(acc[r], wr[s], bcur, q == 0 && dx == 0 && dy == 0);  // row r's first: y = r, dx = dy = 0
      }
      hook(q, rem);
      if (rem == PRD - 1) {
        lds_barrier();  // every wave is past its reads of part q (in-flight unit requests stay in flight)
        bound(q);
      }
      // pin the order: read i + D with read i's MFMAs (the scheduler otherwise pulls every read
      // down next to its consumers, exposing the LDS latency on each one)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogue: bias, bf16 NHWC store, InstanceNorm partial
  // sums: lane (px, g) holds channels 16 wv + 4g .. +3 of pixel px of every tile row.  Exactly
  // TH + 1 vector-memory instructions (the unit waits above count on it) ----
  auto epilogue = [&](const Work& wk, Acc& acc) {
    // the last MFMAs' results: 8-pass XDL write -> VALU read needs >= 12 wait states (20 here)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    const int c0 = 16 * wv + 4 * g;
    const f32x4_t bias = NST_WS_BIAS_C ? (f32x4_t){0.f, 0.f, 0.f, 0.f} : *(const f32x4_t*)(smem + C::BIAS_OFF + c0 * 4);
    const __amdgpu_buffer_rsrc_t ors = launch_rsrc(p.out, ob);
    const int ox = wk.tx0 + px;
    const uint32_t row_bytes = (uint32_t)p.ow * p.cout_stride * 2;
    const uint32_t fo = (uint32_t)wk.n * ob;
    const uint32_t off0 = fo + (uint32_t)(((wk.ty0 * p.ow + ox) * p.cout_stride + c0) * 2);
    f32x4_t s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};  // packed-math statistics
    // lane-derived LDS addresses recomputed per tile (opaque), not held across the K loop
    int obase = C::OUT_OFF + px * 256 + (((4 * wv + g) ^ (2 * (px & 7))) * 8);
    asm volatile("" : "+v"(obase));
    auto rows = [&](auto all_valid) {
#pragma unroll
      for (int r = 0; r < TH; ++r) {
        const bool valid = decltype(all_valid)::value || (wk.ty0 + r < p.oh && ox < p.ow);
        const f32x4_t v = NST_WS_BIAS_C ? acc[r] : add4(acc[r], bias);
        const u32x2_t pk = {pack16<T>(v[0], v[1]), pack16<T>(v[2], v[3])};
        if constexpr (C::OST) {
          *(u32x2_t*)(smem + obase + r * C::TW * 256) = pk;
        } else {
          __builtin_amdgcn_raw_buffer_store_b64(pk, ors, valid ? off0 + r * row_bytes : OOB, 0, ST_AUX);
        }
        const f32x4_t x = valid ? v : (f32x4_t){0.f, 0.f, 0.f, 0.f};
        if constexpr (NST_WS_PK_STATS) {
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
    // every tile but those on the bottom / right edge: no per-row validity
    if (wk.ty0 + TH <= p.oh && wk.tx0 + C::TW <= p.ow)
      rows(std::true_type{});
    else
      rows(std::false_type{});
    const float vv[8] = {s1[0], s2[0], s1[1], s2[1], s1[2], s2[2], s1[3], s2[3]};
    // reduce-scatter of the 8 statistics over the 16 pixel lanes of the DPP row, then the xor-1
    // partner: lane px (even) ends with statistic idx & 1 of channel c0 + (idx >> 1),
    // idx = 4 (px >= 8) + 2 (px & 4) + (px & 2) / 2
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
    if constexpr (C::OST) {
      // the staged tile, 4 whole pixels (1 KB contiguous in a tile row) per store instruction
      lds_barrier();
      int t0 = tid;
      asm volatile("" : "+v"(t0));
#pragma unroll
      for (int k = 0; k < C::NST; ++k) {
        const int off = (k * C::NT + t0) * 16;
        const int pp = off >> 8, cb = off & 255;
        const int x = pp & (C::TW - 1), oy = wk.ty0 + pp / C::TW, ox = wk.tx0 + x;
        const u32x4_t v = *(const u32x4_t*)(smem + C::OUT_OFF + pp * 256 + (((cb >> 3) ^ (2 * (x & 7))) << 3));
        const bool ok = oy < p.oh && ox < p.ow;
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, ok ? fo + (uint32_t)((oy * p.ow + ox) * 256 + cb) : OOB, 0, ST_AUX);
      }
    }
  };

  // ---- persistent walk ----
  Work cur = decode(w0);
  int wn = w0 + G;
  const int last = p.n_work - 1;
  build_maps(cur, 0);
  build_maps(decode(min(wn, last)), 1);
  __syncthreads();
  // prologue: the first tile's units (units 6, 7 and the next tile's 0, 1 stay in flight, as in
  // the steady state); then drain once, so every later wait counts only steady-state instructions
  Item xx = items(cur, 0);  // sources of the tile being consumed
  Item xd = xx;             // ... and of the tile being requested
#pragma unroll
  for (int u = 0; u < C::NSLOT; ++u) request(u, xd);
  {
    const Work n1 = decode(min(wn, last));
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      vm_wait<0>();
      consume(cur, u, xx, stage_read(u));
      if (u + 4 < C::NUNIT) {
        request(u + 4, xd);
      } else {
        if (u + 4 == C::NUNIT) xd = items(n1, 1);
        request(u + 4 - C::NUNIT, xd);
      }
    }
  }
  vm_wait<0>();
  __syncthreads();
  if (NST_WS_PRIO && team) __builtin_amdgcn_s_setprio(1);
  // Unit schedule (u = 2q + half; region q is free once the barrier ending part q has passed):
  //   part 0: A: unit 6 of cur, request 2 of nxt    | B: unit 7 of cur, request 3 of nxt
  //   part 1: A: unit 0 of nxt, request 4 of nxt    | B: unit 1, request 5
  //   part 2: A: unit 2, request 6                  | B: unit 3, request 7
  //   part 3: A: unit 4, request 0 of the tile after nxt | B: unit 5, request 1 of it
  // A is right after the part's first reads, B half a part later; team 1 runs a quarter part
  // behind team 0 so the two waves of a SIMD never stage at the same time.
  constexpr int POS_A = 0, POS_B = PRD / 2, DT = PRD / 4;
  Acc acc;
  Staged stg_u;  // the unit between its staging read and its transform
  for (int it = 0;; ++it) {
    // past the last work item the hooks restage LDS with whatever they are given (never read
    // again) and store nothing, so they need no branch
    const bool more = wn < p.n_work;
    const Work nxt = more ? decode(wn) : cur;
    const Work nxt2 = decode(min(wn + G, last));
    const int cs = it & 1, ns = cs ^ 1;  // map slots of cur and nxt
    kloop(
        acc,
        [&](int q, int rem) {  // after read rem of part q
          // unit work at pa / pb (staging read) and WS_SPLIT reads later (transform + next request)
          const int pa = POS_A + (team ? DT : 0), pb = POS_B + (team ? DT : 0);
          const bool rd = rem == pa || rem == pb;
          const bool wr = rem == pa + WS_SPLIT || rem == pb + WS_SPLIT;
          if (!rd && !wr) return;
          const int half = (rem == pa || rem == pa + WS_SPLIT) ? 0 : 1;
          if (q == 0) {
            if (rd) {
              vm_wait<KEP>();
              stg_u = stage_read(6 + half);
            }
            if (wr) {
              consume(cur, 6 + half, xx, stg_u);
              request(2 + half, xd);
              if (SOUT && half == 0) store_region(cur, 0);
            }
          } else {
            const int u = 2 * (q - 1) + half;
            if (rd) {
              if (u == 0) xx = items(nxt, ns);
              if (u <= 1) vm_wait<KEP>(); else vm_wait<KIN>();
              stg_u = stage_read(u);
            }
            if (wr) {
              consume(nxt, u, xx, stg_u);
              if (u + 4 < C::NUNIT) {
                request(u + 4, xd);
              } else {
                if (u == 4) xd = items(nxt2, cs);
                request(u - 4, xd);
              }
              if (SOUT && half == 0) store_region(cur, q);
            }
          }
        },
        [&](int q) {  // after the barrier that ends part q
          // the tile after nxt into cur's slot: cur's sources were last resolved in the previous
          // iteration, and the barriers ending parts 1 and 2 publish it before part 3 resolves it
          if (q == 0) build_maps(nxt2, cs);
        });
    epilogue(cur, acc);
    if (!more) break;
    cur = nxt;
    wn += G;
  }
  vm_wait<0>();  // no LDS-DMA may land after the workgroup has released its LDS
}

template <typename T, int TH, bool RES>
struct WstatInst {
  using C = WsCfg<TH, RES ? WF_RES : WF_NORM>;  // NFMAX, LDS and weight sizes shared by the FILL variants
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
    hipLaunchKernelGGL((wstat_kernel<T, TH, FILL, ZPAD, XO>), dim3(nb), dim3(C::NT), 0, st, p);
  }
  // grid.x = tiles per frame, grid.y = frames; launched in chunks of <= NFMAX frames (the IN tables
  // of a launch's frames live in LDS)
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    const int ntile = (int)grid.x, n = (int)grid.y;
    const size_t fin = (size_t)p0.hs * p0.ws * p0.cs * 2, fout = (size_t)p0.oh * p0.ow * p0.cout_stride * 2;
    // frames per launch: the LDS IN tables' capacity, and every offset (frame * bytes) below OOB
    const int fmax = (int)std::min<size_t>(C::NFMAX, (size_t)OOB / std::max(fin, fout));
    if (fmax < 1) return;  // nst_api validates sizes before launching
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
      const int nb = std::min(p.n_work, cus());  // one workgroup per CU (registers, LDS)
      const bool zp = p.axis_mode != AX_REFLECT;  // zero-padded trunk (transformer_net_nst.py ConvBlock)
      if constexpr (RES) {
        // joins a stored residual stream (block 1's conv1 exports x_0; nst_api rejects a
        // normalised residual here)
        zp ? go<WF_RES, true>(p, nb, st) : go<WF_RES, false>(p, nb, st);
      } else {
        if (p.in_norm != nullptr && p.res_out != nullptr)  // block 1's conv1, exporting x_0
          zp ? go<WF_NORM, true, true>(p, nb, st) : go<WF_NORM, false, true>(p, nb, st);
        else if (p.in_norm != nullptr)
          zp ? go<WF_NORM, true>(p, nb, st) : go<WF_NORM, false>(p, nb, st);
        else  // the residual stream itself (unfused joins)
          zp ? go<WF_RAW, true>(p, nb, st) : go<WF_RAW, false>(p, nb, st);
      }
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
#ifndef NST_WSTAT_TH_RES
#define NST_WSTAT_TH_RES NST_WSTAT_TH
#endif
constexpr int WSTAT_TH = NST_WSTAT_TH;          // tile rows (plain trunk conv)
constexpr int WSTAT_TH_RES = NST_WSTAT_TH_RES;  // ... of the joined variant (its staging ring takes twice the LDS)
#define E(...) WstatInst<__VA_ARGS__>::info()
const ConvKernelInfo* conv_table_wstat(int* count) {
  static const ConvKernelInfo table[] = {
      E(__bf16, WSTAT_TH, false),    // residual trunk
      E(__bf16, WSTAT_TH_RES, true),     // + residual join in the fill
      E(_Float16, WSTAT_TH, false),  // fp16 mode
      E(_Float16, WSTAT_TH_RES, true),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E

}  // namespace nst
