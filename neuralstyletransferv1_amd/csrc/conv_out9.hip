// conv_out9.hip — the output conv of the Johnson / NST / ReCoNet nets (9x9, C -> 3 channels:
// transformer_net.py:37-38 deconv3, transformer_net_nst.py:91 final, model.py:78 ConvTanhLayer)
// as a row-streaming "ky-rotation" GEMM on v_mfma_f32_32x32x16_{bf16,f16}.
//
// Why a separate mapping: with N = 3 output channels a plain implicit GEMM wastes 13 of 16 MFMA
// columns, and any 2-D halo tile re-reads 9 input rows per output row.  Here
//   * the 32 MFMA rows are (slot k, channel c) pairs, rho = 3k + c (27 used): slot k accumulates
//     output row o with o % 9 == k;
//   * K = (kx, input channel) of ONE input row v; N = 32 output columns;
//   * input row v contributes W[.][.][ky][.] to output row o = v - ky, so at row v the A operand
//     of slot k holds kernel row ky = (v - k) mod 9 ("rotation" v mod 9 of the weights, read from
//     a per-lane LDS offset); after row v, slot (v+1) mod 9 holds the finished output row v - 8:
//     it is decoded and stored, then zeroed for output row v + 1.
// So every input row is staged once per column strip and read by 9 x C/16 MFMAs per 32 columns:
// 27/32 = 84 % of the MFMA rows are useful and there is no K padding.
//
// Structure: one wave = one column strip (32*G output columns) x one vertical segment of output
// rows; waves are independent (no barrier after the weight upload).  Each wave keeps a 2-row
// LDS ring of its strip's input rows: row v+1 is loaded into registers at the start of row v,
// normalised (producer InstanceNorm + ReLU) and written to the other ring slot at its end.  The
// 9x9 weights (one copy, 15.5 KB bf16 for C = 32) sit in LDS for the whole kernel.
#include <algorithm>
#include <cstring>

#include "conv_impl.h"

namespace nst {

typedef __attribute__((address_space(3))) uint64_t lds_u64;  // volatile LDS loads: never merged

// ESZ: LDS bytes per channel, 2 for the 16-bit modes, 4 for the split-fp16 mode (NST_DT_F32S: each 16-B chunk is
// [hi0..3, lo0..3] of 4 fp32 channels, conv_impl.h F32Split; one 32x32x16 K step = 8 channels)
template <int CINP, int G, int NW, int ESZ = 2>
struct Out9Cfg {
  static constexpr int KC = CINP * ESZ / 32;      // 32-byte K blocks per tap (16 channels, 8 split)
  static constexpr int NCH = CINP * ESZ / 16;     // 16-B chunks per pixel
  static constexpr int CPCH = 16 / ESZ;           // channels per chunk
  // LDS bytes per pixel: one 16-B pad makes the stride an odd number of 16-B slots, so the 16
  // lanes of every ds_read_b128 lane group hit 16 distinct slots (consecutive columns)
  static constexpr int EB = CINP * ESZ + 16;
  static constexpr int SW = 32 * G;               // output columns per strip
  static constexpr int LWS = SW + 8;              // input columns per strip row
  static constexpr int ROWB = LWS * EB;
  static constexpr int WAVE_LDS = 2 * ROWB;
  // weight table: [part p][block (kx, kc)][K half h][row i = 3*ky + c] x 8 bytes (4 x 16 bit); a lane's
  // 16-B A fragment is two ds_read_b64 (parts 0 and 1, PART_BYTES apart).  Split mode: part 0 = Wh, part 1 = Wl
  // of the same 4 channels (the two MFMAs' fragments [Wh Wh] x [xh xl] and [Wl 0] x [xh xl]).  The 32 lanes of one
  // half read 27 different rows (the rotation permutes them), i.e. 27 consecutive 8-B slots: no
  // bank conflict for any rotation (ds_read_b64 banks 32-lane groups mod 64 dwords); the 5 unused
  // rows re-read row 0's address (broadcast).  The two reads stay separate instructions: hipcc
  // would merge them into one ds_read2_b64, which banks 16-lane groups mod 32 dwords, where rows
  // r and r + 16 collide.
  static constexpr int NBLK = 9 * KC;
  static constexpr int BLK_BYTES = 2 * 27 * 8;
  static constexpr int PART_BYTES = NBLK * BLK_BYTES;
  static constexpr int W_BYTES = 2 * PART_BYTES;
  static constexpr int W_OFF = NW * WAVE_LDS;
  static constexpr int LDS = W_OFF + W_BYTES;
  static constexpr int ITEMS = LWS * NCH;         // 16-B loads per strip row
  static constexpr int IPL = (ITEMS + 63) / 64;   // per lane
  // fill item lane + 64 j = chunk lane / PPJ of column PPJ j + lane % PPJ: the 8 lanes of a
  // ds_write_b128 group write one chunk of 8 consecutive columns, 8 distinct 16-B bank slots (EB is an
  // odd number of them); a wave's load still covers PPJ whole pixels
  static constexpr int PPJ = 64 / NCH;
  static_assert(64 % NCH == 0, "a lane keeps one channel chunk");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// CLD: input channels stored (<= CINP; ReCoNet's unpadded 48-channel decoder output): the chunks past them stage zeros
template <typename T, int CINP, int G, int NW, int OUTK, bool TANH, int CLD = CINP>
__global__ __launch_bounds__(64 * NW) void out9_kernel(ConvParams p) {
  constexpr bool SPLIT = IS_SPLIT<T>;
  using TM = std::conditional_t<SPLIT, _Float16, T>;  // the MFMA operand type
  using C = Out9Cfg<CINP, G, NW, SPLIT ? 4 : 2>;
  constexpr int KC = C::KC, EB = C::EB;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: work-item math in SGPRs

  // ---- weights -> LDS (packed host-side in table order) ----
  {
    const uint4* src = (const uint4*)p.wpk;
    uint4* dst = (uint4*)(smem + C::W_OFF);
    for (int i = tid; i < C::W_BYTES / 16; i += 64 * NW) dst[i] = src[i];
  }
  __syncthreads();

  // ---- work item: (frame, segment of output rows, column strip) ----
  const int item = blockIdx.x * NW + wave;
  if (item >= p.n_work) return;
  const int strips = p.tiles_x, nseg = p.tiles_y;
  const int strip = item % strips;
  const int rest = item / strips;
  const int seg = rest % nseg;
  const int n = rest / nseg;
  const int x0 = strip * C::SW;
  const int o0 = seg * p.seg_len;
  const int L = min(p.seg_len, p.oh - o0);
  if (L <= 0) return;
  const int NV = L + 8;  // input rows streamed: output rows o0..o0+L-1 need virtual rows o0-4 .. o0+L+3

  // ---- per-lane constants ----
  // A operand (weights): lane row rho = lane & 31 -> (slot k, channel c); K half h = lane >> 5
  const int rho = lane & 31, h = lane >> 5;
  int a_off[9];
  {
    const int k = rho < 27 ? rho / 3 : 0;  // unused rows 27..31 re-read row 0's address (broadcast)
    const int c = rho < 27 ? rho - 3 * (rho / 3) : 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      a_off[t] = C::W_OFF + (h * 27 + 3 * ((t - k + 9) % 9) + c) * 8;
      asm volatile("" : "+v"(a_off[t]));  // keep the 9 bases opaque: no per-tap address re-derivation
    }
  }
  // B operand (pixels): column rho of the 32-column group, K half h
  char* ring = smem + wave * C::WAVE_LDS;
  const int b_lane = rho * EB + 16 * h;
  // fill: item lane + 64*j -> strip column PPJ*j + lane % PPJ, chunk lane / PPJ (fixed per lane)
  const int chunk = lane / C::PPJ;
  const int pix_bytes = p.cs * (SPLIT ? 4 : 2);  // HBM activations: fp32 in the split mode
  const int row_bytes = p.ws * pix_bytes;
  int coloff[C::IPL];
#pragma unroll
  for (int j = 0; j < C::IPL; ++j) {
    const int col = C::PPJ * j + lane % C::PPJ;
    const int sx = map_axis(x0 + p.crop_x - p.pad + col, p.ws, p.axis_mode, p.pre);
    coloff[j] = (col < C::LWS && sx >= 0 && chunk * C::CPCH < CLD) ? sx * pix_bytes + chunk * 16 : -1;
  }
  float2 nm[C::CPCH];
#pragma unroll
  for (int j = 0; j < C::CPCH; ++j)
    nm[j] = chunk * C::CPCH < CLD ? p.in_norm[(size_t)n * p.cs + chunk * C::CPCH + j] : make_float2(0.f, 0.f);
  const char* img = (const char*)p.in + (size_t)n * p.hs * row_bytes;
  const int vy0 = o0 + p.crop_y - p.pad;

  auto row_src = [&](int v) -> int {
    const int sy = map_axis(vy0 + v, p.hs, p.axis_mode, p.pre);
    return sy < 0 ? -1 : sy * row_bytes;
  };
  uint4 raw[C::IPL];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)img, (short)0, p.hs * row_bytes, 0x00020000);
  // an out-of-range buffer offset reads 0 (zero padding); the IN+ReLU is skipped for those items
  constexpr uint32_t OOB = 0x80000000u;
  auto issue = [&](int ro) {
#pragma unroll
    for (int j = 0; j < C::IPL; ++j) {
      const bool ok = ro >= 0 && coloff[j] >= 0;
      raw[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (uint32_t)(ro + coloff[j]) : OOB, 0, 0));
    }
  };
  // zero padding stays zero (the pad applies after the producer's IN + ReLU)
  auto store_row = [&](int v, int ro) {
    char* dst = ring + (v & 1) * C::ROWB + (lane % C::PPJ) * EB + chunk * 16;
#pragma unroll
    for (int j = 0; j < C::IPL; ++j) {
      if (C::PPJ * j + lane % C::PPJ < C::LWS) {
        const bool ok = ro >= 0 && coloff[j] >= 0;
        const uint4 v4 = lds_form<T>(norm_chunk<T>(raw[j], nm));  // split: IN + ReLU in fp32, then hi / lo
        *(uint4*)(dst + j * C::PPJ * EB) = ok ? v4 : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };

  // ---- output ----
  // decode v = ((y + p) * q) / r + s as a multiply by 1/r (bf16 throughput mode: within one ulp of
  // the division, bar a truncation boundary)
  const float bias[3] = {p.bias[0], p.bias[1], p.bias[2]};
  float dp[3], dq[3], dri[3], ds[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int ch = p.dec_perm[c];  // the presets' channel permutations are involutions
    dp[c] = p.dec_p[ch]; dq[c] = p.dec_q[ch]; dri[c] = 1.0f / p.dec_r[ch]; ds[c] = p.dec_s[ch];
  }
  // stores through a buffer resource: masked-out lanes get an out-of-range offset and are dropped,
  // so the emission is branch-free
  const int out_bytes = OUTK == OUT_F32_NCHW ? 3 * p.oh * p.ow * 4 : p.oh * p.ow * 3;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((char*)p.out + (size_t)n * out_bytes), (short)0, out_bytes, 0x00020000);
  int perm[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) perm[c] = p.dec_perm[c];
  auto emit = [&](const f32x16_t (&acc)[G], int reg, int c, int oy, bool on) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int ox = x0 + gi * 32 + rho;
      const bool ok = on && ox < p.ow;
      float y = acc[gi][reg] + bias[c];
      if constexpr (TANH) y = tanhf(y);  // ReCoNet ConvTanhLayer (model.py:77-80)
      if constexpr (OUTK == OUT_F32_NCHW) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(y), ors, ok ? (uint32_t)(((c * p.oh + oy) * p.ow + ox) * 4) : OOB, 0, 0);
      } else {
        const float v = fminf(fmaxf((y + dp[c]) * dq[c] * dri[c] + ds[c], 0.f), 1.f);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v * 255.0f), ors,  // pic.mul(255).byte()
                                             ok ? (uint32_t)((oy * p.ow + ox) * 3 + perm[c]) : OOB, 0, 0);
      }
    }
  };

  f32x16_t acc[G];
#pragma unroll
  for (int gi = 0; gi < G; ++gi)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[gi][r] = 0.f;

  {
    const int ro0 = row_src(0);
    issue(ro0);
    store_row(0, ro0);
  }
  for (int vb = 0; vb < NV; vb += 9) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int v = vb + t;
      if (v >= NV) break;
      const bool next = v + 1 < NV;
      const int ro_next = next ? row_src(v + 1) : -1;
      if (next) issue(ro_next);
      const char* rb = ring + (v & 1) * C::ROWB + b_lane;
      const char* ab = smem + a_off[t];
      // operands of tap column kx, double-buffered: tap kx+1's reads are issued before tap kx's
      // MFMAs, one scheduling region per tap (keeps the live operand set at two taps)
      constexpr int AF = SPLIT ? 2 : 1;  // A fragments per K block
      uint4 av[2][KC][AF], bv[2][KC][G];
      auto ld = [&](int kx, uint4 (&a)[KC][AF], uint4 (&b)[KC][G]) {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const uint64_t a0 = *(const volatile lds_u64*)(ab + (kx * KC + kc) * C::BLK_BYTES);
          const uint64_t a1 = *(const volatile lds_u64*)(ab + (kx * KC + kc) * C::BLK_BYTES + C::PART_BYTES);
          if constexpr (SPLIT) {  // [Wh Wh] and [Wl 0] for the lane's chunk [xh0..3 xl0..3]
            a[kc][0] = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a0, (uint32_t)(a0 >> 32));
            a[kc][AF - 1] = make_uint4((uint32_t)a1, (uint32_t)(a1 >> 32), 0u, 0u);
          } else {
            a[kc][0] = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32));
          }
#pragma unroll
          for (int gi = 0; gi < G; ++gi) b[kc][gi] = *(const uint4*)(rb + (gi * 32 + kx) * EB + kc * 32);
        }
      };
      ld(0, av[0], bv[0]);
#pragma unroll
      for (int kx = 0; kx < 9; ++kx) {
        if (kx + 1 < 9) ld(kx + 1, av[(kx + 1) & 1], bv[(kx + 1) & 1]);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc)
#pragma unroll
          for (int gi = 0; gi < G; ++gi)
#pragma unroll
            for (int f = 0; f < AF; ++f)  // split: Wh * (xh + xl) + Wl * xh (~22-bit products, fp32 sums)
              acc[gi] = mfma32x32x16<TM>(av[kx & 1][kc][f], bv[kx & 1][kc][gi], acc[gi]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // slot (t+1) % 9 now holds output row v - 8: store it, then clear it for output row v + 1
      const int kk = (t + 1) % 9;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int r3 = 3 * kk + c;
        const int reg = (r3 & 3) + 4 * (r3 >> 3), hh = (r3 >> 2) & 1;
        emit(acc, reg, c, o0 + v - 8, v >= 8 && h == hh);
#pragma unroll
        for (int gi = 0; gi < G; ++gi) acc[gi][reg] = (h == hh) ? 0.f : acc[gi][reg];
      }
      if (next) store_row(v + 1, ro_next);
    }
  }
}

template <typename T, int CINP, int G, int NW, int OUTK, bool TANH, int CLD = CINP>
struct Out9Inst {
  using C = Out9Cfg<CINP, G, NW, IS_SPLIT<T> ? 4 : 2>;
  static constexpr auto kernel = out9_kernel<T, CINP, G, NW, OUTK, TANH, CLD>;
  static int cus() {
    static const int v = [] {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        c = 256;
      return c;
    }();
    return v;
  }
  // grid.y = frames (one channel block); the segment count fills the chip's wave slots once
  static void launch(const ConvParams& p0, dim3 grid, hipStream_t st) {
    ConvParams p = p0;
    const int n = (int)grid.y;
    const int strips = (p.ow + C::SW - 1) / C::SW;
    const int slots = cus() * NW;  // one workgroup per CU (LDS)
    int nseg = std::max(1, slots / std::max(1, n * strips));
    nseg = std::min(nseg, std::max(1, p.oh / 16));  // segments of >= 16 rows (8 rows of lead-in each)
    p.seg_len = (p.oh + nseg - 1) / nseg;
    nseg = (p.oh + p.seg_len - 1) / p.seg_len;
    p.tiles_x = strips;
    p.tiles_y = nseg;
    p.n_work = n * nseg * strips;
    const int blocks = (p.n_work + NW - 1) / NW;
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(64 * NW), 0, st, p);
  }
  static ConvKernelInfo info() {
    ConvKernelInfo k;
    std::memset(&k, 0, sizeof(k));
    k.dtype = dtype_code<T>();
    k.mode = MODE_KYROT;
    k.ks = 9; k.stride = 1; k.cinp = CLD; k.bn = 16;
    k.cinp_k = CLD != CINP ? CINP : 0; k.th = 1; k.tw = C::SW; k.wm = NW; k.wn = 1;
    k.in_kind = IN_ACT; k.out_kind = OUTK;
    k.cpc = C::CPCH; k.nch = C::NCH; k.lds_bytes = C::LDS;
    k.in_esz = IS_SPLIT<T> ? 4 : 0;
    k.wbytes = C::W_BYTES;
    k.part_rows = 1;
    k.tanh_out = TANH ? 1 : 0;
    k.launch = &launch;
    return k;
  }
};

// ReCoNet's 48 (64-padded) -> 3 output conv: strip groups G and waves NW (build-time, for sweeps)
// (r04 sweep, 8 x 1080p: G 3 / NW 4 0.869 ms, G 2 / NW 4 0.800, G 2 / NW 6 0.686, G 1 / NW 8 0.643)
#ifndef NST_OUT9_R_G
#define NST_OUT9_R_G 1
#endif
#ifndef NST_OUT9_R_NW
#define NST_OUT9_R_NW 8
#endif
#ifndef NST_OUT9_J_G
#define NST_OUT9_J_G 3
#endif
#ifndef NST_OUT9_J_NW
#define NST_OUT9_J_NW 8
#endif
#ifndef NST_OUT9_S_G
#define NST_OUT9_S_G 1
#endif
#ifndef NST_OUT9_S_NW
#define NST_OUT9_S_NW 8
#endif
#define E(...) Out9Inst<__VA_ARGS__>::info()
const ConvKernelInfo* conv_table_out9(int* count) {
  static const ConvKernelInfo table[] = {
      //  T     CINP G NW OUT          TANH
      E(__bf16, 32, NST_OUT9_J_G, NST_OUT9_J_NW, OUT_U8_NHWC, false),    // Johnson deconv3 / NST final (frames)
      E(__bf16, 32, 3, 8, OUT_F32_NCHW, false),   // tensor API
      E(__bf16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_U8_NHWC, true),   // ReCoNet (48 channels, padded to 64; tanh)
      E(__bf16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_F32_NCHW, true),
      E(__bf16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_U8_NHWC, true, 48),  // ... reading 48 unpadded channels
      E(__bf16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_F32_NCHW, true, 48),
      E(_Float16, 32, 3, 8, OUT_U8_NHWC, false),  // fp16 mode
      E(_Float16, 32, 3, 8, OUT_F32_NCHW, false),
      E(_Float16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_U8_NHWC, true),
      E(_Float16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_F32_NCHW, true),
      E(_Float16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_U8_NHWC, true, 48),
      E(_Float16, 64, NST_OUT9_R_G, NST_OUT9_R_NW, OUT_F32_NCHW, true, 48),
      // split-fp16 mode (NST_DT_F32S): fp32 activations, two f16 MFMAs per K step (the x-shift generic kernel's
      // 9-chunk LDS entries were 2-way bank-conflicted on most operand reads: 5.2 ms per batch of 8)
      E(F32Split, 32, NST_OUT9_S_G, NST_OUT9_S_NW, OUT_U8_NHWC, false),
      E(F32Split, 32, NST_OUT9_S_G, NST_OUT9_S_NW, OUT_F32_NCHW, false),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E

}  // namespace nst
