// conv_out9.hip — the output conv of the Johnson / NST / ReCoNet nets (9x9, C -> 3 channels:
// transformer_net.py:37-38 deconv3, transformer_net_nst.py:91 final, model.py:78 ConvTanhLayer)
// as a row-streaming "ky-rotation" GEMM on v_mfma_f32_32x32x16_bf16.
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

typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <int CINP, int G, int NW>
struct Out9Cfg {
  static constexpr int KC = CINP / 16;            // 16-channel K blocks per tap
  static constexpr int NCH = CINP / 8;            // 16-B chunks per pixel
  // LDS bytes per pixel: one 16-B pad makes the stride an odd number of 16-B slots, so the 16
  // lanes of every ds_read_b128 lane group hit 16 distinct slots (consecutive columns)
  static constexpr int EB = CINP * 2 + 16;
  static constexpr int SW = 32 * G;               // output columns per strip
  static constexpr int LWS = SW + 8;              // input columns per strip row
  static constexpr int ROWB = LWS * EB;
  static constexpr int WAVE_LDS = 2 * ROWB;
  static constexpr int KSTRIDE = 9 * KC * 96;     // bytes per kernel row ky in the weight table
  static constexpr int W_BYTES = 9 * KSTRIDE;
  static constexpr int Z_BYTES = KSTRIDE;         // zero block read by the unused rows 27..31
  static constexpr int W_OFF = NW * WAVE_LDS;
  static constexpr int Z_OFF = W_OFF + W_BYTES;
  static constexpr int LDS = Z_OFF + Z_BYTES;
  static constexpr int ITEMS = LWS * NCH;         // 16-B loads per strip row
  static constexpr int IPL = (ITEMS + 63) / 64;   // per lane
  static_assert(64 % NCH == 0, "a lane keeps one channel chunk");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <int CINP, int G, int NW, int OUTK>
__global__ __launch_bounds__(64 * NW) void out9_kernel(ConvParams p) {
  using C = Out9Cfg<CINP, G, NW>;
  constexpr int KC = C::KC, NCH = C::NCH, EB = C::EB;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- weights -> LDS (packed host-side in table order), zero block ----
  {
    const uint4* src = (const uint4*)p.wpk;
    uint4* dst = (uint4*)(smem + C::W_OFF);
    for (int i = tid; i < C::W_BYTES / 16; i += 64 * NW) dst[i] = src[i];
    uint4* z = (uint4*)(smem + C::Z_OFF);
    for (int i = tid; i < C::Z_BYTES / 16; i += 64 * NW) z[i] = make_uint4(0u, 0u, 0u, 0u);
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
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    if (rho < 27) {
      const int k = rho / 3, c = rho - 3 * (rho / 3);
      const int ky = (t - k + 9) % 9;
      a_off[t] = C::W_OFF + ky * C::KSTRIDE + c * 32 + 16 * h;
    } else {
      a_off[t] = C::Z_OFF + 16 * h;
    }
  }
  // B operand (pixels): column rho of the 32-column group, K half h
  char* ring = smem + wave * C::WAVE_LDS;
  const int b_lane = rho * EB + 16 * h;
  // fill: item i = lane + 64*j -> strip column i / NCH, chunk lane % NCH (fixed per lane)
  const int chunk = lane % NCH;
  const int pix_bytes = p.cs * 2;
  const int row_bytes = p.ws * pix_bytes;
  int coloff[C::IPL];
#pragma unroll
  for (int j = 0; j < C::IPL; ++j) {
    const int i = lane + 64 * j;
    const int col = i / NCH;
    const int sx = map_axis(x0 + p.crop_x - p.pad + col, p.ws, p.axis_mode, p.pre);
    coloff[j] = (i < C::ITEMS && sx >= 0) ? sx * pix_bytes + chunk * 16 : -1;
  }
  float2 nm[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) nm[j] = p.in_norm[(size_t)n * p.cs + chunk * 8 + j];
  const char* img = (const char*)p.in + (size_t)n * p.hs * row_bytes;
  const int vy0 = o0 + p.crop_y - p.pad;

  auto row_src = [&](int v) -> int {
    const int sy = map_axis(vy0 + v, p.hs, p.axis_mode, p.pre);
    return sy < 0 ? -1 : sy * row_bytes;
  };
  uint4 raw[C::IPL];
  auto issue = [&](int v) {
    const int ro = row_src(v);
#pragma unroll
    for (int j = 0; j < C::IPL; ++j) {
      const bool ok = ro >= 0 && coloff[j] >= 0;
      raw[j] = *(const uint4*)(img + (ok ? (unsigned)(ro + coloff[j]) : 0u));
      if (!ok) raw[j] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  // zero padding stays zero (the pad applies after the producer's IN + ReLU)
  auto store_row = [&](int v) {
    const int ro = row_src(v);
    char* dst = ring + (v & 1) * C::ROWB + (lane / NCH) * EB + chunk * 16;
#pragma unroll
    for (int j = 0; j < C::IPL; ++j) {
      if (lane + 64 * j < C::ITEMS) {
        const bool ok = ro >= 0 && coloff[j] >= 0;
        const uint4 v4 = ok ? norm_chunk<__bf16>(raw[j], nm) : make_uint4(0u, 0u, 0u, 0u);
        *(uint4*)(dst + j * (64 / NCH) * EB) = v4;
      }
    }
  };

  // ---- output ----
  const float bias0 = p.bias[0], bias1 = p.bias[1], bias2 = p.bias[2];
  auto emit = [&](const f32x16_t (&acc)[G], int reg, int c, int oy) {
    const float b = c == 0 ? bias0 : (c == 1 ? bias1 : bias2);
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int ox = x0 + gi * 32 + rho;
      if (ox < p.ow) {
        float y = acc[gi][reg] + b;
        if (p.dec_tanh) y = tanhf(y);
        if constexpr (OUTK == OUT_F32_NCHW) {
          ((float*)p.out)[(((size_t)n * 3 + c) * p.oh + oy) * p.ow + ox] = y;
        } else {
          const int ch = p.dec_perm[c];  // the presets' channel permutations are involutions
          ((uint8_t*)p.out)[(((size_t)n * p.oh + oy) * p.ow + ox) * 3 + ch] =
              (uint8_t)(decode_ch(y, ch, p) * 255.0f);  // ToPILImage: pic.mul(255).byte()
        }
      }
    }
  };

  f32x16_t acc[G];
#pragma unroll
  for (int gi = 0; gi < G; ++gi)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[gi][r] = 0.f;

  issue(0);
  store_row(0);
  for (int vb = 0; vb < NV; vb += 9) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int v = vb + t;
      if (v >= NV) break;
      const bool next = v + 1 < NV;
      if (next) issue(v + 1);
      const char* rb = ring + (v & 1) * C::ROWB + b_lane;
      const char* ab = smem + a_off[t];
#pragma unroll
      for (int kx = 0; kx < 9; ++kx) {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const uint4 a = *(const uint4*)(ab + (kx * KC + kc) * 96);
#pragma unroll
          for (int gi = 0; gi < G; ++gi) {
            const uint4 b = *(const uint4*)(rb + (gi * 32 + kx) * EB + kc * 32);
            acc[gi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                              __builtin_bit_cast(bf16x8_t, b), acc[gi], 0, 0, 0);
          }
        }
      }
      // slot (t+1) % 9 now holds output row v - 8: store it, then clear it for output row v + 1
      const int kk = (t + 1) % 9;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int r3 = 3 * kk + c;
        const int reg = (r3 & 3) + 4 * (r3 >> 3), hh = (r3 >> 2) & 1;
        if (v >= 8 && h == hh) emit(acc, reg, c, o0 + v - 8);
#pragma unroll
        for (int gi = 0; gi < G; ++gi) acc[gi][reg] = (h == hh) ? 0.f : acc[gi][reg];
      }
      if (next) store_row(v + 1);
    }
  }
}

template <int CINP, int G, int NW, int OUTK>
struct Out9Inst {
  using C = Out9Cfg<CINP, G, NW>;
  static constexpr auto kernel = out9_kernel<CINP, G, NW, OUTK>;
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
    k.dtype = NST_DT_BF16;
    k.mode = MODE_KYROT;
    k.ks = 9; k.stride = 1; k.cinp = CINP; k.bn = 16; k.th = 1; k.tw = C::SW; k.wm = NW; k.wn = 1;
    k.in_kind = IN_ACT; k.out_kind = OUTK;
    k.cpc = 8; k.nch = C::NCH; k.lds_bytes = C::LDS;
    k.wbytes = C::W_BYTES;
    k.part_rows = 1;
    k.launch = &launch;
    return k;
  }
};

#define E(...) Out9Inst<__VA_ARGS__>::info()
const ConvKernelInfo* conv_table_out9(int* count) {
  static const ConvKernelInfo table[] = {
      //  CINP G NW OUT
      E(32, 3, 8, OUT_U8_NHWC),   // Johnson deconv3 / NST final (frames)
      E(32, 3, 8, OUT_F32_NCHW),  // tensor API
      E(64, 3, 4, OUT_U8_NHWC),   // ReCoNet (48 channels, bf16 padded to 64)
      E(64, 3, 4, OUT_F32_NCHW),
  };
  *count = (int)(sizeof(table) / sizeof(table[0]));
  return table;
}
#undef E

}  // namespace nst
