// conv_gemm.hip — K-streaming implicit-GEMM convolution for the DeepLab v3+ ResNet-101 mask network
// (modeling/backbone/resnet.py:6-43 Bottleneck, :61-65 stem; modeling/aspp.py:7-78; modeling/decoder.py:19-43).
//
// The stylization kernels stage a tile's whole input halo (all channels) in LDS once; ResNet-101's
// 1024/2048-channel layers do not fit that, so this kernel streams K instead: one STAGE = one tap x
// 128 bytes of input channels (64 bf16 / fp16 or 32 fp32), double-buffered in LDS through registers (the
// next stage's global loads are in flight while the current stage's MFMAs run; one barrier per stage).
//
//   * GEMM rows = output channels (A = packed weights, one contiguous 8 KiB piece per 64 rows and
//     stage: [cout/64][stage][64][128 B]); columns = output pixels (B = an im2col row gathered on the
//     fly: pixel (n,oy,ox), tap (ky,kx) -> source (oy*s - pad + ky*d, ox*s - pad + kx*d), zero outside
//     the image: Conv2d zero padding, any stride and dilation — the atrous convs of layer4 / ASPP).
//   * 4 waves in 2x2, each (BM/2)x(BN/2) of the BMxBN tile; bf16 / fp16: v_mfma_f32_16x16x32_{bf16,f16}, one per
//     16x16 sub-tile and half-stage; fp32 (parity mode): v_mfma_f32_16x16x4_f32, 4 per half-stage over
//     a 16-byte operand read (the K permutation is the same for A and B, so the sum is over the same
//     products).
//   * LDS image per stage: [half][row][4 x 16-B chunks] with the chunk index XOR (((row >> 3) & 1) << 1):
//     each of ds_read_b128's four 16-lane groups (lanes {0-3,12-15,20-27}, ...) then touches 16
//     distinct 16-B bank slots (MI355X_MICROARCH.md §LDS).
//   * epilogue: eval BatchNorm as y = acc * scale + shift (torch's inference form: alpha = gamma /
//     sqrt(var + eps), beta = bias - mean * alpha), + residual, ReLU, NHWC store at a channel offset.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "conv_ws_common.h"
#include "nst_hip.h"
#include "seg_internal.h"

namespace nst {

namespace {

typedef __bf16 bf16x8_g __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_g __attribute__((ext_vector_type(8)));
typedef float f32x4_g __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_g __attribute__((ext_vector_type(4)));

// a use of the operand fragments after a stage's MFMAs: hipcc (ROCm 7.2) otherwise may allocate an MFMA's
// destination partially over a source register that dies at that MFMA (tools/check_mfma_overlap.py), which the
// matrix pipeline does not support
template <int N>
__device__ __forceinline__ void keep_live(const u32x4_g (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(v[i]));
}
__device__ __forceinline__ int chunk_swz(int row) { return ((row >> 3) & 1) << 1; }

// 16-bit activation formats (dt = NST_DT_BF16 / NST_DT_F16): exact unpack, round-to-nearest-even pack
__device__ __forceinline__ float h_to_f(uint16_t v, int dt) {
  return dt == NST_DT_F16 ? (float)__builtin_bit_cast(_Float16, v) : __uint_as_float((uint32_t)v << 16);
}
__device__ __forceinline__ uint16_t f_to_h(float f, int dt) {
  if (dt == NST_DT_F16) return __builtin_bit_cast(uint16_t, (_Float16)f);
  const uint32_t u = __float_as_uint(f);  // bf16 (finite inputs)
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// DT: the compute dtype (NST_DT_F32 = the exact-f32 parity mode, NST_DT_BF16, NST_DT_F16, or NST_DT_F32S: the fp32
// layout of the parity mode with each 16-B operand fragment (4 fp32 values of A and of B) split into fp16 pairs in
// registers, v = RNE16(v) + RNE16(v - RNE16(v)), and two v_mfma_f32_16x16x32_f16 per fragment pair instead of four
// v_mfma_f32_16x16x4_f32: [Ah Ah] x [Bh Bl] + [Al 0] x [Bh Bl] = Ah Bh + Ah Bl + Al Bh over the same 4 products per
// lane group (Al Bl, ~2^-22 of the product, dropped): ~22-bit products, fp32 accumulation)
__device__ __forceinline__ void split4(const u32x4_g& v, uint2& hi, uint2& lo) {
  float f[4] = {__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
  _Float16 h[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    h[k] = (_Float16)f[k];
    l[k] = (_Float16)(f[k] - (float)h[k]);
  }
  auto pk = [](_Float16 a, _Float16 b) {
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
  };
  hi = make_uint2(pk(h[0], h[1]), pk(h[2], h[3]));
  lo = make_uint2(pk(l[0], l[1]), pk(l[2], l[3]));
}
template <int BM, int BN, int DT, bool PF2>
__global__ __launch_bounds__(256, 2) void gemm_conv_kernel(GemmConvParams p) {
  constexpr bool SPL = DT == NST_DT_F32S;
  constexpr bool F32 = DT == NST_DT_F32 || SPL;  // fp32 activations and weights in memory and LDS
  constexpr int MI = BM / 32, NI = BN / 32;      // 16x16 sub-tiles per wave along rows / columns
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, BUF = A_BYTES + B_BYTES;
  constexpr int A_TPR = 256 / BM, A_CPT = 8 / A_TPR;  // loader threads per row, 16-B chunks per thread
  constexpr int B_TPR = 256 / BN, B_CPT = 8 / B_TPR;
  constexpr int ESZ = F32 ? 4 : 2;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  // the live-tap table in LDS: read from the kernel arguments with a dynamic index it is a vector memory load,
  // and the wait for it would also wait for every K stage still in flight
  __shared__ unsigned char s_taps[64];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 64) s_taps[tid] = p.taps[tid];
  __syncthreads();
  const int wm = wave & 1, wn = wave >> 1;
  const int pix0 = blockIdx.x * BN, row0 = blockIdx.y * BM;

  // ---- loader roles ----
  const int a_row = tid / A_TPR, a_c0 = (tid % A_TPR) * A_CPT;
  const int b_pix = tid / B_TPR, b_c0 = (tid % B_TPR) * B_CPT;
  const int gp = pix0 + b_pix;
  const bool pvalid = gp < p.npix;
  int img = 0, oy = 0, ox = 0;
  if (pvalid) {
    const int hw = p.ho * p.wo;
    img = gp / hw;
    const int r = gp - img * hw;
    oy = r / p.wo;
    ox = r - oy * p.wo;
  }
  const int iy0 = oy * p.stride - p.pad, ix0 = ox * p.stride - p.pad;
  const char* in_img = (const char*)p.in + (size_t)img * p.hi * p.wi * p.cs * ESZ + b_c0 * 16;
  // PF2 (launched only when the input tensor is under 2 GiB): the same addresses as 32-bit buffer offsets
  const uint32_t in_off0 = (uint32_t)((size_t)img * p.hi * p.wi * p.cs * ESZ + b_c0 * 16);
  const int n_img_all = p.npix / (p.ho * p.wo);
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.in, (short)0,
      __builtin_amdgcn_readfirstlane((int)std::min<long long>((long long)n_img_all * p.hi * p.wi * p.cs * ESZ, 0x7fffffffLL)),
      0x00020000);
  const int nck = p.cin / (128 / ESZ);
  const int nstage_all = p.kh * p.kw * nck;   // packed stages per 64-row block (every tap)
  const int nstage = p.ntaps * nck;           // stages this launch runs (live taps only)
  const int ablk = (row0 + a_row) >> 6;
  const char* wsrc = (const char*)p.wpk + ((size_t)ablk * nstage_all * 64 + (a_row & 63)) * 128 + a_c0 * 16;
  const size_t wstage = 64 * 128;
  // this workgroup's K slice (split-K: blockIdx.z of ksplit)
  const int s_begin = (int)(((long)nstage * blockIdx.z) / p.ksplit);
  const int s_end = (int)(((long)nstage * (blockIdx.z + 1)) / p.ksplit);

  u32x4_g ra[A_CPT], rb[B_CPT];
  auto load_into = [&](int s, u32x4_g (&ra)[A_CPT], u32x4_g (&rb)[B_CPT]) {
    const int ti = s / nck, cc = s - ti * nck;
    const int tap = __builtin_amdgcn_readfirstlane(s_taps[ti]);
    const char* wa = wsrc + (size_t)(tap * nck + cc) * wstage;
#pragma unroll
    for (int j = 0; j < A_CPT; ++j) ra[j] = *(const u32x4_g*)(wa + j * 16);
    const int ky = tap / p.kw, kx = tap - ky * p.kw;
    const int iy = iy0 + ky * p.dil, ix = ix0 + kx * p.dil;
    const bool ok = pvalid && (unsigned)iy < (unsigned)p.hi && (unsigned)ix < (unsigned)p.wi;
    if constexpr (PF2) {
      // buffer loads, zero past the tensor (offset 2^31): no branch around the loads, so the wait before a stage's
      // LDS store counts only the older stage's loads and the newer stage's stay in flight
      const uint32_t off = ok ? in_off0 + (uint32_t)(((iy * p.wi + ix) * p.cs) * ESZ + cc * 128) : 0x80000000u;
#pragma unroll
      for (int j = 0; j < B_CPT; ++j)
        rb[j] = __builtin_bit_cast(u32x4_g, __builtin_amdgcn_raw_buffer_load_b128(rs_in, off + j * 16, 0, 0));
    } else {
      const char* src = in_img + ((size_t)iy * p.wi + ix) * p.cs * ESZ + cc * 128;
#pragma unroll
      for (int j = 0; j < B_CPT; ++j) {
        u32x4_g v = {0u, 0u, 0u, 0u};
        if (ok) v = *(const u32x4_g*)(src + j * 16);
        rb[j] = v;
      }
    }
  };
  auto store_from = [&](int buf, const u32x4_g (&ra)[A_CPT], const u32x4_g (&rb)[B_CPT]) {
    char* A = lds + buf * BUF;
    char* B = A + A_BYTES;
#pragma unroll
    for (int j = 0; j < A_CPT; ++j) {
      const int c = a_c0 + j, half = c >> 2, q = c & 3;
      *(u32x4_g*)(A + half * (BM * 64) + a_row * 64 + ((q ^ chunk_swz(a_row)) << 4)) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_CPT; ++j) {
      const int c = b_c0 + j, half = c >> 2, q = c & 3;
      *(u32x4_g*)(B + half * (BN * 64) + b_pix * 64 + ((q ^ chunk_swz(b_pix)) << 4)) = rb[j];
    }
  };

  // ---- fragment addressing: lane (r16, g) reads row r16 of a 16-row sub-tile, chunk g (swizzled) ----
  const int r16 = lane & 15, g = lane >> 4;
  const int frag_off = r16 * 64 + ((g ^ chunk_swz(r16)) << 4);
  const int a_off = (wm * (BM / 2)) * 64 + frag_off;
  const int b_off = A_BYTES + (wn * (BN / 2)) * 64 + frag_off;

  f32x4_g acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4_g{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* base) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      u32x4_g a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = *(const u32x4_g*)(base + half * (BM * 64) + a_off + i * 16 * 64);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = *(const u32x4_g*)(base + half * (BN * 64) + b_off + j * 16 * 64);
      if constexpr (SPL) {
        u32x4_g ah[MI], al[MI], bb[NI];  // [Ah Ah], [Al 0], [Bh Bl] operand fragments
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          uint2 h, l;
          split4(a[i], h, l);
          ah[i] = u32x4_g{h.x, h.y, h.x, h.y};
          al[i] = u32x4_g{l.x, l.y, 0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          uint2 h, l;
          split4(b[j], h, l);
          bb[j] = u32x4_g{h.x, h.y, l.x, l.y};
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_g, ah[i]),
                                                               __builtin_bit_cast(f16x8_g, bb[j]), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_g, al[i]),
                                                               __builtin_bit_cast(f16x8_g, bb[j]), acc[i][j], 0, 0, 0);
          }
        keep_live(ah);
        keep_live(al);
        keep_live(bb);
        continue;
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if constexpr (F32) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].x), __uint_as_float(b[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].y), __uint_as_float(b[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].z), __uint_as_float(b[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].w), __uint_as_float(b[j].w), acc[i][j], 0, 0, 0);
          } else if constexpr (DT == NST_DT_F16) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_g, a[i]),
                                                               __builtin_bit_cast(f16x8_g, b[j]), acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_g, a[i]),
                                                                __builtin_bit_cast(bf16x8_g, b[j]), acc[i][j], 0, 0, 0);
          }
        }
      keep_live(a);
      keep_live(b);
    }
  };
  if constexpr (PF2) {
    // two stages in flight: stage s + 2's global loads go out before stage s's MFMAs, into the register set
    // stage s left (stored to LDS one step earlier); the loop is unrolled by two so both sets stay in registers.
    // The loads past the slice's end re-read its last stage (never stored).
    u32x4_g ra2[A_CPT], rb2[B_CPT];
    const int last = s_end - 1;
    load_into(s_begin, ra, rb);
    load_into(min(s_begin + 1, last), ra2, rb2);
    store_from(0, ra, rb);
    __syncthreads();
    for (int s = s_begin; s < s_end; s += 2) {
      load_into(min(s + 2, last), ra, rb);
      compute(lds);
      if (s + 1 < s_end) store_from(1, ra2, rb2);
      __syncthreads();
      if (s + 1 >= s_end) break;
      load_into(min(s + 3, last), ra2, rb2);
      compute(lds + BUF);
      if (s + 2 < s_end) store_from(0, ra, rb);
      __syncthreads();
    }
  } else {
    load_into(s_begin, ra, rb);
    store_from(0, ra, rb);
    __syncthreads();
    for (int s = s_begin; s < s_end; ++s) {
      const int cur = (s - s_begin) & 1;
      const bool more = s + 1 < s_end;
      if (more) load_into(s + 1, ra, rb);
      compute(lds + cur * BUF);
      if (more) store_from(cur ^ 1, ra, rb);
      __syncthreads();
    }
  }

  // ---- epilogue: lane owns output channels co..co+3 of one pixel per sub-tile ----
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int px = pix0 + wn * (BN / 2) + j * 16 + r16;
    if (px >= p.npix) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int co = row0 + wm * (BM / 2) + i * 16 + 4 * g;
      if (co >= p.cout_store) continue;
      if (p.ksplit > 1) {  // raw partial sums of this K slice; gemm_splitk_reduce applies the epilogue
        *(f32x4_g*)(p.partial + ((size_t)blockIdx.z * p.npix + px) * p.cout_store + co) = acc[i][j];
        continue;
      }
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = acc[i][j][q] * p.scale[co + q] + p.shift[co + q];
      if (p.res) {
        if constexpr (F32) {
          const float4 r = *(const float4*)((const float*)p.res + (size_t)px * p.res_cs + co);
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        } else {
          const uint2 r = *(const uint2*)((const uint16_t*)p.res + (size_t)px * p.res_cs + co);
          v[0] += h_to_f((uint16_t)(r.x & 0xffff), DT); v[1] += h_to_f((uint16_t)(r.x >> 16), DT);
          v[2] += h_to_f((uint16_t)(r.y & 0xffff), DT); v[3] += h_to_f((uint16_t)(r.y >> 16), DT);
        }
      }
      if (p.relu) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
      }
      const size_t o = (size_t)px * p.out_cs + p.out_off + co;
      if (F32 || p.out_f32) {
        *(float4*)((float*)p.out + o) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint2 w;
        w.x = (uint32_t)f_to_h(v[0], DT) | ((uint32_t)f_to_h(v[1], DT) << 16);
        w.y = (uint32_t)f_to_h(v[2], DT) | ((uint32_t)f_to_h(v[3], DT) << 16);
        *(uint2*)((uint16_t*)p.out + o) = w;
      }
    }
  }
}

// ---- LDS-DMA form (bf16 / fp16): BM x BN tiles (BM 128, or 64 for 64-channel outputs), 8 waves, one workgroup per CU ----
// The register-staged kernel above keeps one stage in flight and spends VGPRs and ds_writes on the staging; here
// every stage lands in LDS by LDS-DMA (buffer_load_dwordx4 ... lds: no VGPR destination, zero for any offset past
// the buffer = the im2col's zero padding) into a 3-slot ring, two stages ahead of the MFMAs, with counted vmcnt
// waits and one raw barrier per stage (MI355X_MICROARCH / cdna_hip_programming 'glds ... 3 LDS buffers').
//   * LDS image of a stage: rows (A: BM output channels, B: BN pixels) x 128 B, lane-linear per DMA
//     instruction (8 rows x 8 16-B slots); slot s of row r holds K chunk s ^ ((r >> 1) & 7), so the four 16-lane
//     groups of every fragment ds_read_b128 (16 consecutive rows, chunk 4h + g) hit 16 distinct bank slots.
//   * waves BM/64 (M) x 8/(BM/64) (N): 64 channels x BN/WN pixels each, v_mfma_f32_16x16x32_{bf16,f16}; the same
//     epilogue (and split-K partials) as the register-staged kernel.  BM = 64 serves 64-channel outputs (VGG's
//     conv1_2 and the dgrads into 64-channel maps) without a half-empty A tile: half the MFMAs and a quarter fewer
//     fragment reads per output than 128 x 256.
constexpr uint32_t GL_OOB = 0xFFFFFF00u;
template <int BM, int BN, int DT, int RING>
__global__ __launch_bounds__(512) void gemm_glds_kernel(GemmConvParams p, uint32_t w_bytes, uint32_t in_bytes) {
  constexpr int NW = 8, WM = BM / 64, WN = NW / WM;   // wave grid
  constexpr int MI = 4, NI = BN / (16 * WN);           // 16x16 sub-tiles per wave
  static_assert(BM == 64 || BM == 128 || BM == 256, "BM");
  static_assert(NI >= 1 && BN % (16 * WN) == 0, "BN");
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, BUF = A_BYTES + B_BYTES;
  constexpr int A_INS = A_BYTES / 1024 / NW, B_INS = B_BYTES / 1024 / NW;  // DMA instructions per wave and stage
  constexpr int NINS = A_INS + B_INS;
  constexpr bool F32 = DT == NST_DT_F32;
  constexpr int ESZ = F32 ? 4 : 2, CK = 128 / ESZ;  // bytes per element, channels per stage
  static_assert(RING >= 2 && RING <= 4, "ring");
  __shared__ __attribute__((aligned(16))) char lds[RING * BUF];
  // live-tap table in LDS (as gemm_conv_kernel): a kernel-argument read with a dynamic index is a vector memory
  // load whose wait (vmcnt(0)) would drain every DMA stage in flight before each issue
  __shared__ unsigned char s_taps[64];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  if (tid < 64) s_taps[tid] = p.taps[tid];
  __syncthreads();
  const int pix0 = blockIdx.x * BN, row0 = blockIdx.y * BM;
  const int nck = p.cin / CK;
  const int nstage_all = p.kh * p.kw * nck;
  const int nstage = p.ntaps * nck;
  const int s_begin = (int)(((long)nstage * blockIdx.z) / p.ksplit);
  const int s_end = (int)(((long)nstage * (blockIdx.z + 1)) / p.ksplit);

  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)p.wpk, (short)0, (int)w_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc((void*)p.in, (short)0, (int)in_bytes, 0x00020000);
  // this lane's rows: DMA instruction j of this wave covers image rows 8 * (j * NW + wave) + lane / 8, slot lane % 8
  const int slot = lane & 7;
  uint32_t a_off[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int r = 8 * (j * NW + wave) + (lane >> 3);
    const int co = row0 + r;
    const int c = slot ^ ((r >> 1) & 7);
    a_off[j] = ((uint32_t)((co >> 6) * nstage_all) * 64u + (uint32_t)(co & 63)) * 128u + (uint32_t)c * 16u;
  }
  uint32_t b_off[B_INS];
  int b_iy[B_INS], b_ix[B_INS];
  const int hw = p.ho * p.wo;
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int r = 8 * (j * NW + wave) + (lane >> 3);
    const int gp = pix0 + r;
    const int c = slot ^ ((r >> 1) & 7);
    if (gp < p.npix) {
      const int img = gp / hw, rr = gp - img * hw;
      const int oy = rr / p.wo, ox = rr - oy * p.wo;
      b_iy[j] = oy * p.stride - p.pad;
      b_ix[j] = ox * p.stride - p.pad;
      b_off[j] = (uint32_t)(((img * p.hi + b_iy[j]) * p.wi + b_ix[j]) * p.cs) * ESZ + (uint32_t)c * 16u;
    } else {
      b_iy[j] = -(1 << 28);  // never in range
      b_ix[j] = 0;
      b_off[j] = 0;
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
  auto issue = [&](int s) {  // stage s -> ring slot s % RING
    const uint32_t base = lds0 + (uint32_t)((s % RING) * BUF);
    const int ti = s / nck, cc = s - ti * nck;
    const int tap = __builtin_amdgcn_readfirstlane(s_taps[ti]);
    const int ky = tap / p.kw, kx = tap - ky * p.kw;
    const uint32_t wst = (uint32_t)(tap * nck + cc) * 8192u;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) dma16(rs_w, a_off[j] + wst, base + (uint32_t)((j * NW + wave) * 1024), 0);
    const int dy = ky * p.dil, dx = kx * p.dil;
    const int toff = ((dy * p.wi + dx) * p.cs + cc * CK) * ESZ;
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const bool ok = (unsigned)(b_iy[j] + dy) < (unsigned)p.hi && (unsigned)(b_ix[j] + dx) < (unsigned)p.wi;
      dma16(rs_in, ok ? b_off[j] + (uint32_t)toff : GL_OOB, base + (uint32_t)(A_BYTES + (j * NW + wave) * 1024), 0);
    }
  };

  // fragment addressing: lane (r16, g) reads row r16 of a 16-row sub-tile, chunk 4h + g
  const int r16 = lane & 15, g = lane >> 4;
  const int sw = (r16 >> 1) & 7;
  const int fo0 = r16 * 128 + (((0 + g) ^ sw) << 4), fo1 = r16 * 128 + (((4 + g) ^ sw) << 4);
  const int a_base = wm * 64 * 128, b_base = A_BYTES + wn * (BN / WN) * 128;

  f32x4_g acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4_g{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int k = 0; k < RING - 1; ++k)
    if (s_begin + k < s_end) issue(s_begin + k);
  for (int s = s_begin; s < s_end; ++s) {
    // stage s landed (the RING - 2 stages after it may stay in flight); the barrier also ends every wave's reads
    // of slot (s + RING - 1) % RING
    const int ahead = std::min(RING - 2, s_end - 1 - s);
    if (ahead >= 2) vm_wait<2 * NINS>();
    else if (ahead == 1) vm_wait<NINS>();
    else vm_wait<0>();
    lds_barrier();
    if (s + RING - 1 < s_end) issue(s + RING - 1);
    const char* base = lds + (s % RING) * BUF;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int fo = h ? fo1 : fo0;
      u32x4_g a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = *(const u32x4_g*)(base + a_base + i * 16 * 128 + fo);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = *(const u32x4_g*)(base + b_base + j * 16 * 128 + fo);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if constexpr (F32) {  // 16x16x4 f32 over the 16-B fragment: the same K permutation for A and B
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].x), __uint_as_float(b[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].y), __uint_as_float(b[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].z), __uint_as_float(b[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].w), __uint_as_float(b[j].w), acc[i][j], 0, 0, 0);
          } else if constexpr (DT == NST_DT_F16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_g, a[i]),
                                                               __builtin_bit_cast(f16x8_g, b[j]), acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_g, a[i]),
                                                                __builtin_bit_cast(bf16x8_g, b[j]), acc[i][j], 0, 0, 0);
        }
      keep_live(a);
      keep_live(b);
    }
  }
  vm_wait<0>();  // no DMA lands after the workgroup releases its LDS

  // ---- epilogue (as gemm_conv_kernel's): lane owns output channels co..co+3 of one pixel per sub-tile ----
  auto finish = [&](int px, int co, const f32x4_g& a) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = a[q] * p.scale[co + q] + p.shift[co + q];
    if (p.res) {
      if constexpr (F32) {
        const float4 r = *(const float4*)((const float*)p.res + (size_t)px * p.res_cs + co);
        v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
      } else {
        const uint2 r = *(const uint2*)((const uint16_t*)p.res + (size_t)px * p.res_cs + co);
        v[0] += h_to_f((uint16_t)(r.x & 0xffff), DT); v[1] += h_to_f((uint16_t)(r.x >> 16), DT);
        v[2] += h_to_f((uint16_t)(r.y & 0xffff), DT); v[3] += h_to_f((uint16_t)(r.y >> 16), DT);
      }
    }
    if (p.relu) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
    }
    const size_t o = (size_t)px * p.out_cs + p.out_off + co;
    if (F32 || p.out_f32) {
      *(float4*)((float*)p.out + o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      uint2 w;
      w.x = (uint32_t)f_to_h(v[0], DT) | ((uint32_t)f_to_h(v[1], DT) << 16);
      w.y = (uint32_t)f_to_h(v[2], DT) | ((uint32_t)f_to_h(v[3], DT) << 16);
      *(uint2*)((uint16_t*)p.out + o) = w;
    }
  };
  if (p.ksplit == 1) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int px = pix0 + wn * (BN / WN) + j * 16 + r16;
      if (px >= p.npix) continue;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int co = row0 + wm * 64 + i * 16 + 4 * g;
        if (co < p.cout_store) finish(px, co, acc[i][j]);
      }
    }
    return;
  }
  // split K: this slice's fp32 partial (gemm_splitk_reduce sums the slices in slice order)
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int px = pix0 + wn * (BN / WN) + j * 16 + r16;
    if (px >= p.npix) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int co = row0 + wm * 64 + i * 16 + 4 * g;
      if (co < p.cout_store) *(f32x4_g*)(p.partial + ((size_t)blockIdx.z * p.npix + px) * p.cout_store + co) = acc[i][j];
    }
  }
}

// split-K epilogue: sum the K slices in slice order, then scale/shift, residual, ReLU, store (as the
// single-pass epilogue does)
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmConvParams p, int dt) {
  const bool f32 = dt == NST_DT_F32 || dt == NST_DT_F32S;
  const int groups = p.cout_store >> 2;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)p.npix * groups) return;
  const int px = (int)(e / groups), co = (int)(e % groups) * 4;
  f32x4_g a = *(const f32x4_g*)(p.partial + (size_t)px * p.cout_store + co);
  for (int z = 1; z < p.ksplit; ++z) a += *(const f32x4_g*)(p.partial + ((size_t)z * p.npix + px) * p.cout_store + co);
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = a[q] * p.scale[co + q] + p.shift[co + q];
  if (p.res) {
    if (f32) {
      const float4 r = *(const float4*)((const float*)p.res + (size_t)px * p.res_cs + co);
      v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
    } else {
      const uint2 r = *(const uint2*)((const uint16_t*)p.res + (size_t)px * p.res_cs + co);
      v[0] += h_to_f((uint16_t)(r.x & 0xffff), dt); v[1] += h_to_f((uint16_t)(r.x >> 16), dt);
      v[2] += h_to_f((uint16_t)(r.y & 0xffff), dt); v[3] += h_to_f((uint16_t)(r.y >> 16), dt);
    }
  }
  if (p.relu) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
  }
  const size_t o = (size_t)px * p.out_cs + p.out_off + co;
  if (f32 || p.out_f32) {
    *(float4*)((float*)p.out + o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 w;
    w.x = (uint32_t)f_to_h(v[0], dt) | ((uint32_t)f_to_h(v[1], dt) << 16);
    w.y = (uint32_t)f_to_h(v[2], dt) | ((uint32_t)f_to_h(v[3], dt) << 16);
    *(uint2*)((uint16_t*)p.out + o) = w;
  }
}

// register-staged kernel: two K stages in flight (NST_GEMM_PF2, default on) instead of one
int gemm_pf2() {
  static const int v = [] {
    const char* e = std::getenv("NST_GEMM_PF2");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}
template <int BM, int BN>
void launch_tile(int dt, const GemmConvParams& p, hipStream_t st) {
  const dim3 grid((unsigned)((p.npix + BN - 1) / BN), (unsigned)((p.cout_store + BM - 1) / BM), (unsigned)p.ksplit);
  // PF2: the 16-bit and split kernels (the exact-f32 one keeps one stage in flight: with two, hipcc allocated
  // 16x16x4f32 MFMA destinations partially over a source, tools/check_mfma_overlap.py), inputs under 2 GiB
  const long long in_bytes = (long long)(p.npix / std::max(1, p.ho * p.wo)) * p.hi * p.wi * p.cs *
                             (dt == NST_DT_F32 || dt == NST_DT_F32S ? 4 : 2);
  if (gemm_pf2() && dt != NST_DT_F32 && in_bytes < 0x7fffffffLL) {
    if (dt == NST_DT_F32S) hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_F32S, true>), grid, dim3(256), 0, st, p);
    else if (dt == NST_DT_F16) hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_F16, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_BF16, true>), grid, dim3(256), 0, st, p);
    return;
  }
  if (dt == NST_DT_F32) hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_F32, false>), grid, dim3(256), 0, st, p);
  else if (dt == NST_DT_F32S) hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_F32S, false>), grid, dim3(256), 0, st, p);
  else if (dt == NST_DT_F16) hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_F16, false>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((gemm_conv_kernel<BM, BN, NST_DT_BF16, false>), grid, dim3(256), 0, st, p);
}

// taps whose source row AND column land inside the image for at least one output pixel
void live_taps(GemmConvParams& p) {
  p.ntaps = 0;
  for (int ky = 0; ky < p.kh; ++ky) {
    bool row = false;
    for (int oy = 0; oy < p.ho && !row; ++oy) {
      const int iy = oy * p.stride - p.pad + ky * p.dil;
      row = iy >= 0 && iy < p.hi;
    }
    if (!row) continue;
    for (int kx = 0; kx < p.kw; ++kx) {
      bool col = false;
      for (int ox = 0; ox < p.wo && !col; ++ox) {
        const int ix = ox * p.stride - p.pad + kx * p.dil;
        col = ix >= 0 && ix < p.wi;
      }
      if (col) p.taps[p.ntaps++] = (unsigned char)(ky * p.kw + kx);
    }
  }
}

// launch shape.  16-bit: the LDS-DMA kernel (128 x 256 tiles when they fill the chip, else 128 x 128, split in
// K up to about a wave of the chip) unless the tensors exceed its 32-bit buffer offsets or the GEMM is too
// small to fill half the chip that way.  Otherwise (and fp32) the register-staged kernel: 128x128 tiles when
// they fill the chip, split in K over them for deep K when they fill a quarter of it (Gatys 512^2 1.74 -> 1.47 ms
// per Adam step from VGG conv4_x; DeepLab's shorter-K layers measured slower that way, hence the floor), else
// 64x64 tiles, split when fewer than a wave of the chip.
#ifndef NST_GEMM_GLDS
#define NST_GEMM_GLDS 1
#endif
// fp32 on the LDS-DMA kernel: measured slower for the configs[4] mask at its 256-px working size (4.07 -> 4.65 ms,
// tools/gpu_gemm_sweep.sh), slightly faster at full 1080p (91 -> 98 TFLOP/s): off
#ifndef NST_GEMM_GLDS_F32
#define NST_GEMM_GLDS_F32 0
#endif
#ifndef NST_GEMM_RING_32K  // ring depth for tiles whose stage is 32 KB (128 x 128); 4 (three stages in flight) measured
#define NST_GEMM_RING_32K 3   // 1.161 -> 1.169 ms per Gatys step (r03_m2)
#endif
// sweep override of the 32 KB-stage ring depth (NST_GEMM_RING32=4)
int gemm_ring32() {
  static const int v = [] {
    const char* e = std::getenv("NST_GEMM_RING32");
    return e ? std::atoi(e) : NST_GEMM_RING_32K;
  }();
  return v;
}
// runtime override (NST_GEMM_GLDS_F32=1): fp32 / fp32s GEMMs on the LDS-DMA kernel (exact-f32 MFMAs)
int gemm_glds_f32() {
  static const int v = [] {
    const char* e = std::getenv("NST_GEMM_GLDS_F32");
    return e ? std::atoi(e) : NST_GEMM_GLDS_F32;
  }();
  return v;
}
#ifndef NST_GEMM_BIG_SPLIT_MIN_STAGES
#define NST_GEMM_BIG_SPLIT_MIN_STAGES 64
#endif
#ifndef NST_GEMM_SPLIT256  // 128 x 256 tiles split in K where 128 x 128 tiles would run unsplit / less split
#define NST_GEMM_SPLIT256 1
#endif
#ifndef NST_GEMM_BM64  // 64 x 256 LDS-DMA tiles for outputs of at most 64 channels
#define NST_GEMM_BM64 1
#endif
// 256 x 256 LDS-DMA tiles (a 128 x 64 block per wave: a quarter fewer LDS fragment bytes per MFMA than 128 x 256,
// one stage in flight in a 2 x 64 KB ring), split in K to fill the chip: NST_GEMM_T256=1 enables them
enum GemmKind { GK_REG64 = 0, GK_REG128 = 1, GK_GLDS256 = 2, GK_GLDS128 = 3, GK_GLDS64x256 = 4, GK_GLDS256x256 = 5 };
int gemm_t256() {
  static const int v = [] {
    const char* e = std::getenv("NST_GEMM_T256");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
// register-staged 64 x 64 tiles: split K while there are fewer than reg_tiles() tiles, to about reg_target()
// workgroups (sweep overrides NST_GEMM_REG_TILES / NST_GEMM_REG_TARGET; defaults 240 / 480)
int gemm_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
int reg_tiles() {
  static const int v = gemm_env("NST_GEMM_REG_TILES", 240);
  return v;
}
int reg_target() {
  static const int v = gemm_env("NST_GEMM_REG_TARGET", 480);
  return v;
}
struct GemmShape {
  int kind;
  int ksplit;
};
GemmShape gemm_shape(int dtype, const GemmConvParams& p) {
  if (dtype == NST_DT_F32S) dtype = NST_DT_F32;  // the fp32 layout and launch shapes (register-staged kernel)
  const int nstage = p.ntaps * (p.cin / gemm_stage_channels(dtype));
  const long mt = (p.cout_store + 127) / 128;
  GemmShape g{GK_REG64, 1};
  if (NST_GEMM_GLDS && (dtype != NST_DT_F32 || gemm_glds_f32())) {
    const int esz = dtype == NST_DT_F32 ? 4 : 2;
    const long n_img = p.npix / std::max(1, p.ho * p.wo);
    const double in_b = (double)n_img * p.hi * p.wi * p.cs * esz;
    const double w_b = (double)((p.cout_store + 63) / 64) * p.kh * p.kw * (p.cin / (128 / esz)) * 8192.0;
    if (in_b < 2147483648.0 && w_b < 2147483648.0) {
      const long t256 = (long)((p.npix + 255) / 256) * mt, t128 = (long)((p.npix + 127) / 128) * mt;
      if (gemm_t256() && dtype != NST_DT_F32 && p.cout_store > 128 && nstage >= 16) {
        const long tt = (long)((p.npix + 255) / 256) * ((p.cout_store + 255) / 256);
        const long k = std::max<long>(1, std::min<long>((256 + tt - 1) / tt, std::min<long>(8, nstage / 8)));
        if (tt * k >= 128) return GemmShape{GK_GLDS256x256, (int)k};
      }
      if (t256 >= 200) return GemmShape{NST_GEMM_BM64 && p.cout_store <= 64 ? GK_GLDS64x256 : GK_GLDS256, 1};
      if (NST_GEMM_SPLIT256 && p.cout_store > 64 && t128 < 200 && t256 >= 32 && nstage >= 16) {
        // a 128 x 256 tile reads a third less LDS per output than 128 x 128 (64 x 64 per wave instead of 64 x 32);
        // only where 128 x 128 tiles would be split anyway (an unsplit conv3_x: 34.3 us, split 128 x 256: 28.6 + a
        // 7.4 us reduce)
        const long k2 = std::max<long>(1, std::min<long>((256 + t256 - 1) / t256, std::min<long>(8, nstage / 8)));
        if (t256 * k2 >= 200) return GemmShape{GK_GLDS256, (int)k2};
      }
      long k = 1;
      if (t128 < 200 && nstage >= 16) k = std::max<long>(1, std::min<long>((256 + t128 - 1) / t128, std::min<long>(8, nstage / 8)));
      if (t128 * k >= 128) return GemmShape{GK_GLDS128, (int)k};
    }
  }
  const long tiles128 = (long)((p.npix + 127) / 128) * mt;
  if (tiles128 >= 256) return GemmShape{GK_REG128, 1};
  if (tiles128 >= 64 && nstage >= NST_GEMM_BIG_SPLIT_MIN_STAGES) {
    long k = (480 + tiles128 - 1) / tiles128;
    k = std::min<long>(k, std::min<long>(8, nstage / 8));
    if (k > 1) return GemmShape{GK_REG128, (int)k};
  }
  // fewer 64x64 tiles than a wave of the chip and a long K loop: split K (at most 8 slices)
  const long tiles = (long)((p.npix + 63) / 64) * ((p.cout_store + 63) / 64);
  if (tiles < reg_tiles() && nstage >= 16) {
    long k = (reg_target() + tiles - 1) / tiles;
    k = std::min<long>(k, std::min<long>(8, nstage / 8));
    g.ksplit = (int)std::max<long>(k, 1);
  }
  return g;
}

template <int BM, int BN>
void launch_glds(int dt, const GemmConvParams& p, hipStream_t st) {
  if (dt == NST_DT_F32S) dt = NST_DT_F32;  // the fp32 layout; exact-f32 MFMAs on this kernel
  const int esz = dt == NST_DT_F32 ? 4 : 2;
  const long n_img = p.npix / std::max(1, p.ho * p.wo);
  const uint32_t in_b = (uint32_t)(n_img * p.hi * p.wi * p.cs * esz);
  const uint32_t w_b = (uint32_t)((p.cout_store + 63) / 64) * (uint32_t)(p.kh * p.kw * (p.cin / (128 / esz))) * 8192u;
  const dim3 grid((unsigned)((p.npix + BN - 1) / BN), (unsigned)((p.cout_store + BM - 1) / BM), (unsigned)p.ksplit);
  // 4 x 32 KB stages fit the LDS, 4 x 48 KB do not, 2 x 64 KB (256 x 256) do
  constexpr int RING = BM * 128 + BN * 128 <= 32768 ? NST_GEMM_RING_32K : (BM * 128 + BN * 128 <= 49152 ? 3 : 2);
  if constexpr (BM * 128 + BN * 128 <= 32768 && NST_GEMM_RING_32K != 4) {
    if (gemm_ring32() == 4 && dt == NST_DT_BF16) {  // sweep override: three 32 KB stages in flight
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, NST_DT_BF16, 4>), grid, dim3(512), 0, st, p, w_b, in_b);
      return;
    }
  }
  if (dt == NST_DT_F16) hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, NST_DT_F16, RING>), grid, dim3(512), 0, st, p, w_b, in_b);
  else if (dt == NST_DT_F32) {
    // (no fp32 256 x 256 form: hipcc gives its 16x16x4f32 MFMAs partially overlapping registers)
    if constexpr (BM < 256) hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, NST_DT_F32, RING>), grid, dim3(512), 0, st, p, w_b, in_b);
  }
  else hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, NST_DT_BF16, RING>), grid, dim3(512), 0, st, p, w_b, in_b);
}

}  // namespace

size_t gemm_partial_bytes(int dtype, const GemmConvParams& p0) {
  GemmConvParams p = p0;
  live_taps(p);
  const GemmShape g = gemm_shape(dtype, p);
  return g.ksplit > 1 ? (size_t)g.ksplit * p.npix * p.cout_store * 4 : 0;
}

hipError_t launch_gemm_conv(int dtype, GemmConvParams& p, hipStream_t st) {
  const int ck = gemm_stage_channels(dtype);
  if (p.npix <= 0 || p.cin <= 0 || p.cin % ck || p.cs % 8 || p.cout_store % 4 || p.out_off % 4 ||
      p.out_cs % 4 || (p.res && p.res_cs % 4) || p.kh * p.kw > 64)
    return hipErrorInvalidValue;
  live_taps(p);
  if (p.ntaps == 0) return hipErrorInvalidValue;
  const GemmShape g = gemm_shape(dtype, p);
  p.ksplit = p.partial ? g.ksplit : 1;
  if (g.kind == GK_GLDS256x256) launch_glds<256, 256>(dtype, p, st);
  else if (g.kind == GK_GLDS64x256) launch_glds<64, 256>(dtype, p, st);
  else if (g.kind == GK_GLDS256) launch_glds<128, 256>(dtype, p, st);
  else if (g.kind == GK_GLDS128) launch_glds<128, 128>(dtype, p, st);
  else if (g.kind == GK_REG128) launch_tile<128, 128>(dtype, p, st);
  else launch_tile<64, 64>(dtype, p, st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.ksplit == 1) return e;
  const size_t n = (size_t)p.npix * (p.cout_store / 4);
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, dtype);
  return hipGetLastError();
}

}  // namespace nst
