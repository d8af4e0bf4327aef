// peak_bench.hip — measured ceilings of the box ("spec values ... must be replaced by
// measured peaks"): dense bf16 MFMA throughput (v_mfma_f32_16x16x32_bf16, the instruction of every
// benchmarked conv) and HBM stream bandwidth.  Standalone tool, not part of the library.
//   hipcc --offload-arch=gfx950 -O3 tools/peak_bench.hip -o tools/peak_bench && tools/peak_bench
// Prints one JSON object.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

// 8 independent accumulation chains per wave (an MFMA's result is not needed by the next 7), operands
// from registers: the loop is MFMAs back to back.  `src` holds random bf16 (the conv kernels' data
// is not zeros, and data toggling sets the power, hence the clock)
__global__ __launch_bounds__(256) void mfma_loop(const u32x4_t* __restrict__ src, float* __restrict__ out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const u32x4_t a = src[t & 4095], b = src[(t + 1024) & 4095];
  f32x4_t c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
  for (int i = 0; i < iters; ++i) {
#define M(c) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b))
    M(c0); M(c1); M(c2); M(c3); M(c4); M(c5); M(c6); M(c7);
#undef M
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  const f32x4_t s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[t] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 v0 = in[i], v1 = in[i + stride], v2 = in[i + 2 * stride], v3 = in[i + 3 * stride];
    out[i] = v0; out[i + stride] = v1; out[i + 2 * stride] = v2; out[i + 3 * stride] = v3;
  }
  for (; i < n; i += stride) out[i] = in[i];
}

__global__ __launch_bounds__(256) void read_kernel(const uint4* __restrict__ in, size_t n, unsigned* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned x = 0;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 v0 = in[i], v1 = in[i + stride], v2 = in[i + 2 * stride], v3 = in[i + 3 * stride];
    x ^= v0.x ^ v1.y ^ v2.z ^ v3.w;
  }
  for (; i < n; i += stride) x ^= in[i].x;
  if (x == 0x9e3779b9u) out[0] = x;  // practically never: keeps the loads live
}

// Contiguous-chunk forms (each workgroup streams one contiguous slice, U float4 loads in flight per thread before
// the first store), with plain or non-temporal (nt) stores: the grid-stride form above interleaves the whole grid's
// accesses and measured 4.65-5.08 TB/s, below the guide's 6.29 TB/s float4 copy.
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunk_kernel(const uint4* __restrict__ in_, uint4* __restrict__ out_,
                                                         size_t n) {
  const u32x4_t* in = (const u32x4_t*)in_;
  u32x4_t* out = (u32x4_t*)out_;
  const size_t per = (size_t)256 * U;
  for (size_t base = (size_t)blockIdx.x * per; base < n; base += (size_t)gridDim.x * per) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256 + threadIdx.x;
      if (i < n) v[u] = NT ? __builtin_nontemporal_load(in + i) : in[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256 + threadIdx.x;
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v[u], out + i);
        else out[i] = v[u];
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_chunk_kernel(const uint4* __restrict__ in, size_t n,
                                                         unsigned* __restrict__ out) {
  const size_t per = (size_t)256 * U;
  unsigned x = 0;
  for (size_t base = (size_t)blockIdx.x * per; base < n; base += (size_t)gridDim.x * per) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256 + threadIdx.x;
      v[u] = i < n ? in[i] : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (x == 0x9e3779b9u) out[0] = x;
}

static uint16_t bf16_of(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_ms = [&](auto&& launch, int reps) -> float {
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
  };

  // ---- MFMA: random bf16 in [-1, 1] and zeros; 2 and 4 waves per SIMD ----
  std::vector<uint16_t> h(4096 * 8);
  uint32_t seed = 12345u;
  for (auto& v : h) {
    seed = seed * 1664525u + 1013904223u;
    v = bf16_of(((seed >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f);
  }
  u32x4_t *d_rand = nullptr, *d_zero = nullptr;
  float* d_out = nullptr;
  CK(hipMalloc(&d_rand, 4096 * 16));
  CK(hipMalloc(&d_zero, 4096 * 16));
  CK(hipMemcpy(d_rand, h.data(), 4096 * 16, hipMemcpyHostToDevice));
  CK(hipMemset(d_zero, 0, 4096 * 16));
  const int iters = 4096;
  double mfma_tf[2][2] = {};
  for (int z = 0; z < 2; ++z) {
    for (int occ = 0; occ < 2; ++occ) {
      const int waves_per_cu = occ ? 16 : 8;  // 4 or 2 waves per SIMD
      const int blocks = cus * waves_per_cu / 4;
      CK(hipMalloc(&d_out, (size_t)blocks * 256 * 4));
      const u32x4_t* src = z ? d_zero : d_rand;
      const float ms = time_ms([&] { hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, src, d_out, iters); }, 5);
      CK(hipGetLastError());
      const double flop = (double)blocks * 4 * iters * 8 * 16384.0;
      mfma_tf[z][occ] = flop / (ms * 1e-3) / 1e12;
      CK(hipFree(d_out));
    }
  }

  // ---- HBM: 2 GiB copy (read + write) and 2 GiB read ----
  const size_t bytes = (size_t)2 << 30, n = bytes / 16;
  uint4 *a = nullptr, *b = nullptr;
  unsigned* sink = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 1, bytes));
  double copy_gbs = 0.0, read_gbs = 0.0;  // best over grid sizes (workgroups per CU)
  for (int wpc : {8, 16, 32, 64, 128}) {
    const int gb = cus * wpc;
    const float copy_ms = time_ms([&] { hipLaunchKernelGGL(copy_kernel, dim3(gb), dim3(256), 0, 0, a, b, n); }, 10);
    const float read_ms = time_ms([&] { hipLaunchKernelGGL(read_kernel, dim3(gb), dim3(256), 0, 0, a, n, sink); }, 10);
    CK(hipGetLastError());
    copy_gbs = std::fmax(copy_gbs, 2.0 * bytes / (copy_ms * 1e-3) / 1e9);
    read_gbs = std::fmax(read_gbs, bytes / (read_ms * 1e-3) / 1e9);
  }
  // contiguous-chunk forms: best over unroll depth, nt, and grid size (1-8 workgroups per CU, or one slice each)
  double chunk_copy_gbs = 0.0, chunk_read_gbs = 0.0;
  char chunk_copy_cfg[64] = "", chunk_read_cfg[64] = "";
  for (int wpc : {1, 2, 4, 8, 0}) {
    auto go = [&](auto kern, int u, bool nt) -> int {
      const size_t per = (size_t)256 * u;
      const int gb = wpc ? cus * wpc : (int)((n + per - 1) / per);
      const float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(gb), dim3(256), 0, 0, a, b, n); }, 10);
      CK(hipGetLastError());
      const double g = 2.0 * bytes / (ms * 1e-3) / 1e9;
      if (g > chunk_copy_gbs) {
        chunk_copy_gbs = g;
        std::snprintf(chunk_copy_cfg, sizeof(chunk_copy_cfg), "U%d%s wg/cu %d", u, nt ? " nt" : "", wpc);
      }
      return 0;
    };
    go(copy_chunk_kernel<4, false>, 4, false);
    go(copy_chunk_kernel<8, false>, 8, false);
    go(copy_chunk_kernel<4, true>, 4, true);
    go(copy_chunk_kernel<8, true>, 8, true);
    go(copy_chunk_kernel<16, true>, 16, true);
    auto rd = [&](auto kern, int u) -> int {
      const size_t per = (size_t)256 * u;
      const int gb = wpc ? cus * wpc : (int)((n + per - 1) / per);
      const float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(gb), dim3(256), 0, 0, a, n, sink); }, 10);
      CK(hipGetLastError());
      const double g = bytes / (ms * 1e-3) / 1e9;
      if (g > chunk_read_gbs) {
        chunk_read_gbs = g;
        std::snprintf(chunk_read_cfg, sizeof(chunk_read_cfg), "U%d wg/cu %d", u, wpc);
      }
      return 0;
    };
    rd(read_chunk_kernel<4>, 4);
    rd(read_chunk_kernel<8>, 8);
    rd(read_chunk_kernel<16>, 16);
  }

  std::printf(
      "{\"device\": \"%s\", \"cus\": %d, \"mfma_bf16_16x16x32_tflops\": {\"random_2w\": %.1f, \"random_4w\": %.1f, "
      "\"zeros_2w\": %.1f, \"zeros_4w\": %.1f}, \"hbm_copy_gbs\": %.1f, \"hbm_read_gbs\": %.1f, "
      "\"hbm_copy_grid_stride_gbs\": %.1f, \"hbm_read_grid_stride_gbs\": %.1f, "
      "\"hbm_copy_chunk_gbs\": %.1f, \"hbm_copy_chunk_cfg\": \"%s\", \"hbm_read_chunk_gbs\": %.1f, "
      "\"hbm_read_chunk_cfg\": \"%s\", \"spec\": {\"mfma_bf16_tflops\": 2500, \"hbm_gbs\": 8000}}\n",
      prop.gcnArchName, cus, mfma_tf[0][0], mfma_tf[0][1], mfma_tf[1][0], mfma_tf[1][1],
      std::fmax(copy_gbs, chunk_copy_gbs), std::fmax(read_gbs, chunk_read_gbs), copy_gbs, read_gbs, chunk_copy_gbs,
      chunk_copy_cfg, chunk_read_gbs, chunk_read_cfg);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  CK(hipFree(d_rand));
  CK(hipFree(d_zero));
  return 0;
}
