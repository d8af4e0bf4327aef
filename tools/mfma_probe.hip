// mfma_probe.hip — cycles per v_mfma_f32_32x32x16_bf16 in conv_wst32.hip's K-loop pattern, one wave per SIMD
// (scratch measurement for the round-6 trunk kernel; not part of the library).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe && ./tools/mfma_probe
// Variants: A operand (weights) from AGPRs or VGPRs; B operands from a fixed register ring or re-read from LDS
// (ds_read_b128, ring of 3 reads ahead as the kernel); the kernel's order (per read: rows y, y-1, y-2; K halves
// kk = 0, 1 back to back) or rows interleaved.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <bool AG>
__device__ __forceinline__ void mf(f32x16_t& c, const u32x4_t& a, const u32x4_t& b) {
  if constexpr (AG) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
  else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

constexpr int TH = 8, LH = 10, NRD = 2 * LH, PRD = 3 * NRD;

// MODE 0: B from a fixed register set; 1: B re-read from LDS (ring 3); A from AGPRs (AG) or the 8 VGPR steps
template <bool AG, int MODE>
__global__ __launch_bounds__(256) void probe(const u32x4_t* w, float* out, long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) char smem[340 * 272];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 340 * 272 / 4; i += 256) ((unsigned*)smem)[i] = (i * 2654435761u) & 0x3f803f80u;
  __syncthreads();
  u32x4_t wa[64];
  u32x4_t wv[8];
#pragma unroll
  for (int s = 0; s < 64; ++s) {
    if constexpr (AG) asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(wa[s]) : "v"(w + s * 64 + lane) : "memory");
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) wv[s] = w[s * 64 + lane];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  f32x16_t acc[TH];
#pragma unroll
  for (int r = 0; r < TH; ++r)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[r][i] = 0.f;
  const int lbase = (lane & 31) * 272 + (lane >> 5) * 16;
  u32x4_t bfix[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) bfix[i] = *(const u32x4_t*)(smem + lbase + i * 272);
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    u32x4_t ring[3];
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 3; ++i) ring[i] = *(const u32x4_t*)(smem + lbase + i * 272);
    }
#pragma unroll
    for (int i = 0; i < 4 * PRD; ++i) {
      const int q = i / PRD, rem = i - q * PRD;
      const int dx = rem / NRD, y = (rem % NRD) >> 1, kk = rem & 1;
      u32x4_t bcur;
      if constexpr (MODE == 1) {
        bcur = ring[i % 3];
        if (i + 3 < 4 * PRD) {
          const int j = i + 3, q2 = j / PRD, r2 = j - q2 * PRD;
          const int dx2 = r2 / NRD, y2 = (r2 % NRD) >> 1, k2 = r2 & 1;
          ring[i % 3] = *(const u32x4_t*)(smem + lbase + (y2 * 34 + dx2) * 272 + (4 * q2 + 2 * k2) * 16);
        }
      } else {
        bcur = bfix[i % 3];
      }
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int r = y - dy;
        if (r < 0 || r >= TH) continue;
        const int s = 2 * (q * 9 + 3 * dy + dx) + kk;
        if constexpr (AG) {
          if (s < 64) mf<true>(acc[r], wa[s], bcur);
          else mf<false>(acc[r], wv[s - 64], bcur);
        } else {
          mf<false>(acc[r], wv[s & 7], bcur);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < TH; ++r)
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[r][i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <bool AG, int MODE>
void run(const char* name, const u32x4_t* w, float* out, long long* cyc, int iters) {
  hipLaunchKernelGGL((probe<AG, MODE>), dim3(256), dim3(256), 0, 0, w, out, cyc, iters);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((probe<AG, MODE>), dim3(256), dim3(256), 0, 0, w, out, cyc, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(1024);
  hipMemcpy(c.data(), cyc, 1024 * sizeof(long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (long long v : c) avg += (double)v;
  avg /= 1024.0;
  const double nmf = 576.0 * iters;
  // s_memtime counts at the shader clock
  printf("%-28s %8.3f ms  %7.1f cyc/MFMA (memtime)  %7.1f TFLOP/s\n", name, ms, avg / nmf,
         256.0 * 4 * nmf * 32768.0 / (ms * 1e-3) / 1e12);
}

int main() {
  u32x4_t* w;
  float* out;
  long long* cyc;
  hipMalloc(&w, 72 * 64 * 16);
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 1024 * sizeof(long long));
  std::vector<unsigned> hw(72 * 64 * 4);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (unsigned)((i * 2654435761u) & 0x3f803f80u) | 0x00400040u;
  hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  const int iters = 200;
  run<true, 0>("A agpr, B regs", w, out, cyc, iters);
  run<false, 0>("A vgpr, B regs", w, out, cyc, iters);
  run<true, 1>("A agpr, B lds ring3", w, out, cyc, iters);
  run<false, 1>("A vgpr, B lds ring3", w, out, cyc, iters);
  run<true, 0>("A agpr, B regs (again)", w, out, cyc, iters);
  return 0;
}
