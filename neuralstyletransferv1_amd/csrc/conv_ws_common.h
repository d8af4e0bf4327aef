// conv_ws_common.h — pieces shared by the weight-stationary persistent convs (conv_wstat.hip,
// conv_wphase.hip): unit-fill kinds and the wait / barrier statements their LDS-DMA staging needs.
#pragma once
#include "conv_impl.h"

namespace nst {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// f32x4 epilogue arithmetic as four scalar VALU instructions.  Packed f32 VALU (v_pk_add_f32,
// v_pk_fma_f32) costs ~22-26 extra cycles per instruction when issued beside MFMAs, scalar f32 ~0
// (MI355X_MICROARCH.md, 'price of one filler beside MFMAs'); the library is built with
// -fno-slp-vectorize so scalar code stays scalar.  Same per-element roundings as the vector forms.
__device__ __forceinline__ f32x4_t add4(const f32x4_t& a, const f32x4_t& b) {
  f32x4_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = a[i] + b[i];
  return r;
}
// s1 += x, s2 += x * x (one fused rounding, as __builtin_elementwise_fma)
__device__ __forceinline__ void stat4(f32x4_t& s1, f32x4_t& s2, const f32x4_t& x) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s1[i] = s1[i] + x[i];
    s2[i] = __builtin_fmaf(x[i], x[i], s2[i]);
  }
}

// v_mfma_f32_16x16x32_{bf16,f16} as asm with the accumulator tied in place (hipcc's VGPR-form selection
// otherwise moves every accumulator into fresh registers and pads the reuse of the old ones with
// s_nops); first: C = 0 (a tile row's first MFMA)
template <typename T>
__device__ __forceinline__ void mfma_tied(f32x4_t& c, const uint4& a, const uint4& bop, bool first) {
  const u32x4_t av = __builtin_bit_cast(u32x4_t, a), bv = __builtin_bit_cast(u32x4_t, bop);
  if constexpr (IS_F16<T>) {
    if (first)
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(av), "v"(bv));
    else
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(av), "v"(bv));
  } else {
    if (first)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(av), "v"(bv));
    else
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(av), "v"(bv));
  }
}

// v_mfma_f32_16x16x16_{f16,bf16} accumulating in place (asm: the accumulator is tied, so hipcc cannot give the
// destination a register of the A / B operands -- conv_ws9.hip's split-weight variant got
// v_mfma_f32_16x16x16_f16 v[178:181], v[92:93], v[178:179], ... from the builtin and two result values came out
// wrong; tools/check_mfma_overlap.py)
template <typename T>
__device__ __forceinline__ void mfma16x16x16_tied(f32x4_t& c, const uint2& a, const uint2& bop) {
  const u32x2_t av = __builtin_bit_cast(u32x2_t, a), bv = __builtin_bit_cast(u32x2_t, bop);
  if constexpr (IS_F16<T>)
    asm volatile("v_mfma_f32_16x16x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(av), "v"(bv));
  else
    asm volatile("v_mfma_f32_16x16x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(av), "v"(bv));
}

// the same with C = cinit for a tile row's first MFMA (the conv bias: the epilogue then adds nothing)
template <typename T>
__device__ __forceinline__ void mfma_tied_c(f32x4_t& c, const uint4& a, const uint4& bop, bool first, const f32x4_t& cinit) {
  const u32x4_t av = __builtin_bit_cast(u32x4_t, a), bv = __builtin_bit_cast(u32x4_t, bop);
  if constexpr (IS_F16<T>) {
    if (first)
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %3" : "=&v"(c) : "v"(av), "v"(bv), "v"(cinit));
    else
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(av), "v"(bv));
  } else {
    if (first)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %3" : "=&v"(c) : "v"(av), "v"(bv), "v"(cinit));
    else
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(av), "v"(bv));
  }
}

// cache policy of the activation stores: nt (streaming).  A store holds vmcnt until the L2 has taken
// it, and every later unit wait counts it (in-order), so the trunk's output and residual-stream
// stores sit in front of the next tile's loads; streaming stores measured ~1 % faster per step.
constexpr int ST_AUX = 2;

// what the fill applies to a staged input chunk
// (join of ReLU(IN(r)): r normalised as a WF_NORM fill stages it, bf16-rounded)
enum WsFill { WF_NORM = 0, WF_RAW = 1, WF_RES = 2, WF_RESRN = 3 };  // IN+ReLU / identity / join / join of ReLU(IN(r))

// s_waitcnt vmcnt(N) / the part barrier, as statements hipcc cannot move memory operations across
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One 16-byte LDS-DMA request: 64 lanes x 16 B from per-lane buffer offsets into LDS at
// lds + lane * 16 (buffer_load ... lds: no VGPR destination).  M0 is saved and restored inside the
// statement (hipcc owns it); the s_nop covers the M0 write -> LDS-DMA hazard.
__device__ __forceinline__ void dma16(const __amdgpu_buffer_rsrc_t& rs, uint32_t voff, uint32_t lds, int soff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(rs), "s"(soff)
      : "memory");
}

}  // namespace nst
