// Shared device helpers for the CDNA4 (gfx950 / MI355X) kernels of codename_symbiont_amd.
//
// Everything here is written for 64-lane wavefronts, MFMA matrix cores and the 160 KiB LDS of a
// gfx950 CU.  No CUDA, no dual paths: hard-coded wave width 64, OCP bf16/fp8 types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace symb {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;   // MFMA A/B operand (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;     // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16;   // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;  // raw 16-byte vector

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(__bf16 h) { return (float)h; }
__device__ __forceinline__ __bf16 f2bf(float f) { return (__bf16)f; }  // RNE, v_cvt_pk_bf16_f32

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// 8 bf16 <-> 8 f32 through one 16-byte access.
__device__ __forceinline__ void load8(const __bf16* p, float (&o)[8]) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
}
__device__ __forceinline__ void store8(__bf16* p, const float (&o)[8]) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (__bf16)o[i];
  *reinterpret_cast<bf16x8*>(p) = v;
}

// erf by Abramowitz & Stegun 7.1.26: |error| < 1.5e-7 (checked on [-6, 6]), i.e. far below the
// bf16 rounding of the GEMM output, at one v_rcp + one v_exp + 7 FMA-class ops -- the libdevice
// erff costs several times that and was ~30 % of the FFN1 GEMM (GELU epilogue 398 vs 583 TF).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.0f), x);
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}

typedef __attribute__((ext_vector_type(2))) float f32x2;

// GELU(erf) of a PAIR of values with no transcendental: erf(y) = y * P(y^2) on |y| <= 3 (degree-8
// minimax-weighted fit in y^2, |erf error| < 1.7e-5), inputs clamped to |x| <= 3 sqrt(2) (erfc(3)
// = 2.2e-5).  |GELU error| < 5e-5 absolute and 1.1e-5 relative for large |x|: below the bf16
// rounding of the GEMM output except in the far negative tail (|y| ~ 1e-4..1e-3, a few tens of
// bf16 ulps there).  The polynomial runs on packed f32 pairs (v_pk_fma_f32 / v_pk_mul_f32): ~8
// issue slots per element against ~22 for gelu_erf, which made the GELU epilogue the largest
// part of MiniLM's K = 384 FFN1 GEMM.
__device__ __forceinline__ f32x2 gelu2_poly(f32x2 x) {
  constexpr float lim = 4.24264068711928515f;   // 3 sqrt(2)
  f32x2 xc;
  xc.x = __builtin_amdgcn_fmed3f(x.x, -lim, lim);
  xc.y = __builtin_amdgcn_fmed3f(x.y, -lim, lim);
  const f32x2 y = xc * 0.70710678118654752f;
  const f32x2 t = y * y;
  f32x2 p = 4.074636806e-08f;
  p = p * t + -1.944968972e-06f;
  p = p * t + 4.106253982e-05f;
  p = p * t + -5.110510974e-04f;
  p = p * t + 4.235480912e-03f;
  p = p * t + -2.510295995e-02f;
  p = p * t + 1.110793948e-01f;
  p = p * t + -3.753148317e-01f;
  p = p * t + 1.128268361e+00f;
  const f32x2 h = x * 0.5f;
  return h * (y * p) + h;
}

// Bijective XCD-aware remap of a linear workgroup id (MI355X deals workgroups round-robin over
// 8 XCDs): consecutive logical tiles land on the same XCD so their shared operand panels hit the
// same private L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Async global->LDS copy of 16 bytes per lane (global_load_lds_dwordx4).  The LDS destination is
// the wave-uniform base; lane l lands at base + 16*l.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gsrc,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// LDS byte address of a __shared__ pointer (for hand-issued ds_read offsets)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// LDS-DMA issued as inline asm (16 / 4 bytes per lane; lane l lands at lds + size * l, lds a
// wave-uniform LDS byte address).  hipcc neither counts these loads nor inserts its conservative
// "any pending LDS-DMA may alias this ds_read" vmcnt(0): the caller retires them with its own
// counted s_waitcnt vmcnt before reading the data (same wave; other waves also need a barrier).
// M0 is written and restored inside the statement (the compiler reserves it).
#define SYMB_DMA_ASM(NAME, INSN)                                                                 \
  __device__ __forceinline__ void NAME(const void* gsrc, uint32_t lds) {                        \
    unsigned keep;                                                                               \
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t" INSN " %1, off\n\t"        \
                 "s_mov_b32 m0, %0"                                                              \
                 : "=&s"(keep)                                                                   \
                 : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds))                          \
                 : "memory");                                                                    \
  }
SYMB_DMA_ASM(dma16_asm, "global_load_lds_dwordx4")
SYMB_DMA_ASM(dma4_asm, "global_load_lds_dword")
#undef SYMB_DMA_ASM

// Raise a kernel's dynamic-LDS limit (hipFuncAttributeMaxDynamicSharedMemorySize) before its
// first launch ON EACH DEVICE: the attribute is per device, so a process driving several GPUs
// must set it once per device, not once per process.  One bit per device id per kernel.
template <auto Kern>
inline void set_max_lds(int bytes) {
  static std::atomic<uint64_t> done{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const uint64_t bit = 1ull << (dev & 63);
  if (!(done.load(std::memory_order_acquire) & bit)) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(Kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    done.fetch_or(bit, std::memory_order_acq_rel);
  }
}

}  // namespace symb
