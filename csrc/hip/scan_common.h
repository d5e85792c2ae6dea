// Shared pieces of the index scan kernels (bf16: index_topk.hip, fp8: index_fp8.hip).
#pragma once
#include "common.h"

namespace symb {

// counted vector-memory wait (loads, LDS-DMA and stores retire in issue order)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int AUX>
__device__ __forceinline__ void glds16_aux(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gsrc,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, AUX);
}

// compile-time loop: f(integral_constant<int, i>) for i = I .. N - 1
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<I + 1, N>(f);
  }
}

// no-op DMA functor for MFMA chains that issue no LDS-DMA pieces
struct NoDma {
  __device__ __forceinline__ void operator()(int) const {}
};

template <int KMAX>
__device__ __forceinline__ void topk_insert(float (&tv)[KMAX], int (&ti)[KMAX], float s, int id) {
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const bool sw = s > tv[i];
    const float ov = tv[i];
    const int oi = ti[i];
    tv[i] = sw ? s : ov;
    ti[i] = sw ? id : oi;
    s = sw ? ov : s;
    id = sw ? oi : id;
  }
}

// Same result as topk_insert but with no serial chain: every slot decides from the ORIGINAL
// sorted list (monotone "s > tv[i]" flags), so the 16 compare/select pairs issue back to back.
template <int KMAX>
__device__ __forceinline__ void topk_insert_par(float (&tv)[KMAX], int (&ti)[KMAX], float s, int id) {
  float nv[KMAX];
  int ni[KMAX];
  nv[0] = s > tv[0] ? s : tv[0];
  ni[0] = s > tv[0] ? id : ti[0];
#pragma unroll
  for (int i = 1; i < KMAX; ++i) {
    const float shv = s > tv[i - 1] ? tv[i - 1] : s;   // value slot i takes if s beats it
    const int shi = s > tv[i - 1] ? ti[i - 1] : id;
    nv[i] = s > tv[i] ? shv : tv[i];
    ni[i] = s > tv[i] ? shi : ti[i];
  }
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    tv[i] = nv[i];
    ti[i] = ni[i];
  }
}

}  // namespace symb
