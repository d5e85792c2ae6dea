// MFMA bf16 GEMM with fused epilogues for the sentence-transformer encoder.
//
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] )        (nn.Linear layout, both operands K-major)
//
// Replaces the reference's per-op cuBLAS SGEMM + broadcast-add + GELU + residual + LayerNorm chain
// (reference call site
//  services/preprocessing_service/src/embedding_generator.rs:198 -> candle BertModel::forward).
//
// CDNA4 design:
//  * v_mfma_f32_16x16x32_bf16, fp32 accumulate; wave tile (BM/WAVES_M) x (BN/WAVES_N).
//  * BK = 64 -> 128-byte LDS rows, filled by global_load_lds_dwordx4 (16 B/lane, no VGPR staging).
//    The LDS image stays lane-linear (a DMA requirement); the bank-conflict XOR swizzle
//    (chunk ^= (row>>1)&7) is applied on the per-lane GLOBAL source address and again on the
//    ds_read_b128 address (both-sides rule).
//  * 2-stage LDS ring: tile k+1 streams in while tile k feeds the MFMAs; one barrier per k-tile.
//  * XCD-aware bijective block remap so the N-tiles that share an A panel share one XCD's L2.
//  * Epilogue stages the fp32 tile through LDS, then every thread emits full 16-byte stores:
//      EPI_BIAS      : + bias
//      EPI_GELU      : gelu_erf(+ bias)                       (BERT intermediate)
//      EPI_RES       : + bias + residual                      (pre-LN sum, for H >= 768)
//      EPI_RES_LN    : LayerNorm(+ bias + residual)           (row-complete tile, BN == N)
#include "common.h"

namespace symb {

enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RES = 2, EPI_RES_LN = 3, EPI_GELU_MX8 = 4 };

constexpr int GEMM_BK = 64;  // bf16 elements per k-tile (128-byte rows)
#ifndef SYMB_GEMM_SCHED
#define SYMB_GEMM_SCHED 1
#endif
constexpr bool GEMM_SCHED = SYMB_GEMM_SCHED;  // pinned read/MFMA interleave (0: compiler's own)

__device__ __forceinline__ int swz_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

// MX block exponent of 32 values spread over 4 consecutive lanes (8 each, `quad` = lane & 3 of
// the first): the smallest e with amax * 2^-e < 448 (e4m3's largest finite), as an int in
// [-127, 127] (E8M0 byte = e + 127).  All 4 lanes must be active.
__device__ __forceinline__ int mx_block_exponent(const float (&y)[8], int quad) {
  (void)quad;
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(y[e]));
  amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
  // amax/448 = m * 2^ex with m in [0.5, 1)  =>  amax * 2^-ex < 448
  const int ex = __builtin_amdgcn_frexp_expf(amax * (1.0f / 448.0f));
  return amax > 0.f ? max(-127, min(ex, 127)) : -127;
}

// 8 floats * 2^-ex -> 8 OCP e4m3 bytes (round to nearest even, saturating).
__device__ __forceinline__ int2 pack_e4m3x8(const float (&y)[8], int ex) {
  const float inv = __builtin_amdgcn_ldexpf(1.0f, -ex);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(y[0] * inv, y[1] * inv, 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(y[2] * inv, y[3] * inv, lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(y[4] * inv, y[5] * inv, 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(y[6] * inv, y[7] * inv, hi, true);
  return make_int2(lo, hi);
}

// F8 = true: A, W are OCP e4m3 bytes and one k-tile is 128 elements (still 128-byte LDS rows, so
// staging and swizzle are shared); v_mfma_scale_f32_16x16x128_f8f6f4 consumes 32 bytes per lane
// (swizzled 16-byte chunks g and g + 4 of lane group g), and the epilogue rescales by sa[row] (per-token activation scale) x
// sw[col] (per-output-channel weight scale) before bias / GELU / residual.
// AMX = true (F8 only): A is MX-scaled instead -- one E8M0 exponent per 32 consecutive k of a row
// (ascale[row * K/32 + k/32]).  The exponent goes straight into the block-scaled MFMA's scale_a
// operand (the 32 k a lane feeds one v_mfma_scale_f32_16x16x128_f8f6f4 are exactly one block),
// so no per-row rescale is left for the epilogue.
// EPI_GELU_MX8 (F8 only): GELU(+ bias) emitted as MX fp8 -- e4m3 bytes in C plus one E8M0 scale
// per 32 output columns in cscale -- which is the A operand format AMX consumes.  The FFN1 -> FFN2
// hand-off then needs no separate quantiser pass over the 4H-wide activation.
//
// Deferred LayerNorm (LNF, bf16 only; the H >= 768 encoders -- VERDICT r5 item 1).  A post-LN
// BERT layer normalises every residual sum y = x + f(x) before two consumers read it: the next
// projection (as its A operand) and the next residual add.  Rather than a separate pass that
// reads y and writes LN(y) (add_ln, twice per layer), the producer's epilogue also writes
// per-row partial statistics of the y it stores, and the consumers normalise algebraically:
//   LNF_STATS : the epilogue writes, per row and 64-column chunk of its output, (chunk mean,
//               sum of squared deviations from it) as float2 into st_out [M][N / 64] -- from the
//               bf16-rounded values it stores, so the statistics describe exactly the tensor the
//               consumers read.
//   LNF_FOLD  : A is a pre-LN y with statistics st_in [M][np_in].  Since
//                 LN(y) W^T + b = rstd (y (W o gamma)^T - mean cs) + (b + W beta),
//               cs = rowsum(W o gamma), the kernel runs on the folded weight W o gamma and the
//               epilogue applies rstd (acc - mean cs[n]) + b'[n] (b' = b + W beta: `bias`).
//   LNF_RESLN : the residual R is a pre-LN y with statistics st_in: the epilogue adds
//               (R - mean) rstd gamma + beta instead of R.
// Row statistics combine the np_in chunk partials (Chan et al.'s pairwise update) once per tile
// row into LDS; ln_eps is the LayerNorm epsilon.
enum { LNF_FOLD = 1, LNF_RESLN = 2, LNF_STATS = 4 };

template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, int NSTAGE = 2, bool F8 = false,
          bool AMX = false, int LNF = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_bf16_kernel(
    const void* __restrict__ Av, int lda, const void* __restrict__ Wv, int ldw,
    const float* __restrict__ bias, const __bf16* __restrict__ R, int ldr,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    __bf16* __restrict__ C, int ldc, int M, int N, int K, const float* __restrict__ sa,
    const float* __restrict__ sw, int group_m, const uint8_t* __restrict__ ascale,
    uint8_t* __restrict__ cscale, const float2* __restrict__ st_in, int np_in,
    const float* __restrict__ cs, float2* __restrict__ st_out, float ln_eps) {
  static_assert(LNF == 0 || (!F8 && EPI != EPI_RES_LN && EPI != EPI_GELU_MX8), "deferred LN: bf16");
  static_assert(!(LNF & LNF_FOLD) || !(LNF & LNF_RESLN), "one statistics input per kernel");
  static_assert(!(LNF & LNF_RESLN) || EPI == EPI_RES, "a normalised residual needs EPI_RES");
  static_assert(!(LNF & LNF_STATS) || BN % 64 == 0, "statistics chunks of 64 columns");
  static_assert(!AMX || (F8 && NSTAGE == 2), "MX activations are an fp8 2-stage mode");
  static_assert(NSTAGE >= 2 && NSTAGE <= 4, "LDS ring depth");
  static_assert(EPI != EPI_GELU_MX8 || (F8 && BN % 32 == 0), "MX output is an fp8 mode");
  constexpr int ES = F8 ? 1 : 2;               // bytes per element
  constexpr int KTILE = 128 / ES;              // elements per 128-byte k-tile row
  const char* A = reinterpret_cast<const char*>(Av);
  const char* W = reinterpret_cast<const char*>(Wv);
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int NT = 64 * NW;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int TILE_BYTES = (BM + BN) * 128;
  // AMX: the A tile's E8M0 exponents (BM rows x 4 blocks of 32 k) ride the same LDS ring
  constexpr int SC_BYTES = (F8 && AMX) ? BM * 4 : 0;
  constexpr int STAGE_BYTES = TILE_BYTES + SC_BYTES;
  // tiles too big to stage in fp32 at once are emitted one wave-row band at a time
  constexpr int EPI_PASSES = (BM * (BN + 4) * 4 > 160 * 1024) ? WAVES_M : 1;
  static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "tile rows must cover the DMA waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int n_tiles = N / BN;
  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  // grouped tile order: consecutive tiles (one XCD's in-flight set after xcd_remap) walk a
  // group_m-row band column by column, so both the A row panels and the W column panels they
  // touch stay resident in that XCD's 4 MB L2 (row-major order re-streamed all of W per band)
  int tm = tile / n_tiles, tn = tile % n_tiles;
  if (group_m > 1) {
    const int m_tiles = nwg / n_tiles, per_group = group_m * n_tiles;
    const int g = tile / per_group, first = g * group_m;
    const int gm = min(group_m, m_tiles - first), local = tile - g * per_group;
    tm = first + local % gm;
    tn = local / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int KT = K / KTILE;

  auto stage = [&](int kt, int buf) {
    char* sA = smem + buf * STAGE_BYTES;
    char* sB = sA + BM * 128;
    const size_t k0 = (size_t)kt * 128;         // byte offset of the k-tile
#pragma unroll
    for (int i = 0; i < (BM * 8) / NT; ++i) {
      const int s = i * NT + tid;
      const int row = s >> 3, pc = s & 7, c = pc ^ ((row >> 1) & 7);
      const int grow = min(m0 + row, M - 1);
      glds16(A + (size_t)grow * lda * ES + k0 + c * 16, sA + (i * NT + wave * 64) * 16);
    }
#pragma unroll
    for (int i = 0; i < (BN * 8) / NT; ++i) {
      const int s = i * NT + tid;
      const int row = s >> 3, pc = s & 7, c = pc ^ ((row >> 1) & 7);
      glds16(W + (size_t)(n0 + row) * ldw * ES + k0 + c * 16, sB + (i * NT + wave * 64) * 16);
    }
    if constexpr (SC_BYTES > 0) {
      // one dword (the 4 block exponents of this k-tile) per A row; the first BM/64 waves
      if (tid < BM) {
        const int grow = min(m0 + tid, M - 1);
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(ascale + (size_t)grow * (K / 32) + kt * 4),
            (__attribute__((address_space(3))) void*)(sB + BN * 128 + wave * 64 * 4), 4, 0, 0);
      }
    }
  };

  // LayerNorm(+ bias + residual) of `rows` staged fp32 rows (row-complete: n0 == 0, BN == N);
  // one wave per row, lane owns 8 consecutive columns.
  auto res_ln_rows = [&](const float* Cs, int rows, int grow0) {
    constexpr int CS = BN + 4;
    constexpr int NV = BN / 8;
    constexpr int PER = (NV + 63) / 64;
    for (int row = wave; row < rows; row += NW) {
      const int grow = grow0 + row;
      if (grow >= M) break;
      float x[PER][8];
      float s = 0.f;
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int v = lane + 64 * p;
#pragma unroll
        for (int e = 0; e < 8; ++e) x[p][e] = 0.f;
        if (v < NV) {
          float r[8];
          load8(R + (size_t)grow * ldr + v * 8, r);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            x[p][e] = Cs[row * CS + v * 8 + e] + bias[v * 8 + e] + r[e];
            s += x[p][e];
          }
        }
      }
      const float mean = wave_sum(s) * (1.0f / BN);
      float ss = 0.f;
#pragma unroll
      for (int p = 0; p < PER; ++p)
        if (lane + 64 * p < NV)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = x[p][e] - mean;
            ss += d * d;
          }
      const float rstd = rsqrtf(wave_sum(ss) * (1.0f / BN) + eps);
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int v = lane + 64 * p;
        if (v < NV) {
          float y[8];
#pragma unroll
          for (int e = 0; e < 8; ++e)
            y[e] = (x[p][e] - mean) * rstd * gamma[v * 8 + e] + beta[v * 8 + e];
          store8(C + (size_t)grow * ldc + v * 8, y);
        }
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int LOADS = (BM * 8) / NT + (BN * 8) / NT;  // glds per thread per stage
  stage(0, 0);
#pragma unroll
  for (int p = 1; p < NSTAGE - 1; ++p)
    if (p < KT) stage(p, p);
  for (int kt = 0; kt < KT; ++kt) {
    if constexpr (NSTAGE == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kt + 1 < KT) stage(kt + 1, (kt + 1) & 1);
    } else {
      // tile kt landed once only the (up to NSTAGE-2) younger tiles' loads remain; a raw barrier
      // (no vmcnt(0) drain) keeps those in flight across it, and it also retires every wave's
      // reads of the buffer that stage(kt+NSTAGE-1) refills (read in iteration kt-1)
      const int younger = min(NSTAGE - 2, KT - 1 - kt);
      if (NSTAGE > 3 && younger >= 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * LOADS) : "memory");
      else if (younger >= 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LOADS) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + NSTAGE - 1 < KT) stage(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    }
    const char* sA = smem + (kt % NSTAGE) * STAGE_BYTES;
    const char* sB = sA + BM * 128;
    if constexpr (F8) {
      // lane group g feeds the MFMA's k = 16g..16g+15 (VGPRs 0-3) and 64+16g.. (VGPRs 4-7), and
      // the hardware applies lane group b's scale to k block 32b..32b+31 (measured:
      // benchmarks/diag/mx_scale_map.hip), so reading 16-byte chunks g and g + 4 keeps the MFMA's
      // k order equal to memory order and every MX block under its own exponent
      const int g = lane >> 4;
      // AMX: this lane's exponent for each 16-row fragment -- row (lane & 15), k block g
      int asc[AMX ? RM : 1] = {127};
      if constexpr (AMX) {
        const uint8_t* sS = reinterpret_cast<const uint8_t*>(sB + BN * 128);
#pragma unroll
        for (int i = 0; i < RM; ++i) asc[i] = sS[(wm * WTM + i * 16 + (lane & 15)) * 4 + g];
      }
      i32x8 a[RM], b[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = wm * WTM + i * 16 + (lane & 15);
        const i32x4 lo = *reinterpret_cast<const i32x4*>(sA + swz_off(row, g));
        const i32x4 hi = *reinterpret_cast<const i32x4*>(sA + swz_off(row, g + 4));
        a[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = wn * WTN + j * 16 + (lane & 15);
        const i32x4 lo = *reinterpret_cast<const i32x4*>(sB + swz_off(row, g));
        const i32x4 hi = *reinterpret_cast<const i32x4*>(sB + swz_off(row, g + 4));
        b[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              a[i], b[j], acc[i][j], 0, 0, 0, AMX ? asc[i] : 127, 0, 127);

    } else {
      // Both k-halves' fragments are read up front and the schedule is pinned: the 8 reads of
      // half 1 are interleaved with half 0's MFMAs (2 MFMAs per read), so only half 0's LDS
      // latency is exposed after each barrier (the compiler's own schedule waited lgkmcnt(0)
      // every 8 MFMAs; profiles/r1_gemm).
      bf16x8 a[2][RM], b[2][RN];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < RM; ++i)
          a[kk][i] = *reinterpret_cast<const bf16x8*>(sA + swz_off(wm * WTM + i * 16 + (lane & 15), chunk));
#pragma unroll
        for (int j = 0; j < RN; ++j)
          b[kk][j] = *reinterpret_cast<const bf16x8*>(sB + swz_off(wn * WTN + j * 16 + (lane & 15), chunk));
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
      if constexpr (GEMM_SCHED) {
        constexpr int NR = RM + RN, NM = RM * RN;
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);        // half 0 reads
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, NM / NR, 0);  // half 0 MFMAs ...
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);        // ... with half 1 reads
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);         // half 1 MFMAs
      }
    }
  }

  // ---- epilogue: fp32 tile -> LDS (padded rows) -> row-contiguous 16-byte stores ----
  // A tile whose fp32 image does not fit LDS (256-row tiles, row-complete LN tiles) is emitted
  // one wave-row band per pass.
  constexpr int CS = BN + 4;
  constexpr int PROWS = BM / EPI_PASSES;
  constexpr bool NEED_RS = (LNF & (LNF_FOLD | LNF_RESLN)) != 0;
  constexpr int NP_MAX = 16;                        // statistics chunks per row (N <= 1024)
  constexpr int PV = NEED_RS ? (PROWS * NP_MAX + NT - 1) / NT : 1;
  float* Cs = reinterpret_cast<float*>(smem);
  // this pass's row statistics (mean, rstd) for LNF_FOLD / LNF_RESLN, after the fp32 tile, and
  // the raw chunk partials they are combined from
  float2* rs = reinterpret_cast<float2*>(smem + PROWS * CS * 4);
  float2* rsraw = rs + PROWS;
  __syncthreads();
#pragma unroll 1
  for (int p = 0; p < EPI_PASSES; ++p) {
    const int band0 = m0 + p * PROWS;  // first global row of this pass
    // the band's partials are ONE contiguous block of st_in: issue every load now (coalesced,
    // all in flight while the accumulators are staged), combine after the staging barrier
    float2 pv[PV];
    if constexpr (NEED_RS) {
      const int nv = max(0, min(PROWS, M - band0)) * np_in;
      const float2* sp = st_in + (size_t)band0 * np_in;
#pragma unroll
      for (int u = 0; u < PV; ++u) {
        const int idx = u * NT + tid;
        pv[u] = idx < nv ? sp[idx] : make_float2(0.f, 0.f);
      }
    }
    if (EPI_PASSES == 1 || wm == p) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = (EPI_PASSES == 1 ? wm * WTM : 0) + i * 16 + (lane >> 4) * 4 + r;
            const int col = wn * WTN + j * 16 + (lane & 15);
            if constexpr (F8 && AMX)
              Cs[row * CS + col] = acc[i][j][r] * sw[n0 + col];
            else if constexpr (F8)
              Cs[row * CS + col] = acc[i][j][r] * sa[min(band0 + row, M - 1)] * sw[n0 + col];
            else
              Cs[row * CS + col] = acc[i][j][r];
          }
    }
    if constexpr (NEED_RS) {
#pragma unroll
      for (int u = 0; u < PV; ++u)
        if (u * NT + tid < PROWS * np_in) rsraw[u * NT + tid] = pv[u];
      __syncthreads();
      for (int t = tid; t < PROWS; t += NT) {
        const float2* sp = rsraw + t * np_in;
        float msum = 0.f;
        for (int i = 0; i < np_in; ++i) msum += sp[i].x;
        const float mean = msum / (float)np_in;
        float m2 = 0.f;
        for (int i = 0; i < np_in; ++i) {
          const float2 v = sp[i];
          const float d = v.x - mean;
          m2 += v.y + 64.f * d * d;
        }
        rs[t] = make_float2(mean, rsqrtf(m2 / (64.f * (float)np_in) + ln_eps));
      }
    }
    __syncthreads();
    if constexpr (EPI == EPI_RES_LN) {
      res_ln_rows(Cs, PROWS, band0);
    } else {
      constexpr int VPR = BN / 8;
      for (int v = tid; v < PROWS * VPR; v += NT) {
        const int row = v / VPR, c8 = (v % VPR) * 8;
        const int grow = band0 + row;
        if (grow >= M) continue;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(Cs + row * CS + c8);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(Cs + row * CS + c8 + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias + n0 + c8);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(bias + n0 + c8 + 4);
        float y[8];
        if constexpr ((LNF & LNF_FOLD) != 0) {
          const float2 st = rs[row];
          const f32x4 c0 = *reinterpret_cast<const f32x4*>(cs + n0 + c8);
          const f32x4 c1 = *reinterpret_cast<const f32x4*>(cs + n0 + c8 + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y[e] = st.y * (x0[e] - st.x * c0[e]) + b0[e];
            y[e + 4] = st.y * (x1[e] - st.x * c1[e]) + b1[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y[e] = x0[e] + b0[e];
            y[e + 4] = x1[e] + b1[e];
          }
        }
        if constexpr (EPI == EPI_GELU || EPI == EPI_GELU_MX8) {
          if (eps != 0.f) {   // GELU epilogues take eps (LayerNorm-only) as the form switch
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const f32x2 v = gelu2_poly(f32x2{y[e], y[e + 1]});
              y[e] = v.x;
              y[e + 1] = v.y;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = gelu_erf(y[e]);
          }
        }
        if constexpr (EPI == EPI_GELU_MX8) {
          // the 4 consecutive threads (tid & 3) of one row hold one 32-column MX block
          uint8_t* C8 = reinterpret_cast<uint8_t*>(C);
          const int ex = mx_block_exponent(y, tid & 3);
          *reinterpret_cast<int2*>(C8 + (size_t)grow * ldc + n0 + c8) = pack_e4m3x8(y, ex);
          if ((tid & 3) == 0) cscale[(size_t)grow * (N / 32) + (n0 + c8) / 32] = (uint8_t)(ex + 127);
          continue;
        }
        if constexpr (EPI == EPI_RES) {
          float r[8];
          load8(R + (size_t)grow * ldr + n0 + c8, r);
          if constexpr ((LNF & LNF_RESLN) != 0) {
            const float2 st = rs[row];
            const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + n0 + c8);
            const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + n0 + c8 + 4);
            const f32x4 e0 = *reinterpret_cast<const f32x4*>(beta + n0 + c8);
            const f32x4 e1 = *reinterpret_cast<const f32x4*>(beta + n0 + c8 + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              y[e] += (r[e] - st.x) * st.y * g0[e] + e0[e];
              y[e + 4] += (r[e + 4] - st.x) * st.y * g1[e] + e1[e];
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] += r[e];
          }
        }
        if constexpr ((LNF & LNF_STATS) != 0) {
          // the 8 lanes (tid & 7) of this row's 64-column chunk: statistics of the stored values
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = (float)(__bf16)y[e];
          float sm = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) sm += y[e];
          sm += __shfl_xor(sm, 1, 64);
          sm += __shfl_xor(sm, 2, 64);
          sm += __shfl_xor(sm, 4, 64);
          const float mc = sm * (1.f / 64.f);
          float d2 = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) d2 += (y[e] - mc) * (y[e] - mc);
          d2 += __shfl_xor(d2, 1, 64);
          d2 += __shfl_xor(d2, 2, 64);
          d2 += __shfl_xor(d2, 4, 64);
          if ((tid & 7) == 0) st_out[(size_t)grow * (N / 64) + (n0 + c8) / 64] = make_float2(mc, d2);
        }
        store8(C + (size_t)grow * ldc + n0 + c8, y);
      }
    }
    if (EPI_PASSES > 1) __syncthreads();
  }
}

// Rows of tiles per group in the grouped tile order (0/1: plain row-major); see symb_gemm_config.
static int g_group_m = 8;
// Waves of the 128x128 fp8 tile: 4 (64x64 wave tiles) or 8 (64x32, default: e5-large fp8
// forward 18.2 -> 17.7 ms, profiles/r1_s4/fp8_waves/).
static int g_fp8_waves = 8;
// GELU epilogue form: 0 = gelu_erf (A&S erf, one rcp + one exp per value), 1 = gelu2_poly
// (packed-pair polynomial, no transcendental).  Passed to the kernel in its eps argument, which
// only the LayerNorm epilogue otherwise reads.
// Measured (profiles/r2_gelu/ab.json, one process): MiniLM FFN1 52.2 -> 47.1 us, bge FFN1 133.9 ->
// 123.9 us (bias-only epilogue: 40.3 / 111.4), same max error vs the fp32 oracle (bf16-bound).
static int g_gelu_poly = 1;

// Deferred-LayerNorm operands of a launch (LNF kernels; see gemm_bf16_kernel).
struct LnArgs {
  const float2* st_in = nullptr;
  int np_in = 0;
  const float* cs = nullptr;
  float2* st_out = nullptr;
  float ln_eps = 0.f;
};

template <int BM, int BN, int WM, int WN, int EPI, int NSTAGE = 2, bool F8 = false,
          bool AMX = false, int LNF = 0>
static int launch_cfg(const void* A, int lda, const void* W, int ldw, const float* bias,
                      const __bf16* R, int ldr, const float* g, const float* b, float eps,
                      __bf16* C, int ldc, int M, int N, int K, hipStream_t st,
                      const float* sa = nullptr, const float* sw = nullptr,
                      const uint8_t* ascale = nullptr, uint8_t* cscale = nullptr,
                      const LnArgs& ln = LnArgs()) {
  auto kern = gemm_bf16_kernel<BM, BN, WM, WN, EPI, NSTAGE, F8, AMX, LNF>;
  constexpr int main_bytes = NSTAGE * ((BM + BN) * 128 + (AMX ? BM * 4 : 0));
  constexpr int full_epi = BM * (BN + 4) * 4;
  constexpr int passes = full_epi > 160 * 1024 ? WM : 1;
  constexpr int epi_bytes = (BM / passes) * (BN + 4) * 4 +
                            ((LNF & (LNF_FOLD | LNF_RESLN)) ? (BM / passes) * 8 * 17 : 0);
  constexpr int lds = main_bytes > epi_bytes ? main_bytes : epi_bytes;
  static_assert(lds <= 160 * 1024, "LDS");
  set_max_lds<gemm_bf16_kernel<BM, BN, WM, WN, EPI, NSTAGE, F8, AMX, LNF>>(lds);
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * WM * WN), lds, st, A, lda, W, ldw, bias, R, ldr,
                     g, b, eps, C, ldc, M, N, K, sa, sw, g_group_m, ascale, cscale, ln.st_in,
                     ln.np_in, ln.cs, ln.st_out, ln.ln_eps);
  return (int)hipGetLastError();
}

}  // namespace symb

using namespace symb;

// Tile height of the row-complete RES_LN GEMM (64 or 128); a tuning knob, see symb_gemm_config.
static int g_resln_bm = 128;
// Tile of the bias / GELU / residual GEMMs (one path per shape class under the default 3):
// 3 = auto: a 256-row big tile (8 waves, 2-stage ring, one workgroup per CU) when K >= 768 and a
//     256 x 256 or 256 x 192 grid fills whole waves of the 256 CUs (or is long enough that a
//     partial last wave costs little) -- of the two, the one with the least
//     (waves of tiles) x (tile area), ties to 256; else 128x128 with 8 waves of 64x32 (4 waves per
//     SIMD at 2 workgroups per CU), a 4-deep ring when the grid is smaller than the 256 CUs (small
//     M: each tile's serial k-loop is the latency);
// 0 = 128x128 with 4 waves, 2-stage ring (A/B baseline);
// 2 = the 256 x 256 tile wherever N % 256 == 0 (A/B);
// 10 = auto without the 256 x 192 tile (the round-3 rule, A/B).
// Why 192: N = 768 at M = 32768 is 384 tiles of 256 x 256 = 1.5 waves on 256 CUs; as 256 x 192
// it is 512 tiles = 2 whole waves of 3/4-size tiles, the last-wave fill a stream-K split gives,
// without partials or a fix-up (a deep-ring kernel with last-wave split-K was built and measured
// slower on every shape: profiles/r4_gemm/).
static int g_tile = 3;
static int big_tile_bn(int tile, int M, int N, int K) {
  if (tile == 2) return N % 256 == 0 ? 256 : 0;
  if (tile != 3 && tile != 10) return 0;
  // short K (MiniLM's 384): the big tile's fill and epilogue outweigh its operand reuse
  if (K < 768) return 0;
  int best = 0;
  long best_cost = 0;
  for (int bn : {256, 192}) {
    if (N % bn != 0 || (bn == 192 && tile == 10)) continue;
    const long tiles = (long)((M + 255) / 256) * (N / bn);
    if (!(tiles % 256 == 0 || tiles >= 4 * 256)) continue;
    const long cost = (tiles + 255) / 256 * bn;
    if (!best || cost < best_cost) {
      best = bn;
      best_cost = cost;
    }
  }
  return best;
}
int symb_gemm_config(int resln_bm, int tile, int group_m) {
  if (resln_bm != 64 && resln_bm != 128) return -1;
  if (tile != 0 && tile != 2 && tile != 3 && tile != 10) return -1;   // (see g_tile)
  if (group_m < 0 || group_m > 64) return -1;
  g_resln_bm = resln_bm;
  g_tile = tile;
  g_group_m = group_m;
  return 0;
}

// Waves of the row-complete 128x384 RES_LN tile: 8 (64x96 wave tiles) or 16 (32x96, default:
// 4 waves per SIMD; MiniLM out-proj+LN 33.3 -> 27.7 us, FFN2+LN 56.3 -> 50.2 us,
// profiles/r1_s4/resln_waves/).
static int g_resln_waves = 16;
int symb_gemm_resln_config(int waves) {
  if (waves != 8 && waves != 16) return -1;
  g_resln_waves = waves;
  return 0;
}

// fp8 256x256 tiles (8 waves of 128x64): 0 off, 1 under the bf16 auto rule, 2 auto (default).
static int g_fp8_big = 2;
int symb_gemm_fp8_config(int waves, int big) {
  if (waves != 4 && waves != 8 && waves != 16) return -1;
  g_fp8_waves = waves;
  if (big < 0 || big > 2) return -1;
  g_fp8_big = big;
  return 0;
}

// hipBLASLt for the plain bias / bias + residual projections (gemm_lt.cpp): 0 = never (every
// projection on this repo's kernels), 1 = the wide shapes (K >= 768, N >= 768, M >= 4096;
// default), 2 = every bias / residual GEMM.  Round 4 measured this repo's best tiles (256 x 256 /
// 256 x 192, and a deep-ring split-K kernel since removed) against it at M = 32768: the QKV
// (N = 2304 / 3072) and FFN2 (K = 3072 / 4096) shapes stay 13-25 % faster in hipBLASLt, so the
// bge / mpnet / e5 encoders run 6.73 / 6.74 / 19.95 ms with it against 7.52 / 7.55 / 22.50 ms
// without (profiles/r4_gemm/README.md); the GELU / LayerNorm-fused and H = 384 GEMMs are ours.
int symb_gemm_lt(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                 const void* R, int ldr, void* C, int ldc, int M, int N, int K, hipStream_t st);
static int g_gemm_lt = 1;
int symb_gemm_lt_config(int mode) {
  if (mode < 0 || mode > 2) return -1;
  g_gemm_lt = mode;
  return 0;
}

// Small-M split-K path (gemm_skinny.hip): M <= symb_gemm_skinny_max_m() (default 256, the
// query-path batches) goes there first.
int symb_gemm_skinny_max_m();
bool symb_gemm_skinny_supported(int epi, int M, int N, int K);
int symb_gemm_skinny(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                     const void* R, int ldr, const float* gamma, const float* beta, float eps,
                     int gelu_poly, void* C, int ldc, int M, int N, int K, hipStream_t st);

// Returns 0 on success, a HIP error code, or -1 for an unsupported shape.
int symb_gemm(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
              const void* R, int ldr, const float* gamma, const float* beta, float eps, void* C,
              int ldc, int M, int N, int K, hipStream_t st) {
  if (M <= 0) return 0;
  // (the skinny path's split-sum kernel does residual + LayerNorm for any row width <= 4096)
  if (M <= symb_gemm_skinny_max_m() && symb_gemm_skinny_supported(epi, M, N, K))
    return symb_gemm_skinny(epi, A, lda, W, ldw, bias, R, ldr, gamma, beta, eps, g_gelu_poly, C,
                            ldc, M, N, K, st);
  if (epi == EPI_GELU) eps = g_gelu_poly ? 1.f : 0.f;
  if (K % GEMM_BK != 0) return -1;
  auto a = (const __bf16*)A;
  auto w = (const __bf16*)W;
  auto r = (const __bf16*)R;
  auto c = (__bf16*)C;
  if (epi == EPI_RES_LN) {
    if (N == 384 && g_resln_bm == 128 && g_resln_waves == 16)
      return launch_cfg<128, 384, 4, 4, EPI_RES_LN>(a, lda, w, ldw, bias, r, ldr, gamma, beta,
                                                    eps, c, ldc, M, N, K, st);
    if (N == 384 && g_resln_bm == 128)
      return launch_cfg<128, 384, 2, 4, EPI_RES_LN>(a, lda, w, ldw, bias, r, ldr, gamma, beta,
                                                    eps, c, ldc, M, N, K, st);
    if (N == 384)
      return launch_cfg<64, 384, 2, 4, EPI_RES_LN>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps,
                                                   c, ldc, M, N, K, st);
    return -1;  // wider rows: EPI_RES + symb_add_ln
  }
  if (N % 128 != 0) return -1;
  if ((epi == EPI_BIAS || epi == EPI_RES) &&
      (g_gemm_lt == 2 || (g_gemm_lt == 1 && K >= 768 && N >= 768 && M >= 4096))) {
    const int rc = symb_gemm_lt(epi, A, lda, W, ldw, bias, R, ldr, C, ldc, M, N, K, st);
    if (rc != -1 && rc != -2) return rc;   // 0, or a HIP error; else this file's kernels
  }
  if (const int bn = big_tile_bn(g_tile, M, N, K)) {
#define SYMB_G(E, BN_) launch_cfg<256, BN_, 2, 4, E>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps, \
                                                    c, ldc, M, N, K, st)
    switch (epi) {
      case EPI_BIAS: return bn == 256 ? SYMB_G(EPI_BIAS, 256) : SYMB_G(EPI_BIAS, 192);
      case EPI_GELU: return bn == 256 ? SYMB_G(EPI_GELU, 256) : SYMB_G(EPI_GELU, 192);
      case EPI_RES: return bn == 256 ? SYMB_G(EPI_RES, 256) : SYMB_G(EPI_RES, 192);
    }
#undef SYMB_G
    return -1;
  }
  if ((g_tile == 3 || g_tile == 10) && ((M + 127) / 128) * (N / 128) < 256) {
    // small M (query-path batches): fewer tiles than CUs, so occupancy is moot and each tile's
    // serial k-loop is the latency -- a 4-deep ring keeps 3 k-tiles' loads in flight
#define SYMB_G(E) launch_cfg<128, 128, 2, 4, E, 4>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps, \
                                                  c, ldc, M, N, K, st)
    switch (epi) {
      case EPI_BIAS: return SYMB_G(EPI_BIAS);
      case EPI_GELU: return SYMB_G(EPI_GELU);
      case EPI_RES: return SYMB_G(EPI_RES);
    }
#undef SYMB_G
    return -1;
  }
  if (g_tile == 3 || g_tile == 10) {
    // 128x128 with 8 waves of 64x32: 4 waves per SIMD at 2 workgroups per CU
#define SYMB_G(E) launch_cfg<128, 128, 2, 4, E>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps, c, \
                                               ldc, M, N, K, st)
    switch (epi) {
      case EPI_BIAS: return SYMB_G(EPI_BIAS);
      case EPI_GELU: return SYMB_G(EPI_GELU);
      case EPI_RES: return SYMB_G(EPI_RES);
    }
#undef SYMB_G
    return -1;
  }
  switch (epi) {
    case EPI_BIAS:
      return launch_cfg<128, 128, 2, 2, EPI_BIAS>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps,
                                                  c, ldc, M, N, K, st);
    case EPI_GELU:
      return launch_cfg<128, 128, 2, 2, EPI_GELU>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps,
                                                  c, ldc, M, N, K, st);
    case EPI_RES:
      return launch_cfg<128, 128, 2, 2, EPI_RES>(a, lda, w, ldw, bias, r, ldr, gamma, beta, eps, c,
                                                 ldc, M, N, K, st);
  }
  return -1;
}

// Deferred-LayerNorm GEMMs (gemm_bf16_kernel's LNF modes) on the same tiles symb_gemm picks for
// the shape (never hipBLASLt or the small-M path): lnf = LNF_FOLD with EPI_BIAS / EPI_GELU (A a
// pre-LN y, W the gamma-folded weight, bias b' = b + W beta, cs = rowsum of the folded weight),
// LNF_STATS with EPI_RES (the residual R already normalised), LNF_RESLN | LNF_STATS with EPI_RES
// (R a pre-LN y normalised on the fly with gamma / beta).  st_in: float2 [M][np_in] partials of
// the pre-LN input; st_out: float2 [M][N / 64] partials of C.
template <int EPI, int LNF>
static int launch_ln(int bn, bool small, const void* A, int lda, const void* W, int ldw,
                     const float* bias, const __bf16* R, int ldr, const float* g, const float* b,
                     float eps, __bf16* C, int ldc, int M, int N, int K, hipStream_t st,
                     const LnArgs& ln) {
  if (bn == 256)
    return launch_cfg<256, 256, 2, 4, EPI, 2, false, false, LNF>(A, lda, W, ldw, bias, R, ldr, g, b,
                                                                 eps, C, ldc, M, N, K, st, nullptr,
                                                                 nullptr, nullptr, nullptr, ln);
  if (bn == 192)
    return launch_cfg<256, 192, 2, 4, EPI, 2, false, false, LNF>(A, lda, W, ldw, bias, R, ldr, g, b,
                                                                 eps, C, ldc, M, N, K, st, nullptr,
                                                                 nullptr, nullptr, nullptr, ln);
  if (small)
    return launch_cfg<128, 128, 2, 4, EPI, 4, false, false, LNF>(A, lda, W, ldw, bias, R, ldr, g, b,
                                                                 eps, C, ldc, M, N, K, st, nullptr,
                                                                 nullptr, nullptr, nullptr, ln);
  return launch_cfg<128, 128, 2, 4, EPI, 2, false, false, LNF>(A, lda, W, ldw, bias, R, ldr, g, b,
                                                               eps, C, ldc, M, N, K, st, nullptr,
                                                               nullptr, nullptr, nullptr, ln);
}

int symb_gemm_ln(int epi, int lnf, const void* A, int lda, const void* W, int ldw,
                 const float* bias, const void* R, int ldr, const float* gamma, const float* beta,
                 float ln_eps, const float* cs, const void* st_in, int np_in, void* st_out,
                 void* C, int ldc, int M, int N, int K, hipStream_t st) {
  if (M <= 0) return 0;
  if (K % GEMM_BK != 0 || N % 128 != 0) return -1;
  const bool fold = lnf & LNF_FOLD, resln = lnf & LNF_RESLN, stats = lnf & LNF_STATS;
  if ((fold || resln) && (st_in == nullptr || np_in < 1 || np_in > 16)) return -1;
  if (fold && cs == nullptr) return -1;
  if (resln && (gamma == nullptr || beta == nullptr || R == nullptr)) return -1;
  if (stats && st_out == nullptr) return -1;
  LnArgs ln;
  ln.st_in = (const float2*)st_in;
  ln.np_in = np_in;
  ln.cs = cs;
  ln.st_out = (float2*)st_out;
  ln.ln_eps = ln_eps;
  // the tile symb_gemm's auto rule (g_tile 3) picks for the shape
  const int bn = big_tile_bn(3, M, N, K);
  const bool small = !bn && ((M + 127) / 128) * (N / 128) < 256;
  auto a = (const __bf16*)A;
  auto w = (const __bf16*)W;
  auto r = (const __bf16*)R;
  auto c = (__bf16*)C;
  const float geps = g_gelu_poly ? 1.f : 0.f;   // the GELU epilogue's form switch
  if (epi == EPI_BIAS && lnf == 0)
    return launch_ln<EPI_BIAS, 0>(bn, small, a, lda, w, ldw, bias, r, ldr, gamma, beta, 0.f, c, ldc,
                                  M, N, K, st, ln);
  if (epi == EPI_BIAS && lnf == LNF_FOLD)
    return launch_ln<EPI_BIAS, LNF_FOLD>(bn, small, a, lda, w, ldw, bias, r, ldr, gamma, beta, 0.f,
                                         c, ldc, M, N, K, st, ln);
  if (epi == EPI_GELU && lnf == LNF_FOLD)
    return launch_ln<EPI_GELU, LNF_FOLD>(bn, small, a, lda, w, ldw, bias, r, ldr, gamma, beta, geps,
                                         c, ldc, M, N, K, st, ln);
  if (epi == EPI_RES && lnf == LNF_STATS)
    return launch_ln<EPI_RES, LNF_STATS>(bn, small, a, lda, w, ldw, bias, r, ldr, gamma, beta, 0.f,
                                         c, ldc, M, N, K, st, ln);
  if (epi == EPI_RES && lnf == (LNF_RESLN | LNF_STATS))
    return launch_ln<EPI_RES, LNF_RESLN | LNF_STATS>(bn, small, a, lda, w, ldw, bias, r, ldr, gamma,
                                                     beta, 0.f, c, ldc, M, N, K, st, ln);
  return -1;
}

// fp8 GEMM: C = epi((A8 . W8^T) * sa[m] * sw[n] + bias); A8 [M,K], W8 [N,K] OCP e4m3 bytes.
// epi: EPI_BIAS / EPI_GELU / EPI_RES (row LayerNorms go through symb_add_ln), or EPI_GELU_MX8
// (C receives MX fp8: e4m3 bytes, ldc in bytes, plus E8M0 exponents in cscale [M, N/32]).
// ascale != nullptr: A8 is MX-scaled (E8M0 per 32 k, [M, K/32]) and sa is unused.
int symb_gemm_fp8(int epi, const void* A8, int lda, const void* W8, int ldw, const float* sa,
                  const float* sw, const float* bias, const void* R, int ldr, void* C, int ldc,
                  int M, int N, int K, hipStream_t st, const void* ascale, void* cscale) {
  if (M <= 0) return 0;
  if (K % 128 != 0 || N % 128 != 0) return -1;
  if (epi == EPI_GELU_MX8 && !cscale) return -1;
  auto r = (const __bf16*)R;
  auto c = (__bf16*)C;
  auto as = (const uint8_t*)ascale;
  auto cs = (uint8_t*)cscale;
  // 256x256: g_fp8_big 1 = wherever the bf16 auto rule takes it; 2 (default) = only where it
  // measured faster -- long-K or wide-N projections (e5 QKV 1337 -> 1458, FFN2 MX-in 1687 -> 1867
  // TFLOP/s), not the square out-projection or the MX-emitting FFN1 (both slower),
  // profiles/r1_s4/fp8_waves/gemmfp8_256.json
  const bool big = g_fp8_big != 0 && big_tile_bn(10, M, N, K) == 256 &&
                   (g_fp8_big == 1 || (K >= 1024 && N != K && epi != EPI_GELU_MX8));
#define SYMB_G8W(E, X, BMN, WM_, WN_) launch_cfg<BMN, BMN, WM_, WN_, E, 2, true, X>(              \
    A8, lda, W8, ldw, bias, r, ldr, nullptr, nullptr, g_gelu_poly ? 1.f : 0.f, c, ldc, M, N, K, \
    st, sa, sw, as, cs)
#define SYMB_G8(E, X)                                                                      \
  (big ? SYMB_G8W(E, X, 256, 2, 4)                                                         \
       : g_fp8_waves == 16 ? SYMB_G8W(E, X, 128, 4, 4)                                     \
                           : g_fp8_waves == 8 ? SYMB_G8W(E, X, 128, 2, 4) : SYMB_G8W(E, X, 128, 2, 2))
  if (as) {
    switch (epi) {
      case EPI_BIAS: return SYMB_G8(EPI_BIAS, true);
      case EPI_GELU: return SYMB_G8(EPI_GELU, true);
      case EPI_RES: return SYMB_G8(EPI_RES, true);
      case EPI_GELU_MX8: return SYMB_G8(EPI_GELU_MX8, true);
    }
    return -1;
  }
  switch (epi) {
    case EPI_BIAS: return SYMB_G8(EPI_BIAS, false);
    case EPI_GELU: return SYMB_G8(EPI_GELU, false);
    case EPI_RES: return SYMB_G8(EPI_RES, false);
    case EPI_GELU_MX8: return SYMB_G8(EPI_GELU_MX8, false);
  }
#undef SYMB_G8
#undef SYMB_G8W
  return -1;
}

// Per-row (token) activation quantiser for the fp8 GEMMs: scale[m] = amax(x[m, :]) / 448 and
// out = e4m3(x / scale).  One wave per row; K <= 4096 and K % 8 == 0.
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const __bf16* __restrict__ x, int ldx,
                                                             uint8_t* __restrict__ out, int ldo,
                                                             float* __restrict__ scale, int M,
                                                             int K) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[8][8];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < K) {
      load8(x + (size_t)row * ldx + col, v[c]);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[c][e]));
    }
  }
  amax = fmaxf(wave_max(amax), 1e-12f);
  const float inv = 448.f / amax;
  if (lane == 0) scale[row] = amax / 448.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col >= K) continue;
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][0] * inv, v[c][1] * inv, 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][2] * inv, v[c][3] * inv, lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4] * inv, v[c][5] * inv, 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][6] * inv, v[c][7] * inv, hi, true);
    *reinterpret_cast<int2*>(out + (size_t)row * ldo + col) = make_int2(lo, hi);
  }
}

int symb_quant_rows_fp8(const void* x, int ldx, void* out, int ldo, float* scale, int M, int K,
                        hipStream_t st) {
  if (M <= 0) return 0;
  if (K % 8 || K > 4096) return -1;
  hipLaunchKernelGGL(quant_rows_fp8_kernel, dim3((M + 3) / 4), dim3(256), 0, st,
                     (const __bf16*)x, ldx, (uint8_t*)out, ldo, scale, M, K);
  return (int)hipGetLastError();
}

int symb_gemm_gelu_config(int poly) {
  if (poly != 0 && poly != 1) return -1;
  g_gelu_poly = poly;
  return 0;
}
int symb_gemm_gelu_poly() { return g_gelu_poly; }
