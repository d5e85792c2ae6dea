// Persistent 4-wave bf16 GEMM for the wide encoders' large projections (bge-base / e5-large QKV,
// out-projection, FFN1, FFN2), same contract as gemm.hip's symb_gemm:
//
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] )      epi = bias | GELU(erf) | + residual
//
// Reference call site: the candle BertModel linears driven by
// services/preprocessing_service/src/embedding_generator.rs:198.
//
// Why another tile: the 8-wave 256x256 kernels (gemm.hip, gemm256.hip) give every wave a 128x64
// output and run two waves per SIMD; hipBLASLt's fastest kernels for these shapes (rocprofv3
// trace, profiles/r3_gemm/) run 4 waves of 128x128 -- one wave per SIMD, 256 accumulator
// registers each -- which halves the LDS fragment bytes per MFMA (16 ds_read_b128 per 64 MFMAs
// instead of 12 per 32).  This kernel is that geometry, written for our epilogues:
//
//  * 256 threads, waves 2 (M) x 2 (N), wave tile (BM/2) x 128, v_mfma_f32_16x16x32_bf16 with the
//    OPERANDS SWAPPED (W fragment first): each accumulator block is C^T, so a lane holds 4
//    consecutive output COLUMNS of one row.  The W rows are permuted when staged (per-lane DMA
//    source address; the LDS image stays lane-linear) so that blocks 2p and 2p + 1 give a lane
//    8 consecutive columns: the epilogue works straight from the accumulators (bias, GELU,
//    residual) and leaves as one 16-byte store per (16-row block, 32-column group) -- no LDS
//    round trip, so the LDS is free for the next tile's first k-tiles during the epilogue.
//  * BK = 64 (128-byte LDS rows, chunk index XORed with (row >> 1) & 7 on the DMA source and on
//    the ds_read address), two LDS stages filled by global_load_lds_dwordx4.
//  * Register double-buffered fragments: the k-tile's second 32-deep half is read under the
//    first half's 64 MFMAs, and the NEXT k-tile's first half under the second half's, so the
//    one barrier per k-tile sits between two MFMA groups and no LDS latency is exposed after it.
//  * Persistent: grid = min(tiles, CUs); a workgroup walks tiles in the XCD-aware grouped order
//    of gemm.hip.  Before each epilogue the next tile's k-tiles 0 and 1 are DMA'd; the epilogue's
//    stores drain under the next tile's first k-tile (counted vmcnt).
#include "common.h"

namespace symb {

enum { G4_BIAS = 0, G4_GELU = 1, G4_RES = 2 };

namespace g4 {
constexpr int BN = 256, NT = 256;
// lane id from v_mbcnt; volatile so that each use recomputes it instead of keeping one copy
// (and everything derived from it) live across the k-loop
__device__ __forceinline__ int lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ void tile_origin(int id, int n_all, int n_tiles, int group_m, int bm,
                                            int& m0, int& n0) {
  const int tile = xcd_remap(id, n_all);
  int tm = tile / n_tiles, tn = tile % n_tiles;
  if (group_m > 1) {
    const int m_tiles = n_all / n_tiles, per_group = group_m * n_tiles;
    const int g = tile / per_group, first = g * group_m;
    const int gm = min(group_m, m_tiles - first), local = tile - g * per_group;
    tm = first + local % gm;
    tn = local / gm;
  }
  m0 = tm * bm;
  n0 = tn * BN;
}
}  // namespace g4

template <int BM, int EPI>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(
    const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ W, int ldw,
    const float* __restrict__ bias, const __bf16* __restrict__ R, int ldr,
    __bf16* __restrict__ C, int ldc, int M, int N, int K, int group_m, float gelu_poly) {
  using namespace g4;
  constexpr int WTM = BM / 2;             // wave tile rows
  constexpr int RM = WTM / 16, RN = 8;    // 16x16 blocks per wave: RM (rows) x 8 (128 columns)
  constexpr int A_BYTES = BM * 128;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int A_LD = BM * 8 / NT, B_LD = BN * 8 / NT;   // 16-byte DMA pieces per thread
  constexpr int LD = A_LD + B_LD;
  constexpr int ZERO = 2 * STAGE;         // 16 KiB of zeros (see the k-loop)
  constexpr int ZERO_BYTES = 16384;
  constexpr int ST = RM * 4;              // 16-byte output stores per lane per tile
  static_assert(BM % 32 == 0 && RM >= 1, "tile rows");
  static_assert(LD + ST <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // wave id in an SGPR: the DMA's LDS destinations (M0) are then scalar arithmetic, not VGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int n_tiles = N / BN, n_all = ((M + BM - 1) / BM) * n_tiles;
  const int KT = K / 64;

  // ---- DMA through buffer descriptors (SGPRs).  Piece i of a stage covers tile rows 32 i +
  // (tid >> 3), 16-byte chunk (tid & 7) ^ ((tid >> 4) & 7) (the swizzle term is the same for every
  // piece).  A rows are clamped to M - 1 per piece (a few VALU ops per k-tile, nothing long-lived);
  // the soffset SGPR carries only the k-tile's byte offset.  W rows are permuted: LDS B row
  // 128 h + 16 j + c' (wave half h, block j, block row c') holds output column
  // 128 h + 32 (j >> 1) + 8 (c' >> 2) + 4 (j & 1) + (c' & 3) = 32 i + gcol for piece i, so one
  // voffset + an SGPR term i * 32 rows address every W piece (W rows never pass N).
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)((size_t)M * lda * 2), 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((size_t)N * ldw * 2), 0x00020000);
  const int chunk16 = ((tid & 7) ^ ((tid >> 4) & 7)) * 16;
  const int cpr = (tid >> 3) & 15;
  const int gcol = 8 * (cpr >> 2) + 4 * (tid >> 7) + (cpr & 3);
  int arow = 0;          // this thread's first A row of the current tile
  uint32_t vb = 0;
  auto set_tile = [&](int m0, int n0) {
    const int t2 = wave * 64 + lane_id();
    const int ch = ((t2 & 7) ^ ((t2 >> 4) & 7)) * 16, cr = (t2 >> 3) & 15;
    arow = m0 + (t2 >> 3);
    vb = (uint32_t)((n0 + 8 * (cr >> 2) + 4 * (t2 >> 7) + (cr & 3)) * ldw * 2 + ch);
  };
  auto stage = [&](int kt, int buf) {
    char* sA = smem + buf * STAGE;
    char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_LD; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(sA + (i * NT + wave * 64) * 16), 16,
          (uint32_t)(min(arow + 32 * i, M - 1) * lda * 2 + chunk16), kt * 128, 0, 0);
#pragma unroll
    for (int i = 0; i < B_LD; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsW, (__attribute__((address_space(3))) void*)(sB + (i * NT + wave * 64) * 16), 16, vb,
          i * 32 * ldw * 2 + kt * 128, 0, 0);
  };
  // ---- fragments: lane row fr, 8 k at chunk kk * 4 + fq; the XOR term is (fr >> 1) & 7 ----
  const int x = (fr >> 1) & 7;
  uint32_t oa[2], ob[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    oa[kk] = (uint32_t)((wm * WTM + fr) * 128 + (((kk * 4 + fq) ^ x) << 4));
    ob[kk] = (uint32_t)(A_BYTES + (wn * 128 + fr) * 128 + (((kk * 4 + fq) ^ x) << 4));
  }
  // ONE fragment set, refilled in place: with the MFMAs of a half-step ordered as pass 1 =
  // (every row i, columns j < 4), pass 2 = (every row i, columns j >= 4), a fragment is dead
  // as soon as its last MFMA has issued -- b[0..3] after pass 1, a[i] after (i, 7), b[4..7] at
  // the end -- and the next half-step's copy is read into the same registers right there.  Each
  // read then has >= 28 MFMAs (~450 cycles) before its first use, no register copies, and the
  // loop-carried values keep their registers (a second, ping-ponged set made hipcc rotate the
  // 256 accumulators through copies).
  bf16x8 a[RM], b[RN];
  // fragment base offsets; zero = the last half-step's "next" reads, which come from an
  // all-zero LDS region (uniform address) so that the trailing MFMA pass adds exact zeros
  auto off_b = [&](int buf, int kk, bool zero) { return zero ? (uint32_t)ZERO : buf * STAGE + ob[kk]; };
  auto off_a = [&](int buf, int kk, bool zero) { return zero ? (uint32_t)ZERO : buf * STAGE + oa[kk]; };
  auto rd_b = [&](uint32_t off, int j0) {
#pragma unroll
    for (int j = j0; j < j0 + 4; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(smem + off + j * 2048);
  };
  auto rd_a = [&](uint32_t off, int i) {
    a[i] = *reinterpret_cast<const bf16x8*>(smem + off + i * 2048);
  };
  f32x4 acc[RM][RN];

  // zero the region the last half-step's reads come from (never a DMA destination)
#pragma unroll
  for (int c = 0; c < ZERO_BYTES / (NT * 16); ++c)
    *reinterpret_cast<f32x4*>(smem + ZERO + (c * NT + tid) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};

  int id = blockIdx.x;
  int m0, n0;
  tile_origin(id, n_all, n_tiles, group_m, BM, m0, n0);
  set_tile(m0, n0);
  stage(0, 0);
  if (KT > 1) stage(1, 1);
  bool pend = false;   // the previous tile's ST stores are still in flight behind these DMAs

#pragma unroll 1
  for (; id < n_all; id += gridDim.x) {
    // k-tile 0 landed (k-tile 1's LD pieces and the previous tile's stores may still fly)
    if (KT > 1) {
      if (pend)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LD + ST) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LD) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RM; ++i) rd_a(off_a(0, 0, false), i);
    rd_b(off_b(0, 0, false), 0);
    rd_b(off_b(0, 0, false), 4);

    // The loop body is rotated so that its one barrier comes first: iteration h = barrier h,
    // DMA batch, reads of half-step h + 1 (interleaved with pass 2 of h), pass 1 of h + 1.  A
    // barrier between MFMA groups of one body made hipcc rotate the 256 accumulators through
    // copies; with it at the top every accumulator keeps its registers.
    auto pass1 = [&]() {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    };
    auto pass2 = [&](uint32_t aoff) {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
#pragma unroll
        for (int j = 4; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        rd_a(aoff, i);
      }
    };
    pass1();
    // 2 KT identical iterations (no peeled tail: hipcc started moving the accumulators out of
    // the AGPRs before a peeled last pass and spilled); the last one's pass 1 runs on the zero
    // fragments
#pragma unroll 1
    for (int h = 0; h < 2 * KT; ++h) {
      const int t = h >> 1;
      // the next half-step: (t, 1) in the same buffer, or (t + 1, 0) in the other one
      const int nbuf = (t + (h & 1)) & 1, nkk = (h & 1) ^ 1;
      const bool last = h + 1 == 2 * KT;
      // odd half-steps: k-tile t + 1 landed everywhere, and every wave's reads issued before
      // this barrier retired, so buffer t (whose fragments are all in registers by now) takes
      // k-tile t + 2; even half-steps only order the LDS reads
      if (h & 1)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if ((h & 1) && t + 2 < KT) stage(t + 2, t & 1);
      __builtin_amdgcn_sched_barrier(0);
      rd_b(off_b(nbuf, nkk, last), 0);
      pass2(off_a(nbuf, nkk, last));   // columns 4-7 of h; row i's A fragment refilled after (i, 7)
      rd_b(off_b(nbuf, nkk, last), 4);
      pass1();                    // columns 0-3 of h + 1 (b[4..7] are first needed in pass 2)
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * RM, 0);
    }
    pend = false;

    // ---- epilogue (registers only): bias / GELU / residual, 16-byte stores ----
    const int cm0 = m0, cn0 = n0;
    const bool full = cm0 + BM <= M;
    // every wave's last ds_read has retired (each waited before its last MFMAs): the LDS is free
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // lane columns: group p covers cn0 + wn * 128 + 32 p + 8 fq + (0..7)
    // lane-derived addresses recomputed here from a fresh lane id (a volatile asm is never
    // CSE'd with the loop's copies): kept live across the k-loop they were spilled, and the
    // reloads' waits drained the next tile's DMA
    const int elane = lane_id();
    const int col0 = cn0 + wn * 128 + 8 * (elane >> 4);
    f32x4 bv[4][2];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      bv[p][0] = *reinterpret_cast<const f32x4*>(bias + col0 + 32 * p);
      bv[p][1] = *reinterpret_cast<const f32x4*>(bias + col0 + 32 * p + 4);
    }
    const int row0 = cm0 + wm * WTM + (elane & 15);   // + 16 i
    // residual rows: the first half of the row blocks is loaded before the next tile's DMA, the
    // second half after the first half's stores (all of them up front spilled)
    constexpr int RH = (RM + 1) / 2;
    bf16x8 res[RM][4];
    auto load_res = [&](int i0, int i1) {
#pragma unroll
      for (int i = i0; i < i1; ++i)
#pragma unroll
        for (int p = 0; p < 4; ++p)
          res[i][p] = *reinterpret_cast<const bf16x8*>(
              R + (size_t)min(row0 + 16 * i, M - 1) * ldr + col0 + 32 * p);
    };
    if constexpr (EPI == G4_RES) load_res(0, RH);
    // bias (and residual) loads land BEFORE the next tile's DMA is issued: a load waited for
    // after it would wait for the DMA too (vmcnt retires in issue order).  A real S_WAITCNT
    // (vmcnt(0)), so hipcc's own bookkeeping knows those registers are ready.
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // the next tile's first two k-tiles stream in under this epilogue
    if (id + (int)gridDim.x < n_all) {
      tile_origin(id + gridDim.x, n_all, n_tiles, group_m, BM, m0, n0);
      set_tile(m0, n0);
      stage(0, 0);
      if (KT > 1) stage(1, 1);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      if constexpr (EPI == G4_RES) {
        if (i == RH) load_res(RH, RM);
      }
      const int row = row0 + 16 * i;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[i][2 * p][r] + bv[p][0][r];
          v[4 + r] = acc[i][2 * p + 1][r] + bv[p][1][r];
        }
        if constexpr (EPI == G4_GELU) {
          if (gelu_poly != 0.f) {
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const f32x2 g = gelu2_poly(f32x2{v[e], v[e + 1]});
              v[e] = g.x;
              v[e + 1] = g.y;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
          }
        }
        if constexpr (EPI == G4_RES) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)res[i][p][e];
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
        if (full || row < M) *reinterpret_cast<bf16x8*>(C + (size_t)row * ldc + col0 + 32 * p) = o;
      }
      // one 16-row block at a time: unfenced, hipcc hoists every accumulator read and spills
      __builtin_amdgcn_sched_barrier(0);
    }
    pend = full;
    if (!full) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace symb

using namespace symb;

// Shapes this kernel takes: N % 256 == 0, K % 64 == 0 (bm: 256 or 192 rows per tile).
bool symb_gemm4w_supported(int M, int N, int K) {
  return M > 0 && N % 256 == 0 && K % 64 == 0 && K >= 64;
}

// epi: 0 bias, 1 GELU, 2 residual (gemm.hip's EPI_BIAS / EPI_GELU / EPI_RES); bm = 256 or 192.
// Returns 0, a HIP error code, or -1 for an unsupported shape / epilogue.
int symb_gemm4w(int epi, int bm, const void* A, int lda, const void* W, int ldw, const float* bias,
                const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                int gelu_poly, hipStream_t st) {
  if (M <= 0) return 0;
  if (!symb_gemm4w_supported(M, N, K) || (bm != 256 && bm != 192)) return -1;
  // buffer descriptors hold byte sizes in 31 bits
  if ((size_t)M * lda * 2 > 0x7fffffffu || (size_t)N * ldw * 2 > 0x7fffffffu) return -1;
  static int n_cus = 0;
  if (n_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cus <= 0)
      n_cus = 256;
  }
  const int tiles = ((M + bm - 1) / bm) * (N / 256);
  const int grid = tiles < n_cus ? tiles : n_cus;   // persistent: one workgroup per CU
  auto go = [&](auto kern, int lds) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, (const __bf16*)A, lda,
                       (const __bf16*)W, ldw, bias, (const __bf16*)R, ldr, (__bf16*)C, ldc, M, N,
                       K, group_m, gelu_poly ? 1.f : 0.f);
    return (int)hipGetLastError();
  };
  constexpr int L256 = 2 * (256 + 256) * 128 + 16384, L192 = 2 * (192 + 256) * 128 + 16384;
  if (bm == 256) {
    switch (epi) {
      case G4_BIAS: return go(gemm4w_kernel<256, G4_BIAS>, L256);
      case G4_GELU: return go(gemm4w_kernel<256, G4_GELU>, L256);
      case G4_RES: return go(gemm4w_kernel<256, G4_RES>, L256);
    }
  } else {
    switch (epi) {
      case G4_BIAS: return go(gemm4w_kernel<192, G4_BIAS>, L192);
      case G4_GELU: return go(gemm4w_kernel<192, G4_GELU>, L192);
      case G4_RES: return go(gemm4w_kernel<192, G4_RES>, L192);
    }
  }
  return -1;
}
