// Fused brute-force cosine scan + top-k over an HBM-resident index shard (replaces Qdrant's
// HNSW search, services/vector_memory_service/src/main.rs:261-308).
//
//   scores = X[rows] · Q^T   (X: unit-norm bf16 rows, Q: unit-norm bf16 queries)  -> per-query
//   top-KMAX candidates, without ever writing the [rows x queries] score matrix to HBM.
//
// CDNA4 design (one 512-thread workgroup per CU, 2 waves per SIMD):
//  * The queries live in REGISTERS as MFMA B fragments: every wave owns 32 queries (D=384,
//    v_mfma_f32_32x32x16_bf16, 24 fragments = 96 VGPRs) or 16 queries (D=768/1024,
//    v_mfma_f32_16x16x32_bf16).  A workgroup therefore scores 256 (or 128) queries at once.
//  * Index rows stream HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging) in tiles of two
//    MFMA sub-tiles (64 rows at D=384) through an NS-deep LDS ring (ScanCfg: 3 x 48 KiB at D=384)
//    with a COUNTED `s_waitcnt vmcnt` and a raw s_barrier, so the next tile stays in flight across
//    the barrier (a __syncthreads would drain vmcnt to 0).  The DMA pieces of tile t+NS-1 are
//    issued inside sub-tile 0's MFMA chain of tile t.  Every tile read from HBM once feeds 8
//    waves x their queries.
//  * A fragments are read by hand-issued ds_read_b128 (inline asm) with counted lgkmcnt waits,
//    6 in flight, so the compiler cannot serialise them behind lgkmcnt(0).
//  * Bank conflicts: the image stays lane-linear for the DMA; the 16-byte chunk index is XORed
//    with (row & 15) on the global source address and on the ds_read_b128 address.
//  * Top-k: with X as the A operand, a lane's accumulator column IS one query, so the running
//    per-query threshold lives in a register and the sorted top-KMAX list in statically indexed
//    registers.  The threshold can be SEEDED (thr_init) with a lower bound on the final k-th
//    score from a sample pre-pass, which removes the record-breaking inserts that otherwise hit
//    nearly every sub-tile of a fresh 64-list wave (profiles/r1_scan/README.md).
//  * A second small kernel merges the per-workgroup candidate lists into the final top-k.
//  * Profiling-only variants (index_scan_ablate): DMA-only, compute-only, L2-sourced DMA,
//    staggered top-k, s_memtime segment stamps, and a 4-wave AGPR-resident "wide" kernel.
#include "scan_common.h"

#include <type_traits>

namespace symb {

constexpr int TOPK_WAVES = 8;

// ---- hand-counted LDS fragment pipeline -------------------------------------------------------
// hipcc will not count ds_reads around the DMA ring (it drains lgkmcnt(0) before every few MFMAs),
// so the A fragments are read by inline asm and each MFMA waits with a counted lgkmcnt(N) whose
// asm names the fragment as "+v" (the MFMA depends on it and cannot be hoisted above the wait).
template <int OFF>
__device__ __forceinline__ void ds_read16(bf16x8& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "i"(N));
}

// Fragment ks lives at  base + voff[ks % M] + (ks / M) * 256  (the XOR swizzle only touches the
// low 4 bits of the 16-byte chunk index, so the per-lane part repeats every M k-steps).
// DMA (functor, may be a no-op): DMA(i) issues LDS-DMA piece i of the next tile; pieces are
// spread one per DMA_EVERY MFMAs so the waves' DMA issue interleaves with their matrix work.
template <int KS, int NKS, int PF, int M, bool M32, int DMA_EVERY = 0, int DMA_PIECES = 0>
struct FragChain {
  static constexpr int R = PF + 1;  // ring slots: a slot is refilled one MFMA after its last use
  template <class Acc, class Dma = NoDma>
  __device__ __forceinline__ static void run(Acc& acc, bf16x8 (&a)[R], const bf16x8 (&qf)[NKS],
                                             const uint32_t (&voff)[M], uint32_t base,
                                             const Dma& dma = Dma()) {
    if constexpr (DMA_EVERY > 0 && KS % DMA_EVERY == 0 && KS / DMA_EVERY < DMA_PIECES)
      dma(KS / DMA_EVERY);
    constexpr int outstanding = (NKS - KS < PF) ? (NKS - KS) : PF;
    lgkm_wait<outstanding - 1>(a[KS % R]);
    if constexpr (M32)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[KS % R], qf[KS], acc, 0, 0, 0);
    else
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[KS % R], qf[KS], acc, 0, 0, 0);
    if constexpr (KS + PF < NKS)
      ds_read16<((KS + PF) / M) * 256>(a[(KS + PF) % R], base + voff[(KS + PF) % M]);
    if constexpr (KS + 1 < NKS)
      FragChain<KS + 1, NKS, PF, M, M32, DMA_EVERY, DMA_PIECES>::run(acc, a, qf, voff, base, dma);
  }
};

template <int J, int PF, int M, int R>
__device__ __forceinline__ void frag_prologue(bf16x8 (&a)[R], const uint32_t (&voff)[M],
                                              uint32_t base) {
  ds_read16<(J / M) * 256>(a[J % R], base + voff[J % M]);
  if constexpr (J + 1 < PF) frag_prologue<J + 1, PF, M, R>(a, voff, base);
}

// MFMA_32 = true : D = 384 path (32x32x16, 32 queries per wave, 2 lists per query per wave)
// MFMA_32 = false: D = 768/1024 path (16x16x32, 16 queries per wave, 4 lists per query per wave)
// A barrier interval covers one TILE = 2 sub-tiles (2 x 32 rows, or 2 x 16 rows); the second
// sub-tile's fragment reads are issued before the first sub-tile's top-k VALU work so LDS latency
// and the VALU tail overlap, and the per-barrier fixed cost is paid once per 2 MFMA chains.
// NS  : LDS ring depth in tiles (NS-2 tiles stay in flight across every barrier)
// AUX : cache policy of the index stream (0 = default, 2 = non-temporal: rows read once)
// ABL (profiling builds only): 0 = full kernel, 1 = DMA ring only (no MFMA / top-k),
// 2 = compute only (no DMA; fragments come from whatever the LDS holds).
// 8/9/10 = 0/5/2 with per-segment s_memtime stamps written over cand_s (diagnostic builds only).
template <int D, bool MFMA_32, int KMAX, int NS, int AUX, int ABLX = 0>
__global__ __launch_bounds__(512) void index_scan_topk_kernel(
    const __bf16* __restrict__ X, int n_valid, int rows_per_blk, const __bf16* __restrict__ Q,
    int NQ, int n_qblk, int xcd, const float* __restrict__ thr_init, float* __restrict__ cand_s,
    int* __restrict__ cand_i, const int* __restrict__ gate) {
  // gate (optional): run only if *gate != 0 -- the exact fallback of the multi-query-block scan
  // (index_mq.hip) is enqueued unconditionally and skips itself unless a candidate buffer
  // overflowed, so no host sync decides it
  if (gate != nullptr && *gate == 0) return;
  constexpr bool STAMP = ABLX >= 8;
  constexpr int ABL = ABLX == 8 ? 0 : ABLX == 9 ? 5 : ABLX == 10 ? 2 : ABLX;
  uint64_t seg[6] = {0, 0, 0, 0, 0, 0};
  uint64_t t_prev = 0, t_start = 0, rt_start = 0;
  auto stamp = [&](int i) {
    if constexpr (STAMP) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      seg[i] += now - t_prev;
      t_prev = now;
    }
  };
  constexpr int CPR = D / 8;                          // 16-byte chunks per row
  constexpr int SUB = MFMA_32 ? 32 : 16;              // rows per MFMA chain (sub-tile)
  constexpr int TR = 2 * SUB;                         // rows per barrier interval
  constexpr int TILE_BYTES = TR * D * 2;
  constexpr int SUB_BYTES = SUB * D * 2;
  // ABL 6/7: only waves 0-3 (one per SIMD) issue the LDS-DMA, so when an issue stalls on a full
  // miss queue the partner wave on that SIMD still has MFMAs to run.
  constexpr bool HALFDMA = (ABL == 6 || ABL == 7);
  constexpr int DMA_WAVES = HALFDMA ? TOPK_WAVES / 2 : TOPK_WAVES;
  constexpr int LOADS = TILE_BYTES / (1024 * DMA_WAVES);  // glds per DMA wave per tile
  constexpr int DMA_EVERY = HALFDMA ? 2 : 4;               // MFMA steps between DMA pieces
  static_assert(TILE_BYTES % (1024 * DMA_WAVES) == 0, "tile must split evenly over waves");
  static_assert(NS >= 2 && NS * TILE_BYTES <= 160 * 1024, "LDS ring exceeds the CU's 160 KiB");
  constexpr int QW = MFMA_32 ? 32 : 16;               // queries per wave
  constexpr int NKS = MFMA_32 ? D / 16 : D / 32;      // MFMA k-steps over D
  constexpr int LISTS = MFMA_32 ? 2 : 4;
  constexpr int M = MFMA_32 ? 8 : 4;                  // period of the per-lane fragment offsets
  constexpr int PF = 6;                               // fragment reads in flight
  using Acc = typename std::conditional<MFMA_32, f32x16, f32x4>::type;
  constexpr int NR = MFMA_32 ? 16 : 4;                // accumulator registers per lane

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // xcd != 0: the n_qblk query blocks of one row block are consecutive logical ids on ONE XCD, so
  // the row block streams from HBM into that XCD's L2 once and feeds all of its query blocks
  // (without it, round-robin dispatch puts them on n_qblk different XCDs: n_qblk HBM reads).
  const int lb = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qb = lb % n_qblk, rb = lb / n_qblk;
  const int row_begin = rb * rows_per_blk;
  const int row_end = min(row_begin + rows_per_blk, n_valid);
  const int n_tiles = row_end > row_begin ? (row_end - row_begin + TR - 1) / TR : 0;

  // ---- query fragments (B operand) ----
  const int qlocal = MFMA_32 ? (lane & 31) : (lane & 15);
  const int query = qb * (QW * TOPK_WAVES) + wave * QW + qlocal;
  const __bf16* qp = Q + (size_t)min(query, NQ - 1) * D;
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int k0 = MFMA_32 ? ks * 16 + (lane >> 5) * 8 : ks * 32 + (lane >> 4) * 8;
    qf[ks] = *reinterpret_cast<const bf16x8*>(qp + k0);
  }

  // ---- per-thread DMA source offsets within a tile (identical for every tile) ----
  uint32_t goff[LOADS];
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {
    const int s = (i * DMA_WAVES + (wave % DMA_WAVES)) * 64 + lane;  // LDS 16-byte slot filled
    const int row = s / CPR, pc = s % CPR;
    const int c = pc ^ (row & 15);
    goff[i] = (uint32_t)(row * D + c * 8);
  }
  auto issue_piece = [&](int t, int i) {
    // ABL==5 (diagnostic): every tile re-loads the block's first NS tiles (L2-resident source)
    const int tt = ABL == 5 ? min(t % NS, n_tiles - 1) : min(t, n_tiles - 1);
    const __bf16* base = X + (size_t)(row_begin + tt * TR) * D;
    char* dst = smem + (t % NS) * TILE_BYTES;
    glds16_aux<AUX>(base + goff[i], dst + ((i * DMA_WAVES + wave) * 64) * 16);
  };
  const bool dma_wave = !HALFDMA || __builtin_amdgcn_readfirstlane(wave) < DMA_WAVES;
  auto issue = [&](int t) {
    if (!dma_wave) return;
    const int tt = min(t, n_tiles - 1);  // past the end: re-load the last tile (keeps vmcnt exact)
    const __bf16* base = X + (size_t)(row_begin + tt * TR) * D;
    char* dst = smem + (t % NS) * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < LOADS; ++i)
      glds16_aux<AUX>(base + goff[i], dst + ((i * DMA_WAVES + wave) * 64) * 16);
  };

  // ---- per-lane LDS fragment offsets within a sub-tile (see FragChain) ----
  const uint32_t lds_smem = lds_addr(smem);
  uint32_t voff[M];
  if constexpr (MFMA_32) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int m = 0; m < M; ++m) voff[m] = (uint32_t)(r * D * 2 + (((2 * m + h) ^ (r & 15)) << 4));
  } else {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int m = 0; m < M; ++m) voff[m] = (uint32_t)(r * D * 2 + (((4 * m + g) ^ r) << 4));
  }

  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    tv[i] = -INFINITY;
    ti[i] = -1;
  }
  // Seeded filter: thr_init[q] (optional) is a LOWER BOUND on query q's final k-th score (the
  // k-th best over a row sample, nudged down one ulp), so every true top-k score still passes.
  // Random-order rows otherwise break a fresh list's record ~16*ln(n/16) times, and with 64
  // lists per wave nearly every sub-tile paid a wave-wide insert (stamps: top-k 2.3x its cost).
  float thr = thr_init ? thr_init[min(query, NQ - 1)] : -INFINITY;
  // row of accumulator register r for this lane (relative to the sub-tile)
  auto acc_row = [&](int r) {
    return MFMA_32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : (lane >> 4) * 4 + r;
  };
  auto topk_update = [&](Acc& acc, int row0) {
    if (row0 + SUB > row_end) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (row0 + acc_row(r) >= row_end) acc[r] = -INFINITY;
    }
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < NR; ++r) mx = fmaxf(mx, acc[r]);
    if (mx > thr) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (acc[r] > thr) {
          topk_insert_par<KMAX>(tv, ti, acc[r], row0 + acc_row(r));
          thr = fmaxf(thr, tv[KMAX - 1]);
        }
      }
    }
  };

  if (n_tiles > 0 && ABL != 2) {
#pragma unroll
    for (int p = 0; p < NS - 1; ++p) issue(p);
  }
  constexpr int R = PF + 1;
  bf16x8 a[R];
  // ABL==4 (stagger): waves 4-7 (the second wave on each SIMD) defer the top-k of their second
  // sub-tile into the next barrier interval, so the two waves sharing a SIMD leave the barrier
  // out of phase and one's MFMA chain covers the other's fragment-read latency.
  constexpr bool STAG = (ABL == 4 || ABL == 7);
  const bool late = STAG && (__builtin_amdgcn_readfirstlane(wave) >= TOPK_WAVES / 2);
  Acc accd;
  int rowd = 0;
  if constexpr (STAMP) {
    t_start = t_prev = __builtin_amdgcn_s_memtime();
    rt_start = __builtin_amdgcn_s_memrealtime();
  }
  for (int t = 0; t < n_tiles; ++t) {
    // tile t landed for this wave once only the (NS-2) younger tiles' loads remain
    if constexpr (ABL != 2) wait_vmcnt<LOADS * (NS - 2)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(0);
    __builtin_amdgcn_s_barrier();
    stamp(1);
    // (the DMA pieces of tile t+NS-1 are issued inside sub-tile 0's MFMA chain below)
    if constexpr (ABL == 1) {
      issue(t + NS - 1);
      continue;
    }
    const uint32_t base0 = lds_smem + (uint32_t)((t % NS) * TILE_BYTES);
    const uint32_t base1 = base0 + SUB_BYTES;
    const int row0 = row_begin + t * TR;

    Acc acc0, acc1;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      acc0[r] = 0.f;
      acc1[r] = 0.f;
    }
    frag_prologue<0, PF, M, R>(a, voff, base0);
    if (STAG && late && t > 0) topk_update(accd, rowd);
    const int tnext = t + NS - 1;
    auto dma = [&](int i) {
      if constexpr (ABL != 2) {
        if (dma_wave) issue_piece(tnext, i);
      }
    };
    static_assert(LOADS * DMA_EVERY <= NKS, "DMA pieces must fit the first chain");
    FragChain<0, NKS, PF, M, MFMA_32, DMA_EVERY, LOADS>::run(acc0, a, qf, voff, base0, dma);
    stamp(2);
    frag_prologue<0, PF, M, R>(a, voff, base1);   // sub-tile 1 reads fly during top-k of sub 0
    topk_update(acc0, row0);
    stamp(3);
    FragChain<0, NKS, PF, M, MFMA_32>::run(acc1, a, qf, voff, base1);
    stamp(4);
    if (STAG && late) {
#pragma unroll
      for (int r = 0; r < NR; ++r) accd[r] = acc1[r];
      rowd = row0 + SUB;
    } else {
      topk_update(acc1, row0 + SUB);
    }
    stamp(5);
  }
  if (STAG && late && n_tiles > 0) topk_update(accd, rowd);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail prefetches before exit
  if constexpr (STAMP) {
    const uint64_t cyc = __builtin_amdgcn_s_memtime() - t_start;
    const uint64_t rt = __builtin_amdgcn_s_memrealtime() - rt_start;
    if (lane == 0) {
      float* o = cand_s + ((size_t)blockIdx.x * TOPK_WAVES + wave) * 8;
      const float nt = (float)max(n_tiles, 1);
#pragma unroll
      for (int i = 0; i < 6; ++i) o[i] = (float)seg[i] / nt;
      o[6] = (float)cyc / nt;
      o[7] = rt ? (float)cyc / (float)rt * 0.1f : 0.f;   // GHz (memrealtime ticks at 100 MHz)
    }
    if (query < NQ) {  // keep the top-k (and so the MFMAs) live: folded into cand_i only
      const int list = MFMA_32 ? (lane >> 5) : (lane >> 4);
      const size_t base = (((size_t)query * (gridDim.x / n_qblk) + rb) * LISTS + list) * KMAX;
#pragma unroll
      for (int i = 0; i < KMAX; ++i) cand_i[base + i] = ti[i] ^ __float_as_int(tv[i]);
    }
    return;
  }

  if (query < NQ) {
    const int list = MFMA_32 ? (lane >> 5) : (lane >> 4);
    const int n_rblk = gridDim.x / n_qblk;
    const size_t base = (((size_t)query * n_rblk + rb) * LISTS + list) * KMAX;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      cand_s[base + i] = tv[i];
      cand_i[base + i] = ti[i];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// "Wide" D=384 variant: 4 waves per CU (one per SIMD, 512-entry unified VGPR+AGPR file), each wave
// owns 64 queries (two 32-query B-fragment sets), so every A fragment read from LDS feeds TWO
// 32x32x16 MFMAs -> half the LDS read bytes per FLOP of the 8-wave kernel (the scan is power-
// limited when HBM streaming and MFMA+LDS run together; LDS traffic is the energy we can remove).
template <int KS, int NKS, int PF, int M, int DMA_EVERY, int DMA_PIECES>
struct FragChain2 {
  static constexpr int R = PF + 1;
  template <class Dma>
  __device__ __forceinline__ static void run(f32x16& acc0, f32x16& acc1, bf16x8 (&a)[R],
                                             const bf16x8 (&q0)[NKS], const bf16x8 (&q1)[NKS],
                                             const uint32_t (&voff)[M], uint32_t base,
                                             const Dma& dma) {
    if constexpr (DMA_EVERY > 0 && KS % DMA_EVERY == 0 && KS / DMA_EVERY < DMA_PIECES)
      dma(KS / DMA_EVERY);
    constexpr int outstanding = (NKS - KS < PF) ? (NKS - KS) : PF;
    lgkm_wait<outstanding - 1>(a[KS % R]);
    // hand-issued so the 192 query registers stay resident in AGPRs as the B operand (the builtin
    // form makes the compiler shuttle them AGPR->VGPR around every MFMA); step 0 zero-inits C.
    if constexpr (KS == 0) {
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc0) : "v"(a[0]), "a"(q0[0]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc1) : "v"(a[0]), "a"(q1[0]));
    } else {
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc0) : "v"(a[KS % R]), "a"(q0[KS]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc1) : "v"(a[KS % R]), "a"(q1[KS]));
    }
    if constexpr (KS + 1 == NKS)  // XDL write -> VALU read of the accumulators: cover the latency
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    if constexpr (KS + PF < NKS)
      ds_read16<((KS + PF) / M) * 256>(a[(KS + PF) % R], base + voff[(KS + PF) % M]);
    if constexpr (KS + 1 < NKS)
      FragChain2<KS + 1, NKS, PF, M, DMA_EVERY, DMA_PIECES>::run(acc0, acc1, a, q0, q1, voff, base, dma);
  }
};

template <int KMAX, int NS, int AUX>
__global__ __launch_bounds__(256, 1) void index_scan_wide_kernel(
    const __bf16* __restrict__ X, int n_valid, int rows_per_blk, const __bf16* __restrict__ Q,
    int NQ, int n_qblk, int xcd, const float* __restrict__ thr_init, float* __restrict__ cand_s,
    int* __restrict__ cand_i) {
  constexpr int D = 384, CPR = D / 8, SUB = 32, TR = 64, NW = 4;
  constexpr int TILE_BYTES = TR * D * 2, SUB_BYTES = SUB * D * 2;
  constexpr int LOADS = TILE_BYTES / (1024 * NW);  // 12 DMA pieces per wave per tile
  constexpr int NKS = D / 16, M = 8, PF = 6, R = PF + 1;
  static_assert(NS * TILE_BYTES <= 160 * 1024, "LDS ring exceeds the CU's 160 KiB");
  static_assert(LOADS * 2 <= NKS, "DMA pieces must fit the first chain");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lb = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qb = lb % n_qblk, rb = lb / n_qblk;
  const int row_begin = rb * rows_per_blk;
  const int row_end = min(row_begin + rows_per_blk, n_valid);
  const int n_tiles = row_end > row_begin ? (row_end - row_begin + TR - 1) / TR : 0;

  const int h = lane >> 5;
  const int query0 = qb * 256 + wave * 64 + (lane & 31);
  const int query1 = query0 + 32;
  bf16x8 q0[NKS], q1[NKS];
  {
    const __bf16* p0 = Q + (size_t)min(query0, NQ - 1) * D;
    const __bf16* p1 = Q + (size_t)min(query1, NQ - 1) * D;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      q0[ks] = *reinterpret_cast<const bf16x8*>(p0 + ks * 16 + h * 8);
      q1[ks] = *reinterpret_cast<const bf16x8*>(p1 + ks * 16 + h * 8);
    }
  }
  uint32_t goff[LOADS];
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {
    const int s = (i * NW + wave) * 64 + lane;
    const int row = s / CPR, pc = s % CPR;
    goff[i] = (uint32_t)(row * D + (pc ^ (row & 15)) * 8);
  }
  auto issue_piece = [&](int t, int i) {
    const int tt = min(t, n_tiles - 1);
    const __bf16* base = X + (size_t)(row_begin + tt * TR) * D;
    char* dst = smem + (t % NS) * TILE_BYTES;
    glds16_aux<AUX>(base + goff[i], dst + ((i * NW + wave) * 64) * 16);
  };
  const uint32_t lds_smem = lds_addr(smem);
  uint32_t voff[M];
  {
    const int r = lane & 31;
#pragma unroll
    for (int m = 0; m < M; ++m) voff[m] = (uint32_t)(r * D * 2 + (((2 * m + h) ^ (r & 15)) << 4));
  }
  float tv0[KMAX], tv1[KMAX];
  int ti0[KMAX], ti1[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    tv0[i] = tv1[i] = -INFINITY;
    ti0[i] = ti1[i] = -1;
  }
  float thr0 = thr_init ? thr_init[min(query0, NQ - 1)] : -INFINITY;
  float thr1 = thr_init ? thr_init[min(query1, NQ - 1)] : -INFINITY;
  auto update = [&](f32x16& acc, float (&tv)[KMAX], int (&ti)[KMAX], float& thr, int row0) {
    const int rb4 = row0 + 4 * h;
    if (row0 + SUB > row_end) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (rb4 + (r & 3) + 8 * (r >> 2) >= row_end) acc[r] = -INFINITY;
    }
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
    if (mx > thr) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (acc[r] > thr) {
          topk_insert_par<KMAX>(tv, ti, acc[r], rb4 + (r & 3) + 8 * (r >> 2));
          thr = fmaxf(thr, tv[KMAX - 1]);
        }
      }
    }
  };

  if (n_tiles > 0) {
    for (int p = 0; p < NS - 1; ++p)
#pragma unroll
      for (int i = 0; i < LOADS; ++i) issue_piece(p, i);
  }
  bf16x8 a[R];
  for (int t = 0; t < n_tiles; ++t) {
    wait_vmcnt<LOADS * (NS - 2)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t base0 = lds_smem + (uint32_t)((t % NS) * TILE_BYTES);
    const uint32_t base1 = base0 + SUB_BYTES;
    const int row0 = row_begin + t * TR;
    const int tnext = t + NS - 1;
    auto dma = [&](int i) { issue_piece(tnext, i); };
    f32x16 acc0, acc1;
    frag_prologue<0, PF, M, R>(a, voff, base0);
    FragChain2<0, NKS, PF, M, 2, LOADS>::run(acc0, acc1, a, q0, q1, voff, base0, dma);
    frag_prologue<0, PF, M, R>(a, voff, base1);
    // (reads of the asm MFMA results stay below the chain-end s_nops: index_i8.hip emit)
    asm volatile("" : "+v"(acc0), "+v"(acc1));
    update(acc0, tv0, ti0, thr0, row0);
    update(acc1, tv1, ti1, thr1, row0);
    FragChain2<0, NKS, PF, M, 0, 0>::run(acc0, acc1, a, q0, q1, voff, base1, NoDma());
    asm volatile("" : "+v"(acc0), "+v"(acc1));
    update(acc0, tv0, ti0, thr0, row0 + SUB);
    update(acc1, tv1, ti1, thr1, row0 + SUB);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int n_rblk = gridDim.x / n_qblk;
  if (query0 < NQ) {
    const size_t base = (((size_t)query0 * n_rblk + rb) * 2 + h) * KMAX;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      cand_s[base + i] = tv0[i];
      cand_i[base + i] = ti0[i];
    }
  }
  if (query1 < NQ) {
    const size_t base = (((size_t)query1 * n_rblk + rb) * 2 + h) * KMAX;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      cand_s[base + i] = tv1[i];
      cand_i[base + i] = ti1[i];
    }
  }
}

// Merge the candidate lists of one query (contiguous: [n_rblk][lists][KMAX]) into the final
// top-k.  One workgroup per query: strided local top-KMAX, then an LDS tree of pairwise merges.
template <int KMAX, int NTH>
__global__ __launch_bounds__(NTH) void topk_merge_kernel(const float* __restrict__ cand_s,
                                                         const int* __restrict__ cand_i,
                                                         int n_cand_per_query, int k,
                                                         float* __restrict__ out_s,
                                                         int* __restrict__ out_i,
                                                         int64_t id_offset,
                                                         int64_t* __restrict__ out_id64,
                                                         const int* __restrict__ gate) {
  if (gate != nullptr && *gate == 0) return;   // see index_scan_topk_kernel
  __shared__ float ls[NTH * KMAX];
  __shared__ int li[NTH * KMAX];
  const int q = blockIdx.x, tid = threadIdx.x;
  const float* cs = cand_s + (size_t)q * n_cand_per_query;
  const int* ci = cand_i + (size_t)q * n_cand_per_query;
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    tv[i] = -INFINITY;
    ti[i] = -1;
  }
  for (int c = tid; c < n_cand_per_query; c += NTH) {
    const float s = cs[c];
    if (s > tv[KMAX - 1]) topk_insert<KMAX>(tv, ti, s, ci[c]);
  }
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    ls[tid * KMAX + i] = tv[i];
    li[tid * KMAX + i] = ti[i];
  }
  __syncthreads();
  for (int half = NTH / 2; half >= 1; half >>= 1) {
    if (tid < half) {
      const float* as = ls + tid * KMAX;
      const int* ai = li + tid * KMAX;
      const float* bs = ls + (tid + half) * KMAX;
      const int* bi = li + (tid + half) * KMAX;
      int pa = 0, pb = 0;
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        const bool take_a = as[pa] >= bs[pb];
        tv[i] = take_a ? as[pa] : bs[pb];
        ti[i] = take_a ? ai[pa] : bi[pb];
        pa += take_a ? 1 : 0;
        pb += take_a ? 0 : 1;
        pa = min(pa, KMAX - 1);
        pb = min(pb, KMAX - 1);
      }
    }
    __syncthreads();
    if (tid < half) {
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        ls[tid * KMAX + i] = tv[i];
        li[tid * KMAX + i] = ti[i];
      }
    }
    __syncthreads();
  }
  if (tid < k) {
    const float s = tid < KMAX ? ls[tid] : -INFINITY;
    const int i = tid < KMAX ? li[tid] : -1;
    out_s[(size_t)q * k + tid] = s;
    out_i[(size_t)q * k + tid] = i;
    if (out_id64) out_id64[(size_t)q * k + tid] = i >= 0 ? id_offset + i : -1;
  }
}

}  // namespace symb

using namespace symb;

// Candidate-buffer geometry the host must allocate: [n_rblk][NQ][lists][kmax] floats and ints.
int symb_topk_geometry(int D, int kmax, int* lists, int* queries_per_blk) {
  if (kmax != 16 && kmax != 32) return -1;
  if (D == 384) {
    *lists = 2;
    *queries_per_blk = 256;
  } else if (D == 768 || D == 1024) {
    *lists = 4;
    *queries_per_blk = 128;
  } else {
    return -1;
  }
  return 0;
}

template <int D, bool M32, int KMAX, int NS, int AUX>
static int launch_scan(const void* X, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                       int NQ, int n_qblk, int xcd, const float* thr, float* cs, int* ci,
                       hipStream_t st, const int* gate) {
  auto kern = index_scan_topk_kernel<D, M32, KMAX, NS, AUX>;
  constexpr int lds = NS * (M32 ? 64 : 32) * D * 2;
  set_max_lds<index_scan_topk_kernel<D, M32, KMAX, NS, AUX>>(lds);
  hipLaunchKernelGGL(kern, dim3(n_rblk * n_qblk), dim3(512), lds, st, (const __bf16*)X, n_valid,
                     rows_per_blk, (const __bf16*)Q, NQ, n_qblk, xcd, thr, cs, ci, gate);
  return (int)hipGetLastError();
}

// Profiling-only entry: time the DMA ring alone (abl=1) or the compute alone (abl=2), D=384.
int symb_index_scan_ablate(const void* X, int n_valid, int rows_per_blk, int n_rblk,
                           const void* Q, int NQ, float* cs, int* ci, hipStream_t st, int abl,
                           const float* thr) {
  const int n_qblk = (NQ + 255) / 256;
  auto go = [&](auto kern) {
    constexpr int lds = 3 * 64 * 384 * 2;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3(n_rblk * n_qblk), dim3(512), lds, st, (const __bf16*)X, n_valid,
                       rows_per_blk, (const __bf16*)Q, NQ, n_qblk, 0, thr, cs, ci, nullptr);
    return (int)hipGetLastError();
  };
  if (abl == 3) {
    auto kern = index_scan_wide_kernel<16, 3, 2>;
    constexpr int lds = 3 * 64 * 384 * 2;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3(n_rblk * n_qblk), dim3(256), lds, st, (const __bf16*)X, n_valid,
                       rows_per_blk, (const __bf16*)Q, NQ, n_qblk, 0, thr, cs, ci);
    return (int)hipGetLastError();
  }
  if (abl == 1) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 1>);
  if (abl == 2) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 2>);
  if (abl == 4) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 4>);
  if (abl == 5) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 5>);
  if (abl == 8) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 8>);
  if (abl == 9) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 9>);
  if (abl == 10) return go(index_scan_topk_kernel<384, true, 16, 3, 0, 10>);
  return go(index_scan_topk_kernel<384, true, 16, 3, 0, 0>);
}

// Default ring depth per D: as many 24-32 KiB tiles in flight as the 160 KiB LDS allows.
template <int D> struct ScanCfg;
template <> struct ScanCfg<384> { static constexpr bool M32 = true; static constexpr int NS = 3; };
template <> struct ScanCfg<768> { static constexpr bool M32 = false; static constexpr int NS = 3; };
template <> struct ScanCfg<1024> { static constexpr bool M32 = false; static constexpr int NS = 2; };

template <int D, int NS>
static int dispatch_k(int kmax, int aux, const void* X, int n_valid, int rows_per_blk, int n_rblk,
                      const void* Q, int NQ, int n_qblk, int xcd, const float* thr, float* cs,
                      int* ci, hipStream_t st, const int* gate) {
  constexpr bool M32 = ScanCfg<D>::M32;
#define SYMB_L(K, A) launch_scan<D, M32, K, NS, A>(X, n_valid, rows_per_blk, n_rblk, Q, NQ, n_qblk, xcd, thr, cs, ci, st, gate)
  if (kmax == 16) return aux ? SYMB_L(16, 2) : SYMB_L(16, 0);
  return aux ? SYMB_L(32, 2) : SYMB_L(32, 0);
#undef SYMB_L
}

// X: [>= round_up(n_valid, 32), D] bf16 unit rows; Q: [NQ, D] bf16 unit rows.
// rows_per_blk must be a multiple of 64; n_rblk * rows_per_blk >= n_valid.
// ns = 0 -> default ring depth; aux = -1 -> non-temporal iff each index row is read by one block.
// thr_init: optional [NQ] per-query lower bounds on the final k-th score (nullptr = none).
// xcd: group the query blocks of each row block on one XCD (L2-shared row stream; NQ > 256).
int symb_index_scan(const void* X, int n_valid, int D, int rows_per_blk, int n_rblk,
                    const void* Q, int NQ, int kmax, float* cand_s, int* cand_i, hipStream_t st,
                    int ns, int aux, const float* thr_init, int xcd, const int* gate) {
  if (NQ <= 0 || n_rblk <= 0) return 0;
  if (rows_per_blk % 64) return -1;
  int lists, qpb;
  if (symb_topk_geometry(D, kmax, &lists, &qpb)) return -1;
  const int n_qblk = (NQ + qpb - 1) / qpb;
  if (aux < 0) aux = n_qblk == 1 ? 2 : 0;
#define SYMB_ARGS kmax, aux, X, n_valid, rows_per_blk, n_rblk, Q, NQ, n_qblk, xcd, thr_init, cand_s, cand_i, st, gate
  if (D == 384) {
    if (ns == 0 || ns == 3) return dispatch_k<384, 3>(SYMB_ARGS);
    if (ns == 2) return dispatch_k<384, 2>(SYMB_ARGS);
    return -1;
  }
  if (D == 768) {
    if (ns == 0 || ns == 3) return dispatch_k<768, 3>(SYMB_ARGS);
    return -1;
  }
  if (D == 1024) {
    if (ns == 0 || ns == 2) return dispatch_k<1024, 2>(SYMB_ARGS);
    return -1;
  }
#undef SYMB_ARGS
  return -1;
}

// cand_* laid out [NQ][n_cand_per_query] -- exactly the scan's [NQ][n_rblk][lists][kmax] output.
// Also merges gathered per-rank top-k lists ([NQ][world*k], padded to kmax) in the sharded path.
int symb_topk_merge(const float* cand_s, const int* cand_i, int NQ, int n_cand_per_query,
                    int kmax, int k, float* out_s, int* out_i, int64_t id_offset,
                    int64_t* out_id64, hipStream_t st, const int* gate) {
  if (NQ <= 0) return 0;
  if (k > kmax) return -1;
  if (kmax == 16)
    hipLaunchKernelGGL((topk_merge_kernel<16, 256>), dim3(NQ), dim3(256), 0, st, cand_s, cand_i,
                       n_cand_per_query, k, out_s, out_i, id_offset, out_id64, gate);
  else if (kmax == 32)
    hipLaunchKernelGGL((topk_merge_kernel<32, 128>), dim3(NQ), dim3(128), 0, st, cand_s, cand_i,
                       n_cand_per_query, k, out_s, out_i, id_offset, out_id64, gate);
  else
    return -1;
  return (int)hipGetLastError();
}
