// EXACT bf16 top-k through an int8 image of the index: a bound-pruned candidate scan followed by an
// exact bf16 re-score (SURVEY.md §2.5 X2/X3 for the 384-wide headline shard).
//
// Why: at 256 queries the bf16 emitting scan (index_mq.hip) is bound by the chip's power limit,
// streaming 768 bytes and 2 x 256 x 384 bf16 MFMA FLOP per row (profiles/r2_rsplit/).  An int8
// image of the rows is half the bytes and v_mfma_i32_16x16x64_i8 runs at twice the bf16 rate, so
// the same row stream costs about half.  int8 scores are only approximate, so they are used to
// PRUNE, never to rank:
//
//   x~ = sx * x8 (per-row scale sx = max|x| / 127, x8 = round(x / sx)), q~ = sq * q8 likewise,
//   s = q . x (the bf16 cosine), s~ = q~ . x~ = sq * sx * (q8 . x8) (exact integer dot).
//   |s - s~| = |q . (x - x~) + (q - q~) . x~| <= |q| * E + |q - q~| * X        (Cauchy-Schwarz)
//   with E = max over rows of |x - x~| and X = max over rows of |x~| (tracked at every write) and
//   |q - q~| computed per query.  If T lower-bounds the query's final k-th score (an exact sample,
//   index/shard.py), every row of the true top-k has s >= T, hence s~ >= T - margin.
//
// So this kernel EMITS every row with s~ >= T - margin (a superset of the true top-k), the
// re-score kernel replaces each candidate's score by its exact bf16 dot product, and the select
// kernel (index_mq.hip) takes the top-k of those: the same rows and the same scores (up to fp32
// summation order) as scanning every row in bf16.  A query whose candidate buffer overflows raises
// the device flag on which the exact bf16 list scan re-runs the batch (gated, no host sync).
//
// Scan geometry: the emitting design of index_mq.hip at half the row bytes.  A 64-row tile is
// 24 KiB; a 16-row x 64-byte piece (one k-step of one 16-row sub-tile) is exactly the bf16
// kernel's 1 KiB piece, so the LDS image, the LDS-DMA source offsets, the conflict-free fragment
// offsets and the candidate stages are the same.  8 waves x 64 queries (4 sets x 6 k-steps x 4
// registers = 96 VGPRs of queries as B operands); RSPLIT = 2: waves w and w + 4 hold the same
// queries and split each tile's rows (256 queries per workgroup), RSPLIT = 1: 512.  The tile's
// 64 row scales ride the ring as one extra 4-byte-per-lane LDS-DMA issued by wave 0.
#include "scan_common.h"

namespace symb {

namespace i8s {
constexpr int WAVES = 8;
constexpr int SETS = 4;                     // 16-query sets per wave
constexpr int SUB = 16;
constexpr int PIECE = 1024;
#ifndef SYMB_I8_PF
#define SYMB_I8_PF 5
#endif
}  // namespace i8s

// Row width: D = 384 (the headline shard) or 768 (the reference's collection,
// vector_memory_service/src/main.rs:22).  v_mfma_i32_16x16x64_i8 k-steps: 6 / 12; the queries'
// B fragments take SETS x NKS x 4 = 96 / 192 VGPRs.
// Fragment reads in flight: PF (NKS % (PF + 1) == 0); 3 at D = 768, whose 192 query registers
// leave no room for a 6-slot fragment ring.
// HK > 0: the SPLIT image (see "split image" below): the first 32 * HK dims of each (rotated) row
// as fp16, HK v_mfma_f32_16x16x32_f16 k-steps of 64 bytes, then the other D - 32 * HK dims as
// int8 -- RB = 448 bytes per 384-wide row.  Only the fused two-sub-tile chains run it.
// HK = MX4 (4): the MX-fp4 image (see "MX-fp4 image" below): every 32-dim block of a row as OCP
// e2m1 nibbles with a power-of-two block scale, 3 v_mfma_scale_f32_16x16x128_f8f6f4 k-steps of 64
// bytes -- RB = 192 bytes per 384-wide row, plus 16 bytes of block scales in a side array.
constexpr int MX4 = 4;
template <int D, int HK = 0> struct I8Dim {
  static constexpr int NKS = HK == MX4 ? D / 128 : (D + 32 * HK) / 64;
  static constexpr int RB = NKS * 64;            // image bytes per row
  static constexpr int PF = HK ? NKS - 1 : (D == 384 ? SYMB_I8_PF : 3);
  static constexpr int R = PF + 1;
  static_assert(D == 384 || D == 768, "int8 scan row width");
  static_assert(HK == 0 || (D == 384 && (HK == 2 || HK == MX4)),
                "split image: 64 fp16 + 320 int8 dims; MX-fp4 image: 384 dims");
  static_assert(NKS % R == 0, "cross-chain prefetch: fragment j of the next chain uses slot j % R");
};

// Tile geometry: TR = 64-row tiles in a 5-deep ring (24 KiB tiles, D = 384) or a 3-deep ring
// (48 KiB: D = 768, or 128-row tiles at D = 384) -- ~96-144 KiB in flight.
// WV = 4 (D = 384): 4-wave workgroups (one wave per SIMD), TWO per CU, each with its own 3-deep
// ring: the two waves sharing a SIMD then belong to different workgroups, so one's barrier,
// prologue and DMA burst fall under the other's MFMAs instead of in lockstep with them.
// Split image (HK = 2): 28 KiB tiles = 28 pieces over 8 waves, so waves 0-3 carry 4 pieces and
// waves 4-7 three (FULLW); a 5-deep ring still fits (156 KiB with the stages).
template <int D, int TR_, int WV_ = 8, int HK = 0> struct Geo {
  static constexpr int TR = TR_;
  static constexpr int WV = WV_;
  static constexpr int NKS = I8Dim<D, HK>::NKS;
  static constexpr int RB = I8Dim<D, HK>::RB;
  static constexpr int NSUB = TR / i8s::SUB;
  static constexpr int TILE_BYTES = TR * RB;
  static constexpr int PIECES = TILE_BYTES / 1024;
  static constexpr int LOADS = (PIECES + WV - 1) / WV;        // LDS-DMA pieces per wave per tile
  static constexpr int FULLW = PIECES % WV ? PIECES % WV : WV;   // waves carrying LOADS (rest: - 1)
  static constexpr int DMA_EVERY = NKS / LOADS;               // k-steps between pieces
  static constexpr int SCW = TR / 64;                         // waves carrying a scale DMA
  static constexpr int SC_BYTES = TR * (HK == MX4 ? 16 : 4);   // row scales (MX4: block scales)
  static constexpr int STW = WV == 4 ? 160 : (TR == 64 ? 192 : 128);   // staged candidates per wave
  static constexpr int STAGE_BYTES = STW * 10;
  // (MX4: 12 KiB tiles, an 8-deep ring keeps ~84 KiB in flight like the int8 5-deep ring)
  static constexpr int NS = WV == 4 ? 3
                            : HK == MX4 ? (TILE_BYTES <= 12 * 1024 ? 8 : 5)
                            : (TILE_BYTES <= 24 * 1024 ||
                               (HK && 5 * (TILE_BYTES + SC_BYTES) + WV * STAGE_BYTES <= 160 * 1024))
                                ? 5 : 3;
  static constexpr int LDS_BYTES = NS * TILE_BYTES + NS * SC_BYTES + WV * STAGE_BYTES;
  static_assert(TILE_BYTES % 1024 == 0 && (HK || PIECES % WV == 0), "tile must split over waves");
  static_assert(SCW <= FULLW, "the scale waves carry a full share of pieces");
  static_assert(WV == 8 || 2 * LDS_BYTES <= 160 * 1024, "two 4-wave workgroups must share a CU");
  static_assert(NSUB * NKS * i8s::PIECE == TILE_BYTES, "a tile is NSUB x NKS pieces");
  static_assert(LOADS * DMA_EVERY <= NKS && DMA_EVERY >= 1, "DMA pieces must fit the first chain");
  static_assert(LDS_BYTES <= 160 * 1024, "ring + scales + stages exceed the CU's 160 KiB");
};

typedef __attribute__((ext_vector_type(4))) int i32x4;

template <int OFF>
__device__ __forceinline__ void i8_read16(i32x4& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void i8_lgkm(i32x4& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "i"(N));
}
template <bool FIRST>
__device__ __forceinline__ void i8_mfma(i32x4& acc, const i32x4& a, const i32x4& q) {
  if constexpr (FIRST)
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(q));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(q));
}
// the split image's fp16 k-steps: the same 16-byte-per-lane operand layout (row / query lane & 15,
// k-bytes 16 * (lane >> 4)), so fragments come from the same LDS offsets as the int8 ones
template <bool FIRST>
__device__ __forceinline__ void h16_mfma(f32x4& acc, const i32x4& a, const i32x4& q) {
  if constexpr (FIRST)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(q));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(q));
}

// the MX-fp4 image's k-steps: 16x16x128 with e2m1 A and B (cbsz / blgp 4: 16 bytes per lane, the
// int8 layout), each lane's 32 elements one scale block; the e8m0 block scales of k-step KS are
// byte KS of the lane's row-scale (rs) and query-scale (qs) dwords (op_sel / op_sel_hi pick it)
template <int KS, bool FIRST>
__device__ __forceinline__ void mx4_mfma(f32x4& acc, const i32x4& a, const i32x4& q, float rs,
                                         float qs) {
  if constexpr (FIRST) {
    static_assert(KS == 0, "the first k-step zero-initialises");
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, 0, %3, %4 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "=&v"(acc) : "v"(a), "v"(q), "v"(rs), "v"(qs));
  } else if constexpr (KS == 0) {
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "+v"(acc) : "v"(a), "v"(q), "v"(rs), "v"(qs));
  } else if constexpr (KS == 1) {
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,1,0] op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "+v"(acc) : "v"(a), "v"(q), "v"(rs), "v"(qs));
  } else {
    static_assert(KS == 2, "three k-steps per 384-wide row");
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[1,1,0] cbsz:4 blgp:4"
                 : "+v"(acc) : "v"(a), "v"(q), "v"(rs), "v"(qs));
  }
}

// k-step KS of one 16-row sub-tile (index_mq.hip MqChain, int8 operands).
template <int D, int KS, int DMA_PIECES, bool NEXT, int DE>
struct I8Chain {
  static constexpr int NKS = I8Dim<D>::NKS, PF = I8Dim<D>::PF, R = I8Dim<D>::R;
  template <class Dma>
  __device__ __forceinline__ static void run(i32x4 (&acc)[i8s::SETS], i32x4 (&a)[R],
                                             const i32x4 (&qf)[i8s::SETS][NKS],
                                             uint32_t base, uint32_t next, const Dma& dma) {
    using namespace i8s;
    static_assert(DMA_PIECES * DE <= NKS, "every DMA piece must be issued in the chain");
    if constexpr (DMA_PIECES > 0 && KS % DE == 0 && KS / DE < DMA_PIECES) dma(KS / DE);
    constexpr int outstanding = (NEXT || NKS - KS >= PF) ? PF : (NKS - KS);
    i8_lgkm<outstanding - 1>(a[KS % R]);
#pragma unroll
    for (int s = 0; s < SETS; ++s) i8_mfma<KS == 0>(acc[s], a[KS % R], qf[s][KS]);
    if constexpr (KS + 1 == NKS) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    if constexpr (KS + PF < NKS)
      i8_read16<(KS + PF) * PIECE>(a[(KS + PF) % R], base);
    else if constexpr (NEXT)
      i8_read16<(KS + PF - NKS) * PIECE>(a[(KS + PF) % R], next);
    if constexpr (KS + 1 < NKS) I8Chain<D, KS + 1, DMA_PIECES, NEXT, DE>::run(acc, a, qf, base, next, dma);
  }
};

// Fused chain of TWO 16-row sub-tiles (the row-split wave's whole share of a tile): per k-step
// one fragment per sub-tile and 2 x SETS MFMAs, so a tile is one 48-MFMA chain and one emission
// block per wave instead of two 24-MFMA chains (half the chain-end pads, waits and tests).
namespace i8s {
constexpr int PF2 = 2;                      // k-steps of fragment reads in flight (2 reads each)
constexpr int R2 = PF2 + 1;
}  // namespace i8s
template <int N>
__device__ __forceinline__ void i8_lgkm2(i32x4& v0, i32x4& v1) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(v0), "+v"(v1) : "i"(N));
}
template <int N>
__device__ __forceinline__ void i8_lgkm2t(i32x4& v0, i32x4& v1, f32x4& t0, f32x4& t1) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(v0), "+v"(v1), "+v"(t0), "+v"(t1) : "i"(N));
}
// (MX4: the two sub-tiles' block-scale dwords are single registers, read by ds_read_b32 straight
// into the registers the MFMAs use -- a copy into a vector before this wait would read them
// before they arrive)
template <int N>
__device__ __forceinline__ void i8_lgkm2s(i32x4& v0, i32x4& v1, float& t0, float& t1) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(v0), "+v"(v1), "+v"(t0), "+v"(t1) : "i"(N));
}
// t0 / t1: the two sub-tiles' row scales, read from LDS just before the prologue; the first
// k-step's wait covers them (older than every fragment read), so the emission after the chain
// finds them in registers
template <int D, int KS, int DMA_PIECES, int DE, int HK = 0>
struct I8Chain2 {
  static constexpr int NKS = I8Dim<D, HK>::NKS;
  template <class Dma>
  __device__ __forceinline__ static void run(i32x4 (&acc)[2][i8s::SETS],
                                             f32x4 (&accf)[HK ? 2 : 1][i8s::SETS],
                                             i32x4 (&a)[i8s::R2][2],
                                             const i32x4 (&qf)[i8s::SETS][NKS],
                                             uint32_t base, const Dma& dma, f32x4& t0, f32x4& t1,
                                             const float (&qsc)[i8s::SETS], float& r0, float& r1) {
    using namespace i8s;
    if constexpr (DMA_PIECES > 0 && KS % DE == 0 && KS / DE < DMA_PIECES) dma(KS / DE);
    constexpr int steps = (NKS - KS < PF2) ? (NKS - KS) : PF2;   // k-steps in flight, this one too
    if constexpr (KS == 0 && HK == MX4)
      i8_lgkm2s<2 * (steps - 1)>(a[KS % R2][0], a[KS % R2][1], r0, r1);
    else if constexpr (KS == 0)
      i8_lgkm2t<2 * (steps - 1)>(a[KS % R2][0], a[KS % R2][1], t0, t1);
    else
      i8_lgkm2<2 * (steps - 1)>(a[KS % R2][0], a[KS % R2][1]);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int s = 0; s < SETS; ++s) {
        if constexpr (HK == MX4)   // (r0 / r1: the two sub-tiles' row block-scale dwords)
          mx4_mfma<KS, KS == 0>(accf[c][s], a[KS % R2][c], qf[s][KS], c ? r1 : r0, qsc[s]);
        else if constexpr (KS < HK)
          h16_mfma<KS == 0>(accf[c][s], a[KS % R2][c], qf[s][KS]);
        else
          i8_mfma<KS == HK>(acc[c][s], a[KS % R2][c], qf[s][KS]);
      }
    if constexpr (KS + 1 == NKS) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    if constexpr (KS + PF2 < NKS) {
      i8_read16<(KS + PF2) * PIECE>(a[(KS + PF2) % R2][0], base);
      i8_read16<(KS + PF2) * PIECE + NKS * PIECE>(a[(KS + PF2) % R2][1], base);
    }
    if constexpr (KS + 1 < NKS)
      I8Chain2<D, KS + 1, DMA_PIECES, DE, HK>::run(acc, accf, a, qf, base, dma, t0, t1, qsc, r0,
                                                   r1);
  }
};
template <int D, int J, int HK = 0>
__device__ __forceinline__ void i8_prologue2(i32x4 (&a)[i8s::R2][2], uint32_t base) {
  i8_read16<J * i8s::PIECE>(a[J % i8s::R2][0], base);
  i8_read16<J * i8s::PIECE + I8Dim<D, HK>::NKS * i8s::PIECE>(a[J % i8s::R2][1], base);
  if constexpr (J + 1 < i8s::PF2) i8_prologue2<D, J + 1, HK>(a, base);
}

template <int D, int J>
__device__ __forceinline__ void i8_prologue(i32x4 (&a)[I8Dim<D>::R], uint32_t base) {
  i8_read16<J * i8s::PIECE>(a[J % I8Dim<D>::R], base);
  if constexpr (J + 1 < I8Dim<D>::PF) i8_prologue<D, J + 1>(a, base);
}

__device__ __forceinline__ const char* i8_uniform(const char* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const char*>(((uint64_t)hi << 32) | lo);
}

// X8: [>= round_up(n_valid, 64), 384] int8 rows; sx: their scales (f32, same padding);
// Q8: [NQ, 384] int8 queries; thr[NQ]: emit a row iff (q8 . x8) * sx >= thr (already divided by
// the query's scale).  cand_s/cand_i: [NQ][cap]; cand_n[NQ] zeroed by the host entry.
// ABL (profiling entry symb_index_scan_i8_ablate only): 1 = no LDS-DMA, 2 = no emission test,
// 3 = full + s_memtime / s_memrealtime around the tile loop into cand_s[2 * blockIdx.x + {0, 1}],
// 4 = LDS-DMA ring only.
//
// HK = 2 (the split image, index/shard.py calibrate_prune): rows and queries are rotated by the
// shard's orthogonal PCA basis, the 64 leading components are kept as fp16 (an fp32 MFMA dot, ~11
// bits each) and only the 320 trailing ones quantised to int8 with their own per-row scale.
// Emit iff acc_f / sq + acc_i * sx >= thr (sq_in: the queries' int8 scales); the bound (prune_
// qquant_h) is the int8 one on the trailing dims plus the fp16 rounding of the leading ones.
// (Round 4's pair pre-test over both sub-tiles of a fused chain measured parity-to-slower,
// profiles/r4_split/pair/, and was removed in round 5: the per-sub-tile pre-tests alone.)
//
// HK = MX4 (the MX-fp4 image, index/shard.py, the first tier of a batch whose k-th scores sit far
// above the corpus bulk): X8 = [rows][192] e2m1 nibbles, sx = [rows][16] bytes of e8m0 block
// scales (dword g = the scales of blocks g, 4 + g, 8 + g), Q8 / sq_in likewise for the queries.
// The MFMA applies the scales, so acc_f is the approximate score itself: emit iff acc_f >= thr
// (thr = T - margin in score units, the bound of quant_rows_mx4).
// gate (optional): the kernel runs only if *gate == gate_want (the device-side tier choice).
template <int D, int RSPLIT, int ABL = 0, int TRK = 64, int WV = 8, int HK = 0>
__global__ __launch_bounds__(64 * WV, 8 / WV) void index_scan_i8_kernel(
    const int8_t* __restrict__ X8, const float* __restrict__ sx, int n_valid, int rows_per_blk,
    const int8_t* __restrict__ Q8, int NQ, int n_qblk, int xcd, const float* __restrict__ thr_in,
    float* __restrict__ cand_s, int* __restrict__ cand_i, int* __restrict__ cand_n, int cap,
    const int* __restrict__ skip, const float* __restrict__ sq_in, const int* __restrict__ gate,
    int gate_want) {
  using namespace i8s;
  using G = Geo<D, TRK, WV, HK>;
  constexpr int NKS = G::NKS, RB = G::RB;
  constexpr int TR = G::TR, NSUB = G::NSUB, NS = G::NS, TILE_BYTES = G::TILE_BYTES;
  constexpr int LOADS = G::LOADS, SC_BYTES = G::SC_BYTES, STW = G::STW;
  constexpr int STAGE_BYTES = G::STAGE_BYTES;
  constexpr int QW = SETS * 16, QWAVES = WV / RSPLIT, QPB = QWAVES * QW;
  constexpr int NSW = NSUB / RSPLIT;
  static_assert(RSPLIT == 1 || RSPLIT == 2, "row split");
  static_assert(TRK == 64 || NSW % 2 == 0, "128-row tiles run the fused two-sub-tile chains");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lb = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qb = lb % n_qblk, rb = lb / n_qblk;
  // skip (optional, one flag per row block): the sampled route (prune_route_kernel) sent this
  // block to the bf16 emitting scan -- the workgroup returns at once (workgroup-uniform, before
  // any barrier)
  if (skip != nullptr && skip[rb] != 0) return;
  if (gate != nullptr && *gate != gate_want) return;
  const int row_begin = rb * rows_per_blk;
  const int row_end = min(row_begin + rows_per_blk, n_valid);
  const int n_tiles = row_end > row_begin ? (row_end - row_begin + TR - 1) / TR : 0;

  // ---- query fragments (B operand: lane holds query lane&15, k-bytes 16*(lane>>4) .. +16) ----
  const int qwave = wave % QWAVES;
  const int j0 = (wave / QWAVES) * NSW;
  const int qbase = qb * QPB + qwave * QW + (lane & 15);
  i32x4 qf[SETS][NKS];
  float thr[SETS];
  float rsq[SETS];   // split image: 1 / the query's int8 scale (acc_f is in score units);
                     // MX4: the lane's query block-scale dword (its bits, as a float register)
#pragma unroll
  for (int s = 0; s < SETS; ++s) {
    const int q = qbase + s * 16;
    const int8_t* qp = Q8 + (size_t)min(q, NQ - 1) * RB + (lane >> 4) * 16;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[s][ks] = *reinterpret_cast<const i32x4*>(qp + ks * 64);
    thr[s] = q < NQ ? thr_in[q] : INFINITY;
    if constexpr (HK == MX4)
      rsq[s] = sq_in[(size_t)min(q, NQ - 1) * 4 + (lane >> 4)];
    else if constexpr (HK > 0)
      rsq[s] = 1.f / sq_in[min(q, NQ - 1)];
  }
#pragma unroll
  for (int s = 0; s < SETS; ++s) {
    asm volatile("" ::"v"(thr[s]));
    if constexpr (HK > 0) asm volatile("" ::"v"(rsq[s]));
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[s][ks]));
  }

  // ---- LDS-DMA (index_mq.hip layout): lane l fetches row l>>2 of a piece, chunk (l&3)^f ------
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t loff = (uint32_t)((lane >> 2) * RB + (((lane & 3) ^ ((lane >> 3) & 2)) * 16));
  char* scl = smem + NS * TILE_BYTES;   // NS x 64 row scales
  auto issue_tile = [&](int t, int i) {  // piece i of tile t (+ the scales: wave 0, piece 0)
    const int tt = min(t, n_tiles - 1);   // past the end: re-load the last tile (vmcnt stays exact)
    const int p = i * WV + wave_u, j = p / NKS, ks = p % NKS;
    const int prow = row_begin + tt * TR;
    const char* base = reinterpret_cast<const char*>(X8 + (size_t)(prow + j * SUB) * RB + ks * 64);
    // (split image: the last round of pieces covers waves < FULLW only; wave-uniform)
    if (G::FULLW == WV || p < G::PIECES)
      glds16_aux<0>(i8_uniform(base) + loff, smem + (t % NS) * TILE_BYTES + p * PIECE);
    if constexpr (HK == MX4) {   // 64 rows x 16 bytes of block scales per scale wave
      if (wave_u < G::SCW && i == 0)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(sx + (size_t)(prow + 64 * wave_u + lane) * 4),
            (__attribute__((address_space(3))) void*)(scl + (t % NS) * SC_BYTES + 1024 * wave_u),
            16, 0, 0);
    } else if (wave_u < G::SCW && i == 0) {   // 64 row scales per scale wave
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(sx + prow + 64 * wave_u + lane),
          (__attribute__((address_space(3))) void*)(scl + (t % NS) * SC_BYTES + 256 * wave_u), 4,
          0, 0);
    }
  };
  const uint32_t lds_smem = lds_addr(smem);
  const uint32_t foff = (uint32_t)((lane & 15) * 64 + (((lane >> 4) ^ ((lane >> 1) & 2)) * 16));

  // ---- candidate emission (index_mq.hip: per-wave LDS stage, ballot slots, rare flushes) ------
  char* stage = smem + NS * TILE_BYTES + NS * SC_BYTES + wave_u * STAGE_BYTES;
  float* st_s = reinterpret_cast<float*>(stage);
  int* st_r = reinterpret_cast<int*>(stage + STW * 4);
  uint16_t* st_q = reinterpret_cast<uint16_t*>(stage + STW * 8);
  int nst = 0;
  auto flush = [&]() {
    int qw = qb * QPB + (wave_u % QWAVES) * QW;
    asm volatile("" : "+v"(qw));
    for (int e = lane; e < nst; e += 64) {
      const int q = qw + st_q[e];
      const int slot = atomicAdd(cand_n + q, 1);
      if (slot < cap) {
        cand_s[(size_t)q * cap + slot] = st_s[e];
        cand_i[(size_t)q * cap + slot] = st_r[e];
      }
    }
    nst = 0;
  };
  // this lane's 4 row scales of sub-tile jj in ring slot `slot`
  auto scales = [&](int slot, int jj) {
    return *reinterpret_cast<const f32x4*>(scl + slot * SC_BYTES + (jj * SUB + 4 * (lane >> 4)) * 4);
  };
  // ---- emission.  The chains' MFMAs are inline asm, invisible to the compiler's MFMA -> VALU
  // hazard recognizer: their results are only safe to read after the chain-end s_nops.  An empty
  // volatile asm "rewriting" the accumulators keeps every read below it (volatile asm stays in
  // program order); without it a plain C++ read was scheduled above the s_nops and saw a stale
  // first accumulator register (the split image's 512-query form lost rows 0 mod 4 of sub-tile 0,
  // set 0: benchmarks/diag/split_emit.py).
  auto fence_acc = [&](i32x4 (&acc)[SETS], auto& af) {
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
      if constexpr (HK != MX4) asm volatile("" : "+v"(acc[s]));   // (MX4: no int accumulators)
      if constexpr (HK > 0) asm volatile("" : "+v"(af[s]));
    }
  };
  // the exact per-row test of one 16-row sub-tile at row0 (this lane's row scales s4; af: the
  // split image's fp16-part accumulators, unused without it) for the sets the pre-test kept
  auto exact = [&](i32x4 (&acc)[SETS], auto& af, int row0, const f32x4 s4, const bool (&hs)[SETS]) {
    // (per-lane values from an opaque copy made here, so nothing derived from them can be
    // hoisted out of the tile loop into the full register budget)
    int lo = lane;
    asm volatile("" : "+v"(lo));
    const int rl = row0 + 4 * (lo >> 4), lq = lo & 15;
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
      if (!__builtin_amdgcn_ballot_w64(hs[s])) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (HK == MX4)
          v[r] = rl + r < row_end ? af[s][r] : -INFINITY;
        else if constexpr (HK > 0)
          v[r] = rl + r < row_end ? fmaf((float)acc[s][r], s4[r], af[s][r] * rsq[s]) : -INFINITY;
        else
          v[r] = rl + r < row_end ? (float)acc[s][r] * s4[r] : -INFINITY;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool p = v[r] >= thr[s];
        const uint64_t m = __builtin_amdgcn_ballot_w64(p);
        if (m) {
          if (nst > STW - 64) flush();
          const int idx = nst + (int)__builtin_amdgcn_mbcnt_hi(
                                    (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
          if (p) {
            st_s[idx] = v[r];
            st_r[idx] = rl + r;
            st_q[idx] = (uint16_t)(s * 16 + lq);
          }
          nst += __builtin_popcountll(m);
        }
      }
    }
  };
  // one 16-row sub-tile (the single-sub-tile chains; plain image only).  Hot path, a conservative
  // integer pre-test per set: max_r(acc_r * sx_r) <= max_r acc_r * (max_r sx_r) for a
  // non-negative max, so a set whose bound misses its threshold has no hit; only the rest take
  // the exact per-row test
  //   max_r acc_r * sx_r >= thr  implies  max_r acc_r >= ceil(thr / max_r sx_r)  (thr > 0),
  // so with one reciprocal per sub-tile each set's test is two v_max3_i32 and an integer
  // compare; a set with thr <= 0 always takes the exact test
  auto emit = [&](i32x4 (&acc)[SETS], int row0, const f32x4 s4) {
    fence_acc(acc, acc);
    if constexpr (ABL == 2 || ABL == 4) {
#pragma unroll
      for (int s = 0; s < SETS; ++s) asm volatile("" ::"v"(acc[s]), "v"(s4));
      return;
    }
    const float rs = __builtin_amdgcn_rcpf(fmaxf(fmaxf(s4[0], s4[1]), fmaxf(s4[2], s4[3])));
    bool hs[SETS];
    bool hit = false;
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
      int im;
      asm volatile("v_max3_i32 %0, %1, %2, %3\n\tv_max3_i32 %0, %0, %4, %4"
                   : "=&v"(im) : "v"(acc[s][0]), "v"(acc[s][1]), "v"(acc[s][2]), "v"(acc[s][3]));
      // (x 0.999: v_rcp_f32 is approximate, so the integer threshold is rounded down, loosely)
      const int it = thr[s] > 0.f ? (int)fminf(thr[s] * rs * 0.999f, 2.0e9f) : INT_MIN;
      hs[s] = im >= it;
      hit |= hs[s];
    }
    if (__builtin_amdgcn_ballot_w64(hit)) exact(acc, acc, row0, s4, hs);
  };
  // the fused chain's TWO sub-tiles (rows row0 .. row0 + 31, this lane's scales sa / sb) under
  // ONE pre-test per set over all 8 of the lane's rows: max_r of the 8 estimates is bounded by
  //   plain: max_r acc_r * max_r sx_r (thr > 0: a negative integer max cannot reach it; a set
  //          with thr <= 0 always takes the exact test)
  //   split: max_r acc_f,r / sq + max_r acc_i,r * (max_r sx_r, or min_r sx_r for a negative
  //          integer max)
  // -- half the pre-test instructions of two per-sub-tile tests (4 v_max3 per set for 8 values
  // against 2 x 2, one convert / multiply / compare instead of two), the exact test as before
  auto emit2 = [&](i32x4 (&acc)[2][SETS], auto& af, int row0, const f32x4 sa, const f32x4 sb) {
    fence_acc(acc[0], af[0]);
    fence_acc(acc[1], af[HK ? 1 : 0]);
    if constexpr (ABL == 2 || ABL == 4) {
#pragma unroll
      for (int s = 0; s < SETS; ++s) asm volatile("" ::"v"(acc[0][s]), "v"(acc[1][s]), "v"(sa), "v"(sb));
      return;
    }
    bool hs[SETS];
#pragma unroll
    for (int s = 0; s < SETS; ++s) hs[s] = true;
    // a pair that reaches a threshold: the per-sub-tile pre-test (as `emit`) before the exact
    // test, so a busy band (held-out queries over random rows: thousands of candidates per query)
    // costs what it did with per-sub-tile tests, while the common miss costs half
    auto sub = [&](i32x4 (&ac)[SETS], auto& afc, int r0, const f32x4 s4) {
      const float sm = fmaxf(fmaxf(s4[0], s4[1]), fmaxf(s4[2], s4[3]));
      float sn = 0.f;
      if constexpr (HK > 0) sn = fminf(fminf(s4[0], s4[1]), fminf(s4[2], s4[3]));
      bool hc[SETS];
      bool any = false;
#pragma unroll
      for (int s = 0; s < SETS; ++s) {
        if constexpr (HK == MX4) {   // the accumulator is the estimate: its max against thr
          float fm;
          asm volatile("v_max3_f32 %0, %1, %2, %3\n\tv_max3_f32 %0, %0, %4, %4"
                       : "=&v"(fm) : "v"(afc[s][0]), "v"(afc[s][1]), "v"(afc[s][2]), "v"(afc[s][3]));
          hc[s] = hs[s] && fm >= thr[s];
          any |= hc[s];
          continue;
        }
        int im;
        asm volatile("v_max3_i32 %0, %1, %2, %3\n\tv_max3_i32 %0, %0, %4, %4"
                     : "=&v"(im) : "v"(ac[s][0]), "v"(ac[s][1]), "v"(ac[s][2]), "v"(ac[s][3]));
        if constexpr (HK > 0) {
          float fm;
          asm volatile("v_max3_f32 %0, %1, %2, %3\n\tv_max3_f32 %0, %0, %4, %4"
                       : "=&v"(fm) : "v"(afc[s][0]), "v"(afc[s][1]), "v"(afc[s][2]), "v"(afc[s][3]));
          const float ub = fmaf((float)im, im >= 0 ? sm : sn, fm * rsq[s]);
          hc[s] = hs[s] && ub + fabsf(ub) * 1e-4f + 1e-6f >= thr[s];
        } else {
          hc[s] = hs[s] && (thr[s] <= 0.f || (float)im * sm >= thr[s]);
        }
        any |= hc[s];
      }
      if (__builtin_amdgcn_ballot_w64(any)) exact(ac, afc, r0, s4, hc);
    };
    sub(acc[0], af[0], row0, sa);
    sub(acc[1], af[HK ? 1 : 0], row0 + SUB, sb);
  };

  // the scale waves carry one extra vector-memory op per tile
  constexpr int W0X = 1;
  if (n_tiles > 0 && ABL != 1) {
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
#pragma unroll
      for (int i = 0; i < LOADS; ++i) issue_tile(p, i);
  }
  uint64_t c0 = 0, r0t = 0;
  if constexpr (ABL == 3) {
    c0 = __builtin_amdgcn_s_memtime();
    r0t = __builtin_amdgcn_s_memrealtime();
  }
  i32x4 a[I8Dim<D>::R];
  i32x4 acc[SETS];
  // fused two-sub-tile chains: the row-split forms (each wave owns 2 or 4 sub-tiles of a tile)
  // (the 512-query form keeps single-sub-tile chains: its two fused groups per tile have no
  // cross-chain prefetch and measured slower, 10.55 -> 11.15 ms at 12.5M x 2048)
  // (D = 768: single-sub-tile chains -- the fused pair's extra fragment and accumulator
  // registers do not fit beside 192 query registers)
  // (the split image always runs fused chains)
  constexpr bool FUSE = D == 384 && NSW % 2 == 0 && (RSPLIT == 2 || TRK == 128 || HK > 0);
  static_assert(HK == 0 || FUSE, "split image: fused chains only");
  constexpr int NG = FUSE ? NSW / 2 : 1;   // fused chains per wave per tile
  i32x4 a2[FUSE ? R2 : 1][2];
  i32x4 acc2[FUSE ? 2 : 1][SETS];
  f32x4 accf2[HK ? 2 : 1][SETS];
  f32x4 s4_prev = {0.f, 0.f, 0.f, 0.f};
  // partner waves (w, w + 4) of an 8-wave workgroup stay half a test apart
  const bool late = WV == 8 && wave_u >= WAVES / 2;
  // the late wave tests its last sub-tile after the NEXT barrier, when wave 0 may already be
  // refilling that tile's scale slot: its scales are read into registers before the barrier
  f32x4 s4_last = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < n_tiles; ++t) {
    if constexpr (ABL != 1) {
      if (wave_u < G::SCW)
        wait_vmcnt<(LOADS + W0X) * (NS - 2)>();
      else if (G::FULLW == WV || wave_u < G::FULLW)
        wait_vmcnt<LOADS * (NS - 2)>();
      else   // (split image: the waves carrying one piece fewer per tile)
        wait_vmcnt<(LOADS - 1) * (NS - 2)>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int slot = t % NS;
    const uint32_t tbase = lds_smem + (uint32_t)(slot * TILE_BYTES);
    const int row0 = row_begin + t * TR;
    const int tnext = t + NS - 1;
    auto dma = [&](int i) {
      if constexpr (ABL != 1) issue_tile(tnext, i);
    };
    const uint32_t fw = tbase + foff + j0 * NKS * PIECE;
    const int last = (j0 + NSW - 1) * SUB;
    if constexpr (ABL == 4) {
#pragma unroll
      for (int i = 0; i < LOADS; ++i) dma(i);
      continue;
    }
    if constexpr (FUSE) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const uint32_t fg = fw + g * 2 * NKS * PIECE;
        const int jg = j0 + 2 * g;
        f32x4 sa, sb;   // this lane's row scales of sub-tiles jg, jg + 1
        float ra = 0.f, rb = 0.f;   // (MX4) the block-scale dwords of the lane's A row (lane & 15)
                                    // and k-group (lane >> 4), both sub-tiles
        if constexpr (HK == MX4) {
          sa = sb = f32x4{0.f, 0.f, 0.f, 0.f};
          const uint32_t sp = lds_addr(scl) +
                              (uint32_t)(slot * SC_BYTES + (jg * SUB + (lane & 15)) * 16 + 4 * (lane >> 4));
          asm volatile("ds_read_b32 %0, %1" : "=v"(ra) : "v"(sp));
          asm volatile("ds_read_b32 %0, %1 offset:256" : "=v"(rb) : "v"(sp));
        } else {
          const uint32_t sp = lds_addr(scl) + (uint32_t)(slot * SC_BYTES + (jg * SUB + 4 * (lane >> 4)) * 4);
          asm volatile("ds_read_b128 %0, %1" : "=v"(sa) : "v"(sp));
          asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(sb) : "v"(sp));
        }
        i8_prologue2<D, 0, HK>(a2, fg);
        // a late wave tests the previous tile's last two sub-tiles here, under its partner's
        // MFMAs
        if (g == 0 && late && t > 0) {
          emit2(acc2, accf2, row0 - TR + last - SUB, s4_prev, s4_last);
        }
        if (g == 0)
          I8Chain2<D, 0, LOADS, G::DMA_EVERY, HK>::run(acc2, accf2, a2, qf, fg, dma, sa, sb, rsq, ra,
                                                      rb);
        else
          I8Chain2<D, 0, 0, G::DMA_EVERY, HK>::run(acc2, accf2, a2, qf, fg, NoDma(), sa, sb, rsq, ra,
                                                  rb);
        if (g + 1 < NG || !late) {
          emit2(acc2, accf2, row0 + jg * SUB, sa, sb);
        } else {
          s4_prev = sa;
          s4_last = sb;
        }
      }
      continue;
    } else {
    i8_prologue<D, 0>(a, fw);
    if (late && t > 0) emit(acc, row0 - TR + last, s4_last);
    if constexpr (NSW > 1)
      I8Chain<D, 0, LOADS, true, G::DMA_EVERY>::run(acc, a, qf, fw, fw + NKS * PIECE, dma);
    else
      I8Chain<D, 0, LOADS, false, G::DMA_EVERY>::run(acc, a, qf, fw, 0, dma);
#pragma unroll
    for (int j = 1; j < NSW; ++j) {
      emit(acc, row0 + (j0 + j - 1) * SUB, scales(slot, j0 + j - 1));
      if (j + 1 < NSW)
        I8Chain<D, 0, 0, true, G::DMA_EVERY>::run(acc, a, qf, fw + j * NKS * PIECE,
                                                 fw + (j + 1) * NKS * PIECE, NoDma());
      else
        I8Chain<D, 0, 0, false, G::DMA_EVERY>::run(acc, a, qf, fw + j * NKS * PIECE, 0, NoDma());
    }
    if (!late)
      emit(acc, row0 + last, scales(slot, j0 + NSW - 1));
    else
      s4_last = scales(slot, j0 + NSW - 1);
    }
  }
  if (late && n_tiles > 0) {
    if constexpr (FUSE) {
      emit2(acc2, accf2, row_begin + (n_tiles - 1) * TR + (j0 + NSW - 2) * SUB, s4_prev, s4_last);
    } else {
      emit(acc, row_begin + (n_tiles - 1) * TR + (j0 + NSW - 1) * SUB, s4_last);
    }
  }
  if (nst) flush();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (ABL == 3) {
    const uint64_t cyc = __builtin_amdgcn_s_memtime() - c0;
    const uint64_t rt = __builtin_amdgcn_s_memrealtime() - r0t;
    if (tid == 0) {
      cand_s[2 * blockIdx.x] = (float)cyc;
      cand_s[2 * blockIdx.x + 1] = (float)rt;
    }
  }
}

// Exact re-score of every candidate: cand_s[q][c] = <Q[q], X[cand_i[q][c]]> over the bf16 rows
// (fp32 accumulation).  SPLIT workgroups per query (blockIdx.y), one wave per candidate with U
// 768-byte row gathers in flight per wave, 6 elements per lane.
template <int D>
__global__ __launch_bounds__(256) void rescore_bf16_kernel(
    const __bf16* __restrict__ X, const __bf16* __restrict__ Q, const int* __restrict__ cand_i,
    const int* __restrict__ cand_n, int cap, float* __restrict__ cand_s) {
  constexpr int PER = D / 64;
  const int q = blockIdx.x, lane = threadIdx.x & 63;
  const int wave = blockIdx.y * 4 + (threadIdx.x >> 6), nwaves = gridDim.y * 4;
  const int n = min(cand_n[q], cap);
  float qv[PER];
  {
    const uint32_t* qp = reinterpret_cast<const uint32_t*>(Q + (size_t)q * D + PER * lane);
#pragma unroll
    for (int i = 0; i < PER / 2; ++i) {
      const uint32_t w = qp[i];
      qv[2 * i] = __uint_as_float(w << 16);
      qv[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
    }
  }
  const int* ci = cand_i + (size_t)q * cap;
  float* cs = cand_s + (size_t)q * cap;
  constexpr int U = 8;   // candidates in flight per wave
  for (int c0 = wave * U; c0 < n; c0 += nwaves * U) {
    uint32_t w[U][PER / 2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(c0 + u, n - 1);
      const uint32_t* xp = reinterpret_cast<const uint32_t*>(X + (size_t)ci[c] * D + PER * lane);
#pragma unroll
      for (int i = 0; i < PER / 2; ++i) w[u][i] = xp[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < PER / 2; ++i) {
        d = fmaf(qv[2 * i], __uint_as_float(w[u][i] << 16), d);
        d = fmaf(qv[2 * i + 1], __uint_as_float(w[u][i] & 0xffff0000u), d);
      }
      d = wave_sum(d);
      if (lane == 0 && c0 + u < n) cs[c0 + u] = d;
    }
  }
}

// Per-row int8 quantiser of D-wide bf16 rows (D = 384 / 768 / 1024): sx = max|x| / 127, x8 = round(x / sx), and the
// per-row |x - sx * x8| (err) and |sx * x8| (xtn) the pruning bound needs.  One wave per row.
// err / xtn (optional) receive the per-row norms; bounds (optional, 2 floats) is raised to
// (max err, max xtn) by one atomic max per workgroup (non-negative floats order as their bits).
template <int D>
__global__ __launch_bounds__(256) void quant_rows_i8_kernel(const __bf16* __restrict__ X, int n,
                                                            int8_t* __restrict__ X8,
                                                            float* __restrict__ sx,
                                                            float* __restrict__ err,
                                                            float* __restrict__ xtn,
                                                            float* __restrict__ bounds) {
  __shared__ float red[2][4];
  constexpr int PER = D / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  if (row >= n) {   // (block-uniform barrier below: idle waves report zeros)
    if (bounds) {
      if (lane == 0) red[0][w] = red[1][w] = 0.f;
      __syncthreads();
    }
    return;
  }
  float x[PER];
  const uint32_t* xp = reinterpret_cast<const uint32_t*>(X + (size_t)row * D + PER * lane);
#pragma unroll
  for (int i = 0; i < PER / 2; ++i) {
    const uint32_t w = xp[i];
    x[2 * i] = __uint_as_float(w << 16);
    x[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) amax = fmaxf(amax, fabsf(x[i]));
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / s;
  float e2 = 0.f, n2 = 0.f;
  int qv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    qv[i] = max(-127, min(127, (int)rintf(x[i] * inv)));
    const float xt = (float)qv[i] * s;
    e2 += (x[i] - xt) * (x[i] - xt);
    n2 += xt * xt;
  }
  e2 = wave_sum(e2);
  n2 = wave_sum(n2);
  uint16_t* op = reinterpret_cast<uint16_t*>(X8 + (size_t)row * D + PER * lane);
#pragma unroll
  for (int i = 0; i < PER / 2; ++i)
    op[i] = (uint16_t)((qv[2 * i] & 0xff) | ((qv[2 * i + 1] & 0xff) << 8));
  if (lane == 0) {
    sx[row] = s;
    if (err) err[row] = sqrtf(e2);
    if (xtn) xtn[row] = sqrtf(n2);
    red[0][w] = sqrtf(e2);
    red[1][w] = sqrtf(n2);
  }
  if (bounds) {
    __syncthreads();
    if (threadIdx.x < 2) {
      const float m = fmaxf(fmaxf(red[threadIdx.x][0], red[threadIdx.x][1]),
                            fmaxf(red[threadIdx.x][2], red[threadIdx.x][3]));
      atomicMax(reinterpret_cast<int*>(bounds) + threadIdx.x, __float_as_int(m));
    }
  }
}

// Query preparation of the pruned search in ONE launch (was the quantiser plus ~10 small torch
// kernels on the search's critical path, ~0.1 ms; profiles/r2_prepass/).  One wave per query:
//   T    = the k-th best of the union of the exact sample's and the tail's per-query top-k lists
//          (any order, -inf padded; k <= 32) minus thr_margin -- a lower bound of the final k-th
//   q8   = the query's int8 image, sq its scale (exactly as quant_rows_i8_kernel)
//   thr  = (T - (|q| E + |q - q~| X + 1e-5)) / sq, (E, X) = bounds (the shard's tracked maxima),
// i.e. the threshold index_scan_i8_kernel emits against (see the bound at the top of this file).
template <int D>
__global__ __launch_bounds__(256) void prune_qprep_kernel(
    const __bf16* __restrict__ Q, int NQ, const float* __restrict__ pre_s,
    const float* __restrict__ tail_s, int k, float thr_margin, const float* __restrict__ bounds,
    int8_t* __restrict__ Q8, float* __restrict__ sq, float* __restrict__ T_out,
    float* __restrict__ thr) {
  constexpr int PER = D / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = blockIdx.x * 4 + w;
  if (q >= NQ) return;   // (no barrier in this kernel)
  // k-th best of 2k values: lane i < 2k holds value i; its rank counts the values above it
  // (ties: lower index first), so exactly one lane has rank k - 1
  float v = -INFINITY;
  if (lane < k) v = pre_s[(size_t)q * k + lane];
  else if (lane < 2 * k) v = tail_s[(size_t)q * k + lane - k];
  int rank = 0;
  for (int j = 0; j < 2 * k; ++j) {
    const float u = __shfl(v, j);
    rank += (u > v) || (u == v && j < lane);
  }
  const unsigned long long hit = __ballot(lane < 2 * k && rank == k - 1);
  const float T = __shfl(v, (int)__builtin_ctzll(hit)) - thr_margin;

  float x[PER];
  const uint32_t* xp = reinterpret_cast<const uint32_t*>(Q + (size_t)q * D + PER * lane);
#pragma unroll
  for (int i = 0; i < PER / 2; ++i) {
    const uint32_t u = xp[i];
    x[2 * i] = __uint_as_float(u << 16);
    x[2 * i + 1] = __uint_as_float(u & 0xffff0000u);
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) amax = fmaxf(amax, fabsf(x[i]));
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / s;
  float e2 = 0.f, x2 = 0.f;
  int qv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    qv[i] = max(-127, min(127, (int)rintf(x[i] * inv)));
    const float xt = (float)qv[i] * s;
    e2 += (x[i] - xt) * (x[i] - xt);
    x2 += x[i] * x[i];
  }
  e2 = wave_sum(e2);
  x2 = wave_sum(x2);
  uint16_t* op = reinterpret_cast<uint16_t*>(Q8 + (size_t)q * D + PER * lane);
#pragma unroll
  for (int i = 0; i < PER / 2; ++i)
    op[i] = (uint16_t)((qv[2 * i] & 0xff) | ((qv[2 * i + 1] & 0xff) << 8));
  if (lane == 0) {
    const float margin = sqrtf(x2) * bounds[0] + sqrtf(e2) * bounds[1] + 1e-5f;
    sq[q] = s;
    T_out[q] = T;
    thr[q] = (T - margin) / s;
  }
}

// The pruned search in two query-side launches around its exact sample (index/shard.py
// _search_pruned), so the sample can decide the route:
//   prune_qquant: q8 / sq (as prune_qprep) and margin = |q| E + |q - q~| X + 1e-5, known before the
//                 sample is scanned, so the sample emits every row within the margin band;
//   prune_route:  T = k-th best of (sample, tail) - thr_margin and thr = (T - margin) / sq (as
//                 prune_qprep), plus the ROUTE: c = the sample rows (1 tile in 2^tshift) with an
//                 exact score >= T - margin estimates the int8 scan's candidates as c << tshift.
//                 The sample emitted every row >= thr0 (its seed threshold), so c is exact when
//                 T - margin >= thr0; below thr0 the band holds at least the cnt rows >= thr0,
//                 and, scores thinning out upwards, at least the density of [thr0, T] times the
//                 band width: c = max(cnt, (cnt - k) * margin / (T - thr0)).
//                 The route is decided PER ROW BLOCK of the int8 scan: each query's sample rows
//                 in the band are binned by block, est[q][b] = (rows of block b) * c / (rows
//                 binned) << tshift.  prune_route_final then sends to the bf16 emitting scan
//                 every block some query would flood (max_q est[q][b] > blk_limit: a crowd of
//                 near-duplicates the int8 bound cannot separate, such as freshly ingested rows
//                 of one document), and EVERY block when a query's estimate over the remaining
//                 blocks still exceeds `limit`, when a sample buffer overflowed (the bins are
//                 then truncated), or when more blocks are listed than the bf16 scan has row
//                 slots (index_mq.hip MqList).  The int8 scan skips the listed blocks
//                 (skip[b]), the bf16 scan at the exact threshold T scans only them, and both
//                 emit into the same candidate buffers: every row is covered by exactly one
//                 exact-bound scan.  Exactness never depends on the route; only the cost does.
// zero (optional): the search's counter workspace (zero_n ints), cleared here so the search's
// later kernels start from zeroed candidate counts and flags without memset launches.
template <int D>
__global__ __launch_bounds__(256) void prune_qquant_kernel(const __bf16* __restrict__ Q, int NQ,
                                                           const float* __restrict__ bounds,
                                                           int8_t* __restrict__ Q8,
                                                           float* __restrict__ sq,
                                                           float* __restrict__ margin,
                                                           int* __restrict__ zero, int zero_n) {
  constexpr int PER = D / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (zero != nullptr)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < zero_n; i += gridDim.x * 256) zero[i] = 0;
  const int q = blockIdx.x * 4 + w;
  if (q >= NQ) return;   // (no barrier in this kernel)
  float x[PER];
  const uint32_t* xp = reinterpret_cast<const uint32_t*>(Q + (size_t)q * D + PER * lane);
#pragma unroll
  for (int i = 0; i < PER / 2; ++i) {
    const uint32_t u = xp[i];
    x[2 * i] = __uint_as_float(u << 16);
    x[2 * i + 1] = __uint_as_float(u & 0xffff0000u);
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) amax = fmaxf(amax, fabsf(x[i]));
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / s;
  float e2 = 0.f, x2 = 0.f;
  int qv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    qv[i] = max(-127, min(127, (int)rintf(x[i] * inv)));
    const float xt = (float)qv[i] * s;
    e2 += (x[i] - xt) * (x[i] - xt);
    x2 += x[i] * x[i];
  }
  e2 = wave_sum(e2);
  x2 = wave_sum(x2);
  uint16_t* op = reinterpret_cast<uint16_t*>(Q8 + (size_t)q * D + PER * lane);
#pragma unroll
  for (int i = 0; i < PER / 2; ++i)
    op[i] = (uint16_t)((qv[2 * i] & 0xff) | ((qv[2 * i + 1] & 0xff) << 8));
  if (lane == 0) {
    sq[q] = s;
    margin[q] = sqrtf(x2) * bounds[0] + sqrtf(e2) * bounds[1] + 1e-5f;
  }
}

// Split image of rotated rows (index_scan_i8_kernel HK = 2): X = [n, D] fp32 rows already in the
// shard's PCA basis (index/shard.py calibrate_prune).  Dims 0 .. H-1 -> fp16 (image bytes 0 .. 2H),
// dims H .. D-1 -> int8 with sx = max |x_l| / 127 (bytes 2H .. 2H + D - H).  One wave per row: lane
// l holds leading dim l and trailing dims H + L l .. + L - 1.
//   rows    (margin == nullptr): bounds[0..3] raised to (max |x_l - x~_l|, max |x~_l|,
//            max |x_h - x^_h|, max |x^_h|) -- E_l, X_l, E_h, X_h;
//   queries (margin != nullptr): sq = sx and the bound of |q . x - est| (est = q~_l . x~_l +
//            q^_h . x^_h, the scan's acc_i * sq * sx + acc_f):
//            margin = |q_l| E_l + |q_l - q~_l| X_l + |q_h| E_h + |q_h - q^_h| X_h + 1e-5.
template <int D, int H>
__global__ __launch_bounds__(256) void quant_rows_split_kernel(const float* __restrict__ X, int n,
                                                               int8_t* __restrict__ X8,
                                                               float* __restrict__ sx,
                                                               float* __restrict__ bounds,
                                                               float* __restrict__ margin) {
  static_assert(H == 64 && (D - H) % 64 == 0, "64 leading dims, whole int8 k-steps");
  constexpr int L = (D - H) / 64;
  constexpr int RB = 2 * H + (D - H);
  __shared__ float red[4][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  const bool rows = margin == nullptr;
  if (row >= n) {   // (block-uniform barrier below: idle waves report zeros)
    if (rows && bounds) {
      if (lane < 4) red[lane][w] = 0.f;
      __syncthreads();
    }
    return;
  }
  const float* xp = X + (size_t)row * D;
  const float xh = xp[lane];
  float xl[L];
#pragma unroll
  for (int i = 0; i < L; ++i) xl[i] = xp[H + L * lane + i];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < L; ++i) amax = fmaxf(amax, fabsf(xl[i]));
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / s;
  float el2 = 0.f, nl2 = 0.f, ql2 = 0.f;
  int8_t* op = X8 + (size_t)row * RB;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int qv = max(-127, min(127, (int)rintf(xl[i] * inv)));
    const float xt = (float)qv * s;
    el2 += (xl[i] - xt) * (xl[i] - xt);
    nl2 += xt * xt;
    ql2 += xl[i] * xl[i];
    op[2 * H + L * lane + i] = (int8_t)qv;
  }
  const _Float16 hh = (_Float16)xh;
  const float xhh = (float)hh;
  reinterpret_cast<uint16_t*>(op)[lane] = __builtin_bit_cast(uint16_t, hh);
  const float el = sqrtf(wave_sum(el2)), nl = sqrtf(wave_sum(nl2)), ql = sqrtf(wave_sum(ql2));
  const float eh = sqrtf(wave_sum((xh - xhh) * (xh - xhh)));
  const float nh = sqrtf(wave_sum(xhh * xhh)), qh = sqrtf(wave_sum(xh * xh));
  if (!rows) {
    if (lane == 0) {
      sx[row] = s;
      margin[row] = ql * bounds[0] + el * bounds[1] + qh * bounds[2] + eh * bounds[3] + 1e-5f;
    }
    return;
  }
  if (lane == 0) {
    sx[row] = s;
    red[0][w] = el;
    red[1][w] = nl;
    red[2][w] = eh;
    red[3][w] = nh;
  }
  if (bounds) {
    __syncthreads();
    if (threadIdx.x < 4) {
      const float m = fmaxf(fmaxf(red[threadIdx.x][0], red[threadIdx.x][1]),
                            fmaxf(red[threadIdx.x][2], red[threadIdx.x][3]));
      atomicMax(reinterpret_cast<int*>(bounds) + threadIdx.x, __float_as_int(m));
    }
  }
}

// MX-fp4 image of bf16 rows (index_scan_i8_kernel HK = MX4): every 32-dim block b gets the
// power-of-two scale s_b = 2^ceil(log2(max |x_b| / 6)) (so |x| / s_b <= 6: no clamping) as an e8m0
// byte, and each element the nearest OCP e2m1 value of x / s_b (0, .5, 1, 1.5, 2, 3, 4, 6; sign in
// bit 3), two per byte, element 2j in the low nibble of byte j.  Block-scale bytes go to a
// 16-byte side record per row, dword g = blocks g, 4 + g, 8 + g (the scan's per-lane operand).
// One wave per row: lane l holds dims l + 64 m (m < 6), so dims of block 2 m + (l >> 5) sit in
// one half-wave.
//   rows    (margin == nullptr): bounds[0..1] raised to (max |x - x~|, max |x~|) -- E4, X4;
//   queries (margin != nullptr): margin = |q| E4 + |q - q~| X4 + 1e-5 from bounds.
__device__ __forceinline__ float half_max(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int e2m1_code(float a, float& q) {   // a = |x| / s <= 6
  int c;
  if (a < 2.f) {
    q = rintf(a * 2.f) * 0.5f;
    c = (int)(q * 2.f);          // 0 .. 4 -> 0, .5, 1, 1.5, 2
  } else if (a < 4.f) {
    q = rintf(a);                // 2, 3, 4
    c = q == 2.f ? 4 : q == 3.f ? 5 : 6;
  } else {
    q = a < 5.f ? 4.f : 6.f;
    c = q == 4.f ? 6 : 7;
  }
  return c;
}
template <int D>
__global__ __launch_bounds__(256) void quant_rows_mx4_kernel(const __bf16* __restrict__ X, int n,
                                                             uint8_t* __restrict__ X4,
                                                             uint8_t* __restrict__ SC,
                                                             float* __restrict__ bounds,
                                                             float* __restrict__ margin) {
  static_assert(D == 384, "12 blocks of 32 dims");
  constexpr int M = D / 64;
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  const bool rows = margin == nullptr;
  if (row >= n) {   // (block-uniform barrier below: idle waves report zeros)
    if (rows && bounds) {
      if (lane < 2) red[lane][w] = 0.f;
      __syncthreads();
    }
    return;
  }
  const uint16_t* xp = reinterpret_cast<const uint16_t*>(X + (size_t)row * D);
  uint8_t* op = X4 + (size_t)row * (D / 2);
  uint8_t* sp = SC + (size_t)row * 16;
  float e2 = 0.f, n2 = 0.f, x2 = 0.f;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float x = __uint_as_float((uint32_t)xp[lane + 64 * m] << 16);
    const float amax = half_max(fabsf(x));
    int e = -127;
    if (amax > 0.f) {
      int k;
      frexpf(amax / 6.f, &k);              // amax / 6 in [2^(k-1), 2^k)
      e = k;
      if (amax <= 6.f * ldexpf(1.f, k - 1)) e = k - 1;
      if (amax > 6.f * ldexpf(1.f, e)) ++e;   // (guard the division's rounding)
      e = max(e, -127);
    }
    const float sc = ldexpf(1.f, e);
    float q;
    const int c = amax > 0.f ? e2m1_code(fabsf(x) * ldexpf(1.f, -e), q) : (q = 0.f, 0);
    const int code = c | (x < 0.f && c ? 8 : 0);
    const float xt = (x < 0.f ? -q : q) * sc;
    e2 += (x - xt) * (x - xt);
    n2 += xt * xt;
    x2 += x * x;
    const int hi = __shfl_down(code, 1);
    if ((lane & 1) == 0) op[(lane >> 1) + 32 * m] = (uint8_t)(code | (hi << 4));
    if ((lane & 31) == 0) {
      const int b = 2 * m + (lane >> 5);
      sp[4 * (b & 3) + (b >> 2)] = (uint8_t)(e + 127);
    }
  }
  if (lane < 4) sp[4 * lane + 3] = 0;
  const float en = sqrtf(wave_sum(e2)), nn = sqrtf(wave_sum(n2)), xn = sqrtf(wave_sum(x2));
  if (!rows) {
    if (lane == 0) margin[row] = xn * bounds[0] + en * bounds[1] + 1e-5f;
    return;
  }
  if (lane == 0) {
    red[0][w] = en;
    red[1][w] = nn;
  }
  if (bounds) {
    __syncthreads();
    if (threadIdx.x < 2) {
      const float mx = fmaxf(fmaxf(red[threadIdx.x][0], red[threadIdx.x][1]),
                             fmaxf(red[threadIdx.x][2], red[threadIdx.x][3]));
      atomicMax(reinterpret_cast<int*>(bounds) + threadIdx.x, __float_as_int(mx));
    }
  }
}

// The first tier's choice (after prune_route): the MX-fp4 scan emits, beyond the int8 scan's
// candidates, the rows whose fp4 estimate reaches T - margin4 although their exact score is
// below the int8 band T - margin8 -- rows scoring at least T - 2 margin4.  Their population per
// query is estimated from exact dense scores of a row probe (every 4th seed tile of the sample,
// `rate` corpus rows per probe row) plus the exact dense tail: the MX-fp4 tier is viable iff for
// EVERY query probe rows in [T - 2 margin4, T - margin8) x rate + such tail rows <= `limit`.  A
// crowd scoring above the int8 band (fresh near-duplicates) is left to the per-block route, as
// in the int8 tier.  *nv ends 1 (not viable: the int8 tier runs) or stays 0 (the MX-fp4 tier
// runs at thr4 = T - margin4).  Exactness never depends on the choice.
// probe_s: [NQ][ld] exact scores; the probe is columns c < n_cols whose 64-row tile c / 64 is a
// multiple of tile_stride (1: every column), scaled by `rate`; tail_cs: [NQ][tail_ld].
// stage (the MX-fp6 tier between the two, margin4 then being the fp6 margin): 0 = the fp4 choice
// (bit 0 of *nv: fp4 not viable); 1 = the fp6 choice after the fp4 one (nothing when fp4 runs,
// else bit 1: fp6 not viable); 2 = the fp6 choice alone (bit 0 always, bit 1 as in 1).  The
// gated scans then want *nv == 0 (fp4), 1 (fp6), 3 (int8).
// The band counted is [T - wa margin4 - wb margin8, T - margin8): (2, 0) -- the fp4 tier's
// worst case -- or (1, 0) for the fp6 tier, whose rounding error on a pair is typically ~1/30 of
// its Cauchy-Schwarz bound, so its emissions are ~ the rows above T - margin6 (an underestimate
// only costs the overflow fallback, never exactness; the limit leaves 4x headroom to the cap).
__global__ __launch_bounds__(256) void mx4_select_kernel(
    int NQ, const float* __restrict__ T, const float* __restrict__ margin4,
    const float* __restrict__ margin8, const float* __restrict__ probe_s, int n_cols, int ld,
    int tile_stride, float rate, const float* __restrict__ tail_cs, int tail_cap, int tail_ld,
    float limit, float* __restrict__ thr4, int* __restrict__ nv, int stage, float wa, float wb) {
  // one 256-thread workgroup per query (a wave per query took 146 us for 256 queries)
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = blockIdx.x;
  if (stage == 1 && (*nv & 1) == 0) return;   // (bit 0 is final: the fp4 choice ran before)
  if (stage == 2 && q == 0 && threadIdx.x == 0) atomicOr(nv, 1);
  const float t = T[q];
  const float lo = t - wa * margin4[q] - wb * margin8[q], hi = t - margin8[q];
  // the probe's columns enumerated directly (probe tile j = tile j * tile_stride), four
  // independent loads in flight per thread: the walk over every column with a per-element tile
  // test waited out one load round trip per probe column (97 us per held-out search)
  float c = 0.f;
  const float* ps = probe_s + (size_t)q * ld;
  const int n_probe = ((n_cols + 63) / 64 + tile_stride - 1) / tile_stride * 64;
  auto pcol = [&](int j) { return ((j >> 6) * tile_stride << 6) + (j & 63); };
  int j = threadIdx.x;
  for (; j + 3 * 256 < n_probe; j += 4 * 256) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int col = pcol(j + u * 256);
      v[u] = col < n_cols ? ps[col] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) c += (v[u] >= lo && v[u] < hi) ? 1.f : 0.f;
  }
  for (; j < n_probe; j += 256) {
    const int col = pcol(j);
    const float v = col < n_cols ? ps[col] : -INFINITY;
    c += (v >= lo && v < hi) ? 1.f : 0.f;
  }
  float tc = 0.f;
  const float* tcs = tail_cs + (size_t)q * tail_ld;
  int i = threadIdx.x;
  for (; i + 3 * 256 < tail_cap; i += 4 * 256) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = tcs[i + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u) tc += (v[u] >= lo && v[u] < hi) ? 1.f : 0.f;
  }
  for (; i < tail_cap; i += 256) tc += (tcs[i] >= lo && tcs[i] < hi) ? 1.f : 0.f;
  c = wave_sum(c);
  tc = wave_sum(tc);
  if (lane == 0) {
    red[0][w] = c;
    red[1][w] = tc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    tc = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    thr4[q] = t - margin4[q];
    if (!(c * rate + tc <= limit)) atomicOr(nv, stage ? 2 : 1);
  }
}

constexpr int ROUTE_MAX_BLOCKS = 1024;   // int8 row blocks the per-block route can bin

// The exact tail scan's candidates (rows >= thr0 of the fresh rows [off, n), ids relative to
// off, one slot per tail row so none is dropped): binned one by one, no sampling scale.
struct RouteTail {
  const float* cs;
  const int* ci;
  const int* cnt;
  int cap;
  int off;
  int ld;    // row stride of cs (dense form; = cap unless the tail shares a wider score matrix)
};

// One 256-thread workgroup per query (was one wave per query, 4 per workgroup: 64 workgroups
// for a 256-query batch on a 256-CU chip, the longest kernel of the pre-pass chain beside the
// encoder); the four waves split its candidate list and tail and share its LDS histograms.
__global__ __launch_bounds__(256) void prune_route_kernel(
    int NQ, const float* __restrict__ pre_s, const float* __restrict__ tail_s, int k,
    float thr_margin, const float* __restrict__ sq, const float* __restrict__ margin,
    const float* __restrict__ thr0, const float* __restrict__ cs_p, const int* __restrict__ ci_p,
    const int* __restrict__ cnt_p, int cap_p, int tshift, int rows_per_blk, int n_rblk,
    float* __restrict__ T_out, float* __restrict__ thr, int* __restrict__ dense,
    float* __restrict__ est, int* __restrict__ blkmax, RouteTail tail) {
  __shared__ int h[ROUTE_MAX_BLOCKS];
  __shared__ int th[ROUTE_MAX_BLOCKS];
  __shared__ float wc[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = blockIdx.x;
  // k-th best of 2k values (prune_qprep_kernel), every wave alike
  float v = -INFINITY;
  if (lane < k) v = pre_s[(size_t)q * k + lane];
  else if (lane < 2 * k) v = tail_s[(size_t)q * k + lane - k];
  int rank = 0;
  for (int j = 0; j < 2 * k; ++j) {
    const float u = __shfl(v, j);
    rank += (u > v) || (u == v && j < lane);
  }
  const unsigned long long hit = __ballot(lane < 2 * k && rank == k - 1);
  const float T = __shfl(v, (int)__builtin_ctzll(hit)) - thr_margin;
  const float m = margin[q];
  const int cnt = cnt_p[q];
  const int n = min(cnt, cap_p);
  const float band = T - m;
  const float t0 = thr0[q];
  const float* cs = cs_p + (size_t)q * cap_p;
  const int* ci = ci_p + (size_t)q * cap_p;
  for (int b = tid; b < n_rblk; b += 256) {
    h[b] = 0;
    th[b] = 0;
  }
  __syncthreads();
  float c = 0.f;
  for (int i = tid; i < n; i += 256) {
    if (cs[i] >= band) {
      c += 1.f;
      atomicAdd(&h[min(ci[i] / rows_per_blk, n_rblk - 1)], 1);
    }
  }
  const bool tail_dense = tail.cs != nullptr && tail.ci == nullptr;
  if (tail_dense) {   // the exact tail as dense scores [NQ][cap] (row i = tail.off + i)
    const float* tcs = tail.cs + (size_t)q * tail.ld;
    for (int i0 = w * 64; i0 < tail.cap; i0 += 256) {
      const int i = i0 + lane;
      const bool hit = i < tail.cap && tcs[i] >= band;
      const int b = min((min(i, tail.cap - 1) + tail.off) / rows_per_blk, n_rblk - 1);
      const int b0 = __shfl(b, 0), b63 = __shfl(b, 63);
      if (b0 == b63) {   // (64 consecutive rows: almost always one block) one add per chunk
        const int nh = __popcll(__ballot(hit));
        if (lane == 0 && nh) atomicAdd(&th[b0], nh);
      } else if (hit) {
        atomicAdd(&th[b], 1);
      }
    }
  } else if (tail.cs != nullptr) {   // the exact tail: every row >= thr0 of it, one by one
    const int tn = min(tail.cnt[q], tail.cap);
    const float* tcs = tail.cs + (size_t)q * tail.cap;
    const int* tci = tail.ci + (size_t)q * tail.cap;
    for (int i = tid; i < tn; i += 256)
      if (tcs[i] >= band) atomicAdd(&th[min((tci[i] + tail.off) / rows_per_blk, n_rblk - 1)], 1);
  }
  c = wave_sum(c);
  if (lane == 0) wc[w] = c;
  __syncthreads();   // (the histograms and the waves' counts)
  c = wc[0] + wc[1] + wc[2] + wc[3];
  const float binned = c;
  float tscale = 1.f;
  if (band < t0) {   // the band reaches below what the sample emitted: extrapolate (see above)
    c = fmaxf((float)cnt, fmaxf(0.f, (float)(cnt - k)) * m / fmaxf(T - t0, 1e-6f));
    // (an emitting tail scan kept only rows >= thr0 too; a dense tail counted every row)
    tscale = tail_dense ? 1.f : binned > 0.f ? fmaxf(1.f, c / binned) : 1.f;
  }
  const float scale = (binned > 0.f ? c / binned : 0.f) * (float)(1 << tshift);
  for (int b = tid; b < n_rblk; b += 256) {
    const float e = (float)h[b] * scale + (float)th[b] * tscale;
    est[(size_t)q * n_rblk + b] = e;
    if (e > 0.f) atomicMax(blkmax + b, __float_as_int(e));   // (non-negative floats order as ints)
  }
  if (tid == 0) {
    T_out[q] = T;
    thr[q] = (T - m) / sq[q];
    if (cnt > cap_p) atomicOr(dense, 1);
  }
}

// What each query would still emit in the int8 scan after the flooded blocks leave it: one wave per
// query over the blocks (coalesced); any query above `limit` ORs *dense (every block then goes to
// the bf16 scan).  (This loop ran inside the single-workgroup final kernel, one thread per query
// striding its own row of est: 121 us per search at 1024 blocks, profiles/r5_step/.)
__global__ __launch_bounds__(256) void prune_route_sum_kernel(int NQ, int n_rblk,
                                                              const float* __restrict__ est,
                                                              const int* __restrict__ blkmax,
                                                              float blk_limit, float limit,
                                                              int* __restrict__ dense) {
  const int lane = threadIdx.x & 63, q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= NQ) return;
  const float* e = est + (size_t)q * n_rblk;
  float s = 0.f;
  for (int b = lane; b < n_rblk; b += 64) s += __int_as_float(blkmax[b]) > blk_limit ? 0.f : e[b];
  s = wave_sum(s);
  if (lane == 0 && s > limit) atomicOr(dense, 1);
}

// The search statistics of HbmIndexShard.mq_stats in one launch (they were ~10 framework
// kernels per search): tot[0] += *ovf; tot[1] = max(tot[1], max of cnt[0 .. NQ)); with dense:
// tot[2] += *dense; with blk too: part = (blk[0] > 0) && !*dense, tot[3] += part,
// tot[4] += blk[0] * part.  One workgroup; the updates are device atomics, so searches whose end
// halves run on different streams (a pipelined loop beside a plain one) never lose a count.
__global__ __launch_bounds__(256) void prune_stats_kernel(const int* __restrict__ ovf,
                                                          const int* __restrict__ cnt, int NQ,
                                                          const int* __restrict__ dense,
                                                          const int* __restrict__ blk,
                                                          int* __restrict__ tot) {
  __shared__ int wm[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int m = 0;
  for (int i = tid; i < NQ; i += 256) m = max(m, cnt[i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
  if (lane == 0) wm[w] = m;
  __syncthreads();
  if (tid != 0) return;
  m = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
  atomicAdd(tot + 0, *ovf);
  atomicMax(tot + 1, m);
  if (dense != nullptr) {
    const int d = *dense;
    atomicAdd(tot + 2, d);
    if (blk != nullptr) {
      const int part = (blk[0] > 0 ? 1 : 0) * (1 - d);
      atomicAdd(tot + 3, part);
      atomicAdd(tot + 4, blk[0] * part);
    }
  }
}

// One workgroup: the per-block decision of prune_route_kernel.  blk: [0] = listed blocks, [1] =
// n_rblk, [2 .. 2 + n_rblk) = the listed blocks in order, [2 + n_rblk .. 2 + 2 n_rblk) = skip
// flags of the int8 scan.  *dense ends as 1 iff every block went to the bf16 scan.
__global__ __launch_bounds__(1024) void prune_route_final_kernel(
    int NQ, int n_rblk, const float* __restrict__ est, const int* __restrict__ blkmax,
    float blk_limit, float limit, int max_list, int* __restrict__ dense, int* __restrict__ blk) {
  __shared__ int flag[ROUTE_MAX_BLOCKS];
  __shared__ int wtot[16];
  __shared__ int all;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) all = *dense;
  for (int b = tid; b < n_rblk; b += 1024) flag[b] = __int_as_float(blkmax[b]) > blk_limit;
  __syncthreads();   // (all: prune_route_sum_kernel's verdict, read above)
  // listed blocks in order: one bin per thread (n_rblk <= 1024), ballot prefix per wave
  const int f = tid < n_rblk && (all || flag[tid]);
  const unsigned long long bal = __ballot(f);
  if (lane == 0) wtot[w] = __popcll(bal);
  __syncthreads();
  int off = 0, nl = 0;
  for (int i = 0; i < 16; ++i) {
    off += i < w ? wtot[i] : 0;
    nl += wtot[i];
  }
  const bool every = all || nl > max_list;
  if (every) nl = n_rblk;
  if (tid < n_rblk) {
    const int pos = every ? tid
                          : off + (int)__builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
    if (every || f) blk[2 + pos] = tid;
    blk[2 + n_rblk + tid] = every || f;
  }
  if (tid == 0) {
    blk[0] = nl;
    blk[1] = n_rblk;
    *dense = every ? 1 : 0;
  }
}

}  // namespace symb

using namespace symb;

// rows per scan tile and waves per workgroup (symb_i8_config): 64 / 128 rows, 8 waves (one
// workgroup per CU) or 4 (64-row tiles, two workgroups per CU, 256 queries each)
static int g_i8_tr = 64;
static int g_i8_waves = 8;
int symb_i8_config(int tile_rows, int waves) {
  if (tile_rows != 64 && tile_rows != 128) return -1;
  if (waves != 8 && !(waves == 4 && tile_rows == 64)) return -1;
  g_i8_tr = tile_rows;
  g_i8_waves = waves;
  return 0;
}
int symb_i8_tile_rows() { return g_i8_tr; }
int symb_i8_wgs_per_cu() { return 8 / g_i8_waves; }
int symb_i8_queries_per_blk(int rsplit) {
  return g_i8_waves == 4 ? 4 * 16 * i8s::SETS : i8s::WAVES / rsplit * 16 * i8s::SETS;
}

// MX-fp4 scan tile rows at 256 queries per workgroup: 64 (12 KiB tiles, 8-deep ring) or 128
// (24 KiB tiles, 5-deep ring: half the barriers per row; default -- headline 7.35 vs 7.72 ms
// per step, same box, profiles/r4_mx4/tile/); symb_mx4_config
static int g_mx4_tr = 128;
int symb_mx4_config(int tile_rows) {
  if (tile_rows != 64 && tile_rows != 128) return -1;
  g_mx4_tr = tile_rows;
  return 0;
}
int symb_mx4_tile_rows() { return g_mx4_tr; }

template <int D, int RSPLIT, int TRK, int WV = 8, int HK = 0>
static int launch_i8(const void* X8, const float* sx, int n_valid, int rows_per_blk, int n_rblk,
                     const void* Q8, int NQ, const float* thr, float* cand_s, int* cand_i,
                     int* cand_n, int cap, int xcd, hipStream_t st, const int* skip,
                     const float* sq = nullptr, const int* gate = nullptr, int gate_want = 0) {
  constexpr int qpb = WV / RSPLIT * 16 * i8s::SETS;
  const int n_qblk = (NQ + qpb - 1) / qpb;
  constexpr int lds = Geo<D, TRK, WV, HK>::LDS_BYTES;
  auto go = [&](auto kern) {
    set_max_lds<decltype(kern)::value>(lds);
    hipLaunchKernelGGL(decltype(kern)::value, dim3(n_rblk * n_qblk), dim3(64 * WV), lds, st,
                       (const int8_t*)X8, sx, n_valid, rows_per_blk, (const int8_t*)Q8, NQ, n_qblk,
                       xcd, thr, cand_s, cand_i, cand_n, cap, skip, sq, gate, gate_want);
    return (int)hipGetLastError();
  };
  return go(std::integral_constant<decltype(&index_scan_i8_kernel<D, RSPLIT, 0, TRK, WV, HK>),
                                   &index_scan_i8_kernel<D, RSPLIT, 0, TRK, WV, HK>>());
}

// Tile rows the D-wide scan runs with (the 128-row and 4-wave forms are D = 384 knobs; the split
// image runs 64-row tiles, 8 waves).
int symb_i8_tile_rows_for(int dim, int heavy) { return dim == 384 && !heavy ? g_i8_tr : 64; }
int symb_i8_split_queries_per_blk(int rsplit) { return i8s::WAVES / rsplit * 16 * i8s::SETS; }

// rows_per_blk % tile rows == 0, n_rblk * rows_per_blk >= n_valid; X8 / sx hold alloc_rows
// rows, which must cover n_valid rounded up to a whole tile (the DMA reads whole tiles).
// rsplit 2 = 256 queries per workgroup, 1 = 512.  dim: 384 or 768.  heavy = 64: the split image
// (448-byte rows and queries, quant_rows_split), sq = the queries' int8 scales; 0: plain int8.
// form: 0 = plain int8 (heavy 0) or split (heavy 64); 1 = the MX-fp4 image (sx = the rows'
// block scales, sq = the queries'; quant_rows_mx4).  gate / gate_want: the launch runs only if
// *gate == gate_want (nullptr: always); cand_n is zeroed only by an ungated launch.
int symb_index_scan_i8(const void* X8, const float* sx, int n_valid, int alloc_rows,
                       int rows_per_blk, int n_rblk, const void* Q8, int NQ, const float* thr,
                       float* cand_s, int* cand_i, int* cand_n, int cap, int xcd, hipStream_t st,
                       int rsplit, const int* skip, int dim, int heavy, const float* sq, int form,
                       const int* gate, int gate_want) {
  if (NQ <= 0) return 0;
  if (dim != 384 && dim != 768) return -1;
  if (heavy != 0 && (heavy != 64 || dim != 384 || sq == nullptr)) return -1;
  if (form != 0 && (form != 1 || heavy != 0 || dim != 384 || sq == nullptr)) return -1;
  const int tr = form ? (rsplit == 2 ? g_mx4_tr : 64) : symb_i8_tile_rows_for(dim, heavy);
  if (rows_per_blk % tr || n_rblk <= 0 || thr == nullptr || cap <= 0 || n_valid <= 0) return -1;
  if ((long long)n_rblk * rows_per_blk < n_valid) return -1;
  if ((long long)(n_valid + tr - 1) / tr * tr > alloc_rows) return -1;   // a tile past the buffer
  if (gate == nullptr) {
    hipError_t e = hipMemsetAsync(cand_n, 0, sizeof(int) * (size_t)NQ, st);
    if (e != hipSuccess) return (int)e;
  }
#define SYMB_I8(D_, RS, T) launch_i8<D_, RS, T>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8, NQ, thr, \
                                                cand_s, cand_i, cand_n, cap, xcd, st, skip,       \
                                                nullptr, gate, gate_want)
  if (form && rsplit == 2 && g_mx4_tr == 128)   // (rows_per_blk: a multiple of 128, the host's)
    return launch_i8<384, 2, 128, 8, MX4>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8, NQ, thr,
                                          cand_s, cand_i, cand_n, cap, xcd, st, skip, sq, gate,
                                          gate_want);
  if (form)
    return rsplit == 2 ? launch_i8<384, 2, 64, 8, MX4>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8,
                                                       NQ, thr, cand_s, cand_i, cand_n, cap, xcd,
                                                       st, skip, sq, gate, gate_want)
                       : launch_i8<384, 1, 64, 8, MX4>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8,
                                                       NQ, thr, cand_s, cand_i, cand_n, cap, xcd,
                                                       st, skip, sq, gate, gate_want);
  if (heavy)
    return rsplit == 2 ? launch_i8<384, 2, 64, 8, 2>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8, NQ,
                                                     thr, cand_s, cand_i, cand_n, cap, xcd, st,
                                                     skip, sq, gate, gate_want)
                       : launch_i8<384, 1, 64, 8, 2>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8, NQ,
                                                     thr, cand_s, cand_i, cand_n, cap, xcd, st,
                                                     skip, sq, gate, gate_want);
  if (dim == 768) return rsplit == 2 ? SYMB_I8(768, 2, 64) : SYMB_I8(768, 1, 64);
  if (g_i8_waves == 4)
    return launch_i8<384, 1, 64, 4>(X8, sx, n_valid, rows_per_blk, n_rblk, Q8, NQ, thr, cand_s,
                                    cand_i, cand_n, cap, xcd, st, skip, nullptr, gate, gate_want);
  if (rsplit == 2) return tr == 128 ? SYMB_I8(384, 2, 128) : SYMB_I8(384, 2, 64);
  // 512 queries per workgroup always run 64-row tiles: the 128-row form (four fused two-sub-tile
  // chains per wave per tile) emitted a few rows per million with wrong scores, differently from
  // run to run (benchmarks/diag/i8_determinism.py: 1100 queries, candidate totals 1317690 ..
  // 1317766 against a constant 1317699 for every other form, profiles/r3_blockroute/), so it is
  // not dispatched until that race is found
  if (rsplit == 1) return SYMB_I8(384, 1, 64);
#undef SYMB_I8
  return -1;
}

// Profiling-only entry: the ablations of index_scan_i8_kernel<384, 2> (ABL above), same arguments.
int symb_index_scan_i8_ablate(const void* X8, const float* sx, int n_valid, int alloc_rows,
                              int rows_per_blk, int n_rblk, const void* Q8, int NQ,
                              const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                              int xcd, hipStream_t st, int abl) {
  if (NQ <= 0) return 0;
  const int tr = g_i8_tr;
  if (rows_per_blk % tr || n_rblk <= 0 || thr == nullptr || cap <= 0 || n_valid <= 0) return -1;
  if ((long long)n_rblk * rows_per_blk < n_valid) return -1;
  if ((long long)(n_valid + tr - 1) / tr * tr > alloc_rows) return -1;
  hipError_t e = hipMemsetAsync(cand_n, 0, sizeof(int) * (size_t)NQ, st);
  if (e != hipSuccess) return (int)e;
  const int n_qblk = (NQ + 255) / 256;
  const int w4 = g_i8_waves == 4;
  const int lds = w4 ? Geo<384, 64, 4>::LDS_BYTES
                     : (tr == 128 ? Geo<384, 128>::LDS_BYTES : Geo<384, 64>::LDS_BYTES);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3(n_rblk * n_qblk), dim3(w4 ? 256 : 512), lds, st, (const int8_t*)X8, sx,
                       n_valid, rows_per_blk, (const int8_t*)Q8, NQ, n_qblk, xcd, thr, cand_s,
                       cand_i, cand_n, cap, (const int*)nullptr, (const float*)nullptr,
                       (const int*)nullptr, 0);
    return (int)hipGetLastError();
  };
  if (w4) {
    switch (abl) {
      case 0: return go(index_scan_i8_kernel<384, 1, 0, 64, 4>);
      case 2: return go(index_scan_i8_kernel<384, 1, 2, 64, 4>);
      case 3: return go(index_scan_i8_kernel<384, 1, 3, 64, 4>);
      case 4: return go(index_scan_i8_kernel<384, 1, 4, 64, 4>);
      default: return -1;
    }
  }
  switch (abl + (tr == 128 ? 8 : 0)) {
    case 0: return go(index_scan_i8_kernel<384, 2, 0, 64>);
    case 1: return go(index_scan_i8_kernel<384, 2, 1, 64>);
    case 2: return go(index_scan_i8_kernel<384, 2, 2, 64>);
    case 3: return go(index_scan_i8_kernel<384, 2, 3, 64>);
    case 4: return go(index_scan_i8_kernel<384, 2, 4, 64>);
    case 8: return go(index_scan_i8_kernel<384, 2, 0, 128>);
    case 9: return go(index_scan_i8_kernel<384, 2, 1, 128>);
    case 10: return go(index_scan_i8_kernel<384, 2, 2, 128>);
    case 11: return go(index_scan_i8_kernel<384, 2, 3, 128>);
    case 12: return go(index_scan_i8_kernel<384, 2, 4, 128>);
    default: return -1;
  }
}

// launch F(D) for the shard's row width (D = 384 / 768 / 1024); -1 for any other
#define SYMB_BY_DIM(dim, F)      \
  do {                           \
    if ((dim) == 384) {          \
      F(384);                    \
    } else if ((dim) == 768) {   \
      F(768);                    \
    } else if ((dim) == 1024) {  \
      F(1024);                   \
    } else {                     \
      return -1;                 \
    }                            \
  } while (0)

int symb_rescore_bf16(const void* X, const void* Q, int NQ, int dim, const int* cand_i,
                      const int* cand_n, int cap, float* cand_s, hipStream_t st) {
  if (NQ <= 0) return 0;
  if (cap <= 0) return -1;
#define L(D_) hipLaunchKernelGGL(rescore_bf16_kernel<D_>, dim3(NQ, 8), dim3(256), 0, st, \
                                 (const __bf16*)X, (const __bf16*)Q, cand_i, cand_n, cap, cand_s)
  SYMB_BY_DIM(dim, L);
#undef L
  return (int)hipGetLastError();
}

int symb_quant_rows_i8(const void* X, int n, int dim, void* X8, float* sx, float* err, float* xtn,
                       float* bounds, hipStream_t st) {
  if (n <= 0) return 0;
#define L(D_) hipLaunchKernelGGL(quant_rows_i8_kernel<D_>, dim3((n + 3) / 4), dim3(256), 0, st, \
                                 (const __bf16*)X, n, (int8_t*)X8, sx, err, xtn, bounds)
  SYMB_BY_DIM(dim, L);
#undef L
  return (int)hipGetLastError();
}

// The split image of D-wide fp32 rows already rotated into the shard's basis
// (quant_rows_split_kernel): rows (margin == nullptr, bounds raised) or queries (margin and sq =
// sx written, bounds read).  X8: [n, D + 64] bytes.
int symb_quant_rows_split(const float* X, int n, int dim, void* X8, float* sx, float* bounds,
                          float* margin, hipStream_t st) {
  if (n <= 0) return 0;
  if (dim != 384 || bounds == nullptr) return -1;
  hipLaunchKernelGGL((quant_rows_split_kernel<384, 64>), dim3((n + 3) / 4), dim3(256), 0, st, X, n,
                     (int8_t*)X8, sx, bounds, margin);
  return (int)hipGetLastError();
}

// MX-fp4 image of bf16 rows / queries (quant_rows_mx4_kernel): X4 = [n][D / 2], SC = [n][16].
int symb_quant_rows_mx4(const void* X, int n, int dim, void* X4, void* SC, float* bounds,
                        float* margin, hipStream_t st) {
  if (n <= 0) return 0;
  if (dim != 384 || bounds == nullptr) return -1;
  hipLaunchKernelGGL(quant_rows_mx4_kernel<384>, dim3((n + 3) / 4), dim3(256), 0, st,
                     (const __bf16*)X, n, (uint8_t*)X4, (uint8_t*)SC, bounds, margin);
  return (int)hipGetLastError();
}

// The MX-fp4 tier choice (mx4_select_kernel); nv (one int) is zeroed here.  probe_s: [NQ][n_probe]
// exact scores of the probe rows, tail_cs: [NQ][tail_cap] exact scores of the tail rows.
int symb_prune_stats(const int* ovf, const int* cnt, int NQ, const int* dense, const int* blk,
                     int* tot, hipStream_t st) {
  if (NQ <= 0 || ovf == nullptr || cnt == nullptr || tot == nullptr) return -1;
  hipLaunchKernelGGL(prune_stats_kernel, dim3(1), dim3(256), 0, st, ovf, cnt, NQ, dense, blk, tot);
  return (int)hipGetLastError();
}

int symb_mx4_select(int NQ, const float* T, const float* margin4, const float* margin8,
                    const float* probe_s, int n_cols, int ld, int tile_stride, float rate,
                    const float* tail_cs, int tail_cap, int tail_ld, float limit, float* thr4,
                    int* nv, hipStream_t st, int nv_zeroed, int stage, float wa, float wb) {
  if (NQ <= 0) return 0;
  if (stage < 0 || stage > 2 || (stage == 1 && !nv_zeroed)) return -1;
  if (ld <= 0) ld = n_cols;
  if (tail_ld <= 0) tail_ld = tail_cap;
  if (n_cols <= 0 || ld < n_cols || tile_stride < 1 || tail_cap < 0 || tail_ld < tail_cap ||
      probe_s == nullptr || (tail_cap > 0 && tail_cs == nullptr))
    return -1;
  if (!nv_zeroed) {
    hipError_t e = hipMemsetAsync(nv, 0, sizeof(int), st);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(mx4_select_kernel, dim3(NQ), dim3(256), 0, st, NQ, T, margin4, margin8,
                     probe_s, n_cols, ld, tile_stride, rate, tail_cs, tail_cap, tail_ld, limit,
                     thr4, nv, stage, wa, wb);
  return (int)hipGetLastError();
}

int symb_prune_qprep(const void* Q, int NQ, int dim, const float* pre_s, const float* tail_s, int k,
                     float thr_margin, const float* bounds, void* Q8, float* sq, float* T,
                     float* thr, hipStream_t st) {
  if (NQ <= 0) return 0;
  if (k < 1 || k > 32) return -1;
#define L(D_) hipLaunchKernelGGL(prune_qprep_kernel<D_>, dim3((NQ + 3) / 4), dim3(256), 0, st, \
                                 (const __bf16*)Q, NQ, pre_s, tail_s, k, thr_margin, bounds,     \
                                 (int8_t*)Q8, sq, T, thr)
  SYMB_BY_DIM(dim, L);
#undef L
  return (int)hipGetLastError();
}

int symb_prune_qquant(const void* Q, int NQ, int dim, const float* bounds, void* Q8, float* sq,
                      float* margin, hipStream_t st, int* zero, int zero_n) {
  if (NQ <= 0) return 0;
  if (zero_n < 0 || (zero_n > 0 && zero == nullptr)) return -1;
#define L(D_) hipLaunchKernelGGL(prune_qquant_kernel<D_>, dim3((NQ + 3) / 4), dim3(256), 0, st, \
                                 (const __bf16*)Q, NQ, bounds, (int8_t*)Q8, sq, margin, zero,    \
                                 zero_n)
  SYMB_BY_DIM(dim, L);
#undef L
  return (int)hipGetLastError();
}
#undef SYMB_BY_DIM

// The per-block route (prune_route_kernel + prune_route_final_kernel).  dense (one int) ends 1
// iff every block went to the bf16 scan; blk holds 2 + 2 n_rblk ints (layout at the final
// kernel); est: NQ x n_rblk floats and blkmax: n_rblk ints of scratch.  ci_p: the sample's
// candidate rows (physical), rows_per_blk / n_rblk: the int8 scan's row blocks (n_rblk <= 1024).
// tail_* (optional): the exact tail scan's candidates (RouteTail).
int symb_prune_route(int NQ, const float* pre_s, const float* tail_s, int k, float thr_margin,
                     const float* sq, const float* margin, const float* thr0, const float* cs_p,
                     const int* ci_p, const int* cnt_p, int cap_p, int tshift, int rows_per_blk,
                     int n_rblk, float blk_limit, float limit, int max_list, float* T, float* thr,
                     int* dense, float* est, int* blkmax, int* blk, hipStream_t st,
                     const float* tail_cs, const int* tail_ci, const int* tail_cnt, int tail_cap,
                     int tail_off, int tail_ld, int zeroed) {
  if (NQ <= 0) return 0;
  if (k < 1 || k > 32 || cap_p <= 0 || tshift < 0 || tshift > 20) return -1;
  if (n_rblk < 1 || n_rblk > ROUTE_MAX_BLOCKS || rows_per_blk < 1 || max_list < 1) return -1;
  // tail_ci == nullptr: tail_cs holds DENSE scores [NQ][tail_cap] of rows tail_off + i
  if (tail_cs != nullptr && ((tail_ci != nullptr) != (tail_cnt != nullptr) || tail_cap < 1 || tail_off < 0))
    return -1;
  if (tail_ld <= 0) tail_ld = tail_cap;
  if (tail_cs != nullptr && tail_ld < tail_cap) return -1;
  if (!zeroed) {   // (zeroed: the caller's workspace, cleared by prune_qquant)
    hipError_t e = hipMemsetAsync(dense, 0, sizeof(int), st);
    if (e == hipSuccess) e = hipMemsetAsync(blkmax, 0, sizeof(int) * (size_t)n_rblk, st);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(prune_route_kernel, dim3(NQ), dim3(256), 0, st, NQ, pre_s, tail_s,
                     k, thr_margin, sq, margin, thr0, cs_p, ci_p, cnt_p, cap_p, tshift,
                     rows_per_blk, n_rblk, T, thr, dense, est, blkmax,
                     RouteTail{tail_cs, tail_ci, tail_cnt, tail_cap, tail_off, tail_ld});
  hipLaunchKernelGGL(prune_route_sum_kernel, dim3((NQ + 3) / 4), dim3(256), 0, st, NQ, n_rblk, est,
                     blkmax, blk_limit, limit, dense);
  hipLaunchKernelGGL(prune_route_final_kernel, dim3(1), dim3(1024), 0, st, NQ, n_rblk, est, blkmax,
                     blk_limit, limit, max_list, dense, blk);
  return (int)hipGetLastError();
}
