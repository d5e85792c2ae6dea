// Streaming pruning scan (the first pass of the EXACT pruned search): the
// index's int8 or MX-fp4 image streamed from HBM straight into VGPRs, one wave per SIMD, no LDS
// ring and no barriers.  Round 5's replacement of index_scan_i8_kernel (index_i8.hip) for the
// plain int8 image and the MX-fp4 tier.
//
// Why (profiles/r4_scan_pmc/): the LDS-ring scan shares each row tile among 8 waves through LDS,
// so every 64-row tile costs a barrier, a fragment-read prologue and an emission block in which
// the two waves of a SIMD meet in lockstep; it ran 3,419 cycles per tile against an MFMA floor of
// 1,536 with waves parked 44 % of their cycles, and its MX-fp4 form moved 4.0 TB/s.  Here a wave
// holds its queries as resident B operands (256 MX-fp4 queries or 128 int8 queries = 192 VGPRs)
// and pulls 32-row sub-tiles of a FRAGMENT-MAJOR image: every 16-byte lane fragment of one
// MFMA k-step is contiguous, so one global_load_dwordx4 per k-step moves a whole 1 KiB piece and
// DEPTH sub-tiles stay in flight per wave (~50-80 KiB per CU).  Waves never wait on each other;
// the two waves of an int8 workgroup read the same rows (their second read hits L1/L2).
//
// MFMA shapes: v_mfma_i32_32x32x32_i8 and v_mfma_scale_f32_32x32x64_f8f6f4 (e2m1 x e2m1, block
// scales per lane): half the instructions of the 16x16 forms and 24 of every 32 issue cycles
// free for the emission test (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost').  The
// accumulator holds 16 rows of one query per lane (col = lane & 31, row = (r & 3) + 8 (r >> 2) +
// 4 (lane >> 5)), so the test per 32 x 32 block is 8 v_max3 + 1 compare (MX-fp4: the MFMA applies
// the block scales, the accumulator IS the estimate) or 16 cvt + 16 mul first (int8: each row's
// own scale, carried in the sub-tile record).  Only a block with a hit branches to the per-row
// emission, which stages (score, row, query) in a per-wave LDS buffer and reserves slots with one
// atomic per staged candidate, 64 at a time.
//
// Images (quant_stream_*_kernel below), per 32-row sub-tile g:
//   int8  : [128 B: the 32 row scales, lane-half h = (r >> 2) & 1 major, index (r & 3) + 4 (r >> 3)]
//           [NKS x 1 KiB: k-step ks, lane l: row l & 31, bytes 32 ks + 16 (l >> 5) .. + 16]
//   MX-fp4: [NKS x 1 KiB, the same byte map over the 192 nibble bytes of a 384-wide row]
//           [NSC x 256 B: dword j of lane l = the e8m0 scales of k-steps 4 j .. 4 j + 3 (byte
//            ks % 4) of row l & 31, block 2 ks + (l >> 5)]
// The int8 image keeps ONE scale per sub-tile (SDim::HDR), so an append into a partly filled
// sub-tile re-quantises the rows already there (and may raise E).  The pruned search therefore
// scans only whole sub-tiles below its visible count and lists the partial sub-tile's rows as
// candidates of every query (prepass.hip prefill_candidates; index/shard.py _pruned_end): a scan
// in flight never reads a sub-tile a concurrent append rewrites.  The MX images are per row.
#include "scan_common.h"

namespace symb {

enum : int { SF_I8 = 0, SF_MX4 = 1, SF_MX6 = 2 };

typedef __attribute__((ext_vector_type(4))) int i32x4s;
typedef __attribute__((ext_vector_type(6))) int i32x6s;
typedef int i32x3a __attribute__((ext_vector_type(3), aligned(4)));   // a 12-byte, dword-aligned piece
typedef __attribute__((ext_vector_type(8))) int i32x8s;
typedef __attribute__((ext_vector_type(16))) int i32x16s;
typedef __attribute__((ext_vector_type(16))) float f32x16s;

template <int FMT, int D>
struct SDim {
  static constexpr int KE = FMT == SF_I8 ? 32 : 64;             // k elements per MFMA k-step
  static constexpr int NKS = D / KE;                             // k-steps per row
  static constexpr int LB = FMT == SF_MX6 ? 24 : 16;              // bytes per lane per k-step
  static constexpr int RB = NKS * 2 * LB;                        // (query) image bytes per row
  static constexpr int NSC = FMT == SF_I8 ? 0 : (NKS + 3) / 4;   // block-scale dwords per lane
  // int8: ONE scale per 32-row sub-tile (f32 at byte 0 of a 16-byte header): the hit test takes
  // max_r acc[r] before its single multiply (per-row scales cost 16 cvt + 16 mul per set and
  // sub-tile, 8 % of the 100M x 384 scan; profiles/r5_scan/ab_i8_tile_scale.jsonl).  The bound
  // E = max |x - x~| is a maximum over rows either way, so pruning keeps its power.
  static constexpr int HDR = FMT == SF_I8 ? 16 : 0;
  // per k-step 64 lanes x LB bytes; MX-fp6: two 768-byte planes of 12 bytes per lane
  static constexpr int FRAG = NKS * 64 * LB;
  static constexpr int REC = HDR + FRAG + NSC * 256;             // bytes per 32-row sub-tile
  static_assert(D % KE == 0 && (D == 384 || D == 768 || D == 1024), "stream image row width");
};

// Scan geometry: SETS 32-query sets per wave (resident B operands: SETS x NKS x 4 VGPRs), NW
// waves per workgroup on the same rows, DEPTH sub-tiles in flight per wave.  MX-fp4 384: 256
// queries per wave; the wider rows hold fewer resident sets (1024: int8 one set, 4 waves = 128
// queries per workgroup).  (Round 5's A/B forms -- a 128-query MX-fp4 form, one sub-tile
// deeper / shallower in flight, the 16 x 16 x 64 int8 MFMA shape and an LDS-landing ring --
// measured slower or equal and were removed in round 6.)
template <int FMT, int D>
struct SGeo {
  static constexpr int NKS = SDim<FMT, D>::NKS;
  static constexpr int SETS = FMT == SF_MX4 ? (D == 384 ? 8 : D == 1024 ? 2 : 4)
                            : FMT == SF_MX6 ? (D == 384 ? 4 : 2)
                                            : (D == 384 ? 4 : D == 768 ? 2 : 1);
  static constexpr int NW0 = 256 / (SETS * 32) > 0 ? 256 / (SETS * 32) : 1;
  static constexpr int NW = NW0 > 4 ? 4 : NW0;
  static constexpr int DEPTH = FMT == SF_MX4 ? 3 : 2;
  static constexpr int QPB = SETS * 32 * NW;                      // queries per workgroup
  static constexpr int STW = 512;                                 // staged candidates per wave
  static constexpr int STAGE = STW * 10;
  static_assert(SETS * NKS * SDim<FMT, D>::LB / 4 <= 192, "resident query operands");
  static_assert(NW >= 1 && NW <= 4, "waves per workgroup");
};

__device__ __forceinline__ float max16(const float (&v)[16]) {
  float a = __builtin_fmaxf(__builtin_fmaxf(v[0], v[1]), v[2]);   // v_max3_f32 chains
  float b = __builtin_fmaxf(__builtin_fmaxf(v[3], v[4]), v[5]);
  float c = __builtin_fmaxf(__builtin_fmaxf(v[6], v[7]), v[8]);
  float d = __builtin_fmaxf(__builtin_fmaxf(v[9], v[10]), v[11]);
  float e = __builtin_fmaxf(__builtin_fmaxf(v[12], v[13]), v[14]);
  a = __builtin_fmaxf(__builtin_fmaxf(a, b), c);
  d = __builtin_fmaxf(__builtin_fmaxf(d, e), v[15]);
  return __builtin_fmaxf(a, d);
}

// img: the stream image (SDim::REC bytes per 32-row sub-tile); Q: the queries' row-major image
// (int8 [NQ][D] from prune_qquant, or MX-fp4 nibbles [NQ][D / 2] from quant_stream_mx4 with
// qsc = its scale record [NQ][2 NSC] dwords); thr[q]: emit a row iff its estimate >= thr (int8:
// (q8 . x8) * sx >= thr, thr already divided by the query's scale; MX-fp4: the scaled dot).
// Workgroup lb = (row block rb, query block qb); cand_n must be zeroed by the caller.
// ABL (timing ablations, wrong results): 1 = no emission test (the accumulators kept live),
// 2 = no sub-tile loads after the prologue (the first DEPTH sub-tiles re-used).
template <int FMT, int D, int ABL = 0>
__global__ __launch_bounds__((64 * SGeo<FMT, D>::NW), 1) void scan_stream_kernel(
    const uint8_t* __restrict__ img, int n_valid, int rows_per_blk, const uint8_t* __restrict__ Q,
    const uint32_t* __restrict__ qsc, int NQ, int n_qblk, int xcd, const float* __restrict__ thr_in,
    float* __restrict__ cand_s, int* __restrict__ cand_i, int* __restrict__ cand_n, int cap,
    const int* __restrict__ skip, const int* __restrict__ gate, int gate_want,
    int* __restrict__ runs, const uint8_t* __restrict__ cent4, const uint32_t* __restrict__ centqs,
    const float* __restrict__ centR, const float* __restrict__ bounds4) {
  using S = SDim<FMT, D>;
  using G = SGeo<FMT, D>;
  constexpr int NKS = S::NKS, NSC = S::NSC ? S::NSC : 1, REC = S::REC;
  constexpr int SETS = G::SETS, DEPTH = G::DEPTH, STW = G::STW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int lb = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qb = lb % n_qblk, rb = lb / n_qblk;
  if (gate != nullptr && *gate != gate_want) return;   // (no barrier in this kernel)
  // runs (optional): counts the launches that passed the gate (the MX-fp4 tier's batches)
  if (runs != nullptr && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(runs, 1);
  if (skip != nullptr && skip[rb] != 0) return;   // (routed to the bf16 scan)
  const int row_begin = rb * rows_per_blk;
  const int row_end = min(row_begin + rows_per_blk, n_valid);
  if (row_end <= row_begin) return;
  const int g0 = row_begin >> 5, ns = (row_end - row_begin + 31) >> 5;
  const int qw = (qb * G::NW + wave) * SETS * 32;   // the wave's first query

  // ---- resident queries: B operand of set s, k-step ks = query qw + 32 s + (lane & 31), bytes
  //      32 ks + 16 h .. + 16 of its row-major image ----
  using FragT = std::conditional_t<FMT == SF_MX6, i32x6s, i32x4s>;
  // a k-step's lane piece: 16 bytes, or (MX-fp6) 24 bytes as two dword-aligned 12-byte halves
  auto frag_at = [](const uint8_t* p, int second) -> FragT {
    if constexpr (FMT == SF_MX6) {
      const i32x3a a = *reinterpret_cast<const i32x3a*>(p);
      const i32x3a b = *reinterpret_cast<const i32x3a*>(p + second);
      return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5);
    } else {
      (void)second;
      return *reinterpret_cast<const i32x4s*>(p);
    }
  };
  FragT qf[SETS][NKS];
  uint32_t qs[SETS][NSC];
  float thr[SETS];
#pragma unroll
  for (int s = 0; s < SETS; ++s) {
    const int q = qw + 32 * s + (lane & 31);
    const int qq = min(q, NQ - 1);
    const uint8_t* qp = Q + (size_t)qq * S::RB + S::LB * h;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[s][ks] = frag_at(qp + 2 * S::LB * ks, 12);
#pragma unroll
    for (int j = 0; j < NSC; ++j) {
      if constexpr (FMT != SF_I8)
        qs[s][j] = qsc[(size_t)qq * 2 * NSC + h * NSC + j];
      else
        qs[s][j] = 0u;
    }
    thr[s] = q < NQ ? thr_in[q] : INFINITY;
  }

  // ---- the centroid test (MX-fp4, optional; mx4_centroids_kernel): one extra B operand holding
  //      the centroids of the wave's SETS query sets (lane j: centroid j), each set's bound
  //      R_s X4 and smallest threshold.  A sub-tile whose rows all satisfy
  //      c~_s . x~ + R_s X4 < min_q thr[q] cannot emit for set s, whose MFMAs are then skipped --
  //      near-duplicate query batches (the headline's) skip every set on almost every sub-tile ----
  const bool cent_on = FMT == SF_MX4 && cent4 != nullptr;
  i32x4s cf[FMT == SF_MX4 ? NKS : 1];
  uint32_t cqs[NSC];
  float cbound[SETS], tmin[SETS];
  if constexpr (FMT == SF_MX4) {
    if (cent_on) {
      const int gs0 = (qb * G::NW + wave) * SETS, n_sets = (NQ + 31) / 32;
      const int gs = min(gs0 + min(lane & 31, SETS - 1), n_sets - 1);
      const uint8_t* cp = cent4 + (size_t)gs * S::RB + 16 * h;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) cf[ks] = *reinterpret_cast<const i32x4s*>(cp + 32 * ks);
#pragma unroll
      for (int j = 0; j < NSC; ++j) cqs[j] = centqs[(size_t)gs * 2 * NSC + h * NSC + j];
      const float x4 = bounds4[1];
#pragma unroll
      for (int s = 0; s < SETS; ++s) {
        cbound[s] = centR[min(gs0 + s, n_sets - 1)] * x4 * 1.0001f + 1e-4f;
        float t = thr[s];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) t = fminf(t, __shfl_xor(t, o));
        tmin[s] = t;
      }
    }
  }

  // ---- per-wave candidate stage (LDS) ----
  char* stage = smem + wave * G::STAGE;
  float* st_s = reinterpret_cast<float*>(stage);
  int* st_r = reinterpret_cast<int*>(stage + STW * 4);
  uint16_t* st_q = reinterpret_cast<uint16_t*>(stage + STW * 8);
  int nst = 0;
  auto flush = [&]() {
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

  // ---- the sub-tile ring: fragments (+ row scales / block scales) of DEPTH sub-tiles ----
  const uint8_t* rec0 = img + (size_t)g0 * REC;
  FragT fk[DEPTH][NKS];
  uint32_t fsc[DEPTH][NSC];
  float fts[DEPTH];   // (int8) the sub-tile's scale
  auto load = [&](auto dc, int i) {
    constexpr int d = decltype(dc)::value;
    const uint8_t* r = rec0 + (size_t)min(i, ns - 1) * REC;   // (past the end: the last again)
    if constexpr (FMT == SF_I8) fts[d] = *reinterpret_cast<const float*>(r);
    // (MX-fp6: lane l's 24 bytes are 12 in the k-step's first 768-byte plane and 12 in its second)
    const uint8_t* f = r + S::HDR + (FMT == SF_MX6 ? 12 : 16) * lane;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) fk[d][ks] = frag_at(f + 64 * S::LB * ks, 768);
    if constexpr (FMT != SF_I8) {
#pragma unroll
      for (int j = 0; j < NSC; ++j)
        fsc[d][j] = *reinterpret_cast<const uint32_t*>(r + S::FRAG + 256 * j + 4 * lane);
    }
  };

  // int8: the 32 x 32 block's integer dot products (16 rows of one query per lane)
  auto acc_i8 = [&](auto dc, auto sc) {
    constexpr int d = decltype(dc)::value, s = decltype(sc)::value;
    i32x16s acc = {};
    if constexpr (FMT == SF_I8) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fk[d][ks], qf[s][ks], acc, 0, 0, 0);
    }
    return acc;
  };
  // the 32 x 32 block of set s over sub-tile slot d, as estimates (16 rows of one query)
  auto block = [&](auto dc, auto sc, float (&v)[16]) {
    constexpr int d = decltype(dc)::value, s = decltype(sc)::value;
    if constexpr (FMT == SF_MX4) {
      f32x16s acc = {};
      static_for<0, NKS>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        const i32x8s a = __builtin_shufflevector(fk[d][ks], (i32x4s){0, 0, 0, 0}, 0, 1, 2, 3, 4, 5, 6, 7);
        const i32x8s b = __builtin_shufflevector(qf[s][ks], (i32x4s){0, 0, 0, 0}, 0, 1, 2, 3, 4, 5, 6, 7);
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, ks & 3,
                                                              (int)fsc[d][ks >> 2], ks & 3,
                                                              (int)qs[s][ks >> 2]);
      });
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[r];
    } else if constexpr (FMT == SF_MX6) {   // e2m3 x e2m3 (cbsz / blgp 2), six-dword operands
      f32x16s acc = {};
      static_for<0, NKS>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        const i32x8s a = __builtin_shufflevector(fk[d][ks], fk[d][ks], 0, 1, 2, 3, 4, 5, -1, -1);
        const i32x8s b = __builtin_shufflevector(qf[s][ks], qf[s][ks], 0, 1, 2, 3, 4, 5, -1, -1);
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 2, 2, ks & 3,
                                                              (int)fsc[d][ks >> 2], ks & 3,
                                                              (int)qs[s][ks >> 2]);
      });
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[r];
    } else {
      const i32x16s acc = acc_i8(dc, sc);
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = (float)acc[r] * fts[d];
    }
  };

  // (a conservative integer pre-test -- max_r acc[r] times the largest of the 16 row scales --
  // was measured 1.8x slower: the row scales spread +-30 %, so it let through most blocks and
  // their exact re-test recomputed the MFMAs; profiles/r5_scan/)
  auto process = [&](auto dc, int i) {
    constexpr int d = decltype(dc)::value;
    const int row0 = (g0 + i) * 32 + 4 * h;   // + (r & 3) + 8 (r >> 2)
    uint32_t hm = 0;                          // sets with a hit in this lane
    uint32_t pass = ~0u;                      // sets the centroid test could not rule out
    if constexpr (FMT == SF_MX4) {
      if (cent_on) {
        f32x16s acc = {};
        static_for<0, NKS>([&](auto kc) {
          constexpr int ks = decltype(kc)::value;
          const i32x8s a = __builtin_shufflevector(fk[d][ks], (i32x4s){0, 0, 0, 0}, 0, 1, 2, 3, 4, 5, 6, 7);
          const i32x8s b = __builtin_shufflevector(cf[ks], (i32x4s){0, 0, 0, 0}, 0, 1, 2, 3, 4, 5, 6, 7);
          acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, ks & 3,
                                                                (int)fsc[d][ks >> 2], ks & 3,
                                                                (int)cqs[ks >> 2]);
        });
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[r];
        float m = max16(v);
        m = fmaxf(m, __shfl_xor(m, 32));      // lane j: centroid j over the 32 rows
        pass = 0u;
#pragma unroll
        for (int s = 0; s < SETS; ++s)
          pass |= (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), s)) + cbound[s] >=
                           tmin[s]
                       ? 1u
                       : 0u)
                  << s;
      }
    }
    if constexpr (ABL == 1) {
      static_for<0, SETS>([&](auto sc) {
        if (!((pass >> decltype(sc)::value) & 1u)) return;
        float v[16];
        block(dc, sc, v);
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" ::"v"(v[r]));
      });
      return;
    } else {
      static_for<0, SETS>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if (!((pass >> s) & 1u)) return;
        if constexpr (FMT == SF_I8) {   // (the sub-tile's scale > 0 keeps the order)
          const i32x16s acc = acc_i8(dc, sc);
          int m = max(max(acc[0], acc[1]), acc[2]);
#pragma unroll
          for (int r = 3; r < 15; r += 2) m = max(max(m, acc[r]), acc[r + 1]);
          m = max(m, acc[15]);
          hm |= ((float)m * fts[d] >= thr[s] ? 1u : 0u) << s;
        } else {
          float v[16];
          block(dc, sc, v);
          hm |= (max16(v) >= thr[s] ? 1u : 0u) << s;
        }
      });
    }
    if (__builtin_amdgcn_ballot_w64(hm != 0)) {   // rare: recompute the hit sets, emit per row
      static_for<0, SETS>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if (!__builtin_amdgcn_ballot_w64((hm >> s) & 1)) return;
        float v[16];
        block(dc, sc, v);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = row0 + (r & 3) + 8 * (r >> 2);
          const int ql = 32 * s + (lane & 31);
          const bool p = v[r] >= thr[s] && row < row_end;
          const uint64_t m = __builtin_amdgcn_ballot_w64(p);
          if (m) {
            if (nst > STW - 64) flush();
            const int idx = nst + (int)__builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            if (p) {
              st_s[idx] = v[r];
              st_r[idx] = row;
              st_q[idx] = (uint16_t)ql;
            }
            nst += __builtin_popcountll(m);
          }
        }
      });
    }
  };

  // prologue: DEPTH sub-tiles in flight, then use one / refill its slot
  static_for<0, DEPTH>([&](auto dc) { load(dc, decltype(dc)::value); });
  // (the last round may run past ns: those slots re-read the last sub-tile and emit nothing, as
  // every row they name is >= row_end -- a branch-free body keeps the loads' waits counted)
  for (int i0 = 0; i0 < ns; i0 += DEPTH) {
    static_for<0, DEPTH>([&](auto dc) {
      constexpr int d = decltype(dc)::value;
      process(dc, i0 + d);
      if (ABL != 2) load(dc, i0 + d + DEPTH);
    });
  }
  if (nst) flush();
}

// ---------------------------------------------------------------------------------------------
// Image writers.  Row r of sub-tile g = r >> 5, rr = r & 31; row byte b (k-step ks = b >> 5,
// half hh = (b >> 4) & 1, byte bi = b & 15) sits at REC g + HDR + 1024 ks + 16 (32 hh + rr) + bi.

__device__ __forceinline__ size_t stream_frag_off(int rec, int hdr, int r, int b) {
  const int rr = r & 31;
  return (size_t)(r >> 5) * rec + hdr + 1024 * (b >> 5) + 16 * (32 * ((b >> 4) & 1) + rr) + (b & 15);
}

// The int8 stream image of one whole 32-row sub-tile g of the bf16 rows X: the tile's scale
// s = max |x| / 127 over its 32 rows (an all-zero tile: 1) at header byte 0, every row's codes
// round(x / s); returns (max_r |x_r - x~_r|, max_r |x~_r|) in every thread.  One 512-thread
// workgroup: wave w quantises rows w, w + 8, w + 16, w + 24; lane l holds elements PER l ..
// PER l + PER - 1 of a row.
template <int D>
__device__ __forceinline__ void i8_stream_tile(const __bf16* __restrict__ X, int g,
                                               uint8_t* __restrict__ img, float& en_max,
                                               float& nn_max) {
  using S = SDim<SF_I8, D>;
  constexpr int PER = D / 64;
  __shared__ float red[3][8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float x[4][PER];
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t* xp =
        reinterpret_cast<const uint32_t*>(X + (size_t)(32 * g + w + 8 * k) * D + PER * lane);
#pragma unroll
    for (int i = 0; i < PER / 2; ++i) {
      const uint32_t u = xp[i];
      x[k][2 * i] = __uint_as_float(u << 16);
      x[k][2 * i + 1] = __uint_as_float(u & 0xffff0000u);
      amax = fmaxf(amax, fmaxf(fabsf(x[k][2 * i]), fabsf(x[k][2 * i + 1])));
    }
  }
  amax = wave_max(amax);
  if (lane == 0) red[0][w] = amax;
  __syncthreads();
  amax = red[0][0];
#pragma unroll
  for (int i = 1; i < 8; ++i) amax = fmaxf(amax, red[0][i]);
  const float sc = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / sc;
  float em = 0.f, nm = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = 32 * g + w + 8 * k;
    float e2 = 0.f, n2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int qv = max(-127, min(127, (int)rintf(x[k][i] * inv)));
      const float xt = (float)qv * sc;
      e2 += (x[k][i] - xt) * (x[k][i] - xt);
      n2 += xt * xt;
      img[stream_frag_off(S::REC, S::HDR, row, PER * lane + i)] = (uint8_t)(qv & 0xff);
    }
    em = fmaxf(em, sqrtf(wave_sum(e2)));
    nm = fmaxf(nm, sqrtf(wave_sum(n2)));
  }
  if (threadIdx.x < 4)
    reinterpret_cast<float*>(img + (size_t)g * S::REC)[threadIdx.x] = threadIdx.x ? 0.f : sc;
  if (lane == 0) {
    red[1][w] = em;
    red[2][w] = nm;
  }
  __syncthreads();
  en_max = red[1][0];
  nn_max = red[2][0];
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    en_max = fmaxf(en_max, red[1][i]);
    nn_max = fmaxf(nn_max, red[2][i]);
  }
}

__device__ __forceinline__ float half_max32(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int e2m1_code_s(float a, float& q) {   // a = |x| / s <= 6
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

__device__ __forceinline__ void store3(uint8_t* p, uint32_t v) {   // bytes 0-2 of v, little-endian
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
}

__device__ __forceinline__ int e2m3_code_s(float a, float& q) {   // a = |x| / s <= 7.5
  // OCP e2m3 (bias 1): code 8 E + m; steps 1/8 below 2, 1/4 below 4, 1/2 up to 7.5
  if (a < 2.f) {
    q = rintf(a * 8.f) * 0.125f;
    return (int)(q * 8.f);               // 0 .. 16 (16 = 2.0)
  }
  if (a < 4.f) {
    q = rintf(a * 4.f) * 0.25f;
    return (int)(q * 4.f) + 8;           // 16 .. 24
  }
  q = fminf(rintf(a * 2.f) * 0.5f, 7.5f);
  return (int)(q * 2.f) + 16;            // 24 .. 31
}

// e8m0 exponent of an MX block: the smallest e with amax <= top 2^e (top = the element format's
// largest value: 6 for e2m1, 7.5 for e2m3); -127 for an all-zero block
__device__ __forceinline__ int mx_block_exp(float amax, float top) {
  if (!(amax > 0.f)) return -127;
  int k;
  frexpf(amax / top, &k);                // amax / top in [2^(k-1), 2^k)
  int e = k;
  if (amax <= top * ldexpf(1.f, k - 1)) e = k - 1;
  if (amax > top * ldexpf(1.f, e)) ++e;  // (guard the division's rounding)
  return max(e, -127);
}

// One row's MX image (FMT SF_MX4: OCP e2m1 nibbles, SF_MX6: OCP e2m3 6-bit codes): every 32-dim
// block b gets s_b = 2^ceil(log2(max |x_b| / top)) (an e8m0 byte) and each element the nearest
// code of x / s_b -- quant_rows_mx4_kernel's numbers for fp4.  Codes are packed little-endian per
// lane piece (element j of a block at bits [w j, w j + w), w = 4 / 6).  One wave, lane l holds
// dims l + 64 m (block 2 m + (l >> 5), element l & 31).
// Xq == nullptr: into the stream image img at row `row` (fp6: the piece's bytes 0-11 in the
// k-step's first 768-byte plane, 12-23 in its second); else the query layout: row-major pieces
// Xq [.][RB] (RB = D / 2 or 3 D / 4 bytes) and the scale record QS [.][2 NSC] dwords (dword
// h NSC + j, byte b = block 2 (4 j + b) + h: the scan's per-lane B scales).
// en / nn / xn = |x - x~| / |x~| / |x|.
template <int FMT, int D, bool QUERY>
__device__ __forceinline__ void mx_stream_row(const __bf16* __restrict__ xrow, int row,
                                              uint8_t* __restrict__ img, uint8_t* __restrict__ Xq,
                                              uint32_t* __restrict__ QS, float& en, float& nn,
                                              float& xn) {
  using S = SDim<FMT, D>;
  constexpr int M = D / 64, NSC = S::NSC;
  constexpr float TOP = FMT == SF_MX6 ? 7.5f : 6.f;
  const int lane = threadIdx.x & 63, j = lane & 31, hh = lane >> 5;
  constexpr bool query = QUERY;
  const uint16_t* xp = reinterpret_cast<const uint16_t*>(xrow);
  // this row's scale record (queries): half 0's words built in lanes 0-31, half 1's in 32-63
  uint32_t scw[NSC];
#pragma unroll
  for (int i = 0; i < NSC; ++i) scw[i] = 0u;
  float e2 = 0.f, n2 = 0.f, x2 = 0.f;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float x = __uint_as_float((uint32_t)xp[lane + 64 * m] << 16);
    const float amax = half_max32(fabsf(x));
    const int e = mx_block_exp(amax, TOP);
    const float sc = ldexpf(1.f, e);
    float qv = 0.f;
    int c = 0;
    if (amax > 0.f) {
      if constexpr (FMT == SF_MX6) c = e2m3_code_s(fabsf(x) * ldexpf(1.f, -e), qv);
      else c = e2m1_code_s(fabsf(x) * ldexpf(1.f, -e), qv);
    }
    const int code = c | (x < 0.f && c ? (FMT == SF_MX6 ? 32 : 8) : 0);
    const float xt = (x < 0.f ? -qv : qv) * sc;
    e2 += (x - xt) * (x - xt);
    n2 += xt * xt;
    x2 += x * x;
    if constexpr (FMT == SF_MX6) {
      // 4 codes = 3 bytes, written by the group's first lane (byte 3 (j / 4) of the piece)
      const uint32_t v = (uint32_t)code | ((uint32_t)__shfl_down(code, 1) << 6) |
                         ((uint32_t)__shfl_down(code, 2) << 12) |
                         ((uint32_t)__shfl_down(code, 3) << 18);
      // (QUERY a template argument: both stores in one function crashed hipcc's inliner)
      if ((j & 3) == 0) {
        const int g = j >> 2;
        if constexpr (query)
          store3(Xq + (size_t)row * S::RB + 48 * m + 24 * hh + 3 * g, v);
        else
          store3(img + (size_t)(row >> 5) * S::REC + 1536 * m + 768 * (g >> 2) +
                     12 * (32 * hh + (row & 31)) + 3 * (g & 3),
                 v);
      }
    } else {
      const int hi = __shfl_down(code, 1);
      const uint8_t byte = (uint8_t)(code | (hi << 4));
      const int bj = (lane >> 1) + 32 * m;     // row byte of the even lane's pair
      if ((lane & 1) == 0) {
        if constexpr (query) Xq[(size_t)row * (D / 2) + bj] = byte;
        else img[stream_frag_off(S::REC, 0, row, bj)] = byte;
      }
    }
    if constexpr (query) {
      scw[m >> 2] |= (uint32_t)(e + 127) << (8 * (m & 3));
    } else if (j == 0) {
      img[(size_t)(row >> 5) * S::REC + S::FRAG + 256 * (m >> 2) + 4 * (32 * hh + (row & 31)) +
          (m & 3)] = (uint8_t)(e + 127);
    }
  }
  en = sqrtf(wave_sum(e2));
  nn = sqrtf(wave_sum(n2));
  xn = sqrtf(wave_sum(x2));
  if constexpr (query) {
    // lanes 0 and 32 built the two halves' scale words (identical within a half-wave)
#pragma unroll
    for (int i = 0; i < NSC; ++i) {
      const uint32_t lo = (uint32_t)__shfl((int)scw[i], 0), hi = (uint32_t)__shfl((int)scw[i], 32);
      if (lane == 0) {
        QS[(size_t)row * 2 * NSC + i] = lo;
        QS[(size_t)row * 2 * NSC + NSC + i] = hi;
      }
    }
  }
}

template <int D>
__device__ __forceinline__ void mx4_stream_row(const __bf16* __restrict__ xrow, int row,
                                               uint8_t* __restrict__ img, uint8_t* __restrict__ Xq,
                                               uint32_t* __restrict__ QS, float& en, float& nn,
                                               float& xn) {
  if (Xq != nullptr) mx_stream_row<SF_MX4, D, true>(xrow, row, img, Xq, QS, en, nn, xn);
  else mx_stream_row<SF_MX4, D, false>(xrow, row, img, Xq, QS, en, nn, xn);
}

__device__ __forceinline__ float e2m1_value(int c) {   // 4-bit code (sign bit 3) -> value
  const int m = c & 7;
  const float v = m < 5 ? 0.5f * m : (m == 5 ? 3.f : m == 6 ? 4.f : 6.f);
  return (c & 8) ? -v : v;
}

// Element d of an MX-fp4 query image (quant_stream_mx4 query mode: row-major nibbles Xq [.][D/2],
// scale record QS [.][2 NSC] dwords, dword h NSC + j byte b = block 2 (4 j + b) + h).
template <int D>
__device__ __forceinline__ float mx4_query_elem(const uint8_t* __restrict__ Xq,
                                                const uint32_t* __restrict__ QS, int q, int d) {
  constexpr int NSC = SDim<SF_MX4, D>::NSC;
  const int byte = Xq[(size_t)q * (D / 2) + (d >> 1)];
  const int nib = (d & 1) ? byte >> 4 : byte & 15;
  const int k = d >> 5, jb = k >> 1;
  const int e8 = (QS[(size_t)q * 2 * NSC + (k & 1) * NSC + (jb >> 2)] >> (8 * (jb & 3))) & 255;
  return e2m1_value(nib) * ldexpf(1.f, e8 - 127);
}

// The query-side bound of the MX-fp4 tier (scan_stream_kernel's centroid test): for each set of
// 32 consecutive queries, the MX-fp4 image c~ of the mean of their decoded images and
// R = max_q |q~ - c~|, so that every query q of the set and every row x satisfy
//   q~ . x~ = c~ . x~ + (q~ - c~) . x~ <= c~ . x~ + R |x~| <= c~ . x~ + R X4.
// Four waves per set, wave w decoding queries w, w + 4, .. of it (8 independent loads each,
// kept in registers for the radius pass; one wave walking all 32 serially took 66 us per search
// beside the encoder, profiles/r5_step/); C4 / CS: the centroids' image in the query layout,
// R [n_sets].
template <int D>
__global__ __launch_bounds__(256) void mx4_centroids_kernel(const uint8_t* __restrict__ Xq,
                                                            const uint32_t* __restrict__ QS, int NQ,
                                                            uint8_t* __restrict__ C4,
                                                            uint32_t* __restrict__ CS,
                                                            float* __restrict__ R) {
  constexpr int M = D / 64, NSC = SDim<SF_MX4, D>::NSC, QW = 8;
  __shared__ float part[4][D];
  __shared__ float rmax[4];
  const int set = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q0 = set * 32, nq = min(32, NQ - q0);
  float xv[QW][M];
  float c[M];
#pragma unroll
  for (int m = 0; m < M; ++m) c[m] = 0.f;
#pragma unroll
  for (int i = 0; i < QW; ++i) {
    const int q = w + 4 * i;
    const int qq = q0 + min(q, nq - 1);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      xv[i][m] = mx4_query_elem<D>(Xq, QS, qq, lane + 64 * m);
      if (q < nq) c[m] += xv[i][m];
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) part[w][lane + 64 * m] = c[m];
  __syncthreads();
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int d = lane + 64 * m;
    c[m] = (part[0][d] + part[1][d]) + (part[2][d] + part[3][d]);   // (the same sum in every wave)
  }
  uint32_t scw[NSC];
#pragma unroll
  for (int i = 0; i < NSC; ++i) scw[i] = 0u;
  float ct[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float x = c[m] / (float)max(nq, 1);
    const float amax = half_max32(fabsf(x));
    const int e = mx_block_exp(amax, 6.f);
    float qv;
    const int cd = amax > 0.f ? e2m1_code_s(fabsf(x) * ldexpf(1.f, -e), qv) : (qv = 0.f, 0);
    const int code = cd | (x < 0.f && cd ? 8 : 0);
    ct[m] = e2m1_value(code) * ldexpf(1.f, e);   // (the value the image holds)
    const int hi = __shfl_down(code, 1);
    if (w == 0 && (lane & 1) == 0)
      C4[(size_t)set * (D / 2) + (lane >> 1) + 32 * m] = (uint8_t)(code | (hi << 4));
    scw[m >> 2] |= (uint32_t)(e + 127) << (8 * (m & 3));
  }
#pragma unroll
  for (int i = 0; i < NSC; ++i) {
    const uint32_t lo = (uint32_t)__shfl((int)scw[i], 0), hi = (uint32_t)__shfl((int)scw[i], 32);
    if (w == 0 && lane == 0) {
      CS[(size_t)set * 2 * NSC + i] = lo;
      CS[(size_t)set * 2 * NSC + NSC + i] = hi;
    }
  }
  float r2 = 0.f;
#pragma unroll
  for (int i = 0; i < QW; ++i) {
    float d2 = 0.f;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float d = xv[i][m] - ct[m];
      d2 += d * d;
    }
    d2 = wave_sum(d2);
    if (w + 4 * i < nq) r2 = fmaxf(r2, d2);
  }
  if (lane == 0) rmax[w] = r2;
  __syncthreads();
  if (threadIdx.x == 0)   // (rounding of the sums above)
    R[set] = sqrtf(fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]))) * 1.0001f + 1e-6f;
}

// raise bounds[0..1] to the maxima of (a, b) over the workgroup's 4 waves (idle waves pass 0)
__device__ __forceinline__ void raise_bounds2(float* bounds, float a, float b) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = a;
    red[1][w] = b;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const float m = fmaxf(fmaxf(red[threadIdx.x][0], red[threadIdx.x][1]),
                          fmaxf(red[threadIdx.x][2], red[threadIdx.x][3]));
    atomicMax(reinterpret_cast<int*>(bounds) + threadIdx.x, __float_as_int(m));
  }
}

// int8 stream image of whole sub-tiles of the bf16 rows X (i8_stream_tile): tiles g_lo +
// blockIdx.x, or (rows != nullptr) the tile of listed row rows[blockIdx.x] -- a tile listed twice
// is written twice with the same bytes; bounds (2 floats) raised to (max |x - x~|, max |x~|).
template <int D>
__global__ __launch_bounds__(512) void quant_stream_i8_kernel(const __bf16* __restrict__ X, int g_lo,
                                                              const int* __restrict__ rows,
                                                              uint8_t* __restrict__ img,
                                                              float* __restrict__ bounds) {
  const int g = rows ? rows[blockIdx.x] >> 5 : g_lo + blockIdx.x;
  float en, nn;
  i8_stream_tile<D>(X, g, img, en, nn);
  if (threadIdx.x < 2) atomicMax(reinterpret_cast<int*>(bounds) + threadIdx.x, __float_as_int(threadIdx.x ? nn : en));
}

// MX-fp4 / MX-fp6 stream image of bf16 rows (margin == nullptr: rows [r0, r0 + n) or the listed
// rows into img, bounds[0..1] raised to (E, X)) or the query image (margin != nullptr: Xq / QS for
// rows 0 .. n - 1 and margin = |q| E + |q - q~| X + 1e-5 from bounds).  One wave per row.
template <int FMT, int D>
__global__ __launch_bounds__(256) void quant_stream_mx_kernel(
    const __bf16* __restrict__ X, int r0, const int* __restrict__ rows, int n,
    uint8_t* __restrict__ img, uint8_t* __restrict__ Xq, uint32_t* __restrict__ QS,
    float* __restrict__ bounds, float* __restrict__ margin) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const bool query = margin != nullptr;
  float en = 0.f, nn = 0.f, xn = 0.f;
  if (query) {
    if (j >= n) return;   // (no barrier on the query path)
    mx_stream_row<FMT, D, true>(X + (size_t)j * D, j, nullptr, Xq, QS, en, nn, xn);
    if ((threadIdx.x & 63) == 0) margin[j] = xn * bounds[0] + en * bounds[1] + 1e-5f;
    return;
  }
  if (j < n) {
    const int row = rows ? rows[j] : r0 + j;
    mx_stream_row<FMT, D, false>(X + (size_t)row * D, row, img, nullptr, nullptr, en, nn, xn);
  }
  raise_bounds2(bounds, en, nn);
}

// An append of n unit bf16 rows at row r0: the rows themselves (src -> rows), their MX-fp4 stream
// image (img4, bounds b4[0..1]) and MX-fp6 stream image (img6, b6) -- either image may be absent
// (nullptr).  One wave per row.  (The int8 image's sub-tiles follow in a second launch: their
// shared scale needs every row of the tile written first.)
template <int D, bool FP6>
__global__ __launch_bounds__(256) void append_rows_kernel(const __bf16* __restrict__ src, int n,
                                                          __bf16* __restrict__ rows, int r0,
                                                          uint8_t* __restrict__ img4,
                                                          float* __restrict__ b4,
                                                          uint8_t* __restrict__ img6,
                                                          float* __restrict__ b6) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  float e4 = 0.f, n4 = 0.f, x4 = 0.f, e6 = 0.f, n6 = 0.f;
  if (j < n) {
    const __bf16* xr = src + (size_t)j * D;
    // the bf16 row: D * 2 bytes as 4-byte words, D / 128 per lane
    const uint32_t* sp = reinterpret_cast<const uint32_t*>(xr);
    uint32_t* dp = reinterpret_cast<uint32_t*>(rows + (size_t)(r0 + j) * D);
#pragma unroll
    for (int i = 0; i < D / 128; ++i) dp[lane + 64 * i] = sp[lane + 64 * i];
    if (img4) mx4_stream_row<D>(xr, r0 + j, img4, nullptr, nullptr, e4, n4, x4);
    if constexpr (FP6) mx_stream_row<SF_MX6, D, false>(xr, r0 + j, img6, nullptr, nullptr, e6, n6, x4);
  }
  if (b4) raise_bounds2(b4, e4, n4);
  if constexpr (FP6) {
    __syncthreads();
    raise_bounds2(b6, e6, n6);
  }
}

// Probe of one v_mfma_scale_f32_32x32x64_f8f6f4 (tests: the operand bit layouts of the f8f6f4
// formats): a / b [64 lanes][8] dwords, sa / sb [64] e8m0 scale bytes (one dword each, byte 0),
// out [64][16] = the accumulator.  F: 0 fp8 e4m3, 2 fp6 e2m3, 3 fp6 e3m2, 4 fp4 e2m1.
template <int F>
__global__ __launch_bounds__(64) void mfma_f8f6f4_probe_kernel(const int* __restrict__ a,
                                                              const int* __restrict__ b,
                                                              const int* __restrict__ sa,
                                                              const int* __restrict__ sb,
                                                              float* __restrict__ out) {
  const int l = threadIdx.x;
  i32x8s av, bv;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    av[i] = a[l * 8 + i];
    bv[i] = b[l * 8 + i];
  }
  f32x16s acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, F, F, 0, sa[l], 0, sb[l]);
#pragma unroll
  for (int r = 0; r < 16; ++r) out[l * 16 + r] = acc[r];
}

}  // namespace symb

using namespace symb;

int symb_mfma_f8f6f4_probe(const int* a, const int* b, const int* sa, const int* sb, float* out,
                           int fmt, hipStream_t st) {
#define L(F_) hipLaunchKernelGGL(mfma_f8f6f4_probe_kernel<F_>, dim3(1), dim3(64), 0, st, a, b, sa, sb, out)
  if (fmt == 0) L(0);
  else if (fmt == 2) L(2);
  else if (fmt == 3) L(3);
  else if (fmt == 4) L(4);
  else return -1;
#undef L
  return (int)hipGetLastError();
}

// bytes per 32-row sub-tile of the stream image (form 0 = int8, 1 = MX-fp4, 2 = MX-fp6);
// 0 = unsupported
int symb_stream_rec_bytes(int dim, int form) {
#define R_(D_) (form == 2 ? SDim<SF_MX6, D_>::REC : form ? SDim<SF_MX4, D_>::REC : SDim<SF_I8, D_>::REC)
  if (form < 0 || form > 2) return 0;
  if (dim == 384) return R_(384);
  if (dim == 768) return R_(768);
  if (dim == 1024) return form == 2 ? 0 : R_(1024);
#undef R_
  return 0;
}

// the kernel's timing ablations (ABL above; wrong results) for benchmarks (symb_stream_config)
static int g_stream_abl = 0;
int symb_stream_config(int abl) {
  if (abl < 0 || abl > 2) return -1;
  g_stream_abl = abl;
  return 0;
}

// queries per workgroup and workgroups per CU (one wave per SIMD) of the stream scan
int symb_stream_geometry(int dim, int form, int* qpb, int* wgs_per_cu) {
#define G_(F, D_)                                    \
  do {                                               \
    *qpb = SGeo<F, D_>::QPB;                         \
    *wgs_per_cu = 4 / SGeo<F, D_>::NW;               \
    return 0;                                        \
  } while (0)
  if (dim == 384) {
    if (form == 2) G_(SF_MX6, 384);
    if (form) G_(SF_MX4, 384);
    G_(SF_I8, 384);
  }
  if (dim == 768) {
    if (form == 2) G_(SF_MX6, 768);
    if (form) G_(SF_MX4, 768);
    G_(SF_I8, 768);
  }
  if (form == 2) return -1;
  if (dim == 1024) {
    if (form) G_(SF_MX4, 1024);
    G_(SF_I8, 1024);
  }
#undef G_
  return -1;
}

struct CentArgs {   // the MX-fp4 centroid test's inputs (all nullptr: off)
  const void* c4;
  const void* cqs;
  const float* R;
  const float* b4;
};

template <int F, int D, int ABL = 0>
static int launch_stream(const void* img, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                         const void* qsc, int NQ, const float* thr, float* cand_s, int* cand_i,
                         int* cand_n, int cap, int xcd, hipStream_t st, const int* skip,
                         const int* gate, int gate_want, int* runs, CentArgs ca) {
  using G = SGeo<F, D>;
  const int n_qblk = (NQ + G::QPB - 1) / G::QPB;
  constexpr int lds = G::STAGE * G::NW;
  if (lds > 64 * 1024) set_max_lds<scan_stream_kernel<F, D, ABL>>(lds);
  hipLaunchKernelGGL((scan_stream_kernel<F, D, ABL>), dim3(n_rblk * n_qblk), dim3(64 * G::NW), lds,
                     st, (const uint8_t*)img, n_valid, rows_per_blk, (const uint8_t*)Q,
                     (const uint32_t*)qsc, NQ, n_qblk, xcd, thr, cand_s, cand_i, cand_n, cap, skip,
                     gate, gate_want, runs, (const uint8_t*)ca.c4, (const uint32_t*)ca.cqs, ca.R,
                     ca.b4);
  return (int)hipGetLastError();
}

// The stream scan over rows [0, n_valid) of a stream image covering alloc_rows rows (a multiple of
// 32 that covers n_valid).  rows_per_blk: a multiple of 32; n_rblk * rows_per_blk >= n_valid.
// form 0: int8 (Q = [NQ][dim] int8, qsc unused); 1: MX-fp4 (Q = [NQ][dim / 2] nibbles, qsc =
// [NQ][2 NSC] scale dwords).  cand_n is zeroed here iff zero_cnt (else the caller's zeroed
// workspace); gate != nullptr: the launch runs only if *gate == gate_want; runs (optional) is
// incremented once by a launch that ran.
int symb_index_scan_stream(const void* img, int n_valid, int alloc_rows, int rows_per_blk,
                           int n_rblk, const void* Q, const void* qsc, int NQ, const float* thr,
                           float* cand_s, int* cand_i, int* cand_n, int cap, int xcd,
                           hipStream_t st, const int* skip, int dim, int form, const int* gate,
                           int gate_want, int zero_cnt, int* runs, const void* cent4,
                           const void* centqs, const float* centR, const float* bounds4) {
  if (NQ <= 0) return 0;
  if (cent4 != nullptr && (form != 1 || centqs == nullptr || centR == nullptr || bounds4 == nullptr))
    return -1;
  const CentArgs ca{cent4, centqs, centR, bounds4};
  if ((dim != 384 && dim != 768 && dim != 1024) || form < 0 || form > 2) return -1;
  if (form == 2 && dim == 1024) return -1;
  if (form != 0 && qsc == nullptr) return -1;
  if (rows_per_blk % 32 || n_rblk <= 0 || thr == nullptr || cap <= 0 || n_valid <= 0) return -1;
  if ((long long)n_rblk * rows_per_blk < n_valid) return -1;
  if (alloc_rows % 32 || (long long)(n_valid + 31) / 32 * 32 > alloc_rows) return -1;
  if (zero_cnt) {
    hipError_t e = hipMemsetAsync(cand_n, 0, sizeof(int) * (size_t)NQ, st);
    if (e != hipSuccess) return (int)e;
  }
#define L(F, D_, A_) launch_stream<F, D_, A_>(img, n_valid, rows_per_blk, n_rblk, Q, qsc, NQ, thr, \
                                              cand_s, cand_i, cand_n, cap, xcd, st, skip, gate,   \
                                              gate_want, runs, ca)
#define LD(F, D_) (g_stream_abl == 1 ? L(F, D_, 1) : g_stream_abl == 2 ? L(F, D_, 2) : L(F, D_, 0))
  if (dim == 384) return form == 2 ? LD(SF_MX6, 384) : form ? LD(SF_MX4, 384) : LD(SF_I8, 384);
  if (dim == 768) return form == 2 ? LD(SF_MX6, 768) : form ? LD(SF_MX4, 768) : LD(SF_I8, 768);
  return form ? LD(SF_MX4, 1024) : LD(SF_I8, 1024);
#undef LD
#undef L
}

// The MX-fp4 tier's query-set centroids (mx4_centroids_kernel) of an MX-fp4 query image: C4
// [ceil(NQ / 32)][dim / 2], CS [.][2 NSC] dwords, R [.].
int symb_mx4_centroids(const void* Xq, const void* QS, int NQ, int dim, void* C4, void* CS,
                       float* R, hipStream_t st) {
  if (NQ <= 0) return 0;
  const int n_sets = (NQ + 31) / 32;
#define L(D_) hipLaunchKernelGGL(mx4_centroids_kernel<D_>, dim3(n_sets), dim3(256), 0, st,             \
                                 (const uint8_t*)Xq, (const uint32_t*)QS, NQ, (uint8_t*)C4,         \
                                 (uint32_t*)CS, R)
  if (dim == 384) L(384);
  else if (dim == 768) L(768);
  else if (dim == 1024) L(1024);
  else return -1;
#undef L
  return (int)hipGetLastError();
}

// Append n unit bf16 rows (src) at row r0 of the shard: rows, int8 stream image (img8 / b8),
// MX-fp4 stream image (img4 / b4) and MX-fp6 stream image (img6 / b6, not at 1024); an image
// pointer may be nullptr (then its bounds too).
int symb_quant_stream_i8(const void* X, int r0, const int* rows, int n, int dim, void* img,
                         float* bounds, hipStream_t st);

int symb_append_rows(const void* src, int n, int dim, void* rows, int r0, void* img8, float* b8,
                     void* img4, float* b4, void* img6, float* b6, hipStream_t st) {
  if (n <= 0) return 0;
  if (r0 < 0 || rows == nullptr || src == nullptr || (img8 && !b8) || (img4 && !b4) ||
      (img6 && !b6) || (img6 && dim == 1024))
    return -1;
#define L(D_, F_) hipLaunchKernelGGL((append_rows_kernel<D_, F_>), dim3((n + 3) / 4), dim3(256), 0,  \
                                     st, (const __bf16*)src, n, (__bf16*)rows, r0, (uint8_t*)img4, \
                                     b4, (uint8_t*)img6, b6)
  if (dim == 384) {
    if (img6) L(384, true);
    else L(384, false);
  } else if (dim == 768) {
    if (img6) L(768, true);
    else L(768, false);
  } else if (dim == 1024) L(1024, false);
  else return -1;
#undef L
  if (img8) return symb_quant_stream_i8(rows, r0, nullptr, n, dim, img8, b8, st);
  return (int)hipGetLastError();
}

// int8 stream image of the sub-tiles covering bf16 rows [r0, r0 + n) of X (rows == nullptr) or
// the n listed rows -- whole 32-row tiles (their shared scale), so X holds the shard's every row.
int symb_quant_stream_i8(const void* X, int r0, const int* rows, int n, int dim, void* img,
                         float* bounds, hipStream_t st) {
  if (n <= 0) return 0;
  if (bounds == nullptr || (rows == nullptr && r0 < 0)) return -1;
  const int g_lo = r0 >> 5, n_wg = rows ? n : ((r0 + n - 1) >> 5) - g_lo + 1;
#define L(D_) hipLaunchKernelGGL(quant_stream_i8_kernel<D_>, dim3(n_wg), dim3(512), 0, st,          \
                                 (const __bf16*)X, g_lo, rows, (uint8_t*)img, bounds)
  if (dim == 384) L(384);
  else if (dim == 768) L(768);
  else if (dim == 1024) L(1024);
  else return -1;
#undef L
  return (int)hipGetLastError();
}

// MX-fp4 stream image of bf16 rows (margin == nullptr: rows [r0, r0 + n) or the listed rows into
// img, bounds raised) or the query image (margin != nullptr: Xq / QS / margin for rows 0 .. n-1).
int symb_quant_stream_mx4(const void* X, int r0, const int* rows, int n, int dim, void* img,
                          void* Xq, void* QS, float* bounds, float* margin, hipStream_t st) {
  if (n <= 0) return 0;
  if (bounds == nullptr) return -1;
  if (margin == nullptr ? (img == nullptr || (rows == nullptr && r0 < 0))
                        : (Xq == nullptr || QS == nullptr))
    return -1;
#define L(D_) hipLaunchKernelGGL((quant_stream_mx_kernel<SF_MX4, D_>), dim3((n + 3) / 4), dim3(256), \
                                 0, st, (const __bf16*)X, r0, rows, n, (uint8_t*)img, (uint8_t*)Xq, \
                                 (uint32_t*)QS, bounds, margin)
  if (dim == 384) L(384);
  else if (dim == 768) L(768);
  else if (dim == 1024) L(1024);
  else return -1;
#undef L
  return (int)hipGetLastError();
}

// MX-fp6 (e2m3) stream image, as symb_quant_stream_mx4 (query image Xq [n][3 dim / 4] bytes; the
// row image's 24-byte lane pieces split over two 768-byte planes per k-step; dim 384 / 768).
int symb_quant_stream_mx6(const void* X, int r0, const int* rows, int n, int dim, void* img,
                          void* Xq, void* QS, float* bounds, float* margin, hipStream_t st) {
  if (n <= 0) return 0;
  if (bounds == nullptr) return -1;
  if (margin == nullptr ? (img == nullptr || (rows == nullptr && r0 < 0))
                        : (Xq == nullptr || QS == nullptr))
    return -1;
#define L(D_) hipLaunchKernelGGL((quant_stream_mx_kernel<SF_MX6, D_>), dim3((n + 3) / 4), dim3(256), \
                                 0, st, (const __bf16*)X, r0, rows, n, (uint8_t*)img, (uint8_t*)Xq, \
                                 (uint32_t*)QS, bounds, margin)
  if (dim == 384) L(384);
  else if (dim == 768) L(768);
  else return -1;
#undef L
  return (int)hipGetLastError();
}
