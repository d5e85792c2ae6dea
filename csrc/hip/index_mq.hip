// Multi-query-block fused scan for bf16 shards of D = 384 / 768 / 1024: the per-rank shape of the
// sharded search at N >= 2 GPUs (every rank scores the 256*N all-gathered queries against its 100M/N rows;
// SURVEY.md §2.5 X2, §2.6 index sharding).  Complements index_topk.hip, whose kernel holds 256
// queries per workgroup and keeps per-lane top-k lists in registers.
//
// Why a second kernel: at 512+ queries the 256-query kernel streams every row block once per
// 256-query block (L2 -> LDS), issues 6 LDS-DMA pieces per 1536 MFMA cycles per wave and reads
// one A fragment from LDS per MFMA.  Its compute-only ablation runs 13.1 ms on 12.5M x 2048 q and
// the full kernel 17.0 ms (profiles/r2_wide/): the row stream, not the MFMAs, is what is left.
//
// This kernel holds 512 queries per workgroup (8 waves x 64 queries):
//  * queries stay RESIDENT IN AGPRs as the B operand of hand-issued v_mfma_f32_16x16x32_bf16
//    (4 sets of 16 queries x 12 k-steps x 4 registers = 192 AGPRs per lane), so one A fragment
//    read from LDS feeds FOUR MFMAs and every row tile DMA'd into LDS feeds 512 queries: half
//    the LDS-DMA issue, L2->LDS bytes and LDS read bytes per FLOP of the 256-query kernel;
//  * the 16x16x32 shape holds a higher clock than 32x32x16 under the chip's power management at
//    equal cycles per FLOP (MI355X_MICROARCH.md, DVFS give-back item 7);
//  * with 192 of the 256 registers a wave may hold at 2 waves/SIMD spent on queries, no per-lane
//    top-k list fits.  The kernel EMITS candidates instead: every score above the query's seeded
//    threshold (a lower bound on its final k-th score, from a row sample: exact by construction)
//    is appended to that query's candidate buffer with a vector atomic, and a select kernel takes
//    the top-k of each buffer.  A sample of 1/64 of the rows puts ~64k candidates per query above
//    the threshold (~640 for k = 10), rare events against 12.5M rows.  A buffer that overflows
//    raises a device flag on which the 256-query kernel re-runs the whole batch (gated launches,
//    no host sync), so the result is exact for any data.
//
// Ring and barrier structure follow index_topk.hip: 64-row tiles (48 KiB) through a 3-deep LDS
// ring by global_load_lds_dwordx4 with counted vmcnt and a raw s_barrier; A fragments by
// hand-issued ds_read_b128 with counted lgkmcnt.  The LDS image of a tile is 48 1-KiB PIECES, one
// per (16-row sub-tile j, 32-column k-step ks): piece j*12 + ks holds rows 16j..16j+15 x 64 bytes,
// so one LDS-DMA instruction fills one piece and one ds_read_b128 per lane reads one MFMA A
// fragment.  Lane l of a piece holds row l>>2, 16-byte slot l&3 = chunk (l&3) ^ f(row), and the
// A-fragment read of lane (r = lane&15, g = lane>>4) takes slot g ^ f(r), f(r) = (r>>1) & 2: every
// 16-lane ds_read_b128 group then covers all 16 slots of a 256-byte bank row once (conflict-free),
// and both the DMA source offset and the fragment offset are ONE per-lane register each.
#include "scan_common.h"

namespace symb {

namespace mq {
constexpr int WAVES = 8;
constexpr int SUB = 16;                     // rows per MFMA chain
constexpr int PIECE = 1024;                 // LDS bytes per (sub-tile, k-step) piece
constexpr int PF = 3;                       // fragment reads in flight
constexpr int R = PF + 1;                   // fragment ring slots
// per-wave candidate stage in LDS after the ring: score f32, row i32, query-in-wave u16
constexpr int STW = 192;                    // staged candidates per wave (flushed past STW - 64)
constexpr int STAGE_BYTES = STW * 10;
}  // namespace mq

// Geometry per row width.  Queries stay resident as B fragments: SETS x D/32 k-steps x 4 VGPRs,
// at most 192 of a wave's 256 registers, so the query sets per wave shrink as D grows --
//   D = 384 : 64-row tiles (48 KiB), 3-deep ring, up to 4 sets (512 queries per workgroup);
//   D = 768 : 32-row tiles (48 KiB), 3-deep ring, 2 sets (256 queries: the reference's 768-d
//             collection, vector_memory_service/src/main.rs:22);
//   D = 1024: 16-row tiles (32 KiB), 4-deep ring, 1 set (128 queries).
template <int D> struct MqGeo {
  static constexpr int NKS = D / 32;                    // 16x16x32 k-steps over D
  static constexpr int TR = D == 384 ? 64 : D == 768 ? 32 : 16;   // rows per barrier interval
  static constexpr int NSUB = TR / mq::SUB;
  static constexpr int NS = D == 1024 ? 4 : 3;          // LDS ring depth in tiles
  static constexpr int TILE_BYTES = TR * D * 2;
  static constexpr int LOADS = TILE_BYTES / (1024 * mq::WAVES);  // LDS-DMA pieces per wave per tile
  static constexpr int DMA_EVERY = NKS / LOADS;         // k-steps between DMA pieces in sub-tile 0
  static constexpr int MAX_SETS = D == 384 ? 4 : D == 768 ? 2 : 1;
  static constexpr int LDS_BYTES = NS * TILE_BYTES + mq::WAVES * mq::STAGE_BYTES;
  static_assert(D == 384 || D == 768 || D == 1024, "row width");
  static_assert(TILE_BYTES % (1024 * mq::WAVES) == 0, "tile must split evenly over waves");
  static_assert(NSUB * NKS * mq::PIECE == TILE_BYTES, "a tile is NSUB x NKS pieces");
  static_assert(LOADS * DMA_EVERY <= NKS && DMA_EVERY >= 1, "DMA pieces must fit the first chain");
  static_assert(LDS_BYTES <= 160 * 1024, "ring + stages exceed the CU's 160 KiB");
  static_assert(NKS % mq::R == 0, "cross-chain prefetch: fragment j of the next chain must use slot j % R");
};

template <int OFF>
__device__ __forceinline__ void mq_read16(bf16x8& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void mq_lgkm(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "i"(N));
}

// One 16x16x32 MFMA per query set.  Hand-issued so the 192 query registers stay put as the B
// operand (VGPRs: naming them as AGPRs makes the compiler split the 256-register budget 128/128
// and shuttle queries between the files).
template <bool FIRST>
__device__ __forceinline__ void mq_mfma(f32x4& acc, const bf16x8& a, const bf16x8& q) {
  if constexpr (FIRST)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(q));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(q));
}

// k-step KS of one 16-row sub-tile: wait for its A fragment, 4 MFMAs (one per query set), then
// refill the ring slot PF steps ahead -- in the last PF steps with the first fragments of the
// NEXT sub-tile (at ``next``, when NEXT), so its chain starts without an LDS round trip.
// DMA(i) issues LDS-DMA piece i of a later tile.
template <int D, int KS, int DMA_PIECES, bool NEXT, int SETS>
struct MqChain {
  static constexpr int NKS = MqGeo<D>::NKS, DMA_EVERY = MqGeo<D>::DMA_EVERY;
  template <class Dma>
  __device__ __forceinline__ static void run(f32x4 (&acc)[SETS], bf16x8 (&a)[mq::R],
                                             const bf16x8 (&qf)[SETS][NKS],
                                             uint32_t base, uint32_t next, const Dma& dma) {
    using namespace mq;
    if constexpr (DMA_PIECES > 0 && KS % DMA_EVERY == 0 && KS / DMA_EVERY < DMA_PIECES)
      dma(KS / DMA_EVERY);
    constexpr int outstanding = (NEXT || NKS - KS >= PF) ? PF : (NKS - KS);
    mq_lgkm<outstanding - 1>(a[KS % R]);
#pragma unroll
    for (int s = 0; s < SETS; ++s) mq_mfma<KS == 0>(acc[s], a[KS % R], qf[s][KS]);
    // XDL result -> VALU read (the emission test reads acc right after the chain): the compiler
    // pads nothing inside asm, so cover the MFMA's result latency here.
    if constexpr (KS + 1 == NKS) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    // base / next: this lane's fragment address in piece 0 of this / the next sub-tile
    if constexpr (KS + PF < NKS)
      mq_read16<(KS + PF) * PIECE>(a[(KS + PF) % R], base);
    else if constexpr (NEXT)  // fragment KS + PF - NKS of the next sub-tile, same ring slot order
      mq_read16<(KS + PF - NKS) * PIECE>(a[(KS + PF) % R], next);
    if constexpr (KS + 1 < NKS)
      MqChain<D, KS + 1, DMA_PIECES, NEXT, SETS>::run(acc, a, qf, base, next, dma);
  }
};

// A pointer the compiler must treat as wave-uniform (SGPR pair): with it the LDS-DMA issues in the
// SGPR-base + 32-bit VGPR-offset form instead of a per-piece 64-bit VGPR address.
__device__ __forceinline__ const char* mq_uniform(const char* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const char*>(((uint64_t)hi << 32) | lo);
}

template <int J>
__device__ __forceinline__ void mq_prologue(bf16x8 (&a)[mq::R], uint32_t base) {
  mq_read16<J * mq::PIECE>(a[J % mq::R], base);
  if constexpr (J + 1 < mq::PF) mq_prologue<J + 1>(a, base);
}

// X: [>= round_up(n_valid, 64), 384] bf16 unit rows; Q: [NQ, 384] bf16 unit queries.
// thr[NQ]: per-query lower bounds on the final k-th score (required).
// cand_s/cand_i: [NQ][cap]; cand_n[NQ] (zeroed): number of candidates each query emitted (may
// exceed cap: the select kernel then raises the overflow flag).
// ABL (profiling entry symb_index_scan_mq_ablate only): 1 = no LDS-DMA (compute on whatever the
// ring holds), 2 = no emission test, 3 = full kernel + per-workgroup s_memtime / s_memrealtime
// around the tile loop written to cand_s[2 * blockIdx.x + {0, 1}] (in-kernel clock), 4 = LDS-DMA
// ring only (same waits and barriers, no MFMA chains, no emission test: the row stream's rate).
//
// RSPLIT = 2 (the 256-query form of the 1-GPU shape): waves w and w + 4 hold the SAME 64 queries
// (4 sets) and split each tile's rows, w the first two 16-row sub-tiles and w + 4 the last two.
// Against the 2-set form (8 waves x 32 queries, every wave reading the whole tile) that halves
// the LDS fragment reads per tile (192 KiB instead of 384) and the chain ends per MFMA, at the
// same MFMA cycles per SIMD: at 256 queries the scan is bound by the chip's power limit (HBM
// streaming + MFMAs hold the in-kernel clock near 1.5 GHz), so bytes moved per FLOP count.
// AUX: cache policy bits of the row stream's LDS-DMA (0 = default, 2 = non-temporal).
// MqList (block-list mode, blist != nullptr): scan only the row blocks that the pruned search's
// route sent to the bf16 path (prune_route_kernel, index_i8.hip) instead of rows [0, n_valid).
// blist[0] = nl listed blocks, blist[1] = the int8 scan's block count, blist[2 + i] = the i-th
// listed block; a block is list_tiles 64-row tiles, rows >= n_valid are never scanned.  The
// launch's n_rblk row slots share the listed blocks: block i gets slots [ceil(i n_rblk / nl),
// ceil((i + 1) n_rblk / nl)) and splits its rows evenly over them (the route never lists more
// blocks than slots), so each workgroup still scans one contiguous physical row range and a
// single crowded block spreads over the whole chip.  Every block listed: rows [0, n_valid) split
// evenly, as without a list.
struct MqList {
  const int* blist;
  int list_tiles;
};

template <int D, int NSET, int ABL = 0, int RSPLIT = 1, int AUX = 0>
__global__ __launch_bounds__(512, 1) void index_scan_mq_kernel(
    const __bf16* __restrict__ X, int n_valid, int rows_per_blk, const __bf16* __restrict__ Q,
    int NQ, int n_qblk, int xcd, const float* __restrict__ thr_in, float* __restrict__ cand_s,
    int* __restrict__ cand_i, int* __restrict__ cand_n, int cap, int tshift,
    const int* __restrict__ gate, MqList lst) {
  // gate (optional): run only if *gate != 0 -- the pruned search's bf16 route (index_i8.hip)
  if (gate != nullptr && *gate == 0) return;
  using namespace mq;
  using G = MqGeo<D>;
  constexpr int NKS = G::NKS, TR = G::TR, NSUB = G::NSUB, NS = G::NS;
  constexpr int TILE_BYTES = G::TILE_BYTES, LOADS = G::LOADS;
  constexpr int SETS = NSET, QW = SETS * 16, QWAVES = WAVES / RSPLIT, QPB = QWAVES * QW;
  constexpr int NSW = NSUB / RSPLIT;          // 16-row sub-tiles per wave per tile
  static_assert(RSPLIT == 1 || (RSPLIT == 2 && NSUB % 2 == 0), "row split");
  static_assert(SETS >= 1 && SETS <= G::MAX_SETS, "query registers");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lb = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qb = lb % n_qblk, rb = lb / n_qblk;
  int row_begin = rb * rows_per_blk;
  int row_end = min(row_begin + rows_per_blk, n_valid);
  if (lst.blist != nullptr) {   // (grid-uniform, before any barrier)
    const int nl = lst.blist[0], n_rblk = gridDim.x / n_qblk;
    if (nl <= 0) return;
    // every block (the route escalates a list longer than the slots to every block; the second
    // test only keeps a corrupt list from dividing by zero below)
    if (nl >= lst.blist[1] || nl > n_rblk) {
      const int per = (n_valid + n_rblk * TR - 1) / (n_rblk * TR) * TR;
      row_begin = min(rb * per, n_valid);
      row_end = min(row_begin + per, n_valid);
    } else {
      const int i = (int)((long long)rb * nl / n_rblk);
      const int s0 = (int)(((long long)i * n_rblk + nl - 1) / nl);
      const int s1 = (int)(((long long)(i + 1) * n_rblk + nl - 1) / nl);
      const int per = (lst.list_tiles + (s1 - s0) - 1) / (s1 - s0);
      const int base = lst.blist[2 + i] * lst.list_tiles;
      const int t0 = base + min((rb - s0) * per, lst.list_tiles);
      const int t1 = base + min((rb - s0 + 1) * per, lst.list_tiles);
      // (list tiles are the caller's 64-row tiles, whatever this width's TR: 768 / 1024 scan
      // 32- / 16-row tiles, and reading t0 * TR there scanned the wrong rows)
      row_begin = min(t0 * 64, n_valid);
      row_end = min(t1 * 64, n_valid);
    }
  }
  const int n_tiles = row_end > row_begin ? (row_end - row_begin + TR - 1) / TR : 0;
  // Row numbers above are VIRTUAL.  tshift = 0: virtual = physical.  tshift > 0 (a row sample for
  // threshold seeding, scanned in place): virtual 64-row tile v is physical tile
  // (v << tshift) + h(v), one pseudo-random tile of every 2^tshift (h: top tshift bits of
  // v * 0x9E3779B1; index/shard.py builds the matching sub-sample).
  auto phys_tile = [&](int v) -> int {
    if (tshift == 0) return v;
    return (v << tshift) + (int)(((uint32_t)v * 0x9E3779B1u) >> (32 - tshift));
  };

  // ---- query fragments (B operand, 16x16x32: lane holds Q[col = lane&15][k = 8*(lane>>4)+j]) --
  const int qwave = wave % QWAVES;                 // this wave's query group
  const int j0 = (wave / QWAVES) * NSW;             // this wave's first sub-tile of a tile
  const int qbase = qb * QPB + qwave * QW + (lane & 15);
  bf16x8 qf[SETS][NKS];
  float thr[SETS];
#pragma unroll
  for (int s = 0; s < SETS; ++s) {
    const int q = qbase + s * 16;
    const __bf16* qp = Q + (size_t)min(q, NQ - 1) * D + (lane >> 4) * 8;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[s][ks] = *reinterpret_cast<const bf16x8*>(qp + ks * 32);
    thr[s] = q < NQ ? thr_in[q] : INFINITY;   // padding queries never emit
  }
  // consume the query/threshold loads here, before any LDS-DMA is in flight: the compiler waits
  // for a load at its first use, and a first use inside the tile loop would be a vmcnt(0) that
  // drains the DMA ring every tile
#pragma unroll
  for (int s = 0; s < SETS; ++s) {
    asm volatile("" ::"v"(thr[s]));
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[s][ks]));
  }

  // ---- LDS-DMA: wave w fills pieces p = i*WAVES + w (i < LOADS) of a tile.  Lane l fetches row
  // l>>2 of the piece, chunk (l&3) ^ f(l>>2): one loop-invariant per-lane offset for every piece
  // (SGPR base + VGPR offset form; a pending LDS-DMA's registers are never rewritten, which would
  // make the compiler drain vmcnt to 0).
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t loff = (uint32_t)((lane >> 2) * D * 2 + (((lane & 3) ^ ((lane >> 3) & 2)) * 16));
  auto issue_piece = [&](int t, int i) {
    const int tt = min(t, n_tiles - 1);  // past the end: re-load the last tile (vmcnt stays exact)
    const int p = i * WAVES + wave_u, j = p / NKS, ks = p % NKS;
    const int prow = phys_tile(row_begin / TR + tt) * TR;
    const char* base = reinterpret_cast<const char*>(X + (size_t)(prow + j * SUB) * D + ks * 32);
    char* dst = smem + (t % NS) * TILE_BYTES + p * PIECE;
    glds16_aux<AUX>(mq_uniform(base) + loff, dst);
  };

  // ---- per-lane A-fragment offset within a piece (lane holds X[row r][k 8g..8g+7] of the k-step)
  const uint32_t lds_smem = lds_addr(smem);
  const uint32_t foff = (uint32_t)((lane & 15) * 64 + (((lane >> 4) ^ ((lane >> 1) & 2)) * 16));

  // ---- candidate emission -------------------------------------------------------------------
  // A hit is staged in this wave's LDS stage at a slot from a wave-wide ballot prefix count (no
  // atomics, no waits), and the stage moves to the per-query global buffers (vector atomics whose
  // returned slot the compiler must wait for, i.e. vmcnt(0), draining the LDS-DMA ring) only when
  // it fills: ~once per 130 candidates instead of once per candidate.
  char* stage = smem + NS * TILE_BYTES + wave_u * STAGE_BYTES;
  float* st_s = reinterpret_cast<float*>(stage);
  int* st_r = reinterpret_cast<int*>(stage + STW * 4);
  uint16_t* st_q = reinterpret_cast<uint16_t*>(stage + STW * 8);
  int nst = 0;  // staged entries (wave-uniform)
  auto flush = [&]() {
    // the candidate addresses derive from an opaque copy of the wave's first query so the
    // compiler cannot hoist 64-bit pointers out of the tile loop into the register budget
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
  // one 16-row sub-tile at virtual row row0 / physical row prow0: lane holds rows
  // 4*(lane>>4) + r of it for the 16 queries of each set (column lane & 15)
  auto emit = [&](f32x4 (&acc)[SETS], int row0, int prow0) {
    // keep every read of the inline-asm MFMA results below the chain-end s_nops (the compiler's
    // hazard recognizer does not see asm MFMAs; index_i8.hip emit has the story)
#pragma unroll
    for (int s = 0; s < SETS; ++s) asm volatile("" : "+v"(acc[s]));
    if constexpr (ABL == 2 || ABL == 4) {
#pragma unroll
      for (int s = 0; s < SETS; ++s) asm volatile("" ::"v"(acc[s]));
      return;
    }
    if (row0 + SUB > row_end) {   // last tile of the block: mask rows past its end
      const int rl = row0 + 4 * (lane >> 4);
#pragma unroll
      for (int s = 0; s < SETS; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (rl + r >= row_end) acc[s][r] = -INFINITY;
    }
    // max of each set's 4 scores by two v_max3 (fmaxf would add NaN-canonicalising maxes)
    float mx[SETS];
#pragma unroll
    for (int s = 0; s < SETS; ++s)
      asm volatile("v_max3_f32 %0, %1, %2, %3\n\tv_max3_f32 %0, %0, %4, %4"
                   : "=&v"(mx[s]) : "v"(acc[s][0]), "v"(acc[s][1]), "v"(acc[s][2]), "v"(acc[s][3]));
    bool hit = false;
#pragma unroll
    for (int s = 0; s < SETS; ++s) hit |= mx[s] > thr[s];
    if (__builtin_amdgcn_ballot_w64(hit)) {
      // cold path: per-lane values come from opaque copies made here, so nothing it derives can
      // be hoisted out of the tile loop into the (full) register budget
      int lo = lane;
      asm volatile("" : "+v"(lo));
      const int lrow = prow0 + 4 * (lo >> 4), lq = lo & 15;
#pragma unroll
      for (int s = 0; s < SETS; ++s) {
        if (!__builtin_amdgcn_ballot_w64(mx[s] > thr[s])) continue;   // usually one set hits
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool p = acc[s][r] > thr[s];
          const uint64_t m = __builtin_amdgcn_ballot_w64(p);
          if (m) {
            if (nst > STW - 64) flush();
            const int idx = nst + (int)__builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            if (p) {
              st_s[idx] = acc[s][r];
              st_r[idx] = lrow + r;
              st_q[idx] = (uint16_t)(s * 16 + lq);
            }
            nst += __builtin_popcountll(m);
          }
        }
      }
    }
  };

  if (n_tiles > 0 && ABL != 1) {
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
#pragma unroll
      for (int i = 0; i < LOADS; ++i) issue_piece(p, i);
  }
  bf16x8 a[R];
  f32x4 acc[SETS];
  // The two waves sharing a SIMD (w, w + 4) run in phase after every barrier, so their emission
  // tests (VALU + branch, ~8 % of the loop) would idle the SIMD together.  The second wave tests
  // its last sub-tile AFTER the barrier, under its partner's first MFMAs: the pair stays half a
  // test apart and each test overlaps the other wave's chain.
  const bool late = wave_u >= WAVES / 2;
  int prow_last = 0;   // physical first row of the previous tile
  uint64_t c0 = 0, r0t = 0;
  if constexpr (ABL == 3) {
    c0 = __builtin_amdgcn_s_memtime();
    r0t = __builtin_amdgcn_s_memrealtime();
  }
  for (int t = 0; t < n_tiles; ++t) {
    // tile t landed for this wave once only the (NS-2) younger tiles' pieces remain; the barrier
    // makes every wave's pieces visible and retires every wave's reads of slot (t-1) % NS
    if constexpr (ABL != 1) wait_vmcnt<LOADS * (NS - 2)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t tbase = lds_smem + (uint32_t)((t % NS) * TILE_BYTES);
    const int row0 = row_begin + t * TR;
    const int prow0 = phys_tile(row0 / TR) * TR;
    const int tnext = t + NS - 1;
    auto dma = [&](int i) {
      if constexpr (ABL != 1) issue_piece(tnext, i);
    };
    const uint32_t fb = tbase + foff;   // this lane's fragment in piece 0 of sub-tile 0
    if constexpr (ABL == 4) {
#pragma unroll
      for (int i = 0; i < LOADS; ++i) dma(i);
      continue;
    }
    mq_prologue<0>(a, fb + j0 * NKS * PIECE);
    // (this wave's sub-tiles are j0 .. j0 + NSW - 1; ``last`` = row offset of its last one)
    const int last = (j0 + NSW - 1) * SUB;
    if (late && t > 0) emit(acc, row0 - TR + last, prow_last + last);
    prow_last = prow0;
    const uint32_t fw = fb + j0 * NKS * PIECE;
    if constexpr (NSW > 1)
      MqChain<D, 0, LOADS, true, SETS>::run(acc, a, qf, fw, fw + NKS * PIECE, dma);
    else
      MqChain<D, 0, LOADS, false, SETS>::run(acc, a, qf, fw, 0, dma);
#pragma unroll
    for (int j = 1; j < NSW; ++j) {
      // sub-tile j's first fragments were read by the previous chain's tail and fly while this
      // wave tests the previous sub-tile's scores
      emit(acc, row0 + (j0 + j - 1) * SUB, prow0 + (j0 + j - 1) * SUB);
      if (j + 1 < NSW)
        MqChain<D, 0, 0, true, SETS>::run(acc, a, qf, fw + j * NKS * PIECE,
                                          fw + (j + 1) * NKS * PIECE, NoDma());
      else
        MqChain<D, 0, 0, false, SETS>::run(acc, a, qf, fw + j * NKS * PIECE, 0, NoDma());
    }
    if (!late) emit(acc, row0 + last, prow0 + last);
  }
  if (late && n_tiles > 0) {
    const int last = (j0 + NSW - 1) * SUB;
    emit(acc, row_begin + (n_tiles - 1) * TR + last, prow_last + last);
  }
  if (nst) flush();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail prefetches and emissions
  if constexpr (ABL == 3) {
    const uint64_t cyc = __builtin_amdgcn_s_memtime() - c0;
    const uint64_t rt = __builtin_amdgcn_s_memrealtime() - r0t;
    if (tid == 0) {
      cand_s[2 * blockIdx.x] = (float)cyc;
      cand_s[2 * blockIdx.x + 1] = (float)rt;
    }
  }
}

// Wave-wide max of a float, valid in lane 63: DPP row shifts fold each 16-lane row, then two row
// broadcasts fold the rows (max is idempotent, so lanes whose DPP source is out of range simply
// keep their own value).
__device__ __forceinline__ float wave_max63(float v) {
  int x = __float_as_int(v);
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x111, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x112, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x114, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x118, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x142, 0xa, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x143, 0xc, 0xf, false))));
  return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

// KMAX rounds of a wave-wide "pop the best head": every lane holds a descending list of L
// candidates; each round the wave max of the heads (DPP, no LDS), the lowest lane holding it gives
// up its head (its list shifts by one) and lane r keeps round r's winner.  Replaces the LDS tree
// of pairwise merges (8 rounds x 2 barriers x a 16-step serial merge per level).
template <int KMAX, int L>
__device__ __forceinline__ void wave_pop_topk(float (&tv)[L], int (&ti)[L], int lane, float& rv,
                                              int& ri) {
  rv = -INFINITY;
  ri = -1;
#pragma unroll
  for (int r = 0; r < KMAX; ++r) {
    const float mx = wave_max63(tv[0]);
    const uint64_t hit = __ballot(tv[0] == mx);
    const int win = hit ? (int)__builtin_ctzll(hit) : 0;
    const int id = __builtin_amdgcn_readlane(ti[0], win);
    if (lane == r) {
      rv = mx;
      ri = id;
    }
    if (lane == win) {
#pragma unroll
      for (int i = 0; i + 1 < L; ++i) {
        tv[i] = tv[i + 1];
        ti[i] = ti[i + 1];
      }
      tv[L - 1] = -INFINITY;
      ti[L - 1] = -1;
    }
  }
}

// A second, dense segment of the same select launch (blockIdx.y == 1): the pruned search's
// exact fresh-row tail, selected in the seed select's launch instead of a serial one of its own.
struct SelSeg2 {
  const float* s;   // [NQ, ld] scores (the same stride as the first segment)
  int cap;          // columns
  float* out_s;     // [NQ, k]
  int* out_i;
};

// Top-k of each query's emitted candidates (or of a dense score row).  One workgroup per query:
// every thread keeps a register top-KMAX over a strided walk (4 independent loads in flight per
// thread), each wave reduces its 64 lists with wave_pop_topk, and wave 0 reduces the waves'
// lists the same way.  A query whose buffer overflowed raises *ovf (the gated 256-query kernel
// then recomputes the batch).
template <int KMAX, int NTH>
__global__ __launch_bounds__(NTH) void topk_select_counted_kernel(
    const float* __restrict__ cand_s, const int* __restrict__ cand_i,
    const int* __restrict__ cand_n, int cap, int k, float* __restrict__ out_s,
    int* __restrict__ out_i, int* __restrict__ ovf, const int* __restrict__ gate, int ld,
    float* __restrict__ kth_out, float kth_margin, SelSeg2 seg2) {
  constexpr int NW = NTH / 64, P = NW * KMAX / 64;   // waves; wave 0's list length per lane
  static_assert(NW * KMAX % 64 == 0 && P >= 1, "wave lists must tile wave 0's lanes");
  if (gate != nullptr && *gate == 0) return;   // (grid-uniform, before any barrier)
  __shared__ float ls[NW * KMAX];
  __shared__ int li[NW * KMAX];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (blockIdx.y == 1) {   // (block-uniform) the dense second segment
    cand_s = seg2.s;
    cand_i = cand_n = nullptr;
    cap = seg2.cap;
    out_s = seg2.out_s;
    out_i = seg2.out_i;
    kth_out = nullptr;
  }
  // cand_n == nullptr: every row holds cap candidates; cand_i == nullptr: a candidate's id is
  // its position (dense score rows, e.g. the pruned search's exact tail)
  const int cnt = cand_n != nullptr ? cand_n[q] : cap;
  const int n = min(cnt, cap);
  if (tid == 0 && cnt > cap) *ovf = 1;
  const float* cs = cand_s + (size_t)q * ld;
  const int* ci = cand_i != nullptr ? cand_i + (size_t)q * ld : nullptr;
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    tv[i] = -INFINITY;
    ti[i] = -1;
  }
  float rv;
  int ri;
  // Long lists: a first pass takes each thread's max; the KMAX-th largest of those maxima is at
  // most the list's KMAX-th largest entry (the KMAX largest maxima are KMAX distinct entries), so
  // the second pass inserts only entries reaching it.  Without it a dense row of random scores
  // inserts most of each thread's first ~3 KMAX entries, a serial 16-step chain each.
  __shared__ float floor_s;
  float floor_v = -INFINITY;
  if (n >= 8 * NTH) {   // (block-uniform)
    float mx = -INFINITY;
    int c = tid;
    for (; c + 3 * NTH < n; c += 4 * NTH) {
      float s[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] = cs[c + u * NTH];
      mx = fmaxf(fmaxf(mx, fmaxf(s[0], s[1])), fmaxf(s[2], s[3]));
    }
    for (; c < n; c += NTH) mx = fmaxf(mx, cs[c]);
    float mv[1] = {mx};
    int mi[1] = {0};
    wave_pop_topk<KMAX, 1>(mv, mi, lane, rv, ri);
    if (lane < KMAX) ls[wave * KMAX + lane] = rv;
    __syncthreads();
    if (wave == 0) {
      float pv[P];
      int pi[P];
#pragma unroll
      for (int j = 0; j < P; ++j) {
        pv[j] = -INFINITY;
        pi[j] = 0;
      }
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const float v = ls[lane + 64 * j];
        if (v > pv[P - 1]) topk_insert<P>(pv, pi, v, 0);
      }
      wave_pop_topk<KMAX, P>(pv, pi, lane, rv, ri);
      if (lane == KMAX - 1) floor_s = rv;
    }
    __syncthreads();
    floor_v = floor_s;
  }
  int c = tid;
  for (; c + 3 * NTH < n; c += 4 * NTH) {
    float s[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] = cs[c + u * NTH];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (s[u] >= floor_v && s[u] > tv[KMAX - 1])
        topk_insert<KMAX>(tv, ti, s[u], ci != nullptr ? ci[c + u * NTH] : c + u * NTH);
  }
  for (; c < n; c += NTH) {
    const float s = cs[c];
    if (s >= floor_v && s > tv[KMAX - 1]) topk_insert<KMAX>(tv, ti, s, ci != nullptr ? ci[c] : c);
  }
  wave_pop_topk<KMAX, KMAX>(tv, ti, lane, rv, ri);
  if (lane < KMAX) {
    ls[wave * KMAX + lane] = rv;
    li[wave * KMAX + lane] = ri;
  }
  __syncthreads();
  if (wave != 0) return;
  float pv[P];
  int pi[P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    pv[j] = -INFINITY;
    pi[j] = -1;
  }
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const float v = ls[lane + 64 * j];
    if (v > pv[P - 1]) topk_insert<P>(pv, pi, v, li[lane + 64 * j]);
  }
  wave_pop_topk<KMAX, P>(pv, pi, lane, rv, ri);
  if (lane < k) {
    out_s[(size_t)q * k + lane] = rv;
    out_i[(size_t)q * k + lane] = ri;
  }
  // (optional) the k-th best minus a margin: a seed threshold for the next scan, no torch op
  if (kth_out != nullptr && lane == k - 1) kth_out[q] = rv - kth_margin;
}

// Top-k of each query's emitted candidates for ANY k <= SEL_MAX (the reference passes top_k
// straight to Qdrant: vector_memory_service/src/main.rs:261-284).  One 256-thread workgroup per
// query: an exact radix select of the k-th largest score over its candidates (3 passes of 11, 11
// and 10 bits over an order-preserving uint32 image of the floats, LDS histograms, block-wide
// suffix sums), then every score above it and as many equal ones as k needs are gathered into LDS
// and bitonic-sorted descending.  Cost: 4 reads of the candidate list, independent of k.
namespace sel {
constexpr int NTH = 256;
constexpr int SEL_MAX = 128;
}  // namespace sel

__device__ __forceinline__ uint32_t ord_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ __launch_bounds__(sel::NTH) void topk_select_radix_kernel(
    const float* __restrict__ cand_s, const int* __restrict__ cand_i,
    const int* __restrict__ cand_n, int cap, int k, float* __restrict__ out_s,
    int* __restrict__ out_i, int* __restrict__ ovf, const int* __restrict__ gate) {
  using namespace sel;
  if (gate != nullptr && *gate == 0) return;   // (grid-uniform, before any barrier)
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t part[NTH];
  __shared__ uint32_t s_bin, s_above;
  __shared__ float ss[SEL_MAX];
  __shared__ int si[SEL_MAX];
  __shared__ int n_gt, n_eq;
  const int q = blockIdx.x, tid = threadIdx.x;
  const int cnt = cand_n[q];
  const int n = min(cnt, cap);
  if (tid == 0 && cnt > cap) *ovf = 1;
  const float* cs = cand_s + (size_t)q * cap;
  const int* ci = cand_i + (size_t)q * cap;
  uint32_t prefix = 0, mask = 0;
  int remaining = k;     // rank of the wanted value among those matching the prefix so far
  if (n > k) {
    constexpr int SHIFT[3] = {21, 10, 0};
    constexpr int BITS[3] = {11, 11, 10};
#pragma unroll
    for (int pass = 0; pass < 3; ++pass) {
      const int nb = 1 << BITS[pass], sh = SHIFT[pass];
      for (int b = tid; b < nb; b += NTH) hist[b] = 0;
      __syncthreads();
      for (int c = tid; c < n; c += NTH) {
        const uint32_t key = ord_key(cs[c]);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> sh) & (nb - 1)], 1u);
      }
      __syncthreads();
      // suffix sums from the TOP bin down: thread t owns bins [t * per, (t + 1) * per)
      const int per = nb / NTH;
      uint32_t local = 0;
      for (int j = 0; j < per; ++j) local += hist[tid * per + j];
      part[tid] = local;
      __syncthreads();
      if (tid == 0) {
        uint32_t above = 0;            // candidates in bins above the current thread's range
        for (int t = NTH - 1; t >= 0; --t) {
          if (above + part[t] >= (uint32_t)remaining) {
            for (int j = per - 1; j >= 0; --j) {
              const uint32_t h = hist[t * per + j];
              if (above + h >= (uint32_t)remaining) {
                s_bin = (uint32_t)(t * per + j);
                s_above = above;
                break;
              }
              above += h;
            }
            break;
          }
          above += part[t];
        }
      }
      __syncthreads();
      prefix |= s_bin << sh;
      mask |= (uint32_t)(nb - 1) << sh;
      remaining -= (int)s_above;
      __syncthreads();
    }
  }
  // gather: every value above the k-th, then `remaining` values equal to it (n <= k: all)
  if (tid == 0) {
    n_gt = 0;
    n_eq = 0;
  }
  for (int j = tid; j < SEL_MAX; j += NTH) {
    ss[j] = -INFINITY;
    si[j] = -1;
  }
  __syncthreads();
  const int take_gt = n > k ? k - remaining : n;
  for (int c = tid; c < n; c += NTH) {
    const float v = cs[c];
    const uint32_t key = ord_key(v);
    if (n <= k || key > prefix) {
      const int pos = atomicAdd(&n_gt, 1);
      if (pos < SEL_MAX) {
        ss[pos] = v;
        si[pos] = ci[c];
      }
    } else if (key == prefix) {
      const int e = atomicAdd(&n_eq, 1);
      if (e < remaining) {
        ss[take_gt + e] = v;
        si[take_gt + e] = ci[c];
      }
    }
  }
  __syncthreads();
  // bitonic sort of SEL_MAX entries, descending (ties: lower row first)
  for (int size = 2; size <= SEL_MAX; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < SEL_MAX / 2; t += NTH) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const float a = ss[lo], b = ss[hi];
        const int ia = si[lo], ib = si[hi];
        const bool a_first = a > b || (a == b && (unsigned)ia <= (unsigned)ib);
        if (a_first != desc) {
          ss[lo] = b;
          ss[hi] = a;
          si[lo] = ib;
          si[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int j = tid; j < k; j += NTH) {
    out_s[(size_t)q * k + j] = ss[j];
    out_i[(size_t)q * k + j] = si[j];
  }
}

}  // namespace symb

using namespace symb;

int symb_mq_queries_per_blk(int sets, int rsplit) { return mq::WAVES / rsplit * 16 * sets; }
// Query sets per wave the D-wide form holds (its 16-query sets x D/32 k-steps stay in registers)
int symb_mq_max_sets(int dim) {
  return dim == 384 ? MqGeo<384>::MAX_SETS : dim == 768 ? MqGeo<768>::MAX_SETS
                                                        : dim == 1024 ? MqGeo<1024>::MAX_SETS : 0;
}

// rows_per_blk must be a multiple of 64; n_rblk * rows_per_blk >= n_valid.  cand_n is zeroed here.
// cache policy of the row stream (symb_mq_config): 0 default, 2 non-temporal
static int g_mq_aux = 0;
int symb_mq_config(int aux) {
  if (aux != 0 && aux != 2) return -1;
  g_mq_aux = aux;
  return 0;
}

template <int D, int NSET, int RSPLIT, int AUX>
static int launch_mq_aux(const void* X, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                     int NQ, const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                     int xcd, hipStream_t st, int tshift, const int* gate, MqList lst) {
  constexpr int qpb = mq::WAVES / RSPLIT * 16 * NSET;
  const int n_qblk = (NQ + qpb - 1) / qpb;
  constexpr int lds = MqGeo<D>::LDS_BYTES;
  set_max_lds<index_scan_mq_kernel<D, NSET, 0, RSPLIT, AUX>>(lds);
  hipLaunchKernelGGL((index_scan_mq_kernel<D, NSET, 0, RSPLIT, AUX>), dim3(n_rblk * n_qblk),
                     dim3(512), lds, st, (const __bf16*)X, n_valid, rows_per_blk, (const __bf16*)Q,
                     NQ, n_qblk, xcd, thr, cand_s, cand_i, cand_n, cap, tshift, gate, lst);
  return (int)hipGetLastError();
}

template <int D, int NSET, int RSPLIT>
static int launch_mq(const void* X, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                     int NQ, const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                     int xcd, hipStream_t st, int tshift, const int* gate, MqList lst) {
  return g_mq_aux == 2
             ? launch_mq_aux<D, NSET, RSPLIT, 2>(X, n_valid, rows_per_blk, n_rblk, Q, NQ, thr,
                                                 cand_s, cand_i, cand_n, cap, xcd, st, tshift,
                                                 gate, lst)
             : launch_mq_aux<D, NSET, RSPLIT, 0>(X, n_valid, rows_per_blk, n_rblk, Q, NQ, thr,
                                                 cand_s, cand_i, cand_n, cap, xcd, st, tshift,
                                                 gate, lst);
}

// dim: 384 (sets 4 or 2; rsplit 2 with sets 4), 768 (sets 2), 1024 (sets 1); rsplit 1 otherwise.
// tshift: 0 = rows [0, n_valid); k > 0 = virtual rows of a 1-in-2^k tile sample (kernel note).
// Queries per workgroup: 8 / rsplit * 16 * sets.
// blist (optional, list mode): scan the row blocks listed there (MqList; list_tiles 64-row tiles
// each, rows >= n_valid never scanned) instead of rows [0, n_valid); rows_per_blk is then unused
// and the n_rblk row slots of the grid share the listed rows.  zero_cnt = 0 appends to cand_n
// (another scan's candidates already there) instead of zeroing it.
int symb_index_scan_mq(const void* X, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                       int NQ, const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                       int xcd, hipStream_t st, int sets, int tshift, int rsplit,
                       const int* gate, const int* blist, int list_tiles, int zero_cnt, int dim) {
  if (NQ <= 0) return 0;
  if (rows_per_blk % 64 || n_rblk <= 0 || thr == nullptr || cap <= 0) return -1;
  if (tshift < 0 || tshift > 12) return -1;
  if (dim == 384 && ((sets != 2 && sets != 4) || (rsplit != 1 && !(rsplit == 2 && sets == 4))))
    return -1;
  if (dim == 768 && (sets != 2 || rsplit != 1)) return -1;
  if (dim == 1024 && (sets != 1 || rsplit != 1)) return -1;
  if (dim != 384 && dim != 768 && dim != 1024) return -1;
  if (blist != nullptr && (tshift != 0 || list_tiles <= 0 || n_valid <= 0)) return -1;
  MqList lst{blist, list_tiles};
  if (zero_cnt) {
    hipError_t e = hipMemsetAsync(cand_n, 0, sizeof(int) * (size_t)NQ, st);
    if (e != hipSuccess) return (int)e;
  }
#define SYMB_MQ(D_, S_, R_) launch_mq<D_, S_, R_>(X, n_valid, rows_per_blk, n_rblk, Q, NQ, thr, \
                                                 cand_s, cand_i, cand_n, cap, xcd, st, tshift, gate, lst)
  if (dim == 768) return SYMB_MQ(768, 2, 1);
  if (dim == 1024) return SYMB_MQ(1024, 1, 1);
  if (rsplit == 2) return SYMB_MQ(384, 4, 2);
  return sets == 4 ? SYMB_MQ(384, 4, 1) : SYMB_MQ(384, 2, 1);
#undef SYMB_MQ
}

// Profiling-only entry: the ablations of index_scan_mq_kernel (ABL above), D = 384, same arguments.
int symb_index_scan_mq_ablate(const void* X, int n_valid, int rows_per_blk, int n_rblk,
                              const void* Q, int NQ, const float* thr, float* cand_s, int* cand_i,
                              int* cand_n, int cap, int xcd, hipStream_t st, int abl, int sets,
                              int rsplit) {
  if (NQ <= 0) return 0;
  if (rows_per_blk % 64 || n_rblk <= 0 || thr == nullptr || cap <= 0) return -1;
  if (sets != 2 && sets != 4) return -1;
  if (rsplit != 1 && !(rsplit == 2 && sets == 4)) return -1;
  hipError_t e = hipMemsetAsync(cand_n, 0, sizeof(int) * (size_t)NQ, st);
  if (e != hipSuccess) return (int)e;
  const int qpb = mq::WAVES / rsplit * 16 * sets;
  const int n_qblk = (NQ + qpb - 1) / qpb;
  constexpr int lds = MqGeo<384>::LDS_BYTES;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3(n_rblk * n_qblk), dim3(512), lds, st, (const __bf16*)X,
                       n_valid, rows_per_blk, (const __bf16*)Q, NQ, n_qblk, xcd, thr, cand_s,
                       cand_i, cand_n, cap, 0, (const int*)nullptr, MqList{nullptr, 0});
    return (int)hipGetLastError();
  };
  switch (abl + 8 * (sets == 2) + 16 * (rsplit == 2)) {
    case 0: return go(index_scan_mq_kernel<384, 4, 0>);
    case 1: return go(index_scan_mq_kernel<384, 4, 1>);
    case 2: return go(index_scan_mq_kernel<384, 4, 2>);
    case 3: return go(index_scan_mq_kernel<384, 4, 3>);
    case 4: return go(index_scan_mq_kernel<384, 4, 4>);
    case 8: return go(index_scan_mq_kernel<384, 2, 0>);
    case 9: return go(index_scan_mq_kernel<384, 2, 1>);
    case 10: return go(index_scan_mq_kernel<384, 2, 2>);
    case 11: return go(index_scan_mq_kernel<384, 2, 3>);
    case 12: return go(index_scan_mq_kernel<384, 2, 4>);
    case 16: return go(index_scan_mq_kernel<384, 4, 0, 2>);
    case 17: return go(index_scan_mq_kernel<384, 4, 1, 2>);
    case 18: return go(index_scan_mq_kernel<384, 4, 2, 2>);
    case 19: return go(index_scan_mq_kernel<384, 4, 3, 2>);
    case 20: return go(index_scan_mq_kernel<384, 4, 4, 2>);
    default: return -1;
  }
}

// ovf (one int) is zeroed here (reset_ovf), then set by any query whose buffer overflowed.
// gate (optional): the launch is skipped on the device unless *gate != 0.
int symb_topk_select_counted(const float* cand_s, const int* cand_i, const int* cand_n, int cap,
                             int NQ, int kmax, int k, float* out_s, int* out_i, int* ovf,
                             hipStream_t st, const int* gate, int reset_ovf, int ld,
                             float* kth_out, float kth_margin, const float* seg2_s, int seg2_cap,
                             float* seg2_out_s, int* seg2_out_i) {
  if (NQ <= 0) return 0;
  if (k > kmax) return -1;
  if (ld <= 0) ld = cap;
  if (ld < cap) return -1;
  const SelSeg2 seg2{seg2_s, seg2_cap, seg2_out_s, seg2_out_i};
  const dim3 grid(NQ, seg2_s != nullptr ? 2 : 1);
  if (seg2_s != nullptr && (kmax == sel::SEL_MAX || seg2_cap <= 0 || seg2_cap > ld ||
                            seg2_out_s == nullptr || seg2_out_i == nullptr))
    return -1;
  if (kmax == sel::SEL_MAX && (cand_i == nullptr || cand_n == nullptr)) return -1;   // (dense rows: KMAX 16 / 32 forms)
  if (kmax == sel::SEL_MAX && (ld != cap || kth_out != nullptr)) return -1;
  if (reset_ovf) {
    hipError_t e = hipMemsetAsync(ovf, 0, sizeof(int), st);
    if (e != hipSuccess) return (int)e;
  }
  if (kmax == sel::SEL_MAX)   // any k <= 128: radix select + bitonic sort
    hipLaunchKernelGGL(topk_select_radix_kernel, dim3(NQ), dim3(sel::NTH), 0, st, cand_s, cand_i,
                       cand_n, cap, k, out_s, out_i, ovf, gate);
  else if (kmax == 16 && cand_n == nullptr && cap >= 8192)   // long dense rows: 16 waves
    hipLaunchKernelGGL((topk_select_counted_kernel<16, 1024>), grid, dim3(1024), 0, st, cand_s,
                       cand_i, cand_n, cap, k, out_s, out_i, ovf, gate, ld, kth_out, kth_margin, seg2);
  else if (kmax == 16)
    hipLaunchKernelGGL((topk_select_counted_kernel<16, 256>), grid, dim3(256), 0, st, cand_s,
                       cand_i, cand_n, cap, k, out_s, out_i, ovf, gate, ld, kth_out, kth_margin, seg2);
  else if (kmax == 32)
    hipLaunchKernelGGL((topk_select_counted_kernel<32, 128>), grid, dim3(128), 0, st, cand_s,
                       cand_i, cand_n, cap, k, out_s, out_i, ovf, gate, ld, kth_out, kth_margin, seg2);
  else
    return -1;
  return (int)hipGetLastError();
}
