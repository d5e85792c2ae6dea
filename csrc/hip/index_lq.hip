// int8 pruning scan with the QUERIES in LDS and the rows streamed through a deep VGPR ring
// (the first pass of the exact pruned search; reference hot path
// services/vector_memory_service/src/main.rs:261-286), over index_stream.hip's fragment-major
// int8 image: the default int8 form at D = 768, stream-config int8 variant 5 at D = 384.
//
// Why (profiles/r5_scan/): scan_stream_kernel keeps 128 queries per wave as resident B operands
// (192 VGPRs) and pairs two waves on the same rows.  What is left for the row ring is two
// 48-register slots, and hipcc lands the next sub-tile in the registers the accumulators need,
// so every sub-tile starts with an `s_waitcnt vmcnt(1)`: effectively one sub-tile in flight per
// wave, ~48 KiB per CU, waves parked on memory 41 % of their cycles, 3.9 TB/s.
//
// Here a 4-wave workgroup (one wave per SIMD) copies its 256 queries' B fragments into LDS once
// (8 sets x 12 k-steps x 1 KiB = 96 KiB, lane-linear, so every ds_read_b128 is conflict-free) and
// each wave streams ITS OWN sub-tiles (wave w: w, w + 4, ...) through a DEPTH-slot register ring
// of 48-register fragments: DEPTH x 12 KiB in flight per wave, all four waves on distinct rows.
// Per sub-tile a wave issues 96 v_mfma_i32_32x32x32_i8 (8 sets x 12 k-steps, B operand from one
// ds_read_b128 each: 128 B/clk/CU of LDS at the MFMA rate, half the array's 256) and the same
// integer-max hit test as scan_stream_kernel; only a block with a hit recomputes and emits.
//
// Measured (profiles/r5_lq/): at D = 384 the stall is gone (waves parked 41 -> 16 %) and the time
// is not -- the chip holds 1.22 GHz with the MFMA pipes 76 % busy, the power limit -- so the
// register-resident stream scan stays the default there.  At D = 768 (two query blocks per row
// block, run on one XCD) it is 23.6 ms against the stream scan's 41.1 ms for 100M held-out rows.
#include "scan_common.h"

namespace symb {

typedef __attribute__((ext_vector_type(4))) int i32x4q;
typedef __attribute__((ext_vector_type(16))) int i32x16q;

template <int D>
struct LqGeo {
  static constexpr int NKS = D / 32;              // 32-deep int8 k-steps per row
  static constexpr int HDR = 16;                  // sub-tile header: the f32 scale at byte 0
  static constexpr int REC = HDR + NKS * 1024;    // bytes per 32-row sub-tile (index_stream.hip)
  static constexpr int SETS = D == 384 ? 8 : 4;   // 32-query sets per workgroup, in LDS
  static constexpr int QPB = SETS * 32;           // queries per workgroup
  static constexpr int NW = 4;                    // waves (one per SIMD), each on its own rows
  static constexpr int QBYTES = SETS * NKS * 1024;
  static constexpr int STW = 512;                 // staged candidates per wave
  static constexpr int STAGE = STW * 10;
  static constexpr int LDS = QBYTES + NW * STAGE;
  static_assert(LDS <= 160 * 1024, "LDS");
};

// NP: sub-tiles (ring slots) each LDS query fragment feeds -- 2 would halve the LDS read bytes per
// MFMA, but NP = 2 with 4 slots spills at 512 VGPRs, so only NP = 1 is instantiated; timing
// ablation ABL 2 (wrong results): no sub-tile loads after the prologue.
template <int D, int DEPTH, int NP = 1, int ABL = 0>
__global__ __launch_bounds__(256, 1) void scan_lq_i8_kernel(
    const uint8_t* __restrict__ img, int n_valid, int rows_per_blk, const uint8_t* __restrict__ Q,
    int NQ, int n_qblk, const float* __restrict__ thr_in, float* __restrict__ cand_s,
    int* __restrict__ cand_i, int* __restrict__ cand_n, int cap, const int* __restrict__ skip,
    const int* __restrict__ gate, int gate_want, int* __restrict__ runs) {
  using G = LqGeo<D>;
  constexpr int NKS = G::NKS, SETS = G::SETS, REC = G::REC, STW = G::STW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: scalar loop control)
  // (XCD-contiguous block order: the query blocks of one row block -- two at D = 768 -- run on
  // one XCD, so the second read of each row hits that XCD's L2 / the Infinity Cache)
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = lb % n_qblk, rb = lb / n_qblk;
  if (gate != nullptr && *gate != gate_want) return;   // (workgroup-uniform exits only)
  if (runs != nullptr && lb == 0 && tid == 0) atomicAdd(runs, 1);
  if (skip != nullptr && skip[rb] != 0) return;
  const int row_begin = rb * rows_per_blk;
  const int row_end = min(row_begin + rows_per_blk, n_valid);
  if (row_end <= row_begin) return;
  const int g0 = row_begin >> 5, ns = (row_end - row_begin + 31) >> 5;
  const int qw = qb * G::QPB;

  // ---- the workgroup's queries -> LDS: chunk (s, ks) = 1 KiB at (s NKS + ks) KiB, lane l's B
  //      fragment (query qw + 32 s + (l & 31), bytes 32 ks + 16 (l >> 5) .. + 16) at 16 l ----
  for (int c = tid; c < SETS * NKS * 64; c += 256) {
    const int l = c & 63, sk = c >> 6, s = sk / NKS, ks = sk - s * NKS;
    const int q = min(qw + 32 * s + (l & 31), NQ - 1);
    *reinterpret_cast<i32x4q*>(smem + 16 * c) =
        *reinterpret_cast<const i32x4q*>(Q + (size_t)q * D + 32 * ks + 16 * (l >> 5));
  }
  float thr[SETS];
#pragma unroll
  for (int s = 0; s < SETS; ++s) {
    const int q = qw + 32 * s + (lane & 31);
    thr[s] = q < NQ ? thr_in[q] : INFINITY;
  }
  __syncthreads();   // (the only barrier: the LDS query image is read-only from here on)

  // ---- per-wave candidate stage (LDS, after the query image) ----
  char* stage = smem + G::QBYTES + wave * G::STAGE;
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

  // ---- the wave's sub-tiles: i = wave + 4 j, j < nsw ----
  const int nsw = ns > wave ? (ns - wave + 3) >> 2 : 0;
  if (nsw == 0) return;   // (no barrier follows)
  const uint8_t* rec0 = img + (size_t)(g0 + wave) * REC;
  // a VGPR zero the compiler cannot see through: keeps the (wave-uniform) scale load a vector
  // load counted with its fragments in vmcnt -- a scalar load would sit on lgkmcnt beside the
  // LDS fragment reads and force lgkmcnt(0) waits
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  i32x4q fk[DEPTH][NKS];
  float fts[DEPTH];
  auto load = [&](auto dc, int j) {
    constexpr int d = decltype(dc)::value;
    const uint8_t* r = rec0 + (size_t)min(j, nsw - 1) * (4 * REC);   // (past the end: the last)
    fts[d] = *reinterpret_cast<const float*>(r + vz);
    const uint8_t* f = r + G::HDR + 16 * lane;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) fk[d][ks] = *reinterpret_cast<const i32x4q*>(f + 1024 * ks);
  };
  auto qfrag = [&](int s, int ks) -> i32x4q {
    return *reinterpret_cast<const i32x4q*>(smem + 1024 * (s * NKS + ks) + 16 * lane);
  };

  // Query fragments double-buffered in registers: while set s's MFMAs run from qf2[s & 1], the
  // 12 ds_read_b128 of set s + 1 (set 0 of the NEXT slot group after set 7) fill qf2[~s & 1], one
  // read per NP MFMAs (sched_group_barrier pins the pairing: left to itself hipcc issued each
  // read right before its MFMA and waited lgkmcnt(0) on it, one LDS round trip per MFMA), and the
  // hit test of set s - 1 rides in the VALU gaps of set s's MFMAs (two accumulator sets).
  static_assert(DEPTH % NP == 0, "slot groups");
  i32x4q qf2[2][NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf2[0][ks] = qfrag(0, ks);
  i32x16q acc[2][NP];
  auto hit_test = [&](const i32x16q& x, float ts, float t) -> bool {
    int m = max(max(x[0], x[1]), x[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) m = max(max(m, x[r]), x[r + 1]);
    m = max(m, x[15]);
    return (float)m * ts >= t;   // (the sub-tile's scale > 0 keeps the order)
  };

  // slots d0 .. d0 + NP - 1 hold the wave's sub-tiles j0 .. j0 + NP - 1
  auto process = [&](auto dc, int j0) {
    constexpr int d0 = decltype(dc)::value;
    uint32_t hm[NP] = {};   // per slot: sets with a hit in this lane
    static_for<0, SETS>([&](auto sc) {
      constexpr int s = decltype(sc)::value, b = s & 1, nb = b ^ 1;
      constexpr int sn = s + 1 < SETS ? s + 1 : 0;
#pragma unroll
      for (int p = 0; p < NP; ++p) acc[b][p] = i32x16q{};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          acc[b][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fk[d0 + p][ks], qf2[b][ks], acc[b][p],
                                                           0, 0, 0);
        qf2[nb][ks] = qfrag(sn, ks);
      }
      if constexpr (s > 0) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          hm[p] |= (hit_test(acc[nb][p], fts[d0 + p], thr[s - 1]) ? 1u : 0u) << (s - 1);
      }
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        __builtin_amdgcn_sched_group_barrier(0x008, NP, 0);   // NP MFMAs ...
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // ... one LDS read
      }
    });
#pragma unroll
    for (int p = 0; p < NP; ++p)
      hm[p] |= (hit_test(acc[(SETS - 1) & 1][p], fts[d0 + p], thr[SETS - 1]) ? 1u : 0u) << (SETS - 1);
    static_for<0, NP>([&](auto pc) {
      constexpr int p = decltype(pc)::value, d = d0 + p;
      if (!__builtin_amdgcn_ballot_w64(hm[p] != 0)) return;   // rare: recompute the hit sets
      const int row0 = (g0 + wave + 4 * (j0 + p)) * 32 + 4 * h;   // + (r & 3) + 8 (r >> 2)
      static_for<0, SETS>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if (!__builtin_amdgcn_ballot_w64((hm[p] >> s) & 1)) return;
        i32x16q a = {};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
          a = __builtin_amdgcn_mfma_i32_32x32x32_i8(fk[d][ks], qfrag(s, ks), a, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = (float)a[r] * fts[d];
          const int row = row0 + (r & 3) + 8 * (r >> 2);
          const bool pr = v >= thr[s] && row < row_end;
          const uint64_t mk = __builtin_amdgcn_ballot_w64(pr);
          if (mk) {
            if (nst > STW - 64) flush();
            const int idx = nst + (int)__builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0));
            if (pr) {
              st_s[idx] = v;
              st_r[idx] = row;
              st_q[idx] = (uint16_t)(32 * s + (lane & 31));
            }
            nst += __builtin_popcountll(mk);
          }
        }
      });
    });
  };

  // prologue: DEPTH sub-tiles in flight; then use one / refill its slot (the last round may run
  // past nsw: those slots re-read the wave's last sub-tile and name rows >= row_end, so they
  // emit nothing -- a branch-free body keeps the loads' waits counted)
  static_for<0, DEPTH>([&](auto dc) { load(dc, decltype(dc)::value); });
  for (int j0 = 0; j0 < nsw; j0 += DEPTH) {
    static_for<0, DEPTH / NP>([&](auto gc) {
      constexpr int d0 = decltype(gc)::value * NP;
      process(std::integral_constant<int, d0>(), j0 + d0);
      if constexpr (ABL < 2)
        static_for<0, NP>([&](auto pc) {
          constexpr int d = d0 + decltype(pc)::value;
          load(std::integral_constant<int, d>(), j0 + d + DEPTH);
        });
    });
  }
  if (nst) flush();
}

template <int D, int DEPTH, int NP = 1, int ABL = 0>
static int launch_lq(const void* img, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                     int NQ, const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                     hipStream_t st, const int* skip, const int* gate, int gate_want, int* runs) {
  using G = LqGeo<D>;
  const int n_qblk = (NQ + G::QPB - 1) / G::QPB;
  set_max_lds<scan_lq_i8_kernel<D, DEPTH, NP, ABL>>(G::LDS);
  hipLaunchKernelGGL((scan_lq_i8_kernel<D, DEPTH, NP, ABL>), dim3(n_rblk * n_qblk), dim3(64 * G::NW), G::LDS,
                     st, (const uint8_t*)img, n_valid, rows_per_blk, (const uint8_t*)Q, NQ, n_qblk,
                     thr, cand_s, cand_i, cand_n, cap, skip, gate, gate_want, runs);
  return (int)hipGetLastError();
}

}  // namespace symb

using namespace symb;

// queries per workgroup (workgroups per CU: 1) of the LDS-query int8 scan; 0 = no such form
int symb_lq_qpb(int dim) { return dim == 384 ? LqGeo<384>::QPB : dim == 768 ? LqGeo<768>::QPB : 0; }

// The LDS-query int8 scan over rows [0, n_valid) of an int8 stream image (the arguments of
// symb_index_scan_stream, form 0); form (A/B): 0 = the default (3 slots), 1 = its no-refill
// timing ablation (wrong results).  (NP = 2 with 4 slots spills at 512 VGPRs.)
int symb_index_scan_lq(const void* img, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                       int NQ, const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                       hipStream_t st, const int* skip, int dim, const int* gate, int gate_want,
                       int* runs, int form) {
#define L(D_, P_, C_, A_)                                                                          \
  launch_lq<D_, P_, C_, A_>(img, n_valid, rows_per_blk, n_rblk, Q, NQ, thr, cand_s, cand_i, cand_n, \
                            cap, st, skip, gate, gate_want, runs)
  if (dim == 384) {
    switch (form) {
      case 1: return L(384, 3, 1, 2);
      default: return L(384, 3, 1, 0);
    }
  }
  if (dim == 768) return L(768, 2, 1, 0);
#undef L
  return -1;
}
