// Pre-pass kernels of the exact pruned search (index/shard.py _pruned_begin), so the per-step
// search runs no vendor or framework kernels between its scans:
//
//  * dense_scores_kernel: exact fp32 scores of NQ bf16 queries against a row list plus a
//    contiguous row range in ONE launch -- the threshold sample's seed tiles (a list) and the
//    fresh-row tail (a range), which the round-4 path gathered with torch.index_select and scored
//    with two fp32 torch.mm calls (hipBLASLt Cijk kernels plus bf16 -> f32 casts).  The products
//    of bf16 values are exact in fp32 and are summed by v_mfma_f32_32x32x16_bf16; the callers
//    take a k-th best minus MQ_THR_MARGIN (2^-12) of them as a LOWER bound, which covers any
//    fp32 summation order.
//  * append_rows_kernel: an upsert of unit bf16 rows into the shard in one launch -- the bf16
//    rows, their int8 stream image and their MX-fp4 stream image (index_stream.hip layouts) and
//    the bound maxima, in place of a torch copy plus two quantiser launches.
#include "common.h"

namespace symb {

// out[q * ld + j] = <Q[q], X[row(j)]>, row(j) = rows[j] for j < n_list (rows == nullptr: the
// threshold sample's seed tiles, computed here -- tile v = (j / 64) div is physical tile
// (v << ts) + (v * 0x9E3779B1 mod 2^32) >> (32 - ts), as index/shard.py _tile_sample_plan and
// index_mq.hip's sample), r_lo + j - n_list for n_list <= j < n_list + n_range.  One wave per 32
// rows x 64 queries (two 32 x 32 blocks that share the row fragments), 4 waves per workgroup side
// by side over the queries: 32 TPW rows x 256 queries per workgroup, grid (row tiles / TPW,
// query blocks).  TPW > 1 (D = 384): the wave's 64 query fragments stay in registers (192
// VGPRs) across its TPW row tiles instead of being re-read from L2 for every 32 rows.
template <int D, int TPW>
__global__ __launch_bounds__(256) void dense_scores_kernel(const __bf16* __restrict__ X,
                                                           const int* __restrict__ rows, int n_list,
                                                           int ts, int div, int r_lo, int n_range,
                                                           const __bf16* __restrict__ Q, int NQ,
                                                           float* __restrict__ out, int ld) {
  constexpr int KS = D / 16;
  constexpr bool RES = TPW > 1;   // resident query fragments
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int m = n_list + n_range;
  const int q0 = (blockIdx.y * 4 + wave) * 64;
  if (q0 >= NQ) return;   // (no barrier in this kernel)
  const __bf16* qa = Q + (size_t)min(q0 + (lane & 31), NQ - 1) * D + 8 * h;
  const __bf16* qb = Q + (size_t)min(q0 + 32 + (lane & 31), NQ - 1) * D + 8 * h;
  bf16x8 rb0[RES ? KS : 1], rb1[RES ? KS : 1];
  if constexpr (RES) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      rb0[ks] = *reinterpret_cast<const bf16x8*>(qa + 16 * ks);
      rb1[ks] = *reinterpret_cast<const bf16x8*>(qb + 16 * ks);
    }
  }
  for (int t = 0; t < TPW; ++t) {
    const int j0 = (blockIdx.x * TPW + t) * 32;
    if (j0 >= m) break;   // (wave-uniform)
    // this lane's A row (row l & 31 of the tile) and its two queries (l & 31 of each set)
    const int j = min(j0 + (lane & 31), m - 1);
    int row;
    if (j >= n_list) {
      row = r_lo + (j - n_list);
    } else if (rows != nullptr) {
      row = rows[j];
    } else {
      const uint32_t v = (uint32_t)(j >> 6) * (uint32_t)div;
      row = (int)(((v << ts) + ((v * 0x9E3779B1u) >> (32 - ts))) * 64u) + (j & 63);
    }
    const __bf16* xp = X + (size_t)row * D + 8 * h;
    f32x16 acc0 = {}, acc1 = {};
    // (fully unrolled with resident fragments: a partially unrolled loop indexes rb0 / rb1
    // dynamically and the compiler puts them in scratch)
#pragma unroll (RES ? KS : 8)
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(xp + 16 * ks);
      bf16x8 b0, b1;
      if constexpr (RES) {
        b0 = rb0[ks];
        b1 = rb1[ks];
      } else {
        b0 = *reinterpret_cast<const bf16x8*>(qa + 16 * ks);
        b1 = *reinterpret_cast<const bf16x8*>(qb + 16 * ks);
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, acc1, 0, 0, 0);
    }
    // accumulator: col = query lane & 31, rows (r & 3) + 8 (r >> 2) + 4 h of the tile
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = q0 + 32 * s + (lane & 31);
      if (q >= NQ) continue;
      float* op = out + (size_t)q * ld + j0 + 4 * h;
      const f32x16& acc = s ? acc1 : acc0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int jj = j0 + 8 * c + 4 * h;
        if (jj + 3 < m && (ld & 3) == 0) {
          *reinterpret_cast<f32x4*>(op + 8 * c) =
              f32x4{acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (jj + r < m) op[8 * c + r] = acc[4 * c + r];
        }
      }
    }
  }
}

// Every query's candidate list starts as rows [r_lo, r_lo + n) (n < 64): cand_n[q] = n and
// cand_i[q * cap + j] = r_lo + j (their scores are written by the re-score).  The pruned search
// lists the rows of a partly filled last 32-row sub-tile this way and its scans stop at the
// sub-tile boundary: an append into that sub-tile re-quantises its rows under a new shared int8
// scale, so a scan in flight beside the append must not read it (index/shard.py _pruned_end).
__global__ __launch_bounds__(256) void prefill_candidates_kernel(int NQ, int r_lo, int n,
                                                                 int* __restrict__ cand_i,
                                                                 int* __restrict__ cand_n,
                                                                 int cap) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= NQ) return;
  if (lane < n) cand_i[(size_t)q * cap + lane] = r_lo + lane;
  if (lane == 0) cand_n[q] = n;
}

}  // namespace symb

using namespace symb;

int symb_prefill_candidates(int NQ, int r_lo, int n, int* cand_i, int* cand_n, int cap,
                            hipStream_t st) {
  if (NQ <= 0) return 0;
  if (n < 0 || n >= 64 || n > cap || r_lo < 0) return -1;
  hipLaunchKernelGGL(prefill_candidates_kernel, dim3((NQ + 3) / 4), dim3(256), 0, st, NQ, r_lo, n,
                     cand_i, cand_n, cap);
  return (int)hipGetLastError();
}

// 32-row tiles per wave of the 384-wide dense scores (query fragments resident across them)
#ifndef SYMB_DS_TPW
#define SYMB_DS_TPW 4
#endif

// Exact fp32 scores (dense_scores_kernel): out [NQ][ld] f32, columns 0 .. n_list - 1 for the
// listed rows, n_list .. n_list + n_range - 1 for rows r_lo ..; ld >= n_list + n_range.
// rows == nullptr with n_list > 0: the hashed seed-tile list of (ts, div) (n_list a multiple of 64).
int symb_dense_scores(const void* X, int dim, const int* rows, int n_list, int ts, int div,
                      int r_lo, int n_range, const void* Q, int NQ, float* out, int ld,
                      hipStream_t st) {
  const int m = n_list + n_range;
  if (NQ <= 0 || m <= 0) return 0;
  if (n_list < 0 || n_range < 0 || ld < m || r_lo < 0) return -1;
  if (n_list > 0 && rows == nullptr && (ts < 1 || ts > 24 || div < 1 || n_list % 64)) return -1;
#define L(D_, T_) hipLaunchKernelGGL((dense_scores_kernel<D_, T_>), dim3((m + 32 * T_ - 1) / (32 * T_), (NQ + 255) / 256), \
                                     dim3(256), 0, st, (const __bf16*)X, rows, n_list, ts, div, r_lo, \
                                     n_range, (const __bf16*)Q, NQ, out, ld)
  if (dim == 384) L(384, SYMB_DS_TPW);
  else if (dim == 768) L(768, 1);
  else if (dim == 1024) L(1024, 1);
  else return -1;
#undef L
  return (int)hipGetLastError();
}
