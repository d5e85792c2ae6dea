// Ping-pong MFMA bf16 GEMM for the wide encoder projections (H >= 768: bge / mpnet / e5 QKV,
// out-projection, FFN1, FFN2 at M >= 2048 tokens), so no projection is left to hipBLASLt
// (the round-4 kernels in gemm.hip ran 15-28 % behind it on QKV and FFN2,
// profiles/r4_gemm/README.md).
//
//   C[M, N] = epi( A[M, K] . W[N, K]^T + bias[N] )      epi: bias / GELU / + residual
//
// Why the round-4 256 x 256 tile lost: its 8 waves met at one barrier per 64-deep k-tile and then
// all issued LDS reads, all ran MFMAs, all waited -- the MFMA pipe of a SIMD idled whenever its two
// waves were both in a memory phase (waves parked in waitcnt / barrier 29 % of their cycles,
// active 21-23 %).  This kernel keeps the 256 x BM tile, 2 x 4 waves and the LDS-DMA staging, but
// runs the two wave ROWS half a phase apart ("ping-pong"):
//
//  * Each k-tile is 4 phases; a phase = [memory section: this phase's fragment reads + one
//    half-tile of LDS-DMA prefetch] barrier [MFMA section: one output quadrant x 64 k, 8 MFMAs of
//    v_mfma_f32_32x32x16_bf16 at raised priority] barrier.
//  * Wave row 1 executes one extra barrier before the loop, so its memory sections coincide with
//    row 0's MFMA sections and vice versa: waves w and w + 4 share a SIMD (a workgroup's waves go
//    to SIMDs cyclically), so every SIMD always has one wave issuing MFMAs while the other issues
//    its LDS reads and DMA.
//  * LDS: 2 k-tile buffers x {A rows 0..BM/2-1, A rows BM/2.., W rows 0..127, W rows 128..255}
//    half-tiles of 128-byte rows (XOR-swizzled 16-byte chunks, swizzle applied on the DMA's global
//    source and on the ds_read address; conflict-free for the 32-row fragment reads).  Wave row g
//    reads only A half g; both rows read both W halves.
//  * Prefetch schedule (tile T's phases a b c d; half-tile loads into the buffer freed two phases
//    earlier): a: W half 1 of T+1, b: A half 0 of T+1, c: A half 1 of T+1, d: W half 0 of T+2,
//    then a counted vmcnt retires everything but that last half (T+1 complete) before the barrier
//    that precedes T+1's reads.  The write-after-read distance of every half-tile is >= 1 full
//    section after the last wave's reads of it retired (lgkmcnt(0) at each MFMA section start),
//    counting the half-phase offset of the two rows (see the schedule table in gemm_pp_kernel).
//  * Epilogue: fp32 tile staged through LDS (one wave-row band per pass), bias / GELU / residual,
//    16-byte row-contiguous bf16 stores.
// The reference runs these projections through candle's cuBLAS SGEMM
// (services/preprocessing_service/src/embedding_generator.rs:198 -> BertModel::forward).
#include "common.h"

namespace symb {
namespace ggp {
constexpr int NT = 512;      // 8 waves: 2 (M) x 4 (N)
constexpr int BN = 256;      // W rows (output columns) per tile
constexpr int BH = 128 * 128;  // bytes of one W half-tile (128 rows x 64 k bf16)
enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RES = 2 };

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// One half-tile (rows [row0, row0 + ROWS) of a K-major bf16 operand, k-tile kt) into LDS by
// LDS-DMA: ROWS * 8 16-byte pieces, piece s = i * 512 + tid -> LDS byte 16 s (wave-uniform base +
// 16 lane), global chunk pre-swizzled so that row r's logical chunk c sits at swz(r, c).
template <int ROWS>
__device__ __forceinline__ void stage_half(const __bf16* __restrict__ src, int ld, int row0,
                                           int rmax, int kt, char* region, int tid, int wave) {
#pragma unroll
  for (int i = 0; i < ROWS * 8 / NT; ++i) {
    const int s = i * NT + tid;
    const int row = s >> 3, c = (s & 7) ^ ((row >> 1) & 7);
    const int grow = min(row0 + row, rmax - 1);
    glds16(src + (size_t)grow * ld + kt * 64 + c * 8, region + (i * NT + wave * 64) * 16);
  }
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace ggp

// BM: tile rows (256: 128 x 64 per wave, 4 x 2 blocks of 32 x 32; 128: 64 x 64 per wave).
// ABL (timing ablations, wrong results): 1 = no vmcnt wait in the k-loop, 2 = no DMA in the k-loop
// either (MFMA + LDS reads + barriers only).  RING (BM = 256): the half-tile ring below instead of
// two k-tile buffers.
template <int BM, int EPI, int ABL = 0, int RING = 0>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(
    const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ W, int ldw,
    const float* __restrict__ bias, const __bf16* __restrict__ R, int ldr, __bf16* __restrict__ C,
    int ldc, int M, int N, int K, int group_m, int gelu_poly) {
  using namespace ggp;
  constexpr int WTM = BM / 2;          // rows per wave
  constexpr int MB = WTM / 32;         // 32-row blocks per wave (4 or 2)
  constexpr int QB = MB / 2;           // ... per quadrant
  constexpr int AH = WTM * 128;        // bytes of one A half-tile
  constexpr int BUFB = 2 * AH + 2 * BH;
  static_assert(MB >= 2 && MB % 2 == 0, "tile rows");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int n_tiles = N / BN;
  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  int tm = tile / n_tiles, tn = tile % n_tiles;
  if (group_m > 1) {   // grouped order: an XCD's in-flight tiles share A and W panels in its L2
    const int m_tiles = nwg / n_tiles, per_group = group_m * n_tiles;
    const int g = tile / per_group, first = g * group_m;
    const int gm = min(group_m, m_tiles - first), local = tile - g * per_group;
    tm = first + local % gm;
    tn = local / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int KT = K / 64;

  // half-tile loads: 0 = A rows [0, WTM), 1 = A rows [WTM, BM), 2 = W rows [0, 128), 3 = W [128, 256)
  auto load = [&](int which, int kt) {
    if (ABL >= 2 && kt > 1) return;
    char* buf = smem + (kt & 1) * BUFB;
    if (which < 2)
      stage_half<WTM>(A, lda, m0 + which * WTM, M, kt, buf + which * AH, tid, wave);
    else
      stage_half<128>(W, ldw, n0 + (which - 2) * 128, N, kt, buf + 2 * AH + (which - 2) * BH, tid,
                      wave);
  };

  f32x16 acc[MB][2];
#pragma unroll
  for (int b = 0; b < MB; ++b)
    acc[b][0] = acc[b][1] = f32x16{};
  bf16x8 af[QB][4], bq0[4], bq1[4];

  // fragment reads: this wave's A rows of quadrant row qm (QB blocks x 4 k-steps), or its W
  // columns of quadrant column qn (one block x 4 k-steps); lane: row / column lane & 31, k-chunk
  // 2 ks + (lane >> 5) of the 64-deep tile
  const int fr = lane & 31, fh = lane >> 5;
  auto read_a = [&](const char* buf, int qm) {
    const char* base = buf + wr * AH;
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        af[b][ks] = *reinterpret_cast<const bf16x8*>(base + swz((qm * QB + b) * 32 + fr, 2 * ks + fh));
  };
  auto read_b = [&](const char* buf, int qn, bf16x8 (&bq)[4]) {
    const char* base = buf + 2 * AH + (wc >> 1) * BH;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      bq[ks] = *reinterpret_cast<const bf16x8*>(base + swz((wc & 1) * 64 + qn * 32 + fr, 2 * ks + fh));
  };
  auto mfma_q = [&](int qm, int qn, const bf16x8 (&bq)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int b = 0; b < QB; ++b)
        acc[qm * QB + b][qn] =
            __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[b][ks], bq[ks], acc[qm * QB + b][qn], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // the start of an MFMA section: this wave's reads of the memory section have landed
  auto mfma_gate = [&]() {
    ggp::pp_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  if constexpr (RING) {
    // v2: ten 16 KiB half-tile slots (the whole 160 KiB LDS) instead of two k-tile buffers.
    // Half-tile h = 4 kt + j (j: A rows 0..127, A rows 128.., W rows 0..127, W rows 128..) lives in
    // slot h % 10 and is issued at global phase h - 7 (one half per phase, the same one-half DMA
    // slice per phase as v1), so three half-tiles are always in flight across the once-per-k-tile
    // counted vmcnt (v1: one, which the waves then stalled on).  The slot h reuses held half h - 10,
    // whose last reads (A: phase c of its tile, by one wave row; W: phase b, both rows) lie >= 1
    // section before the DMA is issued, wave-row offset included (the table above, shifted: A half
    // g of tile t is re-filled at d of t (g = 0) / a of t+1 (g = 1), W halves at b / c of t+1).
    static_assert(BM == 256 && AH == BH, "ring slots are one half-tile");
    constexpr int SLOT = BH, NSLOT = 10, LEAD = 7;
    const int NH = 4 * KT;
    auto issue = [&](int h) {
      if (h >= NH) return;
      const int kt = h >> 2, j = h & 3;
      char* dst = smem + (h % NSLOT) * SLOT;
      if (j < 2)
        stage_half<WTM>(A, lda, m0 + j * WTM, M, kt, dst, tid, wave);
      else
        stage_half<128>(W, ldw, n0 + (j - 2) * 128, N, kt, dst, tid, wave);
    };
    auto read_a2 = [&](const char* base, int qm) {
#pragma unroll
      for (int b = 0; b < QB; ++b)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          af[b][ks] = *reinterpret_cast<const bf16x8*>(base + swz((qm * QB + b) * 32 + fr, 2 * ks + fh));
    };
    auto read_b2 = [&](const char* base, int qn, bf16x8 (&bq)[4]) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        bq[ks] = *reinterpret_cast<const bf16x8*>(base + swz((wc & 1) * 64 + qn * 32 + fr, 2 * ks + fh));
    };
    for (int h = 0; h < LEAD; ++h) issue(h);
    if (KT > 1)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile 1's first three halves in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ggp::pp_barrier();
    if (wr == 1) ggp::pp_barrier();
    for (int kt = 0; kt < KT; ++kt) {
      const int hb = 4 * kt;
      const char* sa = smem + ((hb + wr) % NSLOT) * SLOT;
      const char* sb = smem + ((hb + 2 + (wc >> 1)) % NSLOT) * SLOT;
      read_a2(sa, 0);
      read_b2(sb, 0, bq0);
      issue(hb + LEAD);
      mfma_gate();
      mfma_q(0, 0, bq0);
      ggp::pp_barrier();
      read_b2(sb, 1, bq1);
      issue(hb + 1 + LEAD);
      mfma_gate();
      mfma_q(0, 1, bq1);
      ggp::pp_barrier();
      read_a2(sa, 1);
      issue(hb + 2 + LEAD);
      mfma_gate();
      mfma_q(1, 1, bq1);
      ggp::pp_barrier();
      issue(hb + 3 + LEAD);
      // tile kt + 1 complete: all but the halves issued in b, c, d of this tile (2 DMAs each)
      if (kt + 2 < KT)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      mfma_gate();
      mfma_q(1, 0, bq0);
      ggp::pp_barrier();
    }
  } else {
  // Schedule (tile T in buffer T & 1; one row of the table per phase, both wave rows):
  //   phase  reads (memory section)        DMA issued               MFMA quadrant
  //   a      A quadrant row 0, W column 0  W half 1 of T+1          (0, 0)
  //   b      W column 1                    A half 0 of T+1          (0, 1)
  //   c      A quadrant row 1              A half 1 of T+1          (1, 1)
  //   d      --                            W half 0 of T+2, vmcnt   (1, 0)
  // Last reads of buffer T & 1: W halves in b, A half g in c (by wave row g only).  With wave row
  // 1 one section behind row 0, the first DMA into a half of it (d of T: W half 0 of T+2; a, b, c
  // of T+1: the rest) is issued at least one section after every reader's lgkmcnt(0) retired its
  // reads.  The vmcnt of d (all but d's own half retired) makes T+1 complete in LDS before the
  // barrier that precedes row 0's reads of it in a of T+1 (row 1's vmcnt lies one section later,
  // still before that barrier... its section ends at it).
  // prologue: tile 0 and W half 0 of tile 1 in flight, tile 0 retired
  load(0, 0);
  load(1, 0);
  load(2, 0);
  load(3, 0);
  if (KT > 1) {
    load(2, 1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  ggp::pp_barrier();
  if (wr == 1) ggp::pp_barrier();   // the half-phase offset of wave row 1

  auto k_tile = [&](int kt, auto bsel) {
    constexpr int BI = decltype(bsel)::value;
    const char* buf = smem + BI * BUFB;
    // a
    read_a(buf, 0);
    read_b(buf, 0, bq0);
    if (kt + 1 < KT) load(3, kt + 1);
    mfma_gate();
    mfma_q(0, 0, bq0);
    ggp::pp_barrier();
    // b
    read_b(buf, 1, bq1);
    if (kt + 1 < KT) load(0, kt + 1);
    mfma_gate();
    mfma_q(0, 1, bq1);
    ggp::pp_barrier();
    // c
    read_a(buf, 1);
    if (kt + 1 < KT) load(1, kt + 1);
    mfma_gate();
    mfma_q(1, 1, bq1);
    ggp::pp_barrier();
    // d
    if (kt + 2 < KT) {
      load(2, kt + 2);
      if (ABL == 0) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // (W half: 2 DMAs per thread)
    } else if (ABL == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mfma_gate();
    mfma_q(1, 0, bq0);
    ggp::pp_barrier();
  };
  for (int kt = 0; kt < KT; kt += 2) {
    k_tile(kt, std::integral_constant<int, 0>());
    if (kt + 1 < KT) k_tile(kt + 1, std::integral_constant<int, 1>());
  }
  }   // (v1)
  if (wr == 0) ggp::pp_barrier();   // rows back in step
  __syncthreads();

  // ---- epilogue: fp32 tile -> LDS (one wave-row band per pass when the tile does not fit) ----
  constexpr int CS = BN + 4;
  constexpr int PASSES = (BM * CS * 4 > 160 * 1024) ? 2 : 1;
  constexpr int PROWS = BM / PASSES;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll 1
  for (int p = 0; p < PASSES; ++p) {
    if (PASSES == 1 || wr == p) {
      const int rbase = PASSES == 1 ? wr * WTM : 0;
#pragma unroll
      for (int b = 0; b < MB; ++b)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + b * 32 + 8 * (r >> 2) + 4 * fh + (r & 3);
            Cs[row * CS + wc * 64 + nb * 32 + fr] = acc[b][nb][r];
          }
    }
    __syncthreads();
    const int band0 = m0 + p * PROWS;
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
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = x0[e] + b0[e];
        y[e + 4] = x1[e] + b1[e];
      }
      if constexpr (EPI == EPI_GELU) {
        if (gelu_poly) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const f32x2 g = gelu2_poly(f32x2{y[e], y[e + 1]});
            y[e] = g.x;
            y[e + 1] = g.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = gelu_erf(y[e]);
        }
      }
      if constexpr (EPI == EPI_RES) {
        float r[8];
        load8(R + (size_t)grow * ldr + n0 + c8, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] += r[e];
      }
      store8(C + (size_t)grow * ldc + n0 + c8, y);
    }
    if (PASSES > 1) __syncthreads();
  }
}

template <int BM, int EPI, int ABL = 0, int RING = 0>
static int launch_pp(const void* A, int lda, const void* W, int ldw, const float* bias,
                     const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                     int gelu_poly, hipStream_t st) {
  constexpr int main_bytes = RING ? 10 * ggp::BH : 2 * (BM * 128 + 2 * ggp::BH);
  constexpr int full = BM * (ggp::BN + 4) * 4;
  constexpr int epi_bytes = full > 160 * 1024 ? full / 2 : full;
  constexpr int lds = main_bytes > epi_bytes ? main_bytes : epi_bytes;
  set_max_lds<gemm_pp_kernel<BM, EPI, ABL, RING>>(lds);
  const int nwg = ((M + BM - 1) / BM) * (N / ggp::BN);
  hipLaunchKernelGGL((gemm_pp_kernel<BM, EPI, ABL, RING>), dim3(nwg), dim3(ggp::NT), lds, st,
                     (const __bf16*)A, lda, (const __bf16*)W, ldw, bias, (const __bf16*)R, ldr,
                     (__bf16*)C, ldc, M, N, K, group_m, gelu_poly);
  return (int)hipGetLastError();
}

}  // namespace symb

using namespace symb;

// Tile rows: 0 = auto (pp_pick_bm), 256 or 128 forced (A/B sweeps); bm + 1 / + 2: the 256-row
// bias kernel's timing ablations (ABL above).
static int g_pp_bm = 0, g_pp_abl = 0, g_pp_ring = 1;
// 256-row tiles on the half-tile ring (1, default) or the two k-tile buffers (0, v1)
int symb_gemm_pp_ring(int ring) {
  if (ring != 0 && ring != 1) return -1;
  g_pp_ring = ring;
  return 0;
}
int symb_gemm_pp_config(int bm) {
  const int abl = bm & 3;
  bm &= ~3;
  if (bm != 0 && bm != 128 && bm != 256) return -1;
  g_pp_bm = bm;
  g_pp_abl = abl;
  return 0;
}

// Auto tile rows: the fewest (waves of 256 tiles) x (tile rows), with a 256-row tile charged
// nothing extra and a 128-row one ~12 % (half the operand reuse per MFMA).
static int pp_pick_bm(int M, int N) {
  if (g_pp_bm) return g_pp_bm;
  const long nt = N / ggp::BN;
  const long w256 = ((M + 255) / 256 * nt + 255) / 256, w128 = ((M + 127) / 128 * nt + 255) / 256;
  return w128 * 128 * 112 < w256 * 256 * 100 ? 128 : 256;
}

bool symb_gemm_pp_supported(int epi, int M, int N, int K) {
  return (epi == ggp::EPI_BIAS || epi == ggp::EPI_GELU || epi == ggp::EPI_RES) && M > 0 &&
         N % ggp::BN == 0 && K % 64 == 0 && K >= 128;
}

// epi: 0 bias, 1 GELU (gelu_poly: the polynomial form), 2 bias + residual R.  -1: unsupported.
int symb_gemm_pp(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                 const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                 int gelu_poly, hipStream_t st) {
  if (M <= 0) return 0;
  if (!symb_gemm_pp_supported(epi, M, N, K)) return -1;
  if (lda % 8 || ldw % 8 || ldc % 8 || (epi == ggp::EPI_RES && (R == nullptr || ldr % 8))) return -1;
  const int bm = pp_pick_bm(M, N);
  if (g_pp_abl == 1 && bm == 256 && epi == ggp::EPI_BIAS)
    return launch_pp<256, ggp::EPI_BIAS, 1>(A, lda, W, ldw, bias, R, ldr, C, ldc, M, N, K, group_m,
                                            gelu_poly, st);
  if (g_pp_abl == 2 && bm == 256 && epi == ggp::EPI_BIAS)
    return launch_pp<256, ggp::EPI_BIAS, 2>(A, lda, W, ldw, bias, R, ldr, C, ldc, M, N, K, group_m,
                                            gelu_poly, st);
#define L(BM_, E_) launch_pp<BM_, E_>(A, lda, W, ldw, bias, R, ldr, C, ldc, M, N, K, group_m, \
                                      gelu_poly, st)
  if (bm == 128) {
    switch (epi) {
      case ggp::EPI_BIAS: return L(128, ggp::EPI_BIAS);
      case ggp::EPI_GELU: return L(128, ggp::EPI_GELU);
      default: return L(128, ggp::EPI_RES);
    }
  }
  if (g_pp_ring) {
#define LR(E_) launch_pp<256, E_, 0, 1>(A, lda, W, ldw, bias, R, ldr, C, ldc, M, N, K, group_m, \
                                        gelu_poly, st)
    switch (epi) {
      case ggp::EPI_BIAS: return LR(ggp::EPI_BIAS);
      case ggp::EPI_GELU: return LR(ggp::EPI_GELU);
      default: return LR(ggp::EPI_RES);
    }
#undef LR
  }
  switch (epi) {
    case ggp::EPI_BIAS: return L(256, ggp::EPI_BIAS);
    case ggp::EPI_GELU: return L(256, ggp::EPI_GELU);
    default: return L(256, ggp::EPI_RES);
  }
#undef L
}
