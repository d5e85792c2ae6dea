// 256x256 "8-phase" persistent bf16 GEMM for the encoder's large projections (bge-base /
// e5-large, the MiniLM FFN1), same contract as gemm.hip's symb_gemm:
//
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] )      epi = bias | GELU(erf) | + residual
//
// Replaces the 2-barrier-per-k-tile loop (gemm.hip) on shapes with N % 256 == 0, K % 128 == 0:
// that loop drains every LDS-DMA with vmcnt(0) before its barrier and, at one 256x256 workgroup
// per CU, exposes the load latency once per k-tile (782 TFLOP/s on bge FFN1 vs hipBLASLt 1.15 PF).
//
// Structure (one 512-thread workgroup per CU, persistent over tiles; 8 waves as 2 (M) x 4 (N),
// wave tile 128 x 64):
//  * A k-tile (BK = 64, 128-byte LDS rows) is four HALF-TILES: A0/A1 = tile rows 0-127 / 128-255,
//    B0/B1 = W rows 0-127 / 128-255, 16 KiB each, two LDS buffers (128 KiB).  A wave's 128 rows
//    are 64 in A0 + 64 in A1 and its 64 columns 32 in B0 + 32 in B1, so a k-tile is consumed in
//    four PHASES, one C quadrant (A half x B half, 16 MFMAs of 16x16x32) each:
//        P1: read A0,B0 -> MFMA(A0,B0)   P2: read B1 -> (A0,B1)   P3: read A1 -> (A1,B1)
//        P4: -> (A1,B0)
//  * Every phase is  ds_reads | LDS-DMA issue | [counted vmcnt] | s_barrier | lgkmcnt(0) |
//    16 MFMAs at raised priority | s_barrier, and the two wave groups (wr = 0 / 1, one wave of
//    each per SIMD) run one barrier apart: one group's reads and DMA issue fly under the other
//    group's MFMAs, and no barrier ever waits for vmcnt(0).
//  * A half-tile is refilled as soon as every wave's last read of it has retired (two phases
//    after the reading phase): {A0,B0} in P3, B1 in P4, A1 in P5 (= the next k-tile's P1), so
//    three half-tiles are in flight when a k-tile is waited for (vmcnt(6), once per k-tile).
//  * LDS image per half-tile: lane-linear for the DMA, 16-byte chunk index XORed with
//    (row >> 1) & 7 on the global source address and on the ds_read address (both sides).
//  * Persistent: grid = min(tiles, CUs); a workgroup walks tiles blockIdx, + grid, ... in the
//    XCD-aware grouped order of gemm.hip.  The next tile's first two k-tiles are DMA'd into the
//    (then idle) k-tile buffers BEFORE this tile's epilogue, which stages its bf16 output through
//    the last 32 KiB of LDS in four 64-row passes: bias / GELU on the accumulators, adjacent
//    columns paired across lanes by one DPP swap (4-byte LDS writes), then row-contiguous
//    16-byte reads -> (+ residual) -> 16-byte global stores, 16 per lane.  Those stores are
//    younger than the next tile's first DMA, so the next tile's counted waits let them drain
//    under its first MFMA phases (the store burst of 256 CUs finishing together was ~5 us of a
//    29 us K = 768 tile when waited for; benchmarks/gemm_one.py --abl).
#include "common.h"

namespace symb {

enum { G256_BIAS = 0, G256_GELU = 1, G256_RES = 2 };

namespace g256 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 512;
constexpr int HALF_BYTES = 128 * 128;          // 128 rows x 128 bytes
constexpr int BUF_BYTES = 4 * HALF_BYTES;      // A0 A1 B0 B1
// bf16 output staging: 64 rows x 512 B beside the two k-tile buffers (all 160 KiB in use); the
// 16-byte chunk index is XORed with (row >> 1) & 7, which keeps both the DPP-paired 4-byte
// writes (8 rows x 16 columns per instruction) and the row-contiguous 16-byte reads conflict-free
constexpr int STAGE_ROW = BN * 2;
constexpr int STAGE = 2 * BUF_BYTES;           // byte offset of the staging rows
constexpr int LDS = STAGE + 64 * STAGE_ROW;    // 163,840 B
constexpr int STORES = 16;                     // 16-byte output stores per lane per full tile
static_assert(LDS <= 160 * 1024, "LDS budget");

__device__ __forceinline__ uint32_t stage_off(int row, int col) {   // col in bf16 elements
  return (uint32_t)(STAGE + row * STAGE_ROW + ((((col >> 3) ^ ((row >> 1) & 7))) << 4) +
                    (col & 7) * 2);
}

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// tile id -> (m0, n0): XCD-aware bijective remap, then grouped order (a group_m-row band walked
// column by column, so A row panels and W column panels stay in that XCD's L2)
__device__ __forceinline__ void tile_origin(int id, int n_all, int n_tiles, int group_m, int& m0,
                                            int& n0) {
  const int tile = xcd_remap(id, n_all);
  int tm = tile / n_tiles, tn = tile % n_tiles;
  if (group_m > 1) {
    const int m_tiles = n_all / n_tiles, per_group = group_m * n_tiles;
    const int g = tile / per_group, first = g * group_m;
    const int gm = min(group_m, m_tiles - first), local = tile - g * per_group;
    tm = first + local % gm;
    tn = local / gm;
  }
  m0 = tm * BM;
  n0 = tn * BN;
}

}  // namespace g256

// ABL (profiling builds only, symb_gemm256_ablate): 0 = full kernel, 1 = epilogue computes but
// stores nothing (the values stay live), 2 = no epilogue work at all (accumulators kept live)
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(
    const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ W, int ldw,
    const float* __restrict__ bias, const __bf16* __restrict__ R, int ldr,
    __bf16* __restrict__ C, int ldc, int M, int N, int K, int group_m) {
  using namespace g256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int n_tiles = N / BN, n_all = ((M + BM - 1) / BM) * n_tiles;
  const int KT = K / BK;
  const bool lagging = __builtin_amdgcn_readfirstlane(wr) == 1;

  // ---- LDS-DMA of one half-tile (h: 0 = A0, 1 = A1, 2 = B0, 3 = B1) of k-tile kt into buf ----
  // per-thread source offsets are k-tile invariant: two 16-byte pieces per thread per half
  uint32_t src_off[4][2];   // element offsets (< 2^32: M*lda and N*ldw stay far below)
  auto set_tile = [&](int m0, int n0) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int s = i * NT + tid;
        const int row = s >> 3, c = (s & 7) ^ ((row >> 1) & 7);
        if (h < 2) {
          const int grow = min(m0 + h * 128 + row, M - 1);
          src_off[h][i] = (uint32_t)(grow * lda + c * 8);
        } else {
          src_off[h][i] = (uint32_t)((n0 + (h - 2) * 128 + row) * ldw + c * 8);
        }
      }
  };
  auto dma = [&](int h, int kt, int buf) {
    const __bf16* base = (h < 2 ? A : W) + (size_t)kt * BK;
    char* dst = smem + buf * BUF_BYTES + h * HALF_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(base + src_off[h][i], dst + (i * NT + wave * 64) * 16);
  };
  auto dma_ktile = [&](int kt, int buf) {
#pragma unroll
    for (int h = 0; h < 4; ++h) dma(h, kt, buf);
  };

  // ---- fragment reads (16x16x32: lane row = lane & 15, 8 k at chunk kk * 4 + lane >> 4) ----
  const int fr = lane & 15, fq = lane >> 4;
  // A fragments of ONE half at a time (A0 is dead after P2 when A1 is read in P3); both B halves
  // stay resident (B0 is used again in P4): 32 + 32 VGPRs beside 128 accumulator registers
  bf16x8 a[2][4];      // [kk][16-row fragment]
  bf16x8 b[2][2][2];   // [B half][kk][16-col fragment]
  // the XOR term (row >> 1) & 7 of every fragment row is (fr >> 1) & 7 (rows step by 16), so a
  // fragment address is one of 2 per-lane bases (kk) + a compile-time offset (buffer, half, i/j)
  const int x = (fr >> 1) & 7;
  uint32_t oa[2], ob[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    oa[kk] = (uint32_t)((wr * 64 + fr) * 128 + (((kk * 4 + fq) ^ x) << 4));
    ob[kk] = (uint32_t)(2 * HALF_BYTES + (wc * 32 + fr) * 128 + (((kk * 4 + fq) ^ x) << 4));
  }
  auto lds_read = [&](uint32_t off) { return *reinterpret_cast<const bf16x8*>(smem + off); };
  auto read_a = [&](int buf, int ha) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[kk][i] = lds_read(oa[kk] + buf * BUF_BYTES + ha * HALF_BYTES + i * 2048);
  };
  auto read_b = [&](int buf, int hb) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[hb][kk][j] = lds_read(ob[kk] + buf * BUF_BYTES + hb * HALF_BYTES + j * 2048);
  };

  f32x4 acc[2][4][2][2];   // [A half][i][B half][j]
  auto mfma_quadrant = [&](int ha, int hb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ha][i][hb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[hb][kk][j],
                                                                       acc[ha][i][hb][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // barrier | retire this phase's reads | (the caller's MFMAs) -- the sched_barrier keeps the
  // register-only MFMAs from being hoisted above the asm wait (hipcc does not order them by it)
  auto enter = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto leave = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };

  int id = blockIdx.x;
  int m0, n0;
  tile_origin(id, n_all, n_tiles, group_m, m0, n0);
  set_tile(m0, n0);
  // first tile: k-tile 0 -> buf 0, k-tile 1 -> buf 1 (later tiles get them during the epilogue)
  dma_ktile(0, 0);
  dma_ktile(1, 1);
  // the previous tile's epilogue left exactly STORES output stores per lane in flight (a full
  // tile), issued AFTER this tile's k-tile 0/1 DMA: the counted waits below let them drain under
  // the first MFMA phases instead of waiting for them (vmcnt retires in issue order)
  bool pend = false;

#pragma unroll 1
  for (; id < n_all; id += gridDim.x) {
    // k-tile 0 landed (k-tile 1's 8 pieces -- and pending stores -- may still fly)
    if (pend)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(8 + STORES) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[ha][i][hb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // PING-PONG: the wr = 1 waves run one barrier behind the wr = 0 waves, so on every SIMD (one
    // wave of each group) one wave's MFMAs cover the other's LDS reads and DMA issue.  Ordering
    // then needs one barrier more: DMA into a half-tile two phases after its last read, reads of
    // a k-tile one phase after every wave's vmcnt for it (both hold for either group's offset).
    if (lagging) __builtin_amdgcn_s_barrier();

    // ---- main loop: two k-tiles (buf 0 = t, buf 1 = t + 1) per iteration, 8 phases ----
#pragma unroll 1
    for (int t = 0; t < KT; t += 2) {
      const bool more = t + 2 < KT;   // k-tiles t+2 / t+3 exist (KT is even)
      // P1: buf 0 A0,B0.  (steady state: buf 1's A1 for k-tile t+1 goes out here)
      read_a(0, 0);
      read_b(0, 0);
      if (t > 0) dma(1, t + 1, 1);
      enter();
      mfma_quadrant(0, 0);
      leave();
      // P2
      read_b(0, 1);
      enter();
      mfma_quadrant(0, 1);
      leave();
      // P3: A0,B0 of buf 0 were last read in P1 -> refill with k-tile t+2
      read_a(0, 1);
      if (more) {
        dma(0, t + 2, 0);
        dma(2, t + 2, 0);
      }
      enter();
      mfma_quadrant(1, 1);
      leave();
      // P4: B1 of buf 0 (read in P2) -> refill; then k-tile t+1 (buf 1) must have landed: three
      // half-tiles of k-tile t+2 may stay in flight (6 DMA instructions)
      if (more) {
        dma(3, t + 2, 0);
        if (pend)   // (first k-tile pair only) the stores are older than P3/P4's DMA
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(6 + STORES) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pend = false;
      enter();
      mfma_quadrant(1, 0);
      leave();
      // P5: buf 1 A0,B0; A1 of buf 0 (read in P3) -> refill
      read_a(1, 0);
      read_b(1, 0);
      if (more) dma(1, t + 2, 0);
      enter();
      mfma_quadrant(0, 0);
      leave();
      // P6
      read_b(1, 1);
      enter();
      mfma_quadrant(0, 1);
      leave();
      // P7: buf 1 A0,B0 (read in P5) -> k-tile t+3
      read_a(1, 1);
      if (more) {
        dma(0, t + 3, 1);
        dma(2, t + 3, 1);
      }
      enter();
      mfma_quadrant(1, 1);
      leave();
      // P8: buf 1 B1 -> k-tile t+3; k-tile t+2 (buf 0) must have landed before the next P1
      if (more) {
        dma(3, t + 3, 1);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
      enter();
      mfma_quadrant(1, 0);
      leave();
    }
    if (!lagging) __builtin_amdgcn_s_barrier();   // re-align: every wave's reads have retired

    // ---- epilogue: residual prefetch, next tile's first k-tiles, 4 passes of 64 staged rows ----
    const int cm0 = m0, cn0 = n0;
    const bool full = cm0 + BM <= M;
    // pass p stages tile rows 64p .. 64p+63 (A half p >> 1, the waves with wr == p & 1); every
    // thread then moves 4 row-contiguous 16-byte chunks of them: chunk c = q * 512 + tid
    bf16x8 res[4][4];
    if constexpr (EPI == G256_RES) {   // before the DMA: waiting for these never waits for it
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = q * NT + tid, row = c >> 5;
          const int grow = min(cm0 + 64 * p + row, M - 1);
          res[p][q] = *reinterpret_cast<const bf16x8*>(R + (size_t)grow * ldr + cn0 + (c & 31) * 8);
        }
    }
    if (id + (int)gridDim.x < n_all) {
      tile_origin(id + gridDim.x, n_all, n_tiles, group_m, m0, n0);
      set_tile(m0, n0);
      dma_ktile(0, 0);
      dma_ktile(1, 1);
    }
    if constexpr (ABL == 2) {
#pragma unroll
      for (int ha = 0; ha < 2; ++ha)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int hb = 0; hb < 2; ++hb)
#pragma unroll
            for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[ha][i][hb][j]));
      continue;
    }
    // A 16x16 accumulator block gives lane (fr, fq) rows fq*4 .. +3 of column fr.  After bias /
    // GELU, one DPP swap with lane fr ^ 1 pairs adjacent columns: an even lane keeps rows 0-1 of
    // columns (fr, fr+1), an odd lane rows 2-3 of (fr-1, fr) -> two 4-byte LDS writes per block.
    const bool odd = fr & 1;
    const int prow = fq * 4 + (odd ? 2 : 0);
    const int pcol = fr & ~1;
    // staging addresses: every row a lane writes has the same XOR term ((prow >> 1) & 7: rows
    // step by 16, and prow + 1 shares prow's pair), so writes are 2 per-lane bases (j) plus
    // compile-time offsets (i: 16 rows, hb: 16 chunks, second row: 512 B)
    const int x2 = (prow >> 1) & 7;
    uint32_t sbase[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      sbase[j] = (uint32_t)(STAGE + prow * STAGE_ROW +
                            (((wc * 4 + j * 2 + (pcol >> 3)) ^ x2) << 4) + (pcol & 7) * 2);
    const uint32_t rbase = stage_off(tid >> 5, (tid & 31) * 8);   // + 16 rows per q
    float bv[2][2];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[hb][j] = bias[cn0 + hb * 128 + wc * 32 + j * 16 + fr];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int ha = p >> 1;
      if ((p & 1) == (int)lagging) {   // this wave's rows are the pass's rows
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int hb = 0; hb < 2; ++hb)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              float v[4], w[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                v[r] = acc[ha][i][hb][j][r] + bv[hb][j];
                if constexpr (EPI == G256_GELU) v[r] = gelu_erf(v[r]);
              }
#pragma unroll
              for (int r = 0; r < 4; ++r)   // quad_perm [1,0,3,2]: the value of column fr ^ 1
                w[r] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[r]), 0xB1,
                                                                  0xF, 0xF, false));
              const bf16x2 p0{(__bf16)(odd ? w[2] : v[0]), (__bf16)(odd ? v[2] : w[0])};
              const bf16x2 p1{(__bf16)(odd ? w[3] : v[1]), (__bf16)(odd ? v[3] : w[1])};
              const uint32_t so = sbase[j] + i * 16 * STAGE_ROW + hb * 256;
              *reinterpret_cast<bf16x2*>(smem + so) = p0;
              *reinterpret_cast<bf16x2*>(smem + so + STAGE_ROW) = p1;
            }
      }
      // raw barriers: a __syncthreads would drain the next tile's DMA (vmcnt(0))
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = q * NT + tid, row = c >> 5, col = (c & 31) * 8;   // row = 16 q + tid / 32
        bf16x8 o = *reinterpret_cast<const bf16x8*>(smem + rbase + q * 16 * STAGE_ROW);
        if constexpr (EPI == G256_RES) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (__bf16)((float)o[e] + (float)res[p][q][e]);
        }
        const int grow = cm0 + 64 * p + row;
        if constexpr (ABL == 1) {
          asm volatile("" ::"v"(o));
        } else if (full || grow < M) {
          *reinterpret_cast<bf16x8*>(C + (size_t)grow * ldc + cn0 + col) = o;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // every read of the staging rows retired before pass p+1
    }
    // a partial tile may have skipped stores: then the next tile start waits for everything
    pend = full && ABL == 0;
    if (!full) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace symb

using namespace symb;

static int g_abl = 0;

// Shapes this kernel takes: N % 256 == 0, K % 128 == 0 (an even number of 64-deep k-tiles).
bool symb_gemm256_supported(int M, int N, int K) {
  return M > 0 && N % 256 == 0 && K % 128 == 0 && K >= 128;
}

// epi: 0 bias, 1 GELU, 2 residual (gemm.hip's EPI_BIAS / EPI_GELU / EPI_RES).
// Returns 0, a HIP error code, or -1 for an unsupported shape / epilogue.
int symb_gemm256(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                 const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                 hipStream_t st) {
  if (M <= 0) return 0;
  if (!symb_gemm256_supported(M, N, K)) return -1;
  static int n_cus = 0;
  if (n_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cus <= 0)
      n_cus = 256;
  }
  const int tiles = ((M + 255) / 256) * (N / 256);
  const int grid = tiles < n_cus ? tiles : n_cus;   // persistent: <= one workgroup per CU
  auto go = [&](auto kern) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                g256::LDS);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), g256::LDS, st, (const __bf16*)A, lda,
                       (const __bf16*)W, ldw, bias, (const __bf16*)R, ldr, (__bf16*)C, ldc, M, N,
                       K, group_m);
    return (int)hipGetLastError();
  };
  if (g_abl == 1) return epi == G256_GELU ? go(gemm256_kernel<G256_GELU, 1>) : go(gemm256_kernel<G256_BIAS, 1>);
  if (g_abl == 2) return go(gemm256_kernel<G256_BIAS, 2>);
  switch (epi) {
    case G256_BIAS: return go(gemm256_kernel<G256_BIAS>);
    case G256_GELU: return go(gemm256_kernel<G256_GELU>);
    case G256_RES: return go(gemm256_kernel<G256_RES>);
  }
  return -1;
}

// profiling-only: 0 full kernel, 1 no output stores, 2 no epilogue (see gemm256_kernel ABL)
int symb_gemm256_ablate(int abl) {
  if (abl < 0 || abl > 2) return -1;
  g_abl = abl;
  return 0;
}
