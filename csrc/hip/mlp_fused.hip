// Fused BERT feed-forward block for 384-wide encoders (all-MiniLM-L6-v2, the headline model):
//
//   out[M, 384] = LayerNorm( GELU(X W1^T + b1) W2^T + b2 + X )      W1: [1536, 384], W2: [384, 1536]
//
// Replaces the reference's intermediate + output linears of each BERT layer (candle BertModel's
// BertIntermediate / BertOutput: /root/reference/services/preprocessing_service/src/
// embedding_generator.rs:198), which this repo otherwise runs as two GEMMs (gemm.hip EPI_GELU,
// then EPI_RES_LN) with a 4H-wide activation round trip through HBM: at 32768 tokens that is a
// 100 MB write plus a 100 MB read per layer, and the FFN1 GEMM's short K (384) leaves its 128x128
// tiles mostly prologue and epilogue (profiles/r4_mlp: 66 + 63 us per layer).
//
// Measured (profiles/r4_mlp/README.md): 110 us per layer against 129 us for the two GEMMs
// (128 us with one k-tile per phase-A stage); still ~3.5x its MFMA floor -- 60 ring steps, each a
// barrier plus an L2 round trip for a 48-64 KiB stage (deeper rings and an LDS-resident X
// measured slower: v3 / v4 there).
//
// CDNA4 design (one 128-row block of tokens per workgroup, 8 waves as 4 x 2):
//  * The 1536-wide intermediate is produced and consumed in 12 chunks of 128 columns that never
//    leave the CU: phase A computes the chunk H_c = GELU(X W1_c^T + b1_c) (128 x 128, K = 384)
//    into fp32 accumulators, rounds it to bf16 (the same rounding the two-GEMM path stores) into
//    LDS; phase B accumulates out += H_c W2_c^T (128 x 384, K = 128) into registers that live
//    across all 12 chunks (24 accumulators per wave).
//  * Operands stream through ONE 2-slot LDS ring of 64 KiB slots: phase A's stages (two k-tiles
//    each of X 128 x 64 and W1_c 128 x 64 = 64 KiB) and phase B's (W2_c 384 x 64 = 48 KiB) form
//    one sequence of 5 steps per chunk; step s+1's global_load_lds DMA is issued right after
//    step s's barrier, so every load overlaps the previous step's MFMAs, across phase and chunk
//    boundaries alike.
//  * X (re-read per chunk) and W1 / W2 (re-read per row block) come from L2: X's 96 KiB row
//    panel is private to the workgroup, the 2.4 MB of weights are shared by all of them.
//  * v_mfma_f32_16x16x32_bf16; 128-byte LDS rows with the XOR chunk swizzle of gemm.hip on both
//    the DMA source address and the ds_read address; H_c is written in the same swizzled layout,
//    so phase B reads it exactly like a DMA'd tile.
//  * Epilogue: + b2 + X (the residual is the block's own input), LayerNorm over the 384 columns,
//    bf16 16-byte stores; the fp32 tile is staged through LDS in two 64-row passes.
#include "common.h"

namespace symb {

namespace {

constexpr int MF_H = 384, MF_FF = 1536, MF_BM = 128, MF_FC = 128;
constexpr int MF_WM = 4, MF_WN = 2, MF_NW = MF_WM * MF_WN, MF_NT = 64 * MF_NW;
constexpr int MF_KA = 2;                             // k-tiles of X and W1_c per phase-A stage
constexpr int MF_SLOT = 64 * 1024;                   // one ring slot (a phase-A stage)
constexpr int MF_HC = 2 * MF_SLOT;                   // H_c: 2 k-tiles of 128 rows x 128 B
constexpr int MF_LDS = MF_HC + 2 * MF_BM * 128;      // 160 KiB: all of it
constexpr int MF_CS = MF_H + 4;                      // epilogue fp32 row stride
static_assert(64 * MF_CS * 4 <= MF_LDS, "epilogue pass fits the LDS");

__device__ __forceinline__ int mf_swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// (Round 4 also built a form that ran the attention out-projection + LayerNorm first in the same
// workgroup; it measured parity-to-slower and was removed in round 5.  Round 6 built a register-
// resident form -- 4 waves of 512 registers, X and the GELU intermediate in VGPRs, k-permuted W2
// fragments, LayerNorm across the 4 lanes of a token, only the weights through a 3-slot LDS ring:
// exact, but 1.56-1.60 ms per MiniLM forward against 1.25-1.27 with this kernel (24 VGPRs
// spilled, reloads draining the ring), so it was removed: profiles/r6_gemm/README.md.)
__global__ __launch_bounds__(MF_NT) void mlp_fused_kernel(
    const __bf16* X, const __bf16* __restrict__ W1, const float* __restrict__ b1,
    const __bf16* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int gelu_poly, __bf16* C, int M) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / MF_WN, wn = wave % MF_WN;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * MF_BM;
  constexpr int KT_A = MF_H / 64 / MF_KA;            // 3 stages of 2 k-tiles of X . W1_c^T
  constexpr int KT_B = MF_FC / 64;                   // 2 k-tiles of H_c . W2_c^T
  constexpr int STEPS = KT_A + KT_B;                 // per chunk
  constexpr int NCHUNK = MF_FF / MF_FC;
  char* hc = smem + MF_HC;

  // step q of the whole sequence -> (chunk, phase step) into slot q & 1: piece p of the step (a
  // 16-byte swizzled chunk per lane, global source src(p), lane-linear LDS position dst(p)), one
  // global_load_lds each.  (Register staging -- global_load_dwordx4 of step q + 1 before step
  // q's MFMAs, ds_write_b128 after them -- measured slower: MiniLM forward 1.32-1.33 vs
  // 1.26-1.27 ms, profiles/r6_gemm/README.md.)
  constexpr int NPB = (MF_H * 8) / MF_NT;                // phase-B pieces per lane (6)
  auto piece = [&](int q, auto fn) {
    const int c = q / STEPS, s = q % STEPS;
    char* base = smem + (q & 1) * MF_SLOT;
    if (s < KT_A) {
      // slot: X k-tiles 2s, 2s+1 (16 KiB each), then W1_c k-tiles 2s, 2s+1
#pragma unroll
      for (int t = 0; t < MF_KA; ++t) {
        const size_t k0 = (size_t)(s * MF_KA + t) * 128;   // byte offset of the k-tile
#pragma unroll
        for (int i = 0; i < (MF_BM * 8) / MF_NT; ++i) {
          const int v = i * MF_NT + tid;
          const int row = v >> 3, pc = v & 7, ch = pc ^ ((row >> 1) & 7);
          const int grow = min(m0 + row, M - 1);
          const char* src = reinterpret_cast<const char*>(X + (size_t)grow * MF_H) + k0 + ch * 16;
          fn(t * 4 + i, src, base + t * (MF_BM * 128) + (i * MF_NT + wave * 64) * 16);
        }
#pragma unroll
        for (int i = 0; i < (MF_FC * 8) / MF_NT; ++i) {
          const int v = i * MF_NT + tid;
          const int row = v >> 3, pc = v & 7, ch = pc ^ ((row >> 1) & 7);
          fn(t * 4 + 2 + i,
             reinterpret_cast<const char*>(W1 + (size_t)(c * MF_FC + row) * MF_H) + k0 + ch * 16,
             base + (MF_KA + t) * (MF_BM * 128) + (i * MF_NT + wave * 64) * 16);
        }
      }
    } else {
      const size_t k0 = (size_t)(c * MF_FC + (s - KT_A) * 64) * 2;
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        const int v = i * MF_NT + tid;
        const int row = v >> 3, pc = v & 7, ch = pc ^ ((row >> 1) & 7);
        fn(i, reinterpret_cast<const char*>(W2 + (size_t)row * MF_FF) + k0 + ch * 16,
           base + (i * MF_NT + wave * 64) * 16);
      }
    }
  };
  auto stage = [&](int q) {
    piece(q, [&](int, const char* src, char* dst) { glds16(src, dst); });
  };

  f32x4 acc[2][12];                                  // out rows wm*32 + 16i, cols wn*192 + 16j
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, g4 = lane >> 4;
  // step q landed; every wave is done with slot (q+1)&1 and with H_c's writes / reads
  auto step_begin = [&](int q) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (q + 1 < NCHUNK * STEPS) stage(q + 1);
  };
  // LayerNorm(acc + bias + R) of the block's 128 rows -> out (bf16); the fp32 tile is staged
  // through LDS (all of it may be overwritten) in two 64-row passes
  float* Cs = reinterpret_cast<float*>(smem);
  auto ln_store = [&](const float* bias, const __bf16* R, const float* g, const float* bt,
                      __bf16* out) {
#pragma unroll 1
  for (int p = 0; p < 2; ++p) {
    __syncthreads();   // (pass 0: every wave's last MFMA reads of the ring are done)
    if ((wm >> 1) == p) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 12; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = (wm & 1) * 32 + i * 16 + g4 * 4 + r;
            Cs[row * MF_CS + wn * 192 + j * 16 + r16] = acc[i][j][r];
          }
    }
    __syncthreads();
    constexpr int NV = MF_H / 8;                     // 48 eight-column groups: lanes 0..47
    for (int row = wave; row < 64; row += MF_NW) {
      const int grow = m0 + p * 64 + row;
      if (grow >= M) break;
      float x[8];
      float sum = 0.f;
      if (lane < NV) {
        float rr[8];
        load8(R + (size_t)grow * MF_H + lane * 8, rr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          x[e] = Cs[row * MF_CS + lane * 8 + e] + bias[lane * 8 + e] + rr[e];
          sum += x[e];
        }
      }
      const float mean = wave_sum(sum) * (1.0f / MF_H);
      float ss = 0.f;
      if (lane < NV)
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += (x[e] - mean) * (x[e] - mean);
      const float rstd = rsqrtf(wave_sum(ss) * (1.0f / MF_H) + eps);
      if (lane < NV) {
        float y[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          y[e] = (x[e] - mean) * rstd * g[lane * 8 + e] + bt[lane * 8 + e];
        store8(out + (size_t)grow * MF_H + lane * 8, y);
      }
    }
  }
  };

  stage(0);
  int q = 0;
#pragma unroll 1
  for (int c = 0; c < NCHUNK; ++c) {
    // phase A: H_c (rows wm*32 + 16i, cols wn*64 + 16j); its registers are dead in phase B
    f32x4 ha[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) ha[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KT_A; ++s, ++q) {
      step_begin(q);
#pragma unroll
      for (int kq = 0; kq < 2 * MF_KA; ++kq) {
        const int kt = kq >> 1, kk = kq & 1;
        const char* sA = smem + (q & 1) * MF_SLOT + kt * (MF_BM * 128);
        const char* sB = smem + (q & 1) * MF_SLOT + (MF_KA + kt) * (MF_BM * 128);
        const int chunk = kk * 4 + g4;
        bf16x8 a[2], b[4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(sA + mf_swz(wm * 32 + i * 16 + r16, chunk));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(sB + mf_swz(wn * 64 + j * 16 + r16, chunk));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ha[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], ha[i][j], 0, 0, 0);
      }
    }
    // H_c = GELU(. + b1) -> bf16 into the swizzled 2-k-tile image.  The MFMA operands are
    // swapped (W1_c rows first), so accumulator (i, j) holds H_c^T: lane element e is token row
    // wm*32 + 16i + (lane & 15), column wn*64 + 16j + 4 (lane >> 4) + e -- 4 consecutive columns
    // of one row, one 8-byte ds_write (a 2-byte scatter of 4 rows per lane bank-conflicted).
    // Element (row, col): k-tile col / 64, 16-byte chunk (col % 64) / 8, position col % 8.
    // (Every wave's phase-B reads of the previous chunk's H_c finished before this chunk's first
    // barrier.)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wn * 64 + j * 16 + g4 * 4;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + c * MF_FC + col);
      char* kt = hc + (col >> 6) * (MF_BM * 128);
      const int off = (col & 63) >> 3, pos = (col & 7) * 2;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 32 + i * 16 + r16;
        f32x2 y0{ha[i][j][0] + bb[0], ha[i][j][1] + bb[1]};
        f32x2 y1{ha[i][j][2] + bb[2], ha[i][j][3] + bb[3]};
        if (gelu_poly) {
          y0 = gelu2_poly(y0);
          y1 = gelu2_poly(y1);
        } else {
          y0.x = gelu_erf(y0.x);
          y0.y = gelu_erf(y0.y);
          y1.x = gelu_erf(y1.x);
          y1.y = gelu_erf(y1.y);
        }
        bf16x4 w;
        w[0] = (__bf16)y0.x;
        w[1] = (__bf16)y0.y;
        w[2] = (__bf16)y1.x;
        w[3] = (__bf16)y1.y;
        *reinterpret_cast<bf16x4*>(kt + mf_swz(row, off) + pos) = w;
      }
    }
    // phase B: out += H_c W2_c^T
#pragma unroll
    for (int t = 0; t < KT_B; ++t, ++q) {
      step_begin(q);
      const char* sA = hc + t * (MF_BM * 128);
      const char* sB = smem + (q & 1) * MF_SLOT;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + g4;
        bf16x8 a[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(sA + mf_swz(wm * 32 + i * 16 + r16, chunk));
#pragma unroll
        for (int j = 0; j < 12; ++j) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(sB + mf_swz(wn * 192 + j * 16 + r16, chunk));
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: + b2 + X, LayerNorm, bf16 ----
  ln_store(b2, X, gamma, beta, C);
}

}  // namespace

}  // namespace symb

using namespace symb;

// The whole FFN block of a 384-wide layer in one launch (X, C: [M, 384] bf16, row stride 384;
// C must not alias X).  Returns 0, a HIP error, or -1 (shape not supported).
int symb_mlp_fused(const void* X, const void* W1, const float* b1, const void* W2, const float* b2,
                   const float* gamma, const float* beta, float eps, int gelu_poly, void* C, int M,
                   int H, int FF, hipStream_t st) {
  if (M <= 0) return 0;
  if (H != MF_H || FF != MF_FF || X == C) return -1;
  const dim3 grid((M + MF_BM - 1) / MF_BM), block(MF_NT);
  set_max_lds<mlp_fused_kernel>(MF_LDS);
  hipLaunchKernelGGL(mlp_fused_kernel, grid, block, MF_LDS, st, (const __bf16*)X,
                     (const __bf16*)W1, b1, (const __bf16*)W2, b2, gamma, beta, eps, gelu_poly,
                     (__bf16*)C, M);
  return (int)hipGetLastError();
}
