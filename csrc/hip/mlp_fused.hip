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
// workgroup; it measured parity-to-slower and was removed in round 5.)
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

  // step q of the whole sequence -> (chunk, phase step); DMA into slot q & 1
  auto stage = [&](int q) {
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
          const void* src = reinterpret_cast<const char*>(X + (size_t)grow * MF_H) + k0 + ch * 16;
          void* dst = base + t * (MF_BM * 128) + (i * MF_NT + wave * 64) * 16;
          glds16(src, dst);
        }
#pragma unroll
        for (int i = 0; i < (MF_FC * 8) / MF_NT; ++i) {
          const int v = i * MF_NT + tid;
          const int row = v >> 3, pc = v & 7, ch = pc ^ ((row >> 1) & 7);
          glds16(reinterpret_cast<const char*>(W1 + (size_t)(c * MF_FC + row) * MF_H) + k0 + ch * 16,
                 base + (MF_KA + t) * (MF_BM * 128) + (i * MF_NT + wave * 64) * 16);
        }
      }
    } else {
      const size_t k0 = (size_t)(c * MF_FC + (s - KT_A) * 64) * 2;
#pragma unroll
      for (int i = 0; i < (MF_H * 8) / MF_NT; ++i) {
        const int v = i * MF_NT + tid;
        const int row = v >> 3, pc = v & 7, ch = pc ^ ((row >> 1) & 7);
        glds16(reinterpret_cast<const char*>(W2 + (size_t)row * MF_FF) + k0 + ch * 16,
               base + (i * MF_NT + wave * 64) * 16);
      }
    }
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

// ---------------------------------------------------------------------------------------------
// Register-resident form (the MiniLM forward's FFN blocks were ~53 % of it).
// Four waves, ONE per SIMD (512 registers each), 32 token rows per wave, 128 per workgroup:
//  * the wave's X rows (32 x 384) are loaded ONCE into VGPRs as B-operand fragments (96 VGPRs)
//    instead of being re-streamed through LDS for each of the 12 chunks (1.1 MiB of the 3.5 MiB
//    the LDS form moved per workgroup);
//  * H_c never touches LDS: phase A computes H_c^T (W1_c rows as the A operand), so a lane holds
//    4 consecutive intermediate columns of one token -- after GELU and the bf16 rounding, two of
//    those tiles ARE the B operand of phase B under a fixed permutation of the k index, and the
//    W2 fragments are read with the same permutation (two 8-byte reads per fragment);
//  * phase B accumulates out^T (W2 rows as the A operand): a lane ends with 4 consecutive output
//    columns of one token, so the residual add, the LayerNorm (row sums over the 4 lanes of a
//    token: two shuffles) and the 8-byte bf16 stores need no LDS staging at all;
//  * LDS holds only the weight stream: a 3-slot ring of 48 KiB steps (W1_c in 2 steps of 3
//    k-tiles, W2_c in 2 steps of one 384-row k-tile), each step's LDS-DMA issued two steps ahead.
constexpr int MR_BM = 128, MR_NW = 4, MR_NT = 64 * MR_NW;
constexpr int MR_SLOT = 48 * 1024, MR_NSLOT = 3;
constexpr int MR_B1 = MR_SLOT * MR_NSLOT;            // b1 (1536 floats) parked in LDS
constexpr int MR_LDS = MR_B1 + MF_FF * 4;
constexpr int MR_SPC = 4;                            // ring steps per 128-column chunk
constexpr int MR_NSTEP = (MF_FF / MF_FC) * MR_SPC;   // 48
constexpr int MR_DMA = 12;                           // LDS-DMA pieces per lane per step

__global__ __launch_bounds__(MR_NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
void mlp_reg_kernel(const __bf16* X, const __bf16* __restrict__ W1, const float* __restrict__ b1,
                    const __bf16* __restrict__ W2, const float* __restrict__ b2,
                    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                    int gelu_poly, __bf16* C, int M) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * MR_BM + wave * 32;   // this wave's rows

  // ring step q -> slot q % 3.  s = q % 4: 0, 1 = W1_c (rows 128c ..) k-tiles 3s .. 3s + 2;
  // 2, 3 = W2 (all 384 rows) k-tile 2c + s - 2 of its 1536 columns.  Piece v = i * 256 + tid is
  // row 32i + (tid >> 3) of a tile; its swizzled chunk (tid & 7) ^ ((tid >> 4) & 7) does not
  // depend on i, so a lane keeps ONE base address per matrix and every piece adds a uniform
  // offset (per-piece 64-bit addresses held across the loop spilled registers)
  const int lrow = tid >> 3, lch = (tid & 7) ^ ((tid >> 4) & 7);
  const char* w1p = reinterpret_cast<const char*>(W1) + (size_t)lrow * MF_H * 2 + lch * 16;
  const char* w2p = reinterpret_cast<const char*>(W2) + (size_t)lrow * MF_FF * 2 + lch * 16;
  auto stage = [&](int q) {
    const int c = q / MR_SPC, s = q % MR_SPC;
    char* base = smem + (q % MR_NSLOT) * MR_SLOT + wave * 64 * 16;
    if (s < 2) {
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < (MF_FC * 8) / MR_NT; ++i)
          glds16(w1p + (size_t)(c * MF_FC + 32 * i) * MF_H * 2 + (3 * s + t) * 128,
                 base + t * (MF_FC * 128) + i * MR_NT * 16);
    } else {
      const int kt = 2 * c + s - 2;
#pragma unroll
      for (int i = 0; i < (MF_H * 8) / MR_NT; ++i)
        glds16(w2p + (size_t)(32 * i) * MF_FF * 2 + kt * 128, base + i * MR_NT * 16);
    }
  };

  // b1 into LDS (read per chunk with ds_read: a global load there would be counted in vmcnt
  // behind the ring's LDS-DMA and its wait would drain the prefetch)
  float* b1s = reinterpret_cast<float*>(smem + MR_B1);
  for (int i = tid; i < MF_FF / 4; i += MR_NT)
    reinterpret_cast<f32x4*>(b1s)[i] = reinterpret_cast<const f32x4*>(b1)[i];
  // the wave's 32 X rows as B fragments: token 16i + r16, k 32ks + 8g4 .. + 7
  bf16x8 xf[2][12];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const __bf16* xr = X + (size_t)min(m0 + 16 * i + r16, M - 1) * MF_H + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) xf[i][ks] = *reinterpret_cast<const bf16x8*>(xr + 32 * ks);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (X and b1 landed before the ring starts)
  stage(0);
  stage(1);

  f32x4 acc[2][24];     // out^T: token 16i + r16, output columns 16j + 4g4 + e
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 24; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // step q's pieces landed (this wave: all but the next step's MR_DMA; every wave: the
  // barrier); slot (q + 2) % 3 was last read in step q - 1, so it is free to refill
  // (a raw s_barrier: __syncthreads would drain vmcnt to 0 -- the next step's pieces too --
  // which serialised the ring; every wave's reads of the slot being refilled retired with its
  // lgkmcnt(0) before the barrier)
  auto step_begin = [&](int q) {
    if (q + 1 < MR_NSTEP)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(MR_DMA) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (q + 2 < MR_NSTEP) stage(q + 2);
  };

#pragma unroll 1
  for (int c = 0; c < MF_FF / MF_FC; ++c) {
    // ---- phase A: H_c^T = W1_c X^T (lane: token 16i + r16, H_c columns 16j + 4g4 + e) ----
    f32x4 ha[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) ha[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = c * MR_SPC + s;
      step_begin(q);
      const char* base = smem + (q % MR_NSLOT) * MR_SLOT;
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int ks = (3 * s + t) * 2 + kk;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bf16x8 wf = *reinterpret_cast<const bf16x8*>(
                base + t * (MF_FC * 128) + mf_swz(16 * j + r16, 4 * kk + g4));
#pragma unroll
            for (int i = 0; i < 2; ++i)
              ha[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf[i][ks], ha[i][j], 0, 0, 0);
          }
        }
    }
    // ---- GELU(+ b1) -> bf16 B fragments of phase B: hb[i][kb] positions 0..3 = H_c columns
    //      32kb + 4g4 + e, positions 4..7 = 32kb + 16 + 4g4 + e (tiles 2kb, 2kb + 1) ----
    bf16x8 hb[2][4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + c * MF_FC + 16 * j + 4 * g4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
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
        const int p = (j & 1) * 4;
        hb[i][j >> 1][p + 0] = (__bf16)y0.x;
        hb[i][j >> 1][p + 1] = (__bf16)y0.y;
        hb[i][j >> 1][p + 2] = (__bf16)y1.x;
        hb[i][j >> 1][p + 3] = (__bf16)y1.y;
      }
    }
    // ---- phase B: out^T += W2_c H_c^T, k in the permuted order of hb ----
    typedef short s16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int s = 2; s < 4; ++s) {
      const int q = c * MR_SPC + s;
      step_begin(q);
      const char* base = smem + (q % MR_NSLOT) * MR_SLOT;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kb = (s - 2) * 2 + kk;
        const int ch = 4 * kk + (g4 >> 1), off = (g4 & 1) * 8;
#pragma unroll
        for (int j = 0; j < 24; ++j) {
          const int row = 16 * j + r16;
          const s16x4 lo = *reinterpret_cast<const s16x4*>(base + mf_swz(row, ch) + off);
          const s16x4 hi = *reinterpret_cast<const s16x4*>(base + mf_swz(row, ch + 2) + off);
          const bf16x8 wf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, hb[i][kb], acc[i][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: + b2 + X, LayerNorm over the token's 384 columns (4 lanes), bf16 stores ----
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int t = m0 + 16 * i + r16;
    const __bf16* xr = X + (size_t)min(t, M - 1) * MF_H + 4 * g4;
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b2 + 16 * j + 4 * g4);
      const bf16x4 rr = *reinterpret_cast<const bf16x4*>(xr + 16 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[i][j][e] += bb[e] + (float)rr[e];
        sm += acc[i][j][e];
      }
    }
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    const float mean = sm * (1.0f / MF_H);
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 24; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) ss += (acc[i][j][e] - mean) * (acc[i][j][e] - mean);
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    const float rstd = rsqrtf(ss * (1.0f / MF_H) + eps);
    if (t < M) {
      __bf16* o = C + (size_t)t * MF_H + 4 * g4;
#pragma unroll
      for (int j = 0; j < 24; ++j) {
        const f32x4 gg = *reinterpret_cast<const f32x4*>(gamma + 16 * j + 4 * g4);
        const f32x4 be = *reinterpret_cast<const f32x4*>(beta + 16 * j + 4 * g4);
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (__bf16)((acc[i][j][e] - mean) * rstd * gg[e] + be[e]);
        *reinterpret_cast<bf16x4*>(o + 16 * j) = v;
      }
    }
  }
}

}  // namespace

}  // namespace symb

using namespace symb;

// FFN block form: 1 = the LDS-staged kernel (mlp_fused_kernel), 2 = the register-resident one
// (mlp_reg_kernel); see symb_mlp_fused_form.
static int g_mlp_form = 2;
int symb_mlp_fused_form(int form) {
  if (form == 0) return g_mlp_form;
  if (form != 1 && form != 2) return -1;
  g_mlp_form = form;
  return 0;
}

// The whole FFN block of a 384-wide layer in one launch (X, C: [M, 384] bf16, row stride 384;
// C must not alias X).  Returns 0, a HIP error, or -1 (shape not supported).
int symb_mlp_fused(const void* X, const void* W1, const float* b1, const void* W2, const float* b2,
                   const float* gamma, const float* beta, float eps, int gelu_poly, void* C, int M,
                   int H, int FF, hipStream_t st) {
  if (M <= 0) return 0;
  if (H != MF_H || FF != MF_FF || X == C) return -1;
  if (g_mlp_form == 2) {
    set_max_lds<mlp_reg_kernel>(MR_LDS);
    hipLaunchKernelGGL(mlp_reg_kernel, dim3((M + MR_BM - 1) / MR_BM), dim3(MR_NT), MR_LDS, st,
                       (const __bf16*)X, (const __bf16*)W1, b1, (const __bf16*)W2, b2, gamma, beta,
                       eps, gelu_poly, (__bf16*)C, M);
    return (int)hipGetLastError();
  }
  const dim3 grid((M + MF_BM - 1) / MF_BM), block(MF_NT);
  set_max_lds<mlp_fused_kernel>(MF_LDS);
  hipLaunchKernelGGL(mlp_fused_kernel, grid, block, MF_LDS, st, (const __bf16*)X,
                     (const __bf16*)W1, b1, (const __bf16*)W2, b2, gamma, beta, eps, gelu_poly,
                     (__bf16*)C, M);
  return (int)hipGetLastError();
}
