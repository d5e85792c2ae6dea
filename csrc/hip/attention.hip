// Varlen (packed, unpadded) bidirectional flash attention for the encoder, head_dim 32 or 64.
//
// Replaces the reference's padded path (every sentence padded to max_position_embeddings=514,
// services/preprocessing_service/src/embedding_generator.rs:75-91) and candle's
// transpose_for_scores -> QK^T -> +mask -> softmax -> PV -> merge-heads chain (SURVEY.md §2.5
// K6-K11).  Sequences are packed back to back ([T, 3H] fused QKV rows, cu_seqlens offsets), so
// no FLOP or byte is spent on padding and no mask tensor exists.
//
// Per workgroup: 16*NWAVE query rows of one (sequence, head); NWAVE waves x 16 queries (NWAVE = 8
// covers a <=128-token sentence in ONE workgroup, so its K/V rows are read from HBM once instead of
// once per 64-query block).  gfx950 layout:
//  * S^T = K Q^T (v_mfma_f32_16x16x32_bf16, K = A operand from LDS, Q = B operand in registers):
//    a lane's accumulators are 4 keys x ONE query, so the softmax row statistics are lane-local
//    up to a 4-lane (shfl 16/32) reduction, and the probabilities feed the PV MFMA straight from
//    registers: P^T tiles n = 2t, 2t+1 (keys 4g+r and 16+4g+r of a 32-key step) ARE the B operand
//    of O^T = V^T P^T under a fixed permutation of the k index -- no LDS round trip for P.
//  * V stays row-major in LDS (16-byte staging writes) and the matching V^T A fragments come from
//    two ds_read_b64_tr_b16 (4 keys x 16 head dims each, hardware transpose).
//  * Bank conflicts: K rows XOR-swizzle their 16-byte chunk with (row >> 1); V rows are padded to
//    D*2 + 32 bytes.  Both layouts are conflict-free for their reads (checked with the LDS lane-
//    group rules, then SQ_LDS_BANK_CONFLICT).
//  * Output O^T: a lane holds 4 consecutive head dims of one query -> 8-byte stores.
//  * exp2 is the raw v_exp_f32 (__builtin_amdgcn_exp2f): its arguments are <= 0 (or -inf for a
//    masked key, which it maps to 0), so exp2f's range handling (v_cmp / v_cndmask / v_ldexp
//    around every exp) is dead weight.
//  * MX8 (fp8 encoder): the output is emitted as MX fp8 for the out-projection's block-scaled
//    MFMA -- e4m3 bytes plus one E8M0 exponent per 32 head dims, computed across the 4 lanes that
//    share a query (a 32-dim block is 2 of a lane's 16-dim output tiles) -- instead of bf16 rows
//    that a per-token quantiser pass would re-read.
#include "common.h"

namespace symb {

template <int D, int KVT, int NWAVE, bool MX8 = false>
__global__ __launch_bounds__(64 * NWAVE) void attn_varlen_kernel(const __bf16* __restrict__ qkv,
                                                          int ld_qkv, const int32_t* __restrict__ cu,
                                                          int H, float scale_log2,
                                                          __bf16* __restrict__ out, int ld_out,
                                                          uint8_t* __restrict__ oscale, int xcd) {
  static_assert(KVT % 32 == 0, "keys per tile");   // 128: a <=128-token sentence in ONE stage
  constexpr int NT = KVT / 16;            // 16-key accumulator tiles
  constexpr int CK = D / 8;               // 16-byte chunks per K/V row
  constexpr int KRB = D * 2;              // K row bytes (unpadded, swizzled)
  constexpr int VRB = D * 2 + 32;         // V row bytes (padded)
  constexpr int NKS = D / 32;             // k-steps of the QK^T product
  constexpr int ND = D / 16;              // 16-dim output tiles
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) char sm[KVT * KRB + KVT * VRB];
  char* Ks = sm;
  char* Vs = sm + KVT * KRB;

  // xcd: workgroups walk (sequence, head, query block) in XCD-contiguous order, so the heads of
  // one sequence run on ONE XCD.  Its K/V/Q rows then share that XCD's L2 lines: a d = 32 head is
  // 64 of a 128-byte line whose other half is the neighbouring head, and with the default
  // round-robin placement the two halves were fetched into two different XCDs' L2s.
  int bx = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  if (xcd) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int lid = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
    bx = lid % gx;
    h = (lid / gx) % gy;
    b = lid / (gx * gy);
  }
  const int s0 = cu[b], L = cu[b + 1] - s0;
  constexpr int NTH = 64 * NWAVE, QB = 16 * NWAVE;  // threads, query rows per workgroup
  const int q0 = bx * QB;
  if (q0 >= L) return;                    // block-uniform: EXEC stays full for the tr reads
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;

  const int qrow = min(q0 + wave * 16 + c16, L - 1);
  const __bf16* qp = qkv + (size_t)(s0 + qrow) * ld_qkv + h * D;
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + ks * 32 + g * 8);

  // per-lane constant LDS offsets
  uint32_t koff[NT][NKS];                 // A fragment of key tile n, k-step ks
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int r = n * 16 + c16, c = ks * 4 + g;
      koff[n][ks] = (uint32_t)(r * KRB + ((c ^ ((r >> 1) & (CK - 1))) << 4));
    }
  // tr read: lane 4q+p of its 16-lane group gives row (4g + q), columns 4p..4p+3 of a 16-dim tile
  const uint32_t vbase = (uint32_t)((4 * g + (c16 >> 2)) * VRB + (c16 & 3) * 8);
  const uint32_t lds_k = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)Ks);
  const uint32_t lds_v = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)Vs);

  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;        // running max / per-lane partial sum of this query

  for (int kv0 = 0; kv0 < L; kv0 += KVT) {
    __syncthreads();
    for (int c = tid; c < KVT * CK; c += NTH) {
      const int r = c / CK, ch = c % CK;
      const int kr = min(kv0 + r, L - 1);
      const __bf16* src = qkv + (size_t)(s0 + kr) * ld_qkv + h * D + ch * 8;
      *reinterpret_cast<bf16x8*>(Ks + r * KRB + ((ch ^ ((r >> 1) & (CK - 1))) << 4)) =
          *reinterpret_cast<const bf16x8*>(src + H);
      *reinterpret_cast<bf16x8*>(Vs + r * VRB + ch * 16) =
          *reinterpret_cast<const bf16x8*>(src + 2 * H);
    }
    __syncthreads();

    f32x4 s[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + koff[n][ks]);
        s[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[n], 0, 0, 0);
      }
    }
    // scale + key mask; s[n][r] is key kv0 + 16n + 4g + r of this lane's query
    float mx = -INFINITY;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = (kv0 + n * 16 + 4 * g + r) < L ? s[n][r] * scale_log2 : -INFINITY;
        s[n][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    lsum *= alpha;
#pragma unroll
    for (int d = 0; d < ND; ++d) o[d] *= alpha;
    bf16x8 pb[NT / 2];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(s[n][r] - mn);
        lsum += p;
        pb[n >> 1][(n & 1) * 4 + r] = (__bf16)p;
      }
#pragma unroll
    for (int t = 0; t < NT / 2; ++t)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const uint32_t a0 = lds_v + vbase + (uint32_t)(t * 32 * VRB + d * 32);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(uintptr_t)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(uintptr_t)(a0 + 16 * VRB));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[t], o[d], 0, 0, 0);
      }
  }

  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const int row = q0 + wave * 16 + c16;
  if constexpr (MX8) {
    // block j (32 dims) = output tiles 2j, 2j+1 of the 4 lanes g = 0..3 of this query
    const float inv = 1.0f / lsum;
    uint8_t* op8 = reinterpret_cast<uint8_t*>(out) + (size_t)(s0 + min(row, L - 1)) * ld_out + h * D + 4 * g;
#pragma unroll
    for (int j = 0; j < D / 32; ++j) {
      float amax = 0.f;
#pragma unroll
      for (int d = 2 * j; d < 2 * j + 2; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(o[d][r] * inv));
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      const int e = __builtin_amdgcn_frexp_expf(amax * (1.0f / 448.0f));
      const int ex = amax > 0.f ? max(-127, min(e, 127)) : -127;
      const float sc = __builtin_amdgcn_ldexpf(inv, -ex);
      if (row < L) {
#pragma unroll
        for (int d = 2 * j; d < 2 * j + 2; ++d) {
          int w = __builtin_amdgcn_cvt_pk_fp8_f32(o[d][0] * sc, o[d][1] * sc, 0, false);
          w = __builtin_amdgcn_cvt_pk_fp8_f32(o[d][2] * sc, o[d][3] * sc, w, true);
          *reinterpret_cast<int*>(op8 + d * 16) = w;
        }
        if (g == 0) oscale[(size_t)(s0 + row) * (H / 32) + (h * D) / 32 + j] = (uint8_t)(ex + 127);
      }
    }
    return;
  }
  if (row < L) {
    const float inv = 1.0f / lsum;
    __bf16* op = out + (size_t)(s0 + row) * ld_out + h * D + 4 * g;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (__bf16)(o[d][r] * inv);
      *reinterpret_cast<bf16x4*>(op + d * 16) = v;
    }
  }
}

// ---- QKV projection fused into attention (head_dim 32, sentences of <= 128 tokens) ------------
//
// The unfused layer writes the [T, 3H] QKV activation (75 MB at 32768 tokens, H = 384) and the
// attention kernel reads it back; both kernels run far from their MFMA floors (QKV GEMM ~47 us,
// attention ~31 us per MiniLM layer, profiles/r6_step/).  Here ONE workgroup per sentence walks
// the heads, and the activation never leaves the CU:
//  * the sentence's X rows are read once: wave w owns tokens 16w .. 16w + 15 and keeps their
//    rows as resident B fragments (12 k-steps x 4 VGPRs);
//  * per head, the projection computes OUT^T = W_h X^T (v_mfma_f32_16x16x32_bf16; A = the
//    head's 96 Q / K / V weight rows, staged in LDS with 16-byte chunks XOR-swizzled by the row's
//    low 4 bits: conflict-free A-fragment reads; k-step outer, the next k-step's six fragments
//    read under the current six independent MFMAs), so a lane ends with dims 4g .. 4g + 3 and
//    16 + 4g .. of ONE token (c16) for each of Q, K, V;
//  * the k index of the attention's QK^T product is permuted to match: chunk g of a head row is
//    dims {4g..4g+3, 16+4g..16+4g+3}.  A lane's Q values ARE its B fragment (no exchange), its K
//    values are one 16-byte store into the attention's swizzled K row; V rows are stored in
//    natural order (read transposed with ds_read_b64_tr_b16 as in attn_varlen_kernel);
//  * software pipeline over heads: head h + 1's projection (MFMA-bound) and head h's attention
//    (latency-bound softmax VALU and small MFMAs) share one barrier interval, with K / V in two
//    LDS buffers; the two waves of a SIMD (w, w + 4) run them in opposite orders, so one's
//    projection overlaps the other's softmax; head h + 2's weight rows are loaded into registers
//    at the top of the interval and stored to LDS after its barrier;
//  * the attention scores a sentence's (<= 128) keys in one pass: 8 S tiles, one max, one
//    exp2 pass, no online rescaling (keys past the sentence masked).
// Measured forms (the GEMM + attention pair: ~78 us per MiniLM layer): one workgroup per
// (sentence, head), re-reading X per head with every head's weight staging exposed -- 91 us;
// one per sentence with the phases in series -- 73.4 us, of which the attention 36 us (its two
// waves per SIMD could not hide the softmax's latency).
// Tokens past the sentence are clamped to its last row (finite values), as there.
template <int NH>
__global__ __launch_bounds__(512, 1) void qkv_attn_kernel(const __bf16* __restrict__ X,
                                                          const __bf16* __restrict__ Wqkv,
                                                          const float* __restrict__ bqkv,
                                                          const int32_t* __restrict__ cu,
                                                          float scale_log2,
                                                          __bf16* __restrict__ out, int B) {
  constexpr int D = 32, H = NH * D, NKX = H / 32;   // k-steps of the projection
  constexpr int WROW = H * 2;                       // weight row bytes in LDS
  constexpr int NCH = WROW / 16;                    // 16-byte chunks per weight row
  constexpr int WPL = 96 * NCH / 512;               // weight chunks per lane per head
  constexpr int KRB = D * 2, VRB = D * 2 + 32, KVB = 128 * KRB + 128 * VRB;
  static_assert((H * 2) % 256 == 0 && (96 * NCH) % 512 == 0, "weight rows of whole 256-byte groups");
  static_assert(NH >= 2, "the head pipeline peels the last head");
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) char sW[96 * WROW];
  __shared__ __attribute__((aligned(16))) char sKV[2 * KVB];   // K | V of heads h, h + 1

  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int s0 = cu[b], L = cu[b + 1] - s0;
  if (L <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int row = wave * 16 + c16;   // this lane's token: query of the attention, key of K / V

  bf16x8 wst[WPL];
  auto load_w = [&](int h) {   // head h's Q / K / V weight rows (row = 32 * section + dim)
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const int i = tid + k * 512, wr = i / NCH, c = i % NCH;
      const int grow = (wr >> 5) * H + h * D + (wr & 31);
      wst[k] = *reinterpret_cast<const bf16x8*>(Wqkv + (size_t)grow * H + c * 8);
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const int i = tid + k * 512, wr = i / NCH, c = i % NCH;
      *reinterpret_cast<bf16x8*>(sW + wr * WROW + ((c ^ (wr & 15)) << 4)) = wst[k];
    }
  };
  load_w(0);
  const __bf16* xp = X + (size_t)(s0 + min(row, L - 1)) * H + g * 8;
  bf16x8 xf[NKX];
#pragma unroll
  for (int ks = 0; ks < NKX; ++ks) xf[ks] = *reinterpret_cast<const bf16x8*>(xp + ks * 32);
  store_w();
  load_w(1);
  __syncthreads();

  // projection of head h from the weight slab: Q as this lane's B fragment, K / V to buffer kb
  auto project = [&](int h, bf16x8& qf, int kb) {
    f32x4 acc[6];
    bf16x8 wf[2][6];
    auto rd = [&](int buf, int ks) {
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int wr = j * 16 + c16;
        wf[buf][j] = *reinterpret_cast<const bf16x8*>(sW + wr * WROW +
                                                      (((ks * 4 + g) ^ (wr & 15)) << 4));
      }
    };
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < NKX; ++ks) {
      if (ks + 1 < NKX) rd((ks + 1) & 1, ks + 1);
#pragma unroll
      for (int j = 0; j < 6; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks & 1][j], xf[ks], acc[j], 0, 0, 0);
    }
    // + bias; lane holds dims (j & 1) * 16 + 4g + r of section j >> 1 for its token
    bf16x8 kv;
    bf16x4 v0, v1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d0 = h * D + 4 * g + r, d1 = d0 + 16;
      qf[r] = (__bf16)(acc[0][r] + bqkv[d0]);
      qf[4 + r] = (__bf16)(acc[1][r] + bqkv[d1]);
      kv[r] = (__bf16)(acc[2][r] + bqkv[H + d0]);
      kv[4 + r] = (__bf16)(acc[3][r] + bqkv[H + d1]);
      v0[r] = (__bf16)(acc[4][r] + bqkv[2 * H + d0]);
      v1[r] = (__bf16)(acc[5][r] + bqkv[2 * H + d1]);
    }
    char* Ks = sKV + kb * KVB;
    char* Vs = Ks + 128 * KRB;
    *reinterpret_cast<bf16x8*>(Ks + row * KRB + ((g ^ ((row >> 1) & 3)) << 4)) = kv;
    *reinterpret_cast<bf16x4*>(Vs + row * VRB + (4 * g) * 2) = v0;
    *reinterpret_cast<bf16x4*>(Vs + row * VRB + (16 + 4 * g) * 2) = v1;
  };

  // attention of head h (queries: this wave's 16 tokens) over K / V buffer kb
  uint32_t koff[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int r = n * 16 + c16;
    koff[n] = (uint32_t)(r * KRB + ((g ^ ((r >> 1) & 3)) << 4));
  }
  const uint32_t vbase = (uint32_t)((4 * g + (c16 >> 2)) * VRB + (c16 & 3) * 8);
  const uint32_t lds_kv = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)sKV);
  auto attend = [&](int h, const bf16x8& qf, int kb) {
    // (the latency-bound half of the interval: its instructions go first on the SIMD, the other
    // wave's projection MFMAs fill the gaps)
    __builtin_amdgcn_s_setprio(1);
    const char* Ks = sKV + kb * KVB;
    f32x4 sc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (n >> 2) * 64 * KRB + koff[n & 3]);
      sc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    if (L < 128) {   // (block-uniform) keys past the sentence
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n * 16 + 4 * g + r >= L) sc[n][r] = -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int n = 0; n < 8; ++n) mx = fmaxf(mx, fmaxf(fmaxf(sc[n][0], sc[n][1]), fmaxf(sc[n][2], sc[n][3])));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mxs = mx * scale_log2;
    float lsum = 0.f;
    bf16x8 pb[4];
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[n][r], scale_log2, -mxs));
        lsum += p;
        pb[n >> 1][(n & 1) * 4 + r] = (__bf16)p;
      }
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const uint32_t vb = lds_kv + (uint32_t)(kb * KVB + 128 * KRB) + vbase;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const uint32_t a0 = vb + (uint32_t)(t * 32 * VRB + d * 32);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(uintptr_t)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(uintptr_t)(a0 + 16 * VRB));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[t], o[d], 0, 0, 0);
      }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (row < L) {
      const float inv = 1.0f / lsum;
      __bf16* op = out + (size_t)(s0 + row) * H + h * D + 4 * g;
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (__bf16)(o[d][r] * inv);
        *reinterpret_cast<bf16x4*>(op + d * 16) = v;
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  bf16x8 q_cur, q_next;
  project(0, q_cur, 0);
  __syncthreads();    // head 0's K / V visible; every wave done with head 0's weights
  store_w();          // head 1's weights
  __syncthreads();
  for (int h = 0; h + 1 < NH; ++h) {
    load_w(min(h + 2, NH - 1));       // (the last head's rows again at the end: harmless)
    // the two waves of a SIMD (w, w + 4) take the two phases in opposite orders, so one's
    // MFMA-bound projection runs under the other's softmax
    if (wave & 4) {
      attend(h, q_cur, h & 1);
      project(h + 1, q_next, (h + 1) & 1);
    } else {
      project(h + 1, q_next, (h + 1) & 1);
      attend(h, q_cur, h & 1);
    }
    q_cur = q_next;
    __syncthreads();  // head h + 1's K / V visible; the weight slab and buffer h & 1 are free
    store_w();
    __syncthreads();
  }
  attend(NH - 1, q_cur, (NH - 1) & 1);
}

}  // namespace symb

using namespace symb;

// X [T, H] bf16 rows (packed sentences, cu_seqlens), Wqkv [3H, H], bqkv [3H] -> out [T, H]: the
// QKV projection and the attention in one launch.  head_dim 32, H = 384 (12 heads), every
// sentence <= 128 tokens; -1 otherwise (the caller runs the GEMM + attention pair).
int symb_qkv_attention(const void* X, const void* Wqkv, const float* bqkv, const int32_t* cu, int B,
                       int max_len, int n_heads, int head_dim, void* out, hipStream_t st) {
  if (B <= 0) return 0;
  if (head_dim != 32 || n_heads != 12 || max_len > 128 || max_len <= 0) return -1;
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)head_dim);
  hipLaunchKernelGGL((qkv_attn_kernel<12>), dim3(B), dim3(512), 0, st, (const __bf16*)X,
                     (const __bf16*)Wqkv, bqkv, cu, scale_log2, (__bf16*)out, B);
  return (int)hipGetLastError();
}

// 8 waves (one workgroup per <=128-token sentence and head) with 64-key tiles: 256 x 128 tokens,
// 12 heads: D=32 40.5 -> 34.0 us, D=64 52.2 -> 43.1 us vs 4 waves (profiles/r1_attn/attn_waves.json)
static int g_attn_waves = 8;  // 4: 64-query workgroups; 8: 128-query workgroups
static int g_attn_kvt = 64;   // keys per LDS tile (64, or 128 = a <=128-token sentence at once)
// XCD-contiguous (sequence, head) order (kernel note): 0 off, 1 on, 2 auto = head_dim 32 only.
// Measured (profiles/r2_attn_xcd/, 256 x 128 tokens, 12 heads, 8 waves): d = 32 35.2 -> 32.0 us,
// d = 64 45.6 -> 47.0 us (a 64-dim head row is a whole 128-byte line: nothing to share).
static int g_attn_xcd = 2;
int symb_attention_config(int waves, int kvt, int xcd) {
  if ((waves != 4 && waves != 8) || (kvt != 64 && kvt != 128) || xcd < 0 || xcd > 2) return -1;
  g_attn_waves = waves;
  g_attn_kvt = kvt;
  g_attn_xcd = xcd;
  return 0;
}

// oscale != nullptr: emit MX fp8 (out = e4m3 bytes with ld_out in bytes, oscale = E8M0 per 32
// columns, [T, H/32]) instead of bf16.
int symb_attention(const void* qkv, int ld_qkv, const int32_t* cu, int B, int max_len, int n_heads,
                   int head_dim, void* out, int ld_out, hipStream_t st, void* oscale) {
  if (B <= 0 || max_len <= 0) return 0;
  const int xcd = g_attn_xcd == 2 ? (head_dim == 32) : g_attn_xcd;
  if (oscale) {
    const int H = n_heads * head_dim;
    const float scale_log2 = 1.4426950408889634f / sqrtf((float)head_dim);
    dim3 grid((max_len + 127) / 128, n_heads, B);
    if (head_dim == 32)
      hipLaunchKernelGGL((attn_varlen_kernel<32, 64, 8, true>), grid, dim3(512), 0, st,
                         (const __bf16*)qkv, ld_qkv, cu, H, scale_log2, (__bf16*)out, ld_out,
                         (uint8_t*)oscale, xcd);
    else if (head_dim == 64)
      hipLaunchKernelGGL((attn_varlen_kernel<64, 64, 8, true>), grid, dim3(512), 0, st,
                         (const __bf16*)qkv, ld_qkv, cu, H, scale_log2, (__bf16*)out, ld_out,
                         (uint8_t*)oscale, xcd);
    else
      return -1;
    return (int)hipGetLastError();
  }
  const int H = n_heads * head_dim;
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)head_dim);
  const int NW = g_attn_waves;
  dim3 grid((max_len + 16 * NW - 1) / (16 * NW), n_heads, B);
#define SYMB_A(DD, KV, W) hipLaunchKernelGGL((attn_varlen_kernel<DD, KV, W>), grid, dim3(64 * W), 0, \
                                             st, (const __bf16*)qkv, ld_qkv, cu, H, scale_log2,     \
                                             (__bf16*)out, ld_out, nullptr, xcd)
#define SYMB_AW(DD)                                             \
  if (NW == 8 && g_attn_kvt == 128) SYMB_A(DD, 128, 8);         \
  else if (NW == 8) SYMB_A(DD, 64, 8);                          \
  else if (g_attn_kvt == 128) SYMB_A(DD, 128, 4);               \
  else SYMB_A(DD, 64, 4);
  if (head_dim == 32) {
    SYMB_AW(32)
  } else if (head_dim == 64) {
    SYMB_AW(64)
  } else {
    return -1;
  }
#undef SYMB_AW
#undef SYMB_A
  return (int)hipGetLastError();
}
