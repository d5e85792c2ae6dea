// Varlen (packed, unpadded) bidirectional flash attention for the encoder, head_dim 32 or 64.
//
// Replaces the reference's padded path (every sentence padded to max_position_embeddings=514,
// services/preprocessing_service/src/embedding_generator.rs:75-91) and candle's
// transpose_for_scores -> QK^T -> +mask -> softmax -> PV -> merge-heads chain (SURVEY.md §2.5
// K6-K11).  Sequences are packed back to back ([T, 3H] fused QKV rows, cu_seqlens offsets), so
// no FLOP or byte is spent on padding and no mask tensor exists.
//
// Per workgroup: 64 query rows of one (sequence, head); 4 waves x 16 rows.
//   S = Q K^T   : v_mfma_f32_16x16x32_bf16, Q fragments in registers, K tile row-major in LDS
//   softmax     : online (running max / sum in fp32, exp2 with log2(e) folded into the scale)
//   O += P V    : P goes through a wave-private LDS slab to become the A operand; V is stored
//                 transposed in LDS so every B fragment is one ds_read_b128.
#include "common.h"

namespace symb {

template <int D>
__global__ __launch_bounds__(256) void attn_varlen_kernel(const __bf16* __restrict__ qkv,
                                                          int ld_qkv, const int32_t* __restrict__ cu,
                                                          int H, float scale_log2,
                                                          __bf16* __restrict__ out, int ld_out) {
  constexpr int KVT = 64;          // keys per tile
  constexpr int KP = D + 8;        // padded K row (elements)
  constexpr int VP = KVT + 8;      // padded V^T row
  constexpr int PP = KVT + 8;      // padded P row
  constexpr int NKS = D / 32;      // k-steps of the QK^T product
  constexpr int ND = D / 16;       // 16-wide output column tiles
  __shared__ __attribute__((aligned(16))) __bf16 sm[KVT * KP + D * VP + 4 * 16 * PP];

  const int b = blockIdx.z, h = blockIdx.y;
  const int s0 = cu[b], L = cu[b + 1] - s0;
  const int q0 = blockIdx.x * 64;
  if (q0 >= L) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __bf16* Ks = sm;
  __bf16* Vt = sm + KVT * KP;
  __bf16* Ps = Vt + D * VP + wave * 16 * PP;

  const int qrow = min(q0 + wave * 16 + (lane & 15), L - 1);
  const __bf16* qp = qkv + (size_t)(s0 + qrow) * ld_qkv + h * D;
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
    qf[ks] = *reinterpret_cast<const bf16x8*>(qp + ks * 32 + (lane >> 4) * 8);

  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }

  for (int kv0 = 0; kv0 < L; kv0 += KVT) {
    __syncthreads();
    for (int c = tid; c < KVT * (D / 8); c += 256) {
      const int r = c / (D / 8), ch = c % (D / 8);
      const int kr = min(kv0 + r, L - 1);
      const __bf16* src = qkv + (size_t)(s0 + kr) * ld_qkv + h * D + ch * 8;
      *reinterpret_cast<bf16x8*>(Ks + r * KP + ch * 8) =
          *reinterpret_cast<const bf16x8*>(src + H);
      const bf16x8 vv = *reinterpret_cast<const bf16x8*>(src + 2 * H);
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(ch * 8 + e) * VP + r] = vv[e];
    }
    __syncthreads();

    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 kb = *reinterpret_cast<const bf16x8*>(Ks + (n * 16 + (lane & 15)) * KP +
                                                           ks * 32 + (lane >> 4) * 8);
        s[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kb, s[n], 0, 0, 0);
      }
    }
    // scale + key mask (keys past the sequence end contribute exp2(-inf) = 0)
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bool valid = (kv0 + n * 16 + (lane & 15)) < L;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = valid ? s[n][r] * scale_log2 : -INFINITY;
        s[n][r] = v;
        mx[r] = fmaxf(mx[r], v);
      }
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int msk = 1; msk < 16; msk <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], msk, 64));
      const float mn = fmaxf(m[r], mx[r]);
      alpha[r] = exp2f(m[r] - mn);
      m[r] = mn;
      rs[r] = 0.f;
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[n][r] - m[r]);
        rs[r] += p;
        Ps[((lane >> 4) * 4 + r) * PP + n * 16 + (lane & 15)] = (__bf16)p;
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int msk = 1; msk < 16; msk <<= 1) rs[r] += __shfl_xor(rs[r], msk, 64);
      l[r] = l[r] * alpha[r] + rs[r];
    }
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[d][r] *= alpha[r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa =
          *reinterpret_cast<const bf16x8*>(Ps + (lane & 15) * PP + ks * 32 + (lane >> 4) * 8);
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vt + (d * 16 + (lane & 15)) * VP +
                                                           ks * 32 + (lane >> 4) * 8);
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[d], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = q0 + wave * 16 + (lane >> 4) * 4 + r;
    if (row < L) {
      const float inv = 1.0f / l[r];
      __bf16* op = out + (size_t)(s0 + row) * ld_out + h * D + (lane & 15);
#pragma unroll
      for (int d = 0; d < ND; ++d) op[d * 16] = (__bf16)(o[d][r] * inv);
    }
  }
}

}  // namespace symb

using namespace symb;

int symb_attention(const void* qkv, int ld_qkv, const int32_t* cu, int B, int max_len, int n_heads,
                   int head_dim, void* out, int ld_out, hipStream_t st) {
  if (B <= 0 || max_len <= 0) return 0;
  const int H = n_heads * head_dim;
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)head_dim);
  dim3 grid((max_len + 63) / 64, n_heads, B);
  if (head_dim == 32)
    hipLaunchKernelGGL(attn_varlen_kernel<32>, grid, dim3(256), 0, st, (const __bf16*)qkv, ld_qkv,
                       cu, H, scale_log2, (__bf16*)out, ld_out);
  else if (head_dim == 64)
    hipLaunchKernelGGL(attn_varlen_kernel<64>, grid, dim3(256), 0, st, (const __bf16*)qkv, ld_qkv,
                       cu, H, scale_log2, (__bf16*)out, ld_out);
  else
    return -1;
  return (int)hipGetLastError();
}
