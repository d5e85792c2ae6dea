// Memory-bound encoder kernels: fused embedding gather + LayerNorm, residual-add + LayerNorm,
// masked mean-pool (+L2 normalise) and the index-side l2norm_cast.
//
// Reference behaviour being replaced:
//   K1-K4  candle BertEmbeddings index_select x3 + add + LayerNorm
//          (services/preprocessing_service/src/embedding_generator.rs:198, inside BertModel::forward)
//   K18    mask->f32, unsqueeze, mul, sum, +1e-9, div (embedding_generator.rs:201-207)
//   X1     Qdrant cosine normalisation of inserted vectors (vector_memory_service/src/main.rs:36)
//
// One wavefront (64 lanes) owns one row; every global access is a 16-byte bf16x8 vector.
#include "common.h"

namespace symb {

// ---------------------------------------------------------------------------------------------
// embed_ln: out[t] = LN(word[ids[t]] + pos[pos_ids[t]] + type[tt[t]]) * gamma + beta  (bf16 out)
// ---------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int32_t* __restrict__ ids, const int32_t* __restrict__ pos_ids,
    const int32_t* __restrict__ type_ids, const __bf16* __restrict__ wemb,
    const __bf16* __restrict__ pemb, const __bf16* __restrict__ temb,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    __bf16* __restrict__ out, int T) {
  constexpr int NV = H / 8;
  constexpr int PER = (NV + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int id = ids[t], p = pos_ids[t], ty = type_ids ? type_ids[t] : 0;
  float x[PER][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[i][e] = 0.f;
    if (v < NV) {
      float a[8], b[8], c[8];
      load8(wemb + (size_t)id * H + v * 8, a);
      load8(pemb + (size_t)p * H + v * 8, b);
      load8(temb + (size_t)ty * H + v * 8, c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        x[i][e] = a[e] + b[e] + c[e];
        s += x[i][e];
      }
    }
  }
  const float mean = wave_sum(s) * (1.0f / H);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (lane + 64 * i < NV)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = x[i][e] - mean;
        ss += d * d;
      }
  const float rstd = rsqrtf(wave_sum(ss) * (1.0f / H) + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = lane + 64 * i;
    if (v < NV) {
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + v * 8);
      const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + v * 8 + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + v * 8);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + v * 8 + 4);
      float y[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = (x[i][e] - mean) * rstd * g0[e] + b0[e];
        y[e + 4] = (x[i][e + 4] - mean) * rstd * g1[e] + b1[e];
      }
      store8(out + (size_t)t * H + v * 8, y);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// add_ln: out[t] = LN(x[t] (+ res[t])) * gamma + beta.  Used after the MFMA GEMMs whose row is
// too wide (H >= 768) for the GEMM's own fused LayerNorm epilogue.
// ---------------------------------------------------------------------------------------------
// LPT lanes per token (16 at H = 384, 32 at 768 / 1024): every lane holds exactly PER 16-byte
// chunks of its token -- with one 64-lane wave per token, 768 / 1024-wide rows left half the lanes
// idle on the last chunk (2.9 TB/s at bge's 32768 x 768).  Sums reduce over the token's LPT lanes.
template <int H>
__global__ __launch_bounds__(256) void add_ln_kernel(
    const __bf16* __restrict__ x_in, const __bf16* __restrict__ res,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    __bf16* __restrict__ out, int T, uint8_t* __restrict__ out8, float* __restrict__ scale8) {
  constexpr int NV = H / 8;                          // 16-byte chunks per row
  constexpr int LPT = H == 384 ? 16 : 32;
  constexpr int PER = NV / LPT;
  static_assert(NV % LPT == 0, "row must split evenly over the token's lanes");
  const int sl = threadIdx.x & (LPT - 1);
  const int t = (blockIdx.x * 256 + threadIdx.x) / LPT;
  if (t >= T) return;                                // whole token groups leave together
  auto group_sum = [](float v) {
#pragma unroll
    for (int m = LPT / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
  };
  float x[PER][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = sl + LPT * i;
    load8(x_in + (size_t)t * H + v * 8, x[i]);
    if (res) {
      float r[8];
      load8(res + (size_t)t * H + v * 8, r);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[i][e] += r[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s += x[i][e];
  }
  const float mean = group_sum(s) * (1.0f / H);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = x[i][e] - mean;
      ss += d * d;
    }
  const float rstd = rsqrtf(group_sum(ss) * (1.0f / H) + eps);
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = sl + LPT * i;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + v * 8);
    const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + v * 8 + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + v * 8);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + v * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[i][e] = (x[i][e] - mean) * rstd * g0[e] + b0[e];
      x[i][e + 4] = (x[i][e + 4] - mean) * rstd * g1[e] + b1[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(x[i][e]));
    store8(out + (size_t)t * H + v * 8, x[i]);
  }
  if (!out8) return;
  // fused per-token e4m3 quantiser for the next fp8 GEMM (same scale rule as
  // quant_rows_fp8_kernel: scale = amax / 448), from the fp32 LN output
#pragma unroll
  for (int m = LPT / 2; m >= 1; m >>= 1) amax = fmaxf(amax, __shfl_xor(amax, m, 64));
  amax = fmaxf(amax, 1e-12f);
  const float inv = 448.f / amax;
  if (sl == 0) scale8[t] = amax / 448.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = sl + LPT * i;
    float q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = x[i][e] * inv;
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], hi, true);
    *reinterpret_cast<int2*>(out8 + (size_t)t * H + v * 8) = make_int2(lo, hi);
  }
}

// ---------------------------------------------------------------------------------------------
// pool: one 256-thread block per sequence of the packed (varlen) batch.
//   mode 0 = masked mean (reference: sum / (count + 1e-9)), mode 1 = CLS (first token).
//   out_f32  : [B,H] pooled (un-normalised, what the wire format carries)
//   out_norm : [B,H] bf16 L2-normalised copy (what the HBM index / query path consumes), optional
//   gamma / beta (optional): `hidden` is the last layer's PRE-LayerNorm residual sum (the deferred
//            LayerNorm of the H >= 768 encoders, gemm.hip LNF): every token row is normalised
//            here, from its own values (the wave holds the whole row), before it is pooled.
// ---------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(256) void pool_kernel(const __bf16* __restrict__ hidden,
                                                   const int32_t* __restrict__ cu_seqlens,
                                                   int mode, int normalize_f32,
                                                   float* __restrict__ out_f32,
                                                   __bf16* __restrict__ out_norm,
                                                   const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, float eps) {
  constexpr int NV = H / 8;
  constexpr int PER = (NV + 63) / 64;
  __shared__ float part[4][H];
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s0 = cu_seqlens[b], L = cu_seqlens[b + 1] - s0;
  float acc[PER][8];
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[i][e] = 0.f;
  const int t_end = mode == 1 ? (L > 0 ? 1 : 0) : L;
  for (int t = wave; t < t_end; t += 4) {
    float r[PER][8];
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = lane + 64 * i;
#pragma unroll
      for (int e = 0; e < 8; ++e) r[i][e] = 0.f;
      if (v < NV) {
        load8(hidden + (size_t)(s0 + t) * H + v * 8, r[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += r[i][e];
      }
    }
    if (gamma != nullptr) {
      const float mean = wave_sum(sm) * (1.0f / H);
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (lane + 64 * i < NV)
#pragma unroll
          for (int e = 0; e < 8; ++e) ss += (r[i][e] - mean) * (r[i][e] - mean);
      const float rstd = rsqrtf(wave_sum(ss) * (1.0f / H) + eps);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int v = lane + 64 * i;
        if (v < NV)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            r[i][e] = (r[i][e] - mean) * rstd * gamma[v * 8 + e] + beta[v * 8 + e];
      }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[i][e] += r[i][e];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = lane + 64 * i;
    if (v < NV)
#pragma unroll
      for (int e = 0; e < 8; ++e) part[wave][v * 8 + e] = acc[i][e];
  }
  __syncthreads();
  const float denom = mode == 1 ? 1.0f : ((float)L + 1e-9f);
  float y[8];
  float ss = 0.f;
  const int v = threadIdx.x;
  if (v < NV) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = v * 8 + e;
      y[e] = (part[0][c] + part[1][c] + part[2][c] + part[3][c]) / denom;
      ss += y[e] * y[e];
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wave] = ss;
  __syncthreads();
  const float nrm = sqrtf(red[0] + red[1] + red[2] + red[3]);
  const float inv = 1.0f / fmaxf(nrm, 1e-12f);
  if (v < NV) {
    float* o = out_f32 + (size_t)b * H + v * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = normalize_f32 ? y[e] * inv : y[e];
    if (out_norm) {
      float z[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = y[e] * inv;
      store8(out_norm + (size_t)b * H + v * 8, z);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// l2norm_cast: rows of f32 (e.g. decoded from a NATS TextWithEmbeddingsMessage) -> unit-norm
// bf16 rows written straight into the HBM index slab.  One wave per row, any D (multiple of 8).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void l2norm_cast_kernel(const float* __restrict__ x,
                                                          __bf16* __restrict__ out, int n,
                                                          int D, int ld_out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const float* xr = x + (size_t)r * D;
  float ss = 0.f;
  for (int c = lane * 4; c < D; c += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
    ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  const float inv = 1.0f / fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
  __bf16* o = out + (size_t)r * ld_out;
  for (int c = lane * 4; c < D; c += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
    bf16x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = (__bf16)(v[e] * inv);
    *reinterpret_cast<bf16x4*>(o + c) = w;
  }
}

}  // namespace symb

// ------------------------------------- host launchers -------------------------------------------
using namespace symb;

#define SYMB_H_DISPATCH(H, ...)                                  \
  switch (H) {                                                   \
    case 384: { constexpr int HH = 384; __VA_ARGS__; } break;     \
    case 768: { constexpr int HH = 768; __VA_ARGS__; } break;     \
    case 1024: { constexpr int HH = 1024; __VA_ARGS__; } break;   \
    default: return -1;                                          \
  }

int symb_embed_ln(const int32_t* ids, const int32_t* pos, const int32_t* tt, const void* wemb,
                  const void* pemb, const void* temb, const float* g, const float* b, float eps,
                  void* out, int T, int H, hipStream_t st) {
  if (T <= 0) return 0;
  dim3 grid((T + 3) / 4);
  SYMB_H_DISPATCH(H, hipLaunchKernelGGL(embed_ln_kernel<HH>, grid, dim3(256), 0, st, ids, pos, tt,
                                        (const __bf16*)wemb, (const __bf16*)pemb,
                                        (const __bf16*)temb, g, b, eps, (__bf16*)out, T));
  return (int)hipGetLastError();
}

// out8/scale8 (both or neither): also emit the per-token e4m3 quantisation of the output.
int symb_add_ln(const void* x, const void* res, const float* g, const float* b, float eps,
                void* out, int T, int H, hipStream_t st, void* out8, float* scale8) {
  if (T <= 0) return 0;
  if ((out8 == nullptr) != (scale8 == nullptr)) return -1;
  const int tpb = 256 / (H == 384 ? 16 : 32);   // tokens per block (add_ln_kernel's LPT)
  dim3 grid((T + tpb - 1) / tpb);
  SYMB_H_DISPATCH(H, hipLaunchKernelGGL(add_ln_kernel<HH>, grid, dim3(256), 0, st,
                                        (const __bf16*)x, (const __bf16*)res, g, b, eps,
                                        (__bf16*)out, T, (uint8_t*)out8, scale8));
  return (int)hipGetLastError();
}

int symb_pool(const void* hidden, const int32_t* cu, int B, int H, int mode, int normalize_f32,
              float* out_f32, void* out_norm, hipStream_t st, const float* gamma,
              const float* beta, float eps) {
  if (B <= 0) return 0;
  if ((gamma == nullptr) != (beta == nullptr)) return -1;
  SYMB_H_DISPATCH(H, hipLaunchKernelGGL(pool_kernel<HH>, dim3(B), dim3(256), 0, st,
                                        (const __bf16*)hidden, cu, mode, normalize_f32, out_f32,
                                        (__bf16*)out_norm, gamma, beta, eps));
  return (int)hipGetLastError();
}

int symb_l2norm_cast(const float* x, void* out, int n, int D, int ld_out, hipStream_t st) {
  if (n <= 0) return 0;
  if (D % 4) return -1;
  hipLaunchKernelGGL(l2norm_cast_kernel, dim3((n + 3) / 4), dim3(256), 0, st, x, (__bf16*)out, n,
                     D, ld_out);
  return (int)hipGetLastError();
}
