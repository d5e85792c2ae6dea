// Small-M ("skinny") split-K GEMM for the query path: C[M,N] = epi(A[M,K] . W[N,K]^T + bias), M <= 64.
//
// A query-embedding forward (B = 1..32 sentences, tens to a few hundred tokens) is bound by the
// serial k-loop of the big-tile GEMM: a 128-row tile holding a handful of real rows still walks
// every k-tile of W one after another, and the row-complete RES_LN tile of MiniLM's FFN2 runs
// 24 k-tiles in ONE workgroup (profiles/r1_gemm/latency.log: 386 us for a 1 x 16 MiniLM-L6
// forward).  Replaces, for that regime, the same reference op as gemm.hip (the K5 / K12-K17
// linears of candle's BertModel, /root/reference/services/preprocessing_service/src/
// embedding_generator.rs:198).
//
// CDNA4 design:
//  * Split K as far as it goes: one WAVE per (64-column block, 128-k granule).  A workgroup is
//    NW waves = NW consecutive granules of one column block; grid = (N/64, ceil(K/128 / NW)).
//    NW = 8 when that makes ONE split of a K of 640..1024 (bge / mpnet / e5 QKV, out-proj and
//    FFN1): the epilogue then runs in this kernel and the second launch goes away; else NW = 4.
//    Every wave issues all of its loads at once (one round trip to HBM/L2) and then 4 x RM x 4
//    v_mfma_f32_16x16x32_bf16 -- no LDS staging, no k-loop.
//  * Each lane loads 64 contiguous bytes of a row (4 x 16-byte loads): the 4 lane groups of a row
//    cover 256 contiguous bytes.  The MFMA's k order is a permutation of memory order (step t,
//    lane group g, element e <-> k = 32g + 8t + e), applied identically to A and W, so the dot
//    products are unchanged.
//  * The 4 waves' accumulators are summed through LDS (every thread then owns 8 consecutive
//    columns of a row: 16-byte reads and stores); the workgroup writes one fp32 partial slice
//    P[split][M][64 cols].  A second kernel (one wave per row) sums the splits in a fixed
//    order (deterministic), adds bias, and applies GELU / residual / residual + LayerNorm, with
//    16-byte bf16 stores.  LayerNorm needs whole rows, which only exist after the split sum.
//    With a single split (K <= 512: MiniLM's QKV and FFN1) and a row-local epilogue, the split
//    kernel applies bias / GELU / residual itself (no second launch).  An opt-in form lets the
//    last workgroup to finish a small multi-split GEMM do the split sum and epilogue (measured
//    slower; see g_skinny_fuse).
#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

#include "common.h"

namespace symb {

namespace {

enum { SK_BIAS = 0, SK_GELU = 1, SK_RES = 2, SK_RES_LN = 3 };   // == gemm.hip's EPI_* values

// Sum the S split partials of one output row (fixed order: deterministic), add bias and apply the
// epilogue; one wave per row, lane owns 8 consecutive columns per PER-chunk (N <= PER * 512).
template <int EPI, int PER>
__device__ __forceinline__ void finish_row(
    const float* __restrict__ P, int S, const float* __restrict__ bias,
    const __bf16* __restrict__ R, int ldr, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int gelu_poly, __bf16* __restrict__ C, int ldc,
    int M, int N, int ldp, int row, int lane) {
  const int NV = N / 8;
  float x[PER][8];
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int v = lane + 64 * p;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[p][e] = 0.f;
    if (v >= NV) continue;
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias + v * 8);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(bias + v * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[p][e] = b0[e];
      x[p][e + 4] = b1[e];
    }
    for (int sp = 0; sp < S; ++sp) {   // fixed order: deterministic
      const float* q = P + ((size_t)sp * M + row) * ldp + v * 8;
      const f32x4 q0 = *reinterpret_cast<const f32x4*>(q);
      const f32x4 q1 = *reinterpret_cast<const f32x4*>(q + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[p][e] += q0[e];
        x[p][e + 4] += q1[e];
      }
    }
    if constexpr (EPI == SK_GELU) {
      if (gelu_poly) {
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 y = gelu2_poly(f32x2{x[p][e], x[p][e + 1]});
          x[p][e] = y.x;
          x[p][e + 1] = y.y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[p][e] = gelu_erf(x[p][e]);
      }
    }
    if constexpr (EPI == SK_RES || EPI == SK_RES_LN) {
      float rr[8];
      load8(R + (size_t)row * ldr + v * 8, rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[p][e] += rr[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s += x[p][e];
  }
  if constexpr (EPI == SK_RES_LN) {
    const float mean = wave_sum(s) / (float)N;
    float ss = 0.f;
#pragma unroll
    for (int p = 0; p < PER; ++p)
      if (lane + 64 * p < NV)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = x[p][e] - mean;
          ss += d * d;
        }
    const float rstd = rsqrtf(wave_sum(ss) / (float)N + eps);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int v = lane + 64 * p;
      if (v >= NV) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        x[p][e] = (x[p][e] - mean) * rstd * gamma[v * 8 + e] + beta[v * 8 + e];
    }
  }
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int v = lane + 64 * p;
    if (v < NV) store8(C + (size_t)row * ldc + v * 8, x[p]);
  }
}

template <int EPI, int PER>
__global__ __launch_bounds__(256) void skinny_epi_kernel(
    const float* __restrict__ P, int S, const float* __restrict__ bias,
    const __bf16* __restrict__ R, int ldr, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int gelu_poly, __bf16* __restrict__ C, int ldc,
    int M, int N) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  // row-local epilogues: blockIdx.y picks a PER * 512-column slice (more waves for wide N)
  const int col0 = blockIdx.y * PER * 512;
  finish_row<EPI, PER>(P + col0, S, bias + col0, R ? R + col0 : R, ldr, gamma, beta, eps,
                       gelu_poly, C + col0, ldc, M, min(PER * 512, N - col0), N, row,
                       threadIdx.x & 63);
}

// EPI = SK_PARTIAL: write the fp32 split partial; else (one split, K <= 512) apply bias / GELU /
// residual here and store bf16 -- no second launch.
constexpr int SK_PARTIAL = -1;

// FIN != SK_PARTIAL (with EPI == SK_PARTIAL; small outputs, N <= 1024): the LAST workgroup to
// finish (agent-scope release / acquire around one counter) sums every split and applies the FIN
// epilogue itself -- no second launch; it re-arms the counter for the next GEMM on the stream.
template <int RM, int EPI, int FIN, int NW>
__global__ __launch_bounds__(NW * 64) void skinny_partial_kernel(
    const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ W, int ldw,
    float* __restrict__ P, int M, int N, int KG, const float* __restrict__ bias,
    const __bf16* __restrict__ R, int ldr, int gelu_poly, __bf16* __restrict__ C, int ldc,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    int* __restrict__ counter) {
  static_assert(FIN == SK_PARTIAL || EPI == SK_PARTIAL, "the finish needs split partials");
  constexpr int MP = RM * 16, LS = 64 + 4;   // LDS row stride: 272 bytes (16-byte aligned)
  extern __shared__ __attribute__((aligned(16))) float red[];   // [NW waves][MP rows][LS]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 64;
  const int m0 = blockIdx.z * 64;                  // 64-row block (M > 64: several, in z)
  const int g = blockIdx.y * NW + wave;           // this wave's 128-k granule
  const int r = lane & 15, grp = lane >> 4;

  f32x4 acc[RM][4];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (g < KG) {
    const size_t k0 = (size_t)g * 128 + grp * 32;
    bf16x8 a[RM][4], b[4][4];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const __bf16* pa = A + (size_t)min(m0 + i * 16 + r, M - 1) * lda + k0;   // rows >= M: ignored
#pragma unroll
      for (int t = 0; t < 4; ++t) a[i][t] = *reinterpret_cast<const bf16x8*>(pa + 8 * t);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const __bf16* pb = W + (size_t)(n0 + j * 16 + r) * ldw + k0;
#pragma unroll
      for (int t = 0; t < 4; ++t) b[j][t] = *reinterpret_cast<const bf16x8*>(pb + 8 * t);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
  }

  // accumulator (i, j)[e] sits at row i*16 + grp*4 + e, column j*16 + r of the 64-column block;
  // all NW waves park theirs in LDS, then every thread finishes 8 consecutive columns of a row
  // (fixed wave order: deterministic) with 16-byte loads and stores
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(wave * MP + i * 16 + grp * 4 + e) * LS + j * 16 + r] = acc[i][j][e];
  __syncthreads();
  for (int q = threadIdx.x; q < MP * 8; q += NW * 64) {
    const int lrow = q >> 3, c8 = (q & 7) * 8, row = m0 + lrow;
    if (row >= M) break;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float* src = red + (w * MP + lrow) * LS + c8;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(src);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += x0[e];
        v[e + 4] += x1[e];
      }
    }
    if constexpr (EPI == SK_PARTIAL) {
      float* dst = P + ((size_t)blockIdx.y * M + row) * N + n0 + c8;
      *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias + n0 + c8);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(bias + n0 + c8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += b0[e];
        v[e + 4] += b1[e];
      }
      if constexpr (EPI == SK_GELU) {
        if (gelu_poly) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const f32x2 y = gelu2_poly(f32x2{v[e], v[e + 1]});
            v[e] = y.x;
            v[e + 1] = y.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
        }
      }
      if constexpr (EPI == SK_RES) {
        float rr[8];
        load8(R + (size_t)row * ldr + n0 + c8, rr);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rr[e];
      }
      store8(C + (size_t)row * ldc + n0 + c8, v);
    }
  }
  if constexpr (FIN != SK_PARTIAL) {
    __shared__ int s_last;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // this thread's partials, device-wide
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(counter, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == (int)(gridDim.x * gridDim.y * gridDim.z) - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every workgroup's partials
    const int S = gridDim.y;
    for (int row = wave; row < M; row += NW)
      finish_row<FIN, 2>(P, S, bias, R, ldr, gamma, beta, eps, gelu_poly, C, ldc, M, N, N, row, lane);
    if (threadIdx.x == 0) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// fp32 split partials.  An encoder forward hands in its own buffer (part of its workspace, so a
// captured hipGraph bakes a pointer that lives as long as the graph): symb_gemm_skinny_set_scratch,
// thread-local, set for the duration of the forward.  Other callers get one fixed-size buffer
// per stream (concurrent streams must not share one), allocated on first use and never moved;
// a stream under capture that has none takes the tiled path instead (no allocation in a capture).
// Layout: a 256-byte header (the last-workgroup counter, zero between launches) + the partials.
constexpr size_t kScratchHeader = 256;
constexpr size_t kStreamScratchBytes = kScratchHeader + (size_t)256 * 4096 * 8 * sizeof(float);
thread_local float* t_scratch = nullptr;
thread_local size_t t_scratch_bytes = 0;
std::mutex g_scratch_mu;
std::map<std::pair<int, hipStream_t>, float*> g_scratch;   // (device, stream): the null stream is per device

float* scratch_for(hipStream_t st, size_t bytes) {
  if (t_scratch && t_scratch_bytes >= bytes) return t_scratch;
  if (bytes > kStreamScratchBytes) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const auto key = std::make_pair(dev, st);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  auto it = g_scratch.find(key);
  if (it != g_scratch.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
    return nullptr;
  float* p = nullptr;
  if (hipMalloc(&p, kStreamScratchBytes) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, kScratchHeader) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  g_scratch[key] = p;
  return p;
}

template <int RM, int EPI, int FIN, int NW>
void launch_partial(dim3 grid, hipStream_t st, const __bf16* a, int lda, const __bf16* w, int ldw,
                    float* P, int M, int N, int KG, const float* bias, const __bf16* r, int ldr,
                    int gelu_poly, __bf16* c, int ldc, const float* g, const float* b, float eps,
                    int* counter) {
  constexpr int lds = NW * RM * 16 * (64 + 4) * (int)sizeof(float);   // <= 136 KiB
  static_assert(lds <= 160 * 1024, "LDS");
  set_max_lds<skinny_partial_kernel<RM, EPI, FIN, NW>>(lds);
  hipLaunchKernelGGL((skinny_partial_kernel<RM, EPI, FIN, NW>), grid, dim3(NW * 64), lds, st, a,
                     lda, w, ldw, P, M, N, KG, bias, r, ldr, gelu_poly, c, ldc, g, b, eps, counter);
}

template <int EPI>
int launch_epi(int per, const float* P, int S, const float* bias, const __bf16* R, int ldr,
               const float* g, const float* b, float eps, int gelu_poly, __bf16* C, int ldc, int M,
               int N, hipStream_t st) {
  // LayerNorm needs whole rows (PER * 512 >= N); the others take 512-column slices, one wave each
  if (EPI != SK_RES_LN) per = 1;
  const dim3 grid((M + 3) / 4, EPI == SK_RES_LN ? 1 : (N + 511) / 512), block(256);
#define SK_E(PER_) hipLaunchKernelGGL((skinny_epi_kernel<EPI, PER_>), grid, block, 0, st, P, S, \
                                      bias, R, ldr, g, b, eps, gelu_poly, C, ldc, M, N)
  switch (per) {
    case 1: SK_E(1); break;
    case 2: SK_E(2); break;
    case 4: SK_E(4); break;
    case 8: SK_E(8); break;
    default: return -1;
  }
#undef SK_E
  return (int)hipGetLastError();
}

}  // namespace

}  // namespace symb

using namespace symb;

// Largest M the skinny path takes (0 = off); symb_gemm consults it first.  256 (the z-blocked
// form: several 64-row blocks in grid z): MiniLM 8 x 32 / 16 x 16 / 4 x 32 / 1 x 128-token
// forwards 280 / 283 / 279 / 286 us against 511 / 512 / 502 / 524 with the tiled GEMMs above 64,
// bge 8 x 32 850 vs 891 us (profiles/r4_small_m/lat.jsonl).
static int g_skinny_max_m = 256;
// bit 0: a single-split bias / GELU / residual GEMM applies its epilogue in the split kernel;
// bit 1 (opt-in): a small multi-split / LayerNorm GEMM is finished by its last workgroup instead
// of the epilogue kernel.  Measured slower (profiles/r3_skinny: MiniLM out-proj/FFN2 + LN 12.7 us
// vs 5.7 + 3.8 us for split + epilogue kernel): one workgroup walks the rows 4 at a time, each
// row a dependent chain of partial loads, while the epilogue kernel spreads them over M waves.
static int g_skinny_fuse = 1;
int symb_gemm_skinny_config(int max_m, int fuse) {
  if (max_m < 0 || max_m > 256 || fuse < 0 || fuse > 3) return -1;
  g_skinny_max_m = max_m;
  g_skinny_fuse = fuse;
  return 0;
}
int symb_gemm_skinny_max_m() { return g_skinny_max_m; }
// 8-wave workgroups (8 granules per split) for 4 < K / 128 <= max_kg, and above it for M > 64
// when the grid keeps >= min_wgs workgroups (0: never); else 4-wave ones.  With fewer, larger
// splits a small-M forward (MiniLM 8 x 32: 2 splits of 48 workgroups; M <= 64) got slower
// (profiles/r4_small_m/nw8.jsonl).
static int g_skinny_nw8_max_kg = 8;
static int g_skinny_nw8_min_wgs = 128;
int symb_gemm_skinny_nw8(int max_kg, int min_wgs) {
  if (max_kg < 0 || max_kg > 32 || min_wgs < 0) return -1;
  g_skinny_nw8_max_kg = max_kg;
  g_skinny_nw8_min_wgs = min_wgs;
  return 0;
}

void symb_gemm_skinny_set_scratch(void* p, size_t bytes) {
  t_scratch = (float*)p;
  t_scratch_bytes = p ? bytes : 0;
}

bool symb_gemm_skinny_supported(int epi, int M, int N, int K) {
  return M >= 1 && M <= 256 && epi >= SK_BIAS && epi <= SK_RES_LN && K % 128 == 0 && K <= 4096 &&
         N % 64 == 0 && N <= 4096;
}

// Split-partial bytes an M x N x K skinny GEMM may need (an upper bound: independent of the
// fused single-split epilogue, which needs none; 0 for shapes the path does not take).
size_t symb_gemm_skinny_scratch_bytes(int epi, int M, int N, int K) {
  if (!symb_gemm_skinny_supported(epi, M, N, K)) return 0;
  const int S = (K / 128 + 3) / 4;
  return kScratchHeader + (size_t)S * M * N * sizeof(float);
}
// Returns 0, a HIP error code, or -1 (shape not supported: the caller takes its other paths).
int symb_gemm_skinny(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                     const void* R, int ldr, const float* gamma, const float* beta, float eps,
                     int gelu_poly, void* C, int ldc, int M, int N, int K, hipStream_t st) {
  if (!symb_gemm_skinny_supported(epi, M, N, K)) return -1;
  const int KG = K / 128;
  // 8 waves: K = 640..1024 in one split; above, when the 8-wave grid still spans >= min_wgs
  // workgroups (bge / e5 FFN2 at M = 256: 642 / 1552 us per 8 x 32 forward vs 684 / 1643)
  const int wgs8 = (N / 64) * ((KG + 7) / 8) * ((M + 63) / 64);
  const int NW = (KG > 4 && (KG <= g_skinny_nw8_max_kg ||
                             (g_skinny_nw8_min_wgs > 0 && M > 64 && wgs8 >= g_skinny_nw8_min_wgs)))
                     ? 8 : 4;
  const int S = (KG + NW - 1) / NW;
  // one split and a row-local epilogue: finished in the one kernel
  const int fused = (S == 1 && epi != SK_RES_LN && (g_skinny_fuse & 1)) ? epi : SK_PARTIAL;
  // small outputs: the last workgroup sums the splits (one CU reads S x M x N floats)
  const int fin = (fused == SK_PARTIAL && (g_skinny_fuse & 2) && N <= 1024 && M * N <= 16384)
                      ? epi : SK_PARTIAL;
  float* P = nullptr;
  int* counter = nullptr;
  if (fused == SK_PARTIAL) {
    char* base = (char*)scratch_for(st, kScratchHeader + (size_t)S * M * N * sizeof(float));
    if (!base) return -1;   // no buffer for this stream (capturing, or out of memory): tiled path
    counter = (int*)base;
    P = (float*)(base + kScratchHeader);
  }
  const dim3 grid(N / 64, S, (M + 63) / 64), block(256);
  auto a = (const __bf16*)A;
  auto w = (const __bf16*)W;
  auto r = (const __bf16*)R;
  auto c = (__bf16*)C;
  const int rm = (std::min(M, 64) + 15) / 16;   // fragments per 64-row block
#define SK_P(RM_, E_, F_)                                                                      \
  (NW == 8 ? launch_partial<RM_, E_, F_, 8>(grid, st, a, lda, w, ldw, P, M, N, KG, bias, r, ldr,  \
                                            gelu_poly, c, ldc, gamma, beta, eps, counter)         \
           : launch_partial<RM_, E_, F_, 4>(grid, st, a, lda, w, ldw, P, M, N, KG, bias, r, ldr,  \
                                            gelu_poly, c, ldc, gamma, beta, eps, counter))
#define SK_PE(RM_)                                                    \
  switch (fused) {                                                    \
    case SK_BIAS: SK_P(RM_, SK_BIAS, SK_PARTIAL); break;              \
    case SK_GELU: SK_P(RM_, SK_GELU, SK_PARTIAL); break;              \
    case SK_RES: SK_P(RM_, SK_RES, SK_PARTIAL); break;                \
    default:                                                          \
      switch (fin) {                                                  \
        case SK_BIAS: SK_P(RM_, SK_PARTIAL, SK_BIAS); break;          \
        case SK_GELU: SK_P(RM_, SK_PARTIAL, SK_GELU); break;          \
        case SK_RES: SK_P(RM_, SK_PARTIAL, SK_RES); break;            \
        case SK_RES_LN: SK_P(RM_, SK_PARTIAL, SK_RES_LN); break;      \
        default: SK_P(RM_, SK_PARTIAL, SK_PARTIAL); break;            \
      }                                                               \
  }
  if (rm == 1) {
    SK_PE(1)
  } else if (rm == 2) {
    SK_PE(2)
  } else {
    SK_PE(4)
  }
#undef SK_PE
#undef SK_P
  int rc = (int)hipGetLastError();
  if (rc || fused != SK_PARTIAL || fin != SK_PARTIAL) return rc;
  const int nv = N / 8;
  const int per = nv <= 64 ? 1 : nv <= 128 ? 2 : nv <= 256 ? 4 : 8;
  switch (epi) {
    case SK_BIAS:
      return launch_epi<SK_BIAS>(per, P, S, bias, r, ldr, gamma, beta, eps, gelu_poly, c, ldc, M, N, st);
    case SK_GELU:
      return launch_epi<SK_GELU>(per, P, S, bias, r, ldr, gamma, beta, eps, gelu_poly, c, ldc, M, N, st);
    case SK_RES:
      return launch_epi<SK_RES>(per, P, S, bias, r, ldr, gamma, beta, eps, gelu_poly, c, ldc, M, N, st);
    case SK_RES_LN:
      return launch_epi<SK_RES_LN>(per, P, S, bias, r, ldr, gamma, beta, eps, gelu_poly, c, ldc, M, N, st);
  }
  return -1;
}
