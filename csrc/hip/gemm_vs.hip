// Wide-projection bf16 GEMM in hipBLASLt's geometry with VGPR-staged operand loads
// (the QKV / out-projection / FFN GEMMs of the 768- and
// 1024-wide encoders; reference call site services/preprocessing_service/src/
// embedding_generator.rs:198 -> candle BertModel::forward).
//
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] )      epi: bias | GELU | bias + residual
//
// Why this kernel (profiles/r3_gemm/, r4_gemm/, r5_gemm/): hipBLASLt runs these shapes as 256 x
// 256 (or 192) tiles of FOUR waves, each wave a 128 x 128 (96) output tile, one wave per SIMD,
// with the operands staged global -> VGPR -> LDS.  This repo's 4-wave kernel of round 3 staged
// through LDS-DMA instead and was issue-bound: one LDS-DMA piece costs ~60-185 issue cycles next
// to MFMAs (MI355X_MICROARCH.md, per-instruction table), 16 of them per wave and k-tile.  A
// global_load_dwordx4 + ds_write_b128 pair costs a few + 13 cycles, which the 8 free issue
// cycles of every v_mfma_f32_16x16x32_bf16 absorb.
//
// Structure per 64-deep k-tile t (one barrier, no LDS-latency bubble after it):
//   phase A: the 64 MFMAs of k-step 0 (fragments read in the previous phase B), while the wave
//            reads k-step 1's fragments, writes tile t + 1 from its staging registers into the
//            other LDS buffer and issues tile t + 2's global loads into those registers;
//   lgkmcnt(0) + barrier (tile t + 1 is in LDS for every wave; every read of tile t - 1 is done);
//   phase B: the 64 MFMAs of k-step 1, while the wave reads tile t + 1's k-step-0 fragments.
// Two staging sets: a tile's global loads have two k-tiles (~4k MFMA cycles) to land; 128 (or 112) KiB of LDS, the
// bank-conflict XOR swizzle of gemm.hip on the write and read addresses, 256 accumulator AGPRs.
#include "common.h"

namespace symb {
namespace gvs {

enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RES = 2 };
constexpr int BM = 256, BK = 64, NT = 256;

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int BN>
struct Geo {
  static constexpr int WTN = BN / 2;                  // wave tile: 128 x WTN
  static constexpr int RM = 8, RN = WTN / 16;         // 16 x 16 fragments per wave
  static constexpr int LA = BM * 8 / NT, LB = BN * 8 / NT;   // 16-byte loads per thread per tile
  static constexpr int BUF = (BM + BN) * 128;         // one k-tile of A and W
  static constexpr int MAIN = 2 * BUF;
  static constexpr int EPI = (BM / 2) * (BN + 4) * 4; // one wave-row band of fp32 output
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static_assert(BN == 256 || BN == 192, "tile columns");
  static_assert(LDS <= 160 * 1024, "LDS");
};

typedef __attribute__((ext_vector_type(4))) int i32x4g;

// NS: staging register sets (1: tile kt + 2's loads issued during k-tile kt; 2: tile kt + 3's)
template <int BN, int EPI, int NS = 1>
__global__ __launch_bounds__(256, 1) void gemm_vs_kernel(
    const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ W, int ldw,
    const float* __restrict__ bias, const __bf16* __restrict__ R, int ldr, __bf16* __restrict__ C,
    int ldc, int M, int N, int K, int group_m, int gelu_poly) {
  using G = Geo<BN>;
  constexpr int RM = G::RM, RN = G::RN, LA = G::LA, LB = G::LB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // tile order: XCD-contiguous, then group_m-row bands walked column by column (gemm.hip)
  const int n_tiles = N / BN, nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  int tm = tile / n_tiles, tn = tile % n_tiles;
  if (group_m > 1) {
    const int m_tiles = nwg / n_tiles, per_group = group_m * n_tiles;
    const int g = tile / per_group, first = g * group_m;
    const int gm = min(group_m, m_tiles - first), local = tile - g * per_group;
    tm = first + local % gm;
    tn = local / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int KT = K / BK;

  // ---- staging: thread t moves 16-byte chunks s = i * 256 + t: row i * 32 + t / 8, chunk t % 8,
  //      so one lane offset serves every i (the row step goes in the scalar offset) and the
  //      swizzled LDS offset of chunk i is the first one + 4 KiB i (rows 32 apart share the XOR).
  //      Buffer loads: rows past M (the ragged last row tile) read as zeros (the descriptor's
  //      extent), with no clamps or per-chunk pointers in VGPRs.
  i32x4g sa[NS][LA], sb[NS][LB];
  const int r0 = tid >> 3, c0 = tid & 7;
  // (descriptor inputs through readfirstlane: provably uniform, so hipcc emits no waterfall
  // loop around each buffer op -- guide T20)
  auto rsrc = [](const void* p, long bytes) {
    const uint64_t u = (uint64_t)p;
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)u);
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)min(bytes, 0x7fffffffl));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi32 << 32) | lo32), 0, nb, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t ra = rsrc(A + (size_t)m0 * lda, (long)(M - m0) * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc(W + (size_t)n0 * ldw, (long)BN * ldw * 2);
  const int va = r0 * lda * 2 + c0 * 16, vb = r0 * ldw * 2 + c0 * 16;
  const int lo = swz(r0, c0);
  auto gload = [&](auto setc, int kt) {
    constexpr int S = decltype(setc)::value;
    const int k0 = kt * BK * 2;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      sa[S][i] = __builtin_amdgcn_raw_buffer_load_b128(ra, va, k0 + i * 32 * lda * 2, 0);
#pragma unroll
    for (int i = 0; i < LB; ++i)
      sb[S][i] = __builtin_amdgcn_raw_buffer_load_b128(rb, vb, k0 + i * 32 * ldw * 2, 0);
  };
  auto dswrite = [&](auto setc, int buf) {
    constexpr int S = decltype(setc)::value;
    char* base = smem + buf * G::BUF + lo;
#pragma unroll
    for (int i = 0; i < LA; ++i) *reinterpret_cast<i32x4g*>(base + i * 4096) = sa[S][i];
#pragma unroll
    for (int i = 0; i < LB; ++i) *reinterpret_cast<i32x4g*>(base + BM * 128 + i * 4096) = sb[S][i];
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;

  // ---- fragments: k-step kk of buffer buf (lane: row (lane & 15), 16-byte chunk 4 kk + lane / 16)
  bf16x8 fa[2][RM], fb[2][RN];
  auto fread = [&](int buf, int kk, int slot) {
    const char* sA = smem + buf * G::BUF;
    const char* sB = sA + BM * 128;
    const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
    for (int i = 0; i < RM; ++i)
      fa[slot][i] = *reinterpret_cast<const bf16x8*>(sA + swz(wm * 128 + i * 16 + (lane & 15), chunk));
#pragma unroll
    for (int j = 0; j < RN; ++j)
      fb[slot][j] = *reinterpret_cast<const bf16x8*>(sB + swz(wn * G::WTN + j * 16 + (lane & 15), chunk));
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](int slot) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[slot][i], fb[slot][j], acc[i][j], 0, 0, 0);
  };
  constexpr int NM = RM * RN, NR = RM + RN, NW = LA + LB;

  // prologue: tile 0 -> LDS buffer 0, tiles 1 and 2 in flight, k-step 0 fragments of tile 0
  gload(S0(), 0);
  dswrite(S0(), 0);
  if constexpr (NS == 2) {
    gload(S1(), min(1, KT - 1));
    gload(S0(), min(2, KT - 1));
  } else {
    gload(S0(), min(1, KT - 1));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  fread(0, 0, 0);

  // one k-tile; LAST: no next tile to write / read.  The body is branch-free (the loads past
  // the end re-read the last k-tile), so the pinned interleave spans one basic block.
  // k-tile kt stages tile kt + 1 from set (kt + 1) % NS and refills that set with tile kt + NS + 1
  auto ktile = [&](int kt, auto setc, auto lastc) {
    constexpr bool LAST = decltype(lastc)::value;
    const int buf = kt & 1;
    // ---- phase A: k-step 0 MFMAs | k-step 1 reads, tile kt + 1 -> LDS, tile kt + 3 loads ----
    mfmas(0);
    fread(buf, 1, 1);
    if constexpr (!LAST) {
      dswrite(setc, buf ^ 1);
      gload(setc, min(kt + NS + 1, KT - 1));
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA | k-step 1 read
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      // the staged tile's writes, THEN the next loads (a load issued before a write of the same
      // staging set would make hipcc's counted wait for that write drain the new loads too)
      constexpr int MW = (NM - NR) / (2 * NW);
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, MW, 0);   // MFMAs | LDS write
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, MW, 0);   // MFMAs | global load
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NM - NR - 2 * NW * MW, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase B: k-step 1 MFMAs | tile kt + 1's k-step 0 reads ----
    mfmas(1);
    if constexpr (!LAST) {
      fread(buf ^ 1, 0, 0);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, NM / NR, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (NS == 1) {
#pragma nounroll
    for (int kt = 0; kt < KT - 1; ++kt) ktile(kt, S0(), std::false_type());
    ktile(KT - 1, S0(), std::true_type());
  } else {
    int kt = 0;
#pragma nounroll
    for (; kt + 2 < KT; kt += 2) {
      ktile(kt, S1(), std::false_type());
      ktile(kt + 1, S0(), std::false_type());
    }
    if (KT - kt == 2) {
      ktile(kt, S1(), std::false_type());
      ktile(kt + 1, S0(), std::true_type());
    } else {
      ktile(kt, S1(), std::true_type());
    }
  }

  // ---- epilogue: fp32 wave-row band -> LDS -> row-contiguous 16-byte stores ----
  constexpr int CS = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
  __syncthreads();
#pragma unroll 1
  for (int p = 0; p < 2; ++p) {
    const int band0 = m0 + p * 128;
    if (wm == p) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(i * 16 + (lane >> 4) * 4 + r) * CS + wn * G::WTN + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    constexpr int VPR = BN / 8;
    for (int v = tid; v < 128 * VPR; v += NT) {
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
            const f32x2 g2 = gelu2_poly(f32x2{y[e], y[e + 1]});
            y[e] = g2.x;
            y[e + 1] = g2.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = gelu_erf(y[e]);
        }
      }
      if constexpr (EPI == EPI_RES) {
        float r8[8];
        load8(R + (size_t)grow * ldr + n0 + c8, r8);
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] += r8[e];
      }
      store8(C + (size_t)grow * ldc + n0 + c8, y);
    }
    __syncthreads();
  }
}

template <int BN, int EPI, int NS = 1>
static int launch_vs(const void* A, int lda, const void* W, int ldw, const float* bias,
                     const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                     int gelu_poly, hipStream_t st) {
  using G = Geo<BN>;
  set_max_lds<gemm_vs_kernel<BN, EPI, NS>>(G::LDS);
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_vs_kernel<BN, EPI, NS>), dim3(nwg), dim3(NT), G::LDS, st, (const __bf16*)A,
                     lda, (const __bf16*)W, ldw, bias, (const __bf16*)R, ldr, (__bf16*)C, ldc, M, N,
                     K, group_m, gelu_poly);
  return (int)hipGetLastError();
}

}  // namespace gvs
}  // namespace symb

using namespace symb;

// tile columns: 0 = auto (the fewer (waves of tiles) x (tile columns), 256 on ties), 256, 192
static int g_vs_bn = 0;
int symb_gemm_vs_config(int bn) {
  if (bn != 0 && bn != 256 && bn != 192) return -1;
  g_vs_bn = bn;
  return 0;
}

static int vs_pick_bn(int M, int N, int n_cus) {
  if (g_vs_bn) return N % g_vs_bn == 0 ? g_vs_bn : 0;
  const long mt = (M + gvs::BM - 1) / gvs::BM;
  long best = -1, bn_best = 0;
  for (int bn : {256, 192}) {
    if (N % bn) continue;
    const long cost = (mt * (N / bn) + n_cus - 1) / n_cus * bn;
    if (best < 0 || cost < best) best = cost, bn_best = bn;
  }
  return (int)bn_best;
}

bool symb_gemm_vs_supported(int epi, int M, int N, int K) {
  return epi >= 0 && epi <= 2 && M > 0 && (N % 256 == 0 || N % 192 == 0) && K % gvs::BK == 0 &&
         K >= gvs::BK;
}

// epi: 0 bias, 1 GELU (gelu_poly: the polynomial form), 2 bias + residual R.  -1: unsupported.
int symb_gemm_vs(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                 const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                 int gelu_poly, hipStream_t st) {
  if (M <= 0) return 0;
  if (!symb_gemm_vs_supported(epi, M, N, K)) return -1;
  if (lda % 8 || ldw % 8 || ldc % 8 || (epi == gvs::EPI_RES && (R == nullptr || ldr % 8))) return -1;
  // (32-bit buffer offsets: one 256-row band of A and of W must stay under 2 GiB)
  if ((long)gvs::BM * lda * 2 >= (1l << 31) || (long)gvs::BM * ldw * 2 >= (1l << 31)) return -1;
  static int n_cus = 0;   // (one device kind per process)
  if (n_cus == 0) {
    int dev = 0, c = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    n_cus = c;
  }
  const int bn = vs_pick_bn(M, N, n_cus);
  if (!bn) return -1;
#define L(BN_, E_) gvs::launch_vs<BN_, E_>(A, lda, W, ldw, bias, R, ldr, C, ldc, M, N, K, group_m, \
                                           gelu_poly, st)
  if (bn == 192) {
    switch (epi) {
      case gvs::EPI_BIAS: return L(192, gvs::EPI_BIAS);
      case gvs::EPI_GELU: return L(192, gvs::EPI_GELU);
      default: return L(192, gvs::EPI_RES);
    }
  }
  switch (epi) {
    case gvs::EPI_BIAS: return L(256, gvs::EPI_BIAS);
    case gvs::EPI_GELU: return L(256, gvs::EPI_GELU);
    default: return L(256, gvs::EPI_RES);
  }
#undef L
}
