// Deep-ring 256x256 bf16 GEMM with last-wave split-K, for the wide encoders' projections
// (bge-base / e5-large / the reference's 768-d mpnet: H >= 768, SURVEY.md §2.5 K5, K12, K14, K16;
// reference forward at services/preprocessing_service/src/embedding_generator.rs:198).
//
//   C[M,N] = epi( A[M,K] . W[N,K]^T + bias[N] )        epi: bias | GELU | + residual
//
// Why not gemm.hip's 256x256 tile: it stages 64-k tiles (64 KiB per stage) in a 2-deep ring, so
// one tile is in flight while the MFMAs run and every k-tile ends in a full vmcnt(0) drain plus a
// barrier -- the waves sat 45 % of their cycles in waits (profiles/r3_gemm/), and a 1.5-wave grid
// (N = 768 at M = 32768: 384 tiles on 256 CUs) idled half the chip for its last wave.
//
// CDNA4 design:
//  * 8 waves (2 x 4) of 128 x 64, v_mfma_f32_16x16x32_bf16, fp32 accumulators (128 VGPRs).
//  * ONE MFMA k-step (32 bf16 = 64-byte rows) per ring slot: a slot is 32 KiB, so the 160 KiB LDS
//    holds an NS = 4 or 5 deep ring and NS - 2 slots stay in flight across every barrier (counted
//    vmcnt, raw s_barrier).  Rows reach LDS by global_load_lds_dwordx4 (no VGPR staging).
//  * Fragments are double-buffered in registers: the 12 ds_read_b128 of k-step i + 1 are issued
//    between the 32 MFMAs of k-step i (hand-ordered inline asm, so the compiler neither serialises
//    them behind lgkmcnt(0) nor drains the DMA ring before them).
//  * Bank conflicts: the image stays lane-linear for the DMA; 16-byte chunk c of row r is stored
//    at chunk c ^ g(r), g(r) = (4 - ((r >> 2) & 3)) & 3, on the global source side and read back
//    the same way: each 16-lane ds_read_b128 group then covers 16 distinct 16-byte bank slots.
//  * Last-wave split-K (a stream-K form without a persistent loop): of T output tiles, the
//    T mod P that would form a partial last wave over the P CUs are cut into S = P / (T mod P)
//    k-slices (S = 2) that run after the full tiles.  Each slice takes an arrival
//    ticket; the non-last ones publish fp32 partials (write-through sc1 stores, done counter),
//    the LAST arriver waits only for slices that already hold a ticket (so they are resident and
//    finishing: no deadlock whatever the dispatch order), adds their partials and runs the
//    epilogue.  The last arriver resets both counters, so graph replays need no memset.
//  * XCD-aware block order and grouped (group_m) tile order as in gemm.hip.
#include "common.h"

#include <map>
#include <mutex>

namespace symb {

namespace gd {
constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NW = WM * WN, NT = 64 * NW;
constexpr int BK = 32;                       // bf16 k per ring slot (one MFMA k-step)
constexpr int ROWB = BK * 2;                 // 64-byte LDS rows
constexpr int WTM = BM / WM, WTN = BN / WN;  // 128 x 64 per wave
constexpr int RM = WTM / 16, RN = WTN / 16;  // 8 x 4 MFMA tiles per wave
constexpr int A_BYTES = BM * ROWB;           // 16 KiB
constexpr int SLOT = (BM + BN) * ROWB;       // 32 KiB
constexpr int LA = BM * 4 / NT, LB = BN * 4 / NT;   // 16-byte DMA pieces per thread per slot
constexpr int LOADS = LA + LB;               // 4 vector-memory ops per thread per slot
constexpr int CS = BN + 4;                   // fp32 epilogue row stride (floats)
constexpr int PROWS = WTM;                   // epilogue rows per pass (one wave-row band)
constexpr int EPI_BYTES = PROWS * CS * 4;    // 130 KiB
constexpr int PART_FLOATS = BM * BN;         // one split partial (256 KiB)
constexpr int MAX_SPLITS = 2;              // (the combine prefetches ONE other slice's band)
static_assert(LA * NT == BM * 4 && LB * NT == BN * 4, "slot rows must cover the threads");
}  // namespace gd

enum { GD_BIAS = 0, GD_GELU = 1, GD_RES = 2 };

__device__ __forceinline__ int gd_swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }

// The split partial hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the
// sc1 table): every partial byte is stored write-through (sc1, 16 B), each storing wave drains
// its vmcnt, ONE lane adds to the tile's done counter behind a workgroup barrier; the consumer
// polls that counter with sc1 loads and reads EVERY partial byte with sc1 loads after a barrier.
// No L2 write-back fence (it would also flush every other dirty line of the producer's XCD L2:
// the tiles' output stores) and no acquire.  Buffer loads / stores with the sc1 cache-policy bit
// (aux 16): the compiler tracks their data registers (inline asm stores read registers whose
// LDS loads it did not wait for).
constexpr int GD_SC1 = 16;
__device__ __forceinline__ void gd_store_wt(__amdgpu_buffer_rsrc_t r, int off, const f32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, GD_SC1);
}
__device__ __forceinline__ f32x4 gd_load_wt(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, GD_SC1));
}

__device__ __forceinline__ bf16x8 gd_lds16(const char* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}
// wait until at most `younger` ring slots' DMA pieces (LOADS each) are still in flight
__device__ __forceinline__ void gd_wait_slots(int younger) {
  if (younger >= 3)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (younger == 2)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (younger == 1)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void gd_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One k-step: the 32 MFMAs (row-major over the 8 x 4 wave tile) with the NEXT k-step's 12
// fragment reads between them.  A fragment i is last read by MFMA (i, 3), so its refill follows
// that MFMA (same registers); the B fragments are read by every row, so the next k-step's B goes
// to the other B set (bn) during the first two rows.  8 A + 2 x 4 B = 64 fragment VGPRs next to
// 128 accumulators.  The order is pinned by sched_group_barrier: (2 MFMA, 1 read) x 12, 8 MFMA.
__device__ __forceinline__ void gd_kstep(f32x4 (&acc)[gd::RM][gd::RN], bf16x8 (&a)[gd::RM],
                                         const bf16x8 (&b)[gd::RN], bf16x8 (&bn)[gd::RN],
                                         const char* na, const char* nb) {
  using namespace gd;
#pragma unroll
  for (int i = 0; i < RM; ++i) {
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      if (i < 2 && (j == 0 || j == 2)) bn[i * 2 + j / 2] = gd_lds16(nb + (i * 2 + j / 2) * 16 * ROWB);
    }
    a[i] = gd_lds16(na + i * 16 * ROWB);
  }
#pragma unroll
  for (int r = 0; r < RM + RN; ++r) {
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // 2 MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
  }
  __builtin_amdgcn_sched_group_barrier(0x008, RM * RN - 2 * (RM + RN), 0);
}

template <int EPI, int NS>
__global__ __launch_bounds__(gd::NT, 1) void gemm_deep_kernel(
    const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ W, int ldw,
    const float* __restrict__ bias, const __bf16* __restrict__ R, int ldr, int gelu_poly,
    __bf16* __restrict__ C, int ldc, int M, int N, int K, int group_m, int dp_tiles, int splits,
    float* __restrict__ part, int* __restrict__ ctr, int dma_mode) {
  using namespace gd;
  static_assert(NS >= 3 && NS * SLOT <= 160 * 1024, "LDS ring depth");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int n_tn = N / BN;
  const int T = ((M + BM - 1) / BM) * n_tn;
  const int KT = K / BK;

  // ---- which tile and which k-range ----
  const int b = blockIdx.x;
  int t, kb = 0, ke = KT, sk = -1, slice = 0;
  if (b < dp_tiles) {
    t = xcd_remap(b, dp_tiles);
  } else {
    sk = b - dp_tiles;                       // split slot
    t = dp_tiles + sk / splits;
    slice = sk % splits;
    kb = (int)((long long)KT * slice / splits);
    ke = (int)((long long)KT * (slice + 1) / splits);
  }
  int tm = t / n_tn, tn = t % n_tn;
  if (group_m > 1) {   // grouped order over all T tiles (gemm.hip)
    const int m_tiles = T / n_tn, per_group = group_m * n_tn;
    const int g = t / per_group, first = g * group_m;
    const int gm = min(group_m, m_tiles - first), local = t - g * per_group;
    tm = first + local % gm;
    tn = local / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = ke - kb;

  // ---- per-lane DMA source offsets (bytes; slot-invariant) ----
  uint32_t aoff[LA], boff[LB];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int s = i * NT + tid, row = s >> 2, c = (s & 3) ^ gd_swz(row);
    aoff[i] = (uint32_t)min(m0 + row, M - 1) * (uint32_t)lda * 2u + (uint32_t)(c * 16);
  }
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int s = i * NT + tid, row = s >> 2, c = (s & 3) ^ gd_swz(row);
    boff[i] = (uint32_t)(n0 + row) * (uint32_t)ldw * 2u + (uint32_t)(c * 16);
  }
  // buffer descriptors: one SGPR base per operand, the per-lane row offsets above in VGPRs and
  // the k-step's byte offset in an SGPR -- one instruction per 1-KiB piece, no address VALU
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A, (short)0, (int)((uint32_t)M * (uint32_t)lda * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)W, (short)0, (int)((uint32_t)N * (uint32_t)ldw * 2u), 0x00020000);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const char* Ab = reinterpret_cast<const char*>(A);
  const char* Wb = reinterpret_cast<const char*>(W);
  auto stage = [&](int kt, int slot) {
    char* sA = smem + slot * SLOT;
    char* sB = sA + A_BYTES;
    const int k0 = kt * ROWB;
    if (dma_mode == 1) {   // (A/B: per-lane 64-bit addresses, global_load_lds)
#pragma unroll
      for (int i = 0; i < LA; ++i) glds16(Ab + aoff[i] + k0, sA + (i * NT + wave_u * 64) * 16);
#pragma unroll
      for (int i = 0; i < LB; ++i) glds16(Wb + boff[i] + k0, sB + (i * NT + wave_u * 64) * 16);
      return;
    }
#pragma unroll
    for (int i = 0; i < LA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)(sA + (i * NT + wave_u * 64) * 16), 16,
          (int)aoff[i], k0, 0, 0);
#pragma unroll
    for (int i = 0; i < LB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, (__attribute__((address_space(3))) void*)(sB + (i * NT + wave_u * 64) * 16), 16,
          (int)boff[i], k0, 0, 0);
  };

  // ---- per-lane fragment addresses: A row wm*128 + i*16 + (lane&15), B row wn*64 + j*16 + ... --
  const int fr = lane & 15, fc = lane >> 4;
  const uint32_t fa = (uint32_t)((wm * WTM + fr) * ROWB + ((fc ^ gd_swz(fr)) << 4));
  const uint32_t fb = (uint32_t)(A_BYTES + (wn * WTN + fr) * ROWB + ((fc ^ gd_swz(fr)) << 4));

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[RM], bf0[RN], bf1[RN];
  // prologue: slots 0 .. NS-2 in flight, slot 0 landed and visible, its fragments in registers
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) stage(kb + p, p);
  gd_wait_slots(min(NS - 2, nk - 1));
  gd_barrier();
#pragma unroll
  for (int i = 0; i < RM; ++i) af[i] = gd_lds16(smem + fa + i * 16 * ROWB);
#pragma unroll
  for (int j = 0; j < RN; ++j) bf0[j] = gd_lds16(smem + fb + j * 16 * ROWB);

  // k-step `it` on B set CB, reading k-step it + 1's fragments (B into NB).  Slot it + 1 landed
  // for this wave once only the younger slots' pieces remain; the barrier makes every wave's
  // pieces visible and retires every wave's reads of slot it - 1, which stage(it + NS - 1)
  // refills.  The last k-step reads a stale slot it never uses: one code shape for every step
  // keeps the MFMA loop's registers allocated once (two shapes spilled).
#define GD_ITER(CB, NB)                                                         \
  {                                                                             \
    if (it + 1 < nk) gd_wait_slots(min(NS - 3, nk - 2 - it));                   \
    gd_barrier();                                                               \
    if (it + NS - 1 < nk) stage(kb + it + NS - 1, (it + NS - 1) % NS);          \
    const char* nbase = smem + ((it + 1) % NS) * SLOT;                          \
    gd_kstep(acc, af, CB, NB, nbase + fa, nbase + fb);                          \
  }
  int it = 0;
  for (; it + 1 < nk; ++it) {
    GD_ITER(bf0, bf1)
    ++it;
    GD_ITER(bf1, bf0)
  }
  if (it < nk) GD_ITER(bf0, bf1)
#undef GD_ITER

  // ---- last-wave split-K: take a ticket; the last arriver combines, the others publish ----
  // Partials are row-major fp32 256 x 256 tiles, one per split slot, written and read in the
  // epilogue's row-contiguous 16-byte pattern (no extra registers beside the accumulators).
  bool publish = false;
  int st = 0;
  __syncthreads();   // every wave is past its last ring read: the LDS is free
  if (sk >= 0 && splits > 1) {
    st = sk / splits;
    int* arrive = ctr + st;
    int* done = ctr + (T - dp_tiles) + st;
    int* s_ticket = reinterpret_cast<int*>(smem);
    if (tid == 0)
      *s_ticket = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    publish = *s_ticket < splits - 1;
    if (!publish && tid == 0) {
      // every other slice holds a ticket, i.e. is resident and publishing: a bounded wait
      while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < splits - 1)
        __builtin_amdgcn_s_sleep(2);
      // reset for the next launch (ordered by the kernel boundary; graph replays need no memset)
      __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();   // (also orders the ticket read before the epilogue's LDS writes)
  }
  const bool combine = sk >= 0 && splits > 1 && !publish;
  // the split partials as one buffer (byte offsets fit 32 bits: <= P x 256 KiB)
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)part, (short)0, part ? (int)((T - dp_tiles) * splits * PART_FLOATS * 4) : 0, 0x00020000);

  // ---- epilogue: fp32 tile -> LDS (one 128-row band per pass) -> 16-byte row stores ----
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll 1
  for (int pass = 0; pass < WM; ++pass) {
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(i * 16 + fc * 4 + r) * CS + wn * WTN + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    const int band0 = m0 + pass * PROWS;
    constexpr int VPR = BN / 8;
    constexpr int PER = PROWS * VPR / NT;    // 16-byte column groups per thread per pass
    static_assert(PER * NT == PROWS * VPR && PER == 8, "epilogue work split (pp ties 4 x 2)");
    // combine: the other slice's band, half a pass in flight at a time (sc1 loads, one wait)
    constexpr int PH = PER / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
    f32x4 pp[PH][2];
    if (combine) {
      const int pb = ((st * splits + (1 - slice)) * PART_FLOATS + pass * PROWS * BN) * 4;
#pragma unroll
      for (int jj = 0; jj < PH; ++jj) {
        const int v = tid + (h * PH + jj) * NT, row = v / VPR, c8 = (v % VPR) * 8;
        pp[jj][0] = gd_load_wt(rp, pb + (row * BN + c8) * 4);
        pp[jj][1] = gd_load_wt(rp, pb + (row * BN + c8 + 4) * 4);
      }
    }
#pragma unroll
    for (int jj = 0; jj < PH; ++jj) {
      const int j = jj;
      const int v = tid + (h * PH + jj) * NT, row = v / VPR, c8 = (v % VPR) * 8;
      const int grow = band0 + row;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(Cs + row * CS + c8);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(Cs + row * CS + c8 + 4);
      if (publish) {
        const int off = (sk * PART_FLOATS + (pass * PROWS + row) * BN + c8) * 4;
        gd_store_wt(rp, off, x0);
        gd_store_wt(rp, off + 16, x1);
        continue;
      }
      if (grow >= M) continue;
      float y[8];
      // two slices summed in slice order whichever arrived last: bit-identical launches
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = combine ? (slice == 0 ? x0[e] + pp[j][0][e] : pp[j][0][e] + x0[e]) : x0[e];
        y[e + 4] = combine ? (slice == 0 ? x1[e] + pp[j][1][e] : pp[j][1][e] + x1[e]) : x1[e];
      }
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias + n0 + c8);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(bias + n0 + c8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] += b0[e];
        y[e + 4] += b1[e];
      }
      if constexpr (EPI == GD_GELU) {
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
      if constexpr (EPI == GD_RES) {
        float r[8];
        load8(R + (size_t)grow * ldr + n0 + c8, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] += r[e];
      }
      store8(C + (size_t)grow * ldc + n0 + c8, y);
    }
    }
    if (pass + 1 < WM) __syncthreads();
  }
  if (publish) {
    // every storing wave drained its write-through stores, then one done count per workgroup
    int* done = ctr + (T - dp_tiles) + st;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static int g_deep_dma = 0;   // 0: buffer-descriptor LDS-DMA, 1: global_load_lds (A/B)

namespace {

// Split partials + counters, one buffer per (device, stream): concurrent streams must never share
// one.  Allocated on first use (never while the stream is being captured: a capture without a
// buffer runs without split-K) and never freed.  Layout: counters (2 x P ints, zero between
// launches: the last arriver of each split tile resets its pair) at 0, partials at 64 KiB.
constexpr size_t kCtrBytes = 64 * 1024;
std::mutex g_ws_mu;
std::map<std::pair<int, hipStream_t>, char*> g_ws;

char* ws_for(hipStream_t st, size_t part_bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const auto key = std::make_pair(dev, st);
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws.find(key);
  if (it != g_ws.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  char* p = nullptr;
  if (hipMalloc(&p, kCtrBytes + part_bytes) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, kCtrBytes) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  g_ws[key] = p;
  return p;
}

int cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

template <int EPI, int NS>
int launch_deep(const void* A, int lda, const void* W, int ldw, const float* bias, const void* R,
                int ldr, int gelu_poly, void* C, int ldc, int M, int N, int K, int group_m,
                int dp_tiles, int splits, float* part, int* ctr, int nwg, hipStream_t st) {
  constexpr int ring = NS * gd::SLOT;
  constexpr int lds = ring > gd::EPI_BYTES ? ring : gd::EPI_BYTES;
  auto kern = gemm_deep_kernel<EPI, NS>;
  set_max_lds<gemm_deep_kernel<EPI, NS>>(lds);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(gd::NT), lds, st, (const __bf16*)A, lda,
                     (const __bf16*)W, ldw, bias, (const __bf16*)R, ldr, gelu_poly, (__bf16*)C, ldc,
                     M, N, K, group_m, dp_tiles, splits, part, ctr, g_deep_dma);
  return (int)hipGetLastError();
}

}  // namespace

}  // namespace symb

using namespace symb;

// Ring depth (4: 2 slots in flight across each barrier, 5: 3) and the split-K mode of the last
// partial wave (0 off, 1 on); symb_gemm_deep_config.
static int g_deep_ns = 5;
static int g_deep_sk = 1;
int symb_gemm_deep_config(int ns, int sk, int dma) {
  if ((ns != 4 && ns != 5) || sk < 0 || sk > 1 || dma < 0 || dma > 1) return -1;
  g_deep_ns = ns;
  g_deep_sk = sk;
  g_deep_dma = dma;
  return 0;
}

bool symb_gemm_deep_supported(int M, int N, int K) {
  return M > 0 && N % gd::BN == 0 && K % gd::BK == 0 && K >= 2 * gd::BK &&
         (size_t)M * (size_t)K * 2 < (1ull << 32) && (size_t)N * (size_t)K * 2 < (1ull << 32);
}

// Split count the last partial wave of an M x N x K launch would take (1 = none), and the tiles
// that run whole.
static void deep_plan(int M, int N, int K, int* dp_tiles, int* splits) {
  const int T = ((M + gd::BM - 1) / gd::BM) * (N / gd::BN);
  const int P = cu_count();
  const int w = T % P;
  *dp_tiles = T;
  *splits = 1;
  if (!g_deep_sk || w == 0 || w > P / 2) return;
  int s = min(P / w, gd::MAX_SPLITS);
  s = min(s, (K / gd::BK) / 4);          // at least 4 k-steps per slice
  if (s < 2) return;
  *dp_tiles = T - w;
  *splits = s;
}

// epi: 0 bias, 1 GELU(+ bias) (gelu_poly: 1 = the packed polynomial, 0 = erf), 2 + bias +
// residual.  Returns 0, a HIP error code, or -1 (unsupported shape: the caller's other paths).
int symb_gemm_deep(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                   const void* R, int ldr, void* C, int ldc, int M, int N, int K, int group_m,
                   int gelu_poly, hipStream_t st) {
  if (!symb_gemm_deep_supported(M, N, K) || epi < 0 || epi > 2) return -1;
  // (32-bit per-lane DMA offsets)
  if ((size_t)M * lda * 2 >= (1ull << 32) || (size_t)N * ldw * 2 >= (1ull << 32)) return -1;
  int dp = 0, splits = 1;
  deep_plan(M, N, K, &dp, &splits);
  const int T = ((M + gd::BM - 1) / gd::BM) * (N / gd::BN);
  float* part = nullptr;
  int* ctr = nullptr;
  if (splits > 1) {
    char* ws = ws_for(st, (size_t)cu_count() * gd::PART_FLOATS * sizeof(float));
    if (ws == nullptr) {
      dp = T;
      splits = 1;
    } else {
      ctr = reinterpret_cast<int*>(ws);
      part = reinterpret_cast<float*>(ws + kCtrBytes);
    }
  }
  const int nwg = dp + (T - dp) * splits;
#define GD_L(E, NS_) launch_deep<E, NS_>(A, lda, W, ldw, bias, R, ldr, gelu_poly, C, ldc, M, N, K, \
                                         group_m, dp, splits, part, ctr, nwg, st)
#define GD_E(NS_)                         \
  switch (epi) {                          \
    case GD_BIAS: return GD_L(GD_BIAS, NS_); \
    case GD_GELU: return GD_L(GD_GELU, NS_); \
    default: return GD_L(GD_RES, NS_);    \
  }
  if (g_deep_ns == 4) {
    GD_E(4)
  }
  GD_E(5)
#undef GD_E
#undef GD_L
}
