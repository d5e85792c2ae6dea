// hipBLASLt path for the encoder's PLAIN projections: C[M,N] = A[M,K] . W[N,K]^T + bias[N]
// (+ R[M,N]).  These are library-shaped GEMMs (bias, or bias + residual through the GEMM's own
// beta * C term); the fused hot ops -- GELU, residual + LayerNorm on a row-complete tile, the MX
// fp8 hand-offs -- stay on the hand-written MFMA kernels in gemm.hip.
//
// Why: on the bge-base / e5-large shapes (K >= 768, N >= 768, M = 32k tokens) hipBLASLt's
// 256x256 one-wave-per-SIMD kernels run 0.97-1.15 PFLOP/s against 0.8-0.85 for gemm.hip's tiles
// (profiles/r1_gemm/gemm_stream_experiment.json, profiles/r2_gemm/); on MiniLM's K = 384 shapes
// gemm.hip is faster (590 vs 397 TFLOP/s for QKV), so symb_gemm only routes here above a size
// rule (gemm.hip: symb_gemm_lt_config).
//
// Layout: hipBLASLt is column-major, so the row-major product is computed as its transpose,
// D^T[N,M] = op(W^T) . A^T with W^T read as a K x N column-major matrix (ld = ldw, transposed)
// and A^T as K x M (ld = lda); bias is then a per-row vector of D^T (length N, fp32), and the
// residual R enters as C with beta = 1.  One plan (descriptors + heuristic algorithm) per shape;
// the service's packed batches give a new M almost every call, so the cache is an LRU of
// kMaxPlans plans per device whose evicted descriptors are destroyed (a plan miss costs one
// heuristic query, ~tens of us, taken outside any stream capture); one 64 MiB workspace per
// device.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <list>
#include <map>
#include <mutex>
#include <tuple>

namespace {

constexpr size_t kWorkspace = 64u << 20;
constexpr size_t kMaxPlans = 64;

using Key = std::tuple<int, int, int, int, int, int, int, int>;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
  std::list<Key>::iterator lru;
};

void destroy_plan(Plan& p) {
  if (p.a) hipblasLtMatrixLayoutDestroy(p.a);
  if (p.b) hipblasLtMatrixLayoutDestroy(p.b);
  if (p.c) hipblasLtMatrixLayoutDestroy(p.c);
  if (p.d) hipblasLtMatrixLayoutDestroy(p.d);
  if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
  p = Plan{};
}

struct DeviceState {
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  std::map<Key, Plan> plans;
  std::list<Key> order;   // most recently used first
};

std::mutex g_mu;
std::map<int, DeviceState> g_dev;

#define LT_TRY(x)                                        \
  do {                                                   \
    if ((x) != HIPBLAS_STATUS_SUCCESS) return -2;        \
  } while (0)

int make_plan(DeviceState& ds, Plan& p, bool res, int M, int N, int K, int lda, int ldw, int ldr,
              int ldc) {
  LT_TRY(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  const hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  const int32_t bias_t = HIP_R_32F;
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_t,
                                         sizeof(bias_t)));
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, ldw));   // W^T, transposed by op
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, lda));   // A^T
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, N, M, res ? ldr : ldc));
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, N, M, ldc));
  hipblasLtMatmulPreference_t pref;
  LT_TRY(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsz = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz,
                                        sizeof(wsz));
  hipblasLtMatmulHeuristicResult_t r{};
  int n = 0;
  const hipblasStatus_t hs = hipblasLtMatmulAlgoGetHeuristic(ds.handle, p.desc, p.a, p.b, p.c,
                                                             p.d, pref, 1, &r, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || n < 1 || r.workspaceSize > kWorkspace) return -1;
  p.algo = r.algo;
  p.ok = true;
  return 0;
}

}  // namespace

// epi: 0 = + bias, 2 = + bias + R (gemm.hip's EPI_BIAS / EPI_RES).  Returns 0, a HIP error, -1
// (no algorithm for the shape, or a first use inside a stream capture) or -2 (a hipBLASLt call
// failed before anything was enqueued); on -1 / -2 symb_gemm falls back to its own kernels.
int symb_gemm_lt(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
                 const void* R, int ldr, void* C, int ldc, int M, int N, int K, hipStream_t st) {
  if (M <= 0) return 0;
  if (epi != 0 && epi != 2) return -1;
  const bool res = epi == 2;
  if (res && R == nullptr) return -1;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceState& ds = g_dev[dev];
  const auto key = std::make_tuple(epi, M, N, K, lda, ldw, res ? ldr : 0, ldc);
  auto it = ds.plans.find(key);
  if (ds.handle == nullptr || it == ds.plans.end()) {
    // first use of this device / shape allocates (workspace) and queries heuristics, neither of
    // which belongs inside a stream capture: decline, the caller runs gemm.hip's kernel instead
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return -1;
  }
  if (ds.handle == nullptr) {
    if (ds.ws == nullptr) {
      e = hipMalloc(&ds.ws, kWorkspace);
      if (e != hipSuccess) {
        ds.ws = nullptr;
        return -2;
      }
    }
    LT_TRY(hipblasLtCreate(&ds.handle));
  }
  if (it == ds.plans.end()) {
    while (ds.plans.size() >= kMaxPlans) {   // evict the least recently used plan
      auto victim = ds.plans.find(ds.order.back());
      ds.order.pop_back();
      if (victim != ds.plans.end()) {
        destroy_plan(victim->second);
        ds.plans.erase(victim);
      }
    }
    Plan p;
    const int rc = make_plan(ds, p, res, M, N, K, lda, ldw, ldr, ldc);
    ds.order.push_front(key);
    p.lru = ds.order.begin();
    it = ds.plans.emplace(key, p).first;
    if (rc != 0) return rc;
  } else {
    ds.order.splice(ds.order.begin(), ds.order, it->second.lru);
  }
  Plan& p = it->second;
  if (!p.ok) return -1;
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                         sizeof(bias)));
  const float alpha = 1.f, beta = res ? 1.f : 0.f;
  LT_TRY(hipblasLtMatmul(ds.handle, p.desc, &alpha, W, p.a, A, p.b, &beta, res ? R : C, p.c, C, p.d,
                         &p.algo, ds.ws, kWorkspace, st));
  return 0;
}

// Plans cached on the current device (tests: the cache stays bounded).
int symb_gemm_lt_plans() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_dev.find(dev);
  return it == g_dev.end() ? 0 : (int)it->second.plans.size();
}
