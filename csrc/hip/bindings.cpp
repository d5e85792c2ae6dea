// Python bindings + native encoder runtime for the HIP kernels (module codename_symbiont_amd._hip).
//
// Pointers cross the boundary as integers (torch tensors' data_ptr()) and streams as the raw
// hipStream_t handle of torch.cuda.current_stream().  The module links the same libamdhip64.so.7
// as torch (SONAME match), so torch's allocator, streams and our launches share one HIP runtime.
//
// EncoderRuntime::forward is the native replacement of the reference's
// EmbeddingGenerator::generate_sentence_embeddings hot loop
// (services/preprocessing_service/src/embedding_generator.rs:134-223): one call issues the whole
// varlen encoder (embed+LN, L x {QKV GEMM, attention, out-proj+res+LN, FFN1+GELU, FFN2+res+LN},
// pool) on one stream with no host synchronisation, so it can be captured in a hipGraph.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

// ---- kernel launchers (defined in the .hip translation units) ----
int symb_embed_ln(const int32_t* ids, const int32_t* pos, const int32_t* tt, const void* wemb,
                  const void* pemb, const void* temb, const float* g, const float* b, float eps,
                  void* out, int T, int H, hipStream_t st);
int symb_add_ln(const void* x, const void* res, const float* g, const float* b, float eps,
                void* out, int T, int H, hipStream_t st, void* out8 = nullptr,
                float* scale8 = nullptr);
int symb_pool(const void* hidden, const int32_t* cu, int B, int H, int mode, int normalize_f32,
              float* out_f32, void* out_norm, hipStream_t st, const float* gamma = nullptr,
              const float* beta = nullptr, float eps = 0.f);
int symb_gemm_ln(int epi, int lnf, const void* A, int lda, const void* W, int ldw,
                 const float* bias, const void* R, int ldr, const float* gamma, const float* beta,
                 float ln_eps, const float* cs, const void* st_in, int np_in, void* st_out,
                 void* C, int ldc, int M, int N, int K, hipStream_t st);
int symb_l2norm_cast(const float* x, void* out, int n, int D, int ld_out, hipStream_t st);
int symb_gemm(int epi, const void* A, int lda, const void* W, int ldw, const float* bias,
              const void* R, int ldr, const float* gamma, const float* beta, float eps, void* C,
              int ldc, int M, int N, int K, hipStream_t st);
int symb_attention(const void* qkv, int ld_qkv, const int32_t* cu, int B, int max_len,
                   int n_heads, int head_dim, void* out, int ld_out, hipStream_t st,
                   void* oscale = nullptr);
int symb_topk_geometry(int D, int kmax, int* lists, int* queries_per_blk);
int symb_attention_config(int waves, int kvt, int xcd);
int symb_qkv_attention(const void* X, const void* Wqkv, const float* bqkv, const int32_t* cu, int B,
                       int max_len, int n_heads, int head_dim, void* out, hipStream_t st);
// The QKV projection fused into the attention (attention.hip qkv_attn_kernel) for 384-wide,
// 32-dim-head bf16 layers whose sentences fit 128 tokens, above the small-M limit (1, default);
// 0: the QKV GEMM + attention pair.
static int g_qkv_attn = 1;
int symb_index_scan(const void* X, int n_valid, int D, int rows_per_blk, int n_rblk,
                    const void* Q, int NQ, int kmax, float* cand_s, int* cand_i, hipStream_t st,
                    int ns, int aux, const float* thr_init, int xcd,
                    const int* gate = nullptr);
int symb_index_scan_ablate(const void* X, int n_valid, int rows_per_blk, int n_rblk,
                           const void* Q, int NQ, float* cs, int* ci, hipStream_t st, int abl,
                           const float* thr);
int symb_gemm_config(int resln_bm, int tile, int group_m);
int symb_gemm_fp8_config(int waves, int big);
int symb_gemm_resln_config(int waves);
int symb_gemm_gelu_config(int poly);
int symb_gemm_gelu_poly();
int symb_mlp_fused(const void* X, const void* W1, const float* b1, const void* W2, const float* b2,
                   const float* gamma, const float* beta, float eps, int gelu_poly, void* C, int M,
                   int H, int FF, hipStream_t st);
// The fused FFN block (mlp_fused.hip) for bf16 384 x 1536 layers above the small-M limit (1,
// default); 0: the two-GEMM path (FFN1 GELU GEMM + FFN2 residual/LayerNorm GEMM).  Measured
// (profiles/r4_mlp): 110 vs 129 us per layer, the bare MiniLM forward 1.297 vs 1.437 ms, the
// headline step 7.33 / 7.30 vs 7.33 / 7.36 ms (same box, interleaved).
static int g_mlp_fused = 1;
int symb_gemm_fp8(int epi, const void* A8, int lda, const void* W8, int ldw, const float* sa,
                  const float* sw, const float* bias, const void* R, int ldr, void* C, int ldc,
                  int M, int N, int K, hipStream_t st, const void* ascale = nullptr,
                  void* cscale = nullptr);
int symb_quant_rows_fp8(const void* x, int ldx, void* out, int ldo, float* scale, int M, int K,
                        hipStream_t st);
int symb_quant_fp8(const void* in, int in_f32, int ld_in, uint8_t* out, int ld_out, int n, int D,
                   float scale, int normalize, hipStream_t st);
int symb_index_scan_fp8(const void* X, int n_valid, int D, int rows_per_blk, int n_rblk,
                        const void* Q, int NQ, int kmax, float* cand_s, int* cand_i,
                        hipStream_t st, int aux, const float* thr_init, int variant, int xcd);
int symb_topk_merge(const float* cand_s, const int* cand_i, int NQ, int n_cand_per_query,
                    int kmax, int k, float* out_s, int* out_i, int64_t id_offset,
                    int64_t* out_id64, hipStream_t st, const int* gate = nullptr);
int symb_mq_queries_per_blk(int sets, int rsplit);
int symb_i8_queries_per_blk(int rsplit);
int symb_index_scan_i8(const void* X8, const float* sx, int n_valid, int alloc_rows,
                       int rows_per_blk, int n_rblk, const void* Q8, int NQ, const float* thr,
                       float* cand_s, int* cand_i, int* cand_n, int cap, int xcd, hipStream_t st,
                       int rsplit, const int* skip, int dim, int heavy, const float* sq, int form,
                       const int* gate, int gate_want);
int symb_quant_rows_mx4(const void* X, int n, int dim, void* X4, void* SC, float* bounds,
                        float* margin, hipStream_t st);
int symb_mx4_select(int NQ, const float* T, const float* margin4, const float* margin8,
                    const float* probe_s, int n_cols, int ld, int tile_stride, float rate,
                    const float* tail_cs, int tail_cap, int tail_ld, float limit, float* thr4,
                    int* nv, hipStream_t st, int nv_zeroed, int stage, float wa, float wb);
int symb_i8_tile_rows_for(int dim, int heavy);
// the streaming pruning scan (index_stream.hip)
int symb_stream_rec_bytes(int dim, int form);
int symb_stream_config(int abl);
int symb_stream_geometry(int dim, int form, int* qpb, int* wgs_per_cu);
int symb_index_scan_stream(const void* img, int n_valid, int alloc_rows, int rows_per_blk,
                           int n_rblk, const void* Q, const void* qsc, int NQ, const float* thr,
                           float* cand_s, int* cand_i, int* cand_n, int cap, int xcd,
                           hipStream_t st, const int* skip, int dim, int form, const int* gate,
                           int gate_want, int zero_cnt, int* runs, const void* cent4,
                           const void* centqs, const float* centR, const float* bounds4);
int symb_mx4_centroids(const void* Xq, const void* QS, int NQ, int dim, void* C4, void* CS,
                       float* R, hipStream_t st);
int symb_append_rows(const void* src, int n, int dim, void* rows, int r0, void* img8, float* b8,
                     void* img4, float* b4, void* img6, float* b6, hipStream_t st);
int symb_dense_scores(const void* X, int dim, const int* rows, int n_list, int ts, int div,
                      int r_lo, int n_range, const void* Q, int NQ, float* out, int ld,
                      hipStream_t st);
int symb_quant_stream_i8(const void* X, int r0, const int* rows, int n, int dim, void* img,
                         float* bounds, hipStream_t st);
int symb_prefill_candidates(int NQ, int r_lo, int n, int* cand_i, int* cand_n, int cap,
                            hipStream_t st);
int symb_quant_stream_mx4(const void* X, int r0, const int* rows, int n, int dim, void* img,
                          void* Xq, void* QS, float* bounds, float* margin, hipStream_t st);
int symb_quant_stream_mx6(const void* X, int r0, const int* rows, int n, int dim, void* img,
                          void* Xq, void* QS, float* bounds, float* margin, hipStream_t st);
int symb_i8_split_queries_per_blk(int rsplit);
int symb_mx4_config(int tile_rows);
int symb_mx4_tile_rows();
int symb_quant_rows_split(const float* X, int n, int dim, void* X8, float* sx, float* bounds,
                          float* margin, hipStream_t st);
int symb_prune_qquant(const void* Q, int NQ, int dim, const float* bounds, void* Q8, float* sq,
                      float* margin, hipStream_t st, int* zero, int zero_n);
int symb_prune_route(int NQ, const float* pre_s, const float* tail_s, int k, float thr_margin,
                     const float* sq, const float* margin, const float* thr0, const float* cs_p,
                     const int* ci_p, const int* cnt_p, int cap_p, int tshift, int rows_per_blk,
                     int n_rblk, float blk_limit, float limit, int max_list, float* T, float* thr,
                     int* dense, float* est, int* blkmax, int* blk, hipStream_t st,
                     const float* tail_cs, const int* tail_ci, const int* tail_cnt, int tail_cap,
                     int tail_off, int tail_ld, int zeroed);
int symb_i8_config(int tile_rows, int waves);
int symb_i8_tile_rows();
int symb_i8_wgs_per_cu();
int symb_rescore_bf16(const void* X, const void* Q, int NQ, int dim, const int* cand_i,
                      const int* cand_n, int cap, float* cand_s, hipStream_t st);
int symb_index_scan_i8_ablate(const void* X8, const float* sx, int n_valid, int alloc_rows,
                              int rows_per_blk, int n_rblk, const void* Q8, int NQ,
                              const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                              int xcd, hipStream_t st, int abl);
int symb_quant_rows_i8(const void* X, int n, int dim, void* X8, float* sx, float* err, float* xtn,
                       float* bounds, hipStream_t st);
int symb_prune_qprep(const void* Q, int NQ, int dim, const float* pre_s, const float* tail_s, int k,
                     float thr_margin, const float* bounds, void* Q8, float* sq, float* T,
                     float* thr, hipStream_t st);
int symb_gemm_lt_config(int mode);
int symb_mfma_f8f6f4_probe(const int* a, const int* b, const int* sa, const int* sb, float* out,
                           int fmt, hipStream_t st);
int symb_gemm_lt_plans();
int symb_gemm_skinny_config(int max_m, int fuse);
int symb_gemm_skinny_max_m();
int symb_gemm_skinny_nw8(int max_kg, int min_wgs);
size_t symb_gemm_skinny_scratch_bytes(int epi, int M, int N, int K);
void symb_gemm_skinny_set_scratch(void* p, size_t bytes);
int symb_mq_config(int aux);
int symb_index_scan_mq(const void* X, int n_valid, int rows_per_blk, int n_rblk, const void* Q,
                       int NQ, const float* thr, float* cand_s, int* cand_i, int* cand_n, int cap,
                       int xcd, hipStream_t st, int sets, int tshift, int rsplit,
                       const int* gate, const int* blist, int list_tiles, int zero_cnt, int dim);
int symb_mq_max_sets(int dim);
int symb_index_scan_mq_ablate(const void* X, int n_valid, int rows_per_blk, int n_rblk,
                              const void* Q, int NQ, const float* thr, float* cand_s, int* cand_i,
                              int* cand_n, int cap, int xcd, hipStream_t st, int abl, int sets,
                              int rsplit);
int symb_prune_stats(const int* ovf, const int* cnt, int NQ, const int* dense, const int* blk,
                     int* tot, hipStream_t st);
int symb_topk_select_counted(const float* cand_s, const int* cand_i, const int* cand_n, int cap,
                             int NQ, int kmax, int k, float* out_s, int* out_i, int* ovf,
                             hipStream_t st, const int* gate, int reset_ovf, int ld = 0,
                             float* kth_out = nullptr, float kth_margin = 0.f,
                             const float* seg2_s = nullptr, int seg2_cap = 0,
                             float* seg2_out_s = nullptr, int* seg2_out_i = nullptr);

namespace {

using uptr = uintptr_t;
template <class T>
inline T* P(uptr p) { return reinterpret_cast<T*>(p); }
inline hipStream_t S(uptr s) { return reinterpret_cast<hipStream_t>(s); }

// GPU debug mode (SYMB_GPU_DEBUG=1, ops/_ext.py): every launch is followed by a device-wide
// synchronize, so an asynchronous fault (bad address, illegal instruction) is raised by the call
// that launched the faulting kernel, named, instead of by some later unrelated sync point.
static bool g_debug = false;

void check(int rc, const char* what) {
  if (rc == 0) {
    if (!g_debug) return;
    rc = (int)hipDeviceSynchronize();
    if (rc == 0) rc = (int)hipGetLastError();
    if (rc == 0) return;
    throw std::runtime_error(std::string(what) + " [serialized, SYMB_GPU_DEBUG]: " +
                             hipGetErrorString((hipError_t)rc));
  }
  if (rc < 0) throw std::invalid_argument(std::string(what) + ": unsupported shape/config");
  throw std::runtime_error(std::string(what) + ": " + hipGetErrorString((hipError_t)rc));
}

enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RES = 2, EPI_RES_LN = 3, EPI_GELU_MX8 = 4 };

struct LayerWeights {
  uptr wqkv, bqkv, wo, bo, ln1_g, ln1_b, wi, bi, wo2, bo2, ln2_g, ln2_b;
  // fp8 layers: the four weight pointers above are e4m3 [N, K] and these are their per-output-
  // channel scales (f32 [N]); activations are quantised per token right before each GEMM
  bool fp8 = false;
  uptr sw_qkv = 0, sw_o = 0, sw_i = 0, sw_o2 = 0;
  // deferred LayerNorm (set_fold): the QKV weight folded with the PREVIOUS layer's ln2 gamma and
  // the FFN1 weight folded with this layer's ln1 gamma, their biases b + W beta and the folded
  // weights' row sums (0 for layer 0's QKV, whose input the embedding LayerNorm normalised)
  uptr fq_w = 0, fq_b = 0, fq_cs = 0, fi_w = 0, fi_b = 0, fi_cs = 0;
  bool folded = false;
};

class EncoderRuntime {
 public:
  EncoderRuntime(int hidden, int n_heads, int ffn, float eps, uptr wemb, uptr pemb, uptr temb,
                 uptr eln_g, uptr eln_b)
      : H_(hidden), nh_(n_heads), hd_(hidden / n_heads), FF_(ffn), eps_(eps), wemb_(wemb),
        pemb_(pemb), temb_(temb), eln_g_(eln_g), eln_b_(eln_b) {
    if (H_ % n_heads) throw std::invalid_argument("hidden % heads != 0");
  }
  void add_layer(const std::vector<uptr>& w) {
    if (w.size() != 12) throw std::invalid_argument("layer needs 12 pointers");
    layers_.push_back(LayerWeights{w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], w[8], w[9],
                                   w[10], w[11]});
  }
  void add_layer_fp8(const std::vector<uptr>& w) {
    if (w.size() != 16) throw std::invalid_argument("fp8 layer needs 12 pointers + 4 scales");
    if (H_ % 128 || FF_ % 128) throw std::invalid_argument("fp8 layers need hidden/ffn % 128 == 0");
    LayerWeights L{w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], w[8], w[9], w[10], w[11]};
    L.fp8 = true;
    L.sw_qkv = w[12];
    L.sw_o = w[13];
    L.sw_i = w[14];
    L.sw_o2 = w[15];
    layers_.push_back(L);
    any_fp8_ = true;
  }
  int num_layers() const { return (int)layers_.size(); }
  // The deferred-LayerNorm operands of bf16 layer li (gemm.hip LNF): pointers 0 for layer 0's QKV.
  void set_fold(int li, const std::vector<uptr>& w) {
    if (li < 0 || li >= (int)layers_.size() || w.size() != 6)
      throw std::invalid_argument("set_fold: layer index and 6 pointers");
    auto& L = layers_[li];
    if (L.fp8) throw std::invalid_argument("set_fold: bf16 layers only");
    if ((li == 0) != (w[0] == 0)) throw std::invalid_argument("set_fold: QKV fold from layer 1 on");
    L.fq_w = w[0]; L.fq_b = w[1]; L.fq_cs = w[2]; L.fi_w = w[3]; L.fi_b = w[4]; L.fi_cs = w[5];
    L.folded = true;
  }
  // 0 = the add_ln path for wide rows, 1 = deferred LayerNorm where every layer is folded
  void set_deferred_ln(int mode) {
    if (mode != 0 && mode != 1) throw std::invalid_argument("deferred_ln: 0 or 1");
    deferred_ln_ = mode;
  }
  bool deferred_ln_ready() const {
    if (layers_.empty()) return false;
    for (const auto& L : layers_)
      if (L.fp8 || !L.folded) return false;
    return true;
  }

  // Split-partial buffer the bf16 layers' small-M (query-path) GEMMs need: skinny_ws_bytes().
  size_t skinny_ws_bytes() const {
    const int H = H_, M = 256;   // the largest M the small-M path may be configured to take
    size_t b = 0;
    auto mx = [&](int epi, int N, int K) { b = std::max(b, symb_gemm_skinny_scratch_bytes(epi, M, N, K)); };
    mx(EPI_BIAS, 3 * H, H);
    mx(H == 384 ? EPI_RES_LN : EPI_RES, H, H);
    mx(EPI_GELU, FF_, H);
    mx(H == 384 ? EPI_RES_LN : EPI_RES, H, FF_);
    return b;
  }

  // ws: {h, h2, qkv, ctx, ff, tmp} device buffers sized for T tokens; fp8 layers add
  // {a8 (T x max(H, FF) bytes), sa (T floats)}.  Optionally one more, last: the small-M GEMMs'
  // split-partial buffer of skinny_ws_bytes() bytes (a captured graph then owns its own).
  void forward(uptr ids, uptr pos, uptr tt, uptr cu, int T, int B, int max_len,
               const std::vector<uptr>& ws_in, int pool_mode, int normalize_f32, uptr out_f32,
               uptr out_norm, uptr stream) {
    const size_t base = any_fp8_ ? 8u : 6u;
    if (ws_in.size() != base && ws_in.size() != base + 1)
      throw std::invalid_argument(any_fp8_ ? "fp8 workspace needs 8 buffers (+ skinny scratch)"
                                           : "workspace needs 6 buffers (+ skinny scratch)");
    std::vector<uptr> ws(ws_in.begin(), ws_in.begin() + base);
    struct ScratchGuard {
      ScratchGuard(uptr p, size_t n) { symb_gemm_skinny_set_scratch(P<void>(p), n); }
      ~ScratchGuard() { symb_gemm_skinny_set_scratch(nullptr, 0); }
    } guard(ws_in.size() > base ? ws_in.back() : 0, skinny_ws_bytes());
    hipStream_t st = S(stream);
    const int H = H_;
    uptr h = ws[0], h2 = ws[1], qkv = ws[2], ctx = ws[3], ff = ws[4], tmp = ws[5];
    check(symb_embed_ln(P<int32_t>(ids), P<int32_t>(pos), P<int32_t>(tt), P<void>(wemb_),
                        P<void>(pemb_), P<void>(temb_), P<float>(eln_g_), P<float>(eln_b_), eps_,
                        P<void>(h), T, H, st),
          "embed_ln");
    // residual + LayerNorm inside the out-proj / FFN2 GEMM: the 384-wide row-complete tiles, or,
    // at any width, the small-M path's split-sum kernel (query-path batches, scratch provided)
    const bool fuse_ln = (H == 384) ||
                         (ws_in.size() > base && T <= symb_gemm_skinny_max_m() &&
                          symb_gemm_skinny_scratch_bytes(EPI_RES_LN, T, H, H) > 0 &&
                          symb_gemm_skinny_scratch_bytes(EPI_RES_LN, T, H, FF_) > 0);
    if (!fuse_ln && H % 64 == 0 && deferred_ln_ && deferred_ln_ready()) {
      deferred_forward(ws, T, B, max_len, cu, st, pool_mode, normalize_f32, out_f32, out_norm);
      return;
    }
    bool h_quantized = false;  // a8/sa hold the per-token e4m3 image of h (fp8 layers)
    for (size_t li = 0; li < layers_.size(); ++li) {
      const auto& L = layers_[li];
      if (L.fp8) {
        const bool next_fp8 = li + 1 < layers_.size() && layers_[li + 1].fp8;
        fp8_layer(L, ws, T, B, max_len, cu, st, h_quantized, next_fp8);
        h_quantized = next_fp8;
        continue;
      }
      h_quantized = false;
      // the QKV activation never leaves the CU: one launch per layer for short-sentence batches
      const bool fused_qkv = g_qkv_attn && H == 384 && hd_ == 32 && nh_ == 12 && max_len <= 128 &&
                             T > symb_gemm_skinny_max_m();
      if (fused_qkv) {
        check(symb_qkv_attention(P<void>(h), P<void>(L.wqkv), P<float>(L.bqkv), P<int32_t>(cu), B,
                                 max_len, nh_, hd_, P<void>(ctx), st),
              "qkv+attention");
      } else {
        check(symb_gemm(EPI_BIAS, P<void>(h), H, P<void>(L.wqkv), H, P<float>(L.bqkv), nullptr,
                        0, nullptr, nullptr, 0.f, P<void>(qkv), 3 * H, T, 3 * H, H, st),
              "qkv gemm");
        check(symb_attention(P<void>(qkv), 3 * H, P<int32_t>(cu), B, max_len, nh_, hd_,
                             P<void>(ctx), H, st),
              "attention");
      }
      // the fused FFN block (mlp_fused.hip) for 384 x 1536 layers above the small-M limit
      const bool fused_ffn = g_mlp_fused && H == 384 && FF_ == 1536 && T > symb_gemm_skinny_max_m();
      if (fuse_ln) {
        check(symb_gemm(EPI_RES_LN, P<void>(ctx), H, P<void>(L.wo), H, P<float>(L.bo),
                        P<void>(h), H, P<float>(L.ln1_g), P<float>(L.ln1_b), eps_, P<void>(h2),
                        H, T, H, H, st),
              "out-proj+LN gemm");
      } else {
        check(symb_gemm(EPI_RES, P<void>(ctx), H, P<void>(L.wo), H, P<float>(L.bo), P<void>(h),
                        H, nullptr, nullptr, 0.f, P<void>(tmp), H, T, H, H, st),
              "out-proj gemm");
        check(symb_add_ln(P<void>(tmp), nullptr, P<float>(L.ln1_g), P<float>(L.ln1_b), eps_,
                          P<void>(h2), T, H, st),
              "ln1");
      }
      if (fused_ffn) {
        // the whole FFN block in one launch: the 1536-wide activation never leaves the CU
        check(symb_mlp_fused(P<void>(h2), P<void>(L.wi), P<float>(L.bi), P<void>(L.wo2),
                             P<float>(L.bo2), P<float>(L.ln2_g), P<float>(L.ln2_b), eps_,
                             symb_gemm_gelu_poly(), P<void>(h), T, H, FF_, st),
              "fused ffn");
        continue;
      }
      check(symb_gemm(EPI_GELU, P<void>(h2), H, P<void>(L.wi), H, P<float>(L.bi), nullptr, 0,
                      nullptr, nullptr, 0.f, P<void>(ff), FF_, T, FF_, H, st),
            "ffn1 gemm");
      if (fuse_ln) {
        check(symb_gemm(EPI_RES_LN, P<void>(ff), FF_, P<void>(L.wo2), FF_, P<float>(L.bo2),
                        P<void>(h2), H, P<float>(L.ln2_g), P<float>(L.ln2_b), eps_, P<void>(h),
                        H, T, H, FF_, st),
              "ffn2+LN gemm");
      } else {
        check(symb_gemm(EPI_RES, P<void>(ff), FF_, P<void>(L.wo2), FF_, P<float>(L.bo2),
                        P<void>(h2), H, nullptr, nullptr, 0.f, P<void>(tmp), H, T, H, FF_, st),
              "ffn2 gemm");
        check(symb_add_ln(P<void>(tmp), nullptr, P<float>(L.ln2_g), P<float>(L.ln2_b), eps_,
                          P<void>(h), T, H, st),
              "ln2");
      }
    }
    if (out_f32)
      check(symb_pool(P<void>(h), P<int32_t>(cu), B, H, pool_mode, normalize_f32, P<float>(out_f32),
                      P<void>(out_norm), st),
            "pool");
  }

 private:
  // Deferred-LayerNorm forward (bf16 layers at H >= 768, above the small-M limit): no add_ln pass
  // and no hipBLASLt.  Per layer, with y2 = the previous layer's pre-LN output in h (layer 0: the
  // embedding LayerNorm's normalised output) and its row statistics in s2:
  //   qkv = LN2(y2) Wqkv^T + b       QKV GEMM on the folded weight, LNF_FOLD epilogue (s2)
  //   y1  = ctx Wo^T + bo + LN2(y2)  out-proj, LNF_RESLN | LNF_STATS epilogue (reads s2, writes s1)
  //   ff  = GELU(LN1(y1) W1^T + b1)  FFN1 on the folded weight, LNF_FOLD epilogue (s1)
  //   y2' = ff W2^T + b2 + LN1(y1)   FFN2, LNF_RESLN | LNF_STATS epilogue (reads s1, writes s2)
  // and the pool kernel applies the last ln2 to every token row before pooling.
  void deferred_forward(const std::vector<uptr>& ws, int T, int B, int max_len, uptr cu,
                        hipStream_t st, int pool_mode, int normalize_f32, uptr out_f32,
                        uptr out_norm) {
    const int H = H_, NP = H / 64;
    uptr h = ws[0], y1 = ws[1], qkv = ws[2], ctx = ws[3], ff = ws[4];
    // the row statistics live in the add_ln path's tmp buffer (T x H bf16 = 2 T H bytes; the two
    // float2 [T][H / 64] sets need T H / 4)
    void* s1 = P<void>(ws[5]);
    void* s2 = P<void>(ws[5] + (uptr)T * NP * 8);
    const float *g2 = nullptr, *b2 = nullptr;   // the previous layer's ln2 (h is pre-LN)
    for (size_t li = 0; li < layers_.size(); ++li) {
      const auto& L = layers_[li];
      const bool pre = li > 0;
      if (pre)
        check(symb_gemm_ln(EPI_BIAS, 1, P<void>(h), H, P<void>(L.fq_w), H, P<float>(L.fq_b),
                           nullptr, 0, nullptr, nullptr, eps_, P<float>(L.fq_cs), s2, NP, nullptr,
                           P<void>(qkv), 3 * H, T, 3 * H, H, st),
              "qkv gemm (folded ln2)");
      else
        check(symb_gemm_ln_plain(EPI_BIAS, h, L.wqkv, L.bqkv, 0, qkv, T, 3 * H, H, st),
              "qkv gemm");
      check(symb_attention(P<void>(qkv), 3 * H, P<int32_t>(cu), B, max_len, nh_, hd_,
                           P<void>(ctx), H, st),
            "attention");
      check(symb_gemm_ln(EPI_RES, pre ? 2 | 4 : 4, P<void>(ctx), H, P<void>(L.wo), H,
                         P<float>(L.bo), P<void>(h), H, g2, b2, eps_, nullptr, pre ? s2 : nullptr,
                         NP, s1, P<void>(y1), H, T, H, H, st),
            "out-proj gemm (+ln2, stats)");
      check(symb_gemm_ln(EPI_GELU, 1, P<void>(y1), H, P<void>(L.fi_w), H, P<float>(L.fi_b),
                         nullptr, 0, nullptr, nullptr, eps_, P<float>(L.fi_cs), s1, NP, nullptr,
                         P<void>(ff), FF_, T, FF_, H, st),
            "ffn1 gemm (folded ln1)");
      check(symb_gemm_ln(EPI_RES, 2 | 4, P<void>(ff), FF_, P<void>(L.wo2), FF_, P<float>(L.bo2),
                         P<void>(y1), H, P<float>(L.ln1_g), P<float>(L.ln1_b), eps_, nullptr, s1,
                         NP, s2, P<void>(h), H, T, H, FF_, st),
            "ffn2 gemm (+ln1, stats)");
      g2 = P<float>(L.ln2_g);
      b2 = P<float>(L.ln2_b);
    }
    if (out_f32)
      check(symb_pool(P<void>(h), P<int32_t>(cu), B, H, pool_mode, normalize_f32, P<float>(out_f32),
                      P<void>(out_norm), st, g2, b2, eps_),
            "pool (+ln2)");
    else   // token states requested: normalise h in place (one pass, last layer only)
      check(symb_add_ln(P<void>(h), nullptr, g2, b2, eps_, P<void>(h), T, H, st), "final ln2");
  }

  // plain bias GEMM on this repo's tiles (layer 0's QKV of the deferred forward: never hipBLASLt)
  static int symb_gemm_ln_plain(int epi, uptr A, uptr W, uptr b, uptr R, uptr C, int M, int N,
                                int K, hipStream_t st) {
    (void)R;
    return symb_gemm_ln(epi, 0, P<void>(A), K, P<void>(W), K, P<float>(b), nullptr, 0, nullptr,
                        nullptr, 0.f, nullptr, nullptr, 0, nullptr, P<void>(C), N, M, N, K, st);
  }

  // e4m3 layer: every projection is an fp8 MFMA GEMM with its scales folded into the epilogue.
  // Activation hand-offs (no separate quantiser pass inside a run of fp8 layers):
  //   h   --(previous layer's ln2, fused per-token quant, or quant_rows here)--> QKV
  //   attention emits ctx as MX fp8 (E8M0 per 32 head dims) --> out-proj's block-scaled MFMA
  //   out-proj --ln1 + fused per-token quant--> FFN1
  //   FFN1 epilogue emits GELU as MX fp8 (E8M0 per 32 columns) --> FFN2's block-scaled MFMA
  // h_quantized: a8/sa already hold h's quantisation; quantize_out: leave the output h quantised
  // in a8/sa for the next (fp8) layer.
  void fp8_layer(const LayerWeights& L, const std::vector<uptr>& ws, int T, int B, int max_len,
                 uptr cu, hipStream_t st, bool h_quantized, bool quantize_out) {
    const int H = H_;
    uptr h = ws[0], h2 = ws[1], qkv = ws[2], tmp = ws[5];
    uptr a8 = ws[6];
    float* sa = P<float>(ws[7]);
    // the bf16 FFN buffer (T x FF x 2 bytes) holds the MX activations: T x FF e4m3 + T x FF/32
    // E8M0 for FFN1 -> FFN2, then T x H/32 E8M0 for the attention output (its e4m3 bytes go to
    // the bf16 ctx buffer, T x H x 2 bytes)
    uptr ff8 = ws[4], ffs = ws[4] + (uptr)T * FF_, ctxs = ffs + (uptr)T * (FF_ / 32);
    uptr ctx8 = ws[3];
    auto q8 = [&](uptr x, int K, const char* what) {
      check(symb_quant_rows_fp8(P<void>(x), K, P<void>(a8), K, sa, T, K, st), what);
    };
    if (!h_quantized) q8(h, H, "quant h");
    check(symb_gemm_fp8(EPI_BIAS, P<void>(a8), H, P<void>(L.wqkv), H, sa, P<float>(L.sw_qkv),
                        P<float>(L.bqkv), nullptr, 0, P<void>(qkv), 3 * H, T, 3 * H, H, st),
          "qkv gemm fp8");
    check(symb_attention(P<void>(qkv), 3 * H, P<int32_t>(cu), B, max_len, nh_, hd_, P<void>(ctx8),
                         H, st, P<void>(ctxs)),
          "attention -> mx8");
    check(symb_gemm_fp8(EPI_RES, P<void>(ctx8), H, P<void>(L.wo), H, nullptr, P<float>(L.sw_o),
                        P<float>(L.bo), P<void>(h), H, P<void>(tmp), H, T, H, H, st, P<void>(ctxs),
                        nullptr),
          "out-proj gemm mx8");
    check(symb_add_ln(P<void>(tmp), nullptr, P<float>(L.ln1_g), P<float>(L.ln1_b), eps_,
                      P<void>(h2), T, H, st, P<void>(a8), sa),
          "ln1 + quant");
    check(symb_gemm_fp8(EPI_GELU_MX8, P<void>(a8), H, P<void>(L.wi), H, sa, P<float>(L.sw_i),
                        P<float>(L.bi), nullptr, 0, P<void>(ff8), FF_, T, FF_, H, st, nullptr,
                        P<void>(ffs)),
          "ffn1 gemm fp8 -> mx8");
    check(symb_gemm_fp8(EPI_RES, P<void>(ff8), FF_, P<void>(L.wo2), FF_, nullptr,
                        P<float>(L.sw_o2), P<float>(L.bo2), P<void>(h2), H, P<void>(tmp), H, T, H,
                        FF_, st, P<void>(ffs), nullptr),
          "ffn2 gemm mx8");
    check(symb_add_ln(P<void>(tmp), nullptr, P<float>(L.ln2_g), P<float>(L.ln2_b), eps_,
                      P<void>(h), T, H, st, quantize_out ? P<void>(a8) : nullptr,
                      quantize_out ? sa : nullptr),
          "ln2");
  }

  bool any_fp8_ = false;
  int deferred_ln_ = 0;
  int H_, nh_, hd_, FF_;
  float eps_;
  uptr wemb_, pemb_, temb_, eln_g_, eln_b_;
  std::vector<LayerWeights> layers_;
};

}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "CDNA4 (gfx950) HIP kernels of codename_symbiont_amd";
  m.def("arch", []() { return std::string("gfx950"); });
  m.def("stream_destroy", [](uptr st) { check((int)hipStreamDestroy(S(st)), "hipStreamDestroy"); },
        py::arg("stream"));
  m.def("cu_count", [](int device) {
    int n = 0;
    check((int)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device),
          "hipDeviceGetAttribute");
    return n;
  }, py::arg("device"));
  m.def("set_debug", [](bool on) { g_debug = on; }, py::arg("on"));
  m.def("debug", []() { return g_debug; });
  m.def("embed_ln", [](uptr ids, uptr pos, uptr tt, uptr wemb, uptr pemb, uptr temb, uptr g,
                       uptr b, float eps, uptr out, int T, int H, uptr st) {
    check(symb_embed_ln(P<int32_t>(ids), P<int32_t>(pos), P<int32_t>(tt), P<void>(wemb),
                        P<void>(pemb), P<void>(temb), P<float>(g), P<float>(b), eps, P<void>(out),
                        T, H, S(st)),
          "embed_ln");
  });
  m.def("add_ln", [](uptr x, uptr res, uptr g, uptr b, float eps, uptr out, int T, int H, uptr st,
                     uptr out8, uptr scale8) {
    check(symb_add_ln(P<void>(x), P<void>(res), P<float>(g), P<float>(b), eps, P<void>(out), T, H,
                      S(st), P<void>(out8), P<float>(scale8)),
          "add_ln");
  }, py::arg("x"), py::arg("res"), py::arg("g"), py::arg("b"), py::arg("eps"), py::arg("out"),
     py::arg("T"), py::arg("H"), py::arg("st"), py::arg("out8") = 0, py::arg("scale8") = 0);
  m.def("pool", [](uptr hidden, uptr cu, int B, int H, int mode, int normalize_f32, uptr out_f32,
                   uptr out_norm, uptr st, uptr g, uptr b, float eps) {
    check(symb_pool(P<void>(hidden), P<int32_t>(cu), B, H, mode, normalize_f32, P<float>(out_f32),
                    P<void>(out_norm), S(st), P<float>(g), P<float>(b), eps),
          "pool");
  }, py::arg("hidden"), py::arg("cu"), py::arg("B"), py::arg("H"), py::arg("mode"),
     py::arg("normalize_f32"), py::arg("out_f32"), py::arg("out_norm"), py::arg("st"),
     py::arg("g") = 0, py::arg("b") = 0, py::arg("eps") = 0.f);
  m.def("l2norm_cast", [](uptr x, uptr out, int n, int D, int ld_out, uptr st) {
    check(symb_l2norm_cast(P<float>(x), P<void>(out), n, D, ld_out, S(st)), "l2norm_cast");
  });
  m.def("gemm", [](int epi, uptr A, int lda, uptr W, int ldw, uptr bias, uptr R, int ldr, uptr g,
                   uptr b, float eps, uptr C, int ldc, int M, int N, int K, uptr st) {
    check(symb_gemm(epi, P<void>(A), lda, P<void>(W), ldw, P<float>(bias), P<void>(R), ldr,
                    P<float>(g), P<float>(b), eps, P<void>(C), ldc, M, N, K, S(st)),
          "gemm");
  });
  m.def("gemm_ln", [](int epi, int lnf, uptr A, int lda, uptr W, int ldw, uptr bias, uptr R,
                      int ldr, uptr g, uptr b, float ln_eps, uptr cs, uptr st_in, int np_in,
                      uptr st_out, uptr C, int ldc, int M, int N, int K, uptr st) {
    check(symb_gemm_ln(epi, lnf, P<void>(A), lda, P<void>(W), ldw, P<float>(bias), P<void>(R), ldr,
                       P<float>(g), P<float>(b), ln_eps, P<float>(cs), P<void>(st_in), np_in,
                       P<void>(st_out), P<void>(C), ldc, M, N, K, S(st)),
          "gemm_ln");
  });
  m.def("attention", [](uptr qkv, int ld_qkv, uptr cu, int B, int max_len, int n_heads,
                        int head_dim, uptr out, int ld_out, uptr st, uptr oscale) {
    check(symb_attention(P<void>(qkv), ld_qkv, P<int32_t>(cu), B, max_len, n_heads, head_dim,
                         P<void>(out), ld_out, S(st), P<void>(oscale)),
          "attention");
  }, py::arg("qkv"), py::arg("ld_qkv"), py::arg("cu"), py::arg("B"), py::arg("max_len"),
     py::arg("n_heads"), py::arg("head_dim"), py::arg("out"), py::arg("ld_out"), py::arg("st"),
     py::arg("oscale") = 0);
  m.def("qkv_attention", [](uptr X, uptr Wqkv, uptr bqkv, uptr cu, int B, int max_len,
                            int n_heads, int head_dim, uptr out, uptr st) {
    check(symb_qkv_attention(P<void>(X), P<void>(Wqkv), P<float>(bqkv), P<int32_t>(cu), B, max_len,
                             n_heads, head_dim, P<void>(out), S(st)),
          "qkv_attention");
  }, py::arg("X"), py::arg("Wqkv"), py::arg("bqkv"), py::arg("cu"), py::arg("B"),
     py::arg("max_len"), py::arg("n_heads"), py::arg("head_dim"), py::arg("out"), py::arg("st"));
  m.def("qkv_attn_config", [](int mode) {   // 0: QKV GEMM + attention, 1: fused (default)
    if (mode < 0 || mode > 1) throw std::invalid_argument("qkv_attn_config: mode 0 or 1");
    g_qkv_attn = mode;
  });
  m.def("topk_geometry", [](int D, int kmax) {
    int lists = 0, qpb = 0;
    check(symb_topk_geometry(D, kmax, &lists, &qpb), "topk_geometry");
    return py::make_tuple(lists, qpb);
  });
  m.def("index_scan", [](uptr X, int n_valid, int D, int rows_per_blk, int n_rblk, uptr Q, int NQ,
                         int kmax, uptr cand_s, uptr cand_i, uptr st, int ns, int aux, uptr thr,
                         int xcd, uptr gate) {
    check(symb_index_scan(P<void>(X), n_valid, D, rows_per_blk, n_rblk, P<void>(Q), NQ, kmax,
                          P<float>(cand_s), P<int>(cand_i), S(st), ns, aux, P<const float>(thr),
                          xcd, P<const int>(gate)),
          "index_scan");
  }, py::arg("X"), py::arg("n_valid"), py::arg("D"), py::arg("rows_per_blk"), py::arg("n_rblk"),
     py::arg("Q"), py::arg("NQ"), py::arg("kmax"), py::arg("cand_s"), py::arg("cand_i"),
     py::arg("stream"), py::arg("ns") = 0, py::arg("aux") = -1, py::arg("thr_init") = 0,
     py::arg("xcd") = 1, py::arg("gate") = 0);
  // multi-query-block D=384 scan (index_mq.hip): candidates above the seeded thresholds
  m.def("i8_queries_per_blk", [](int rsplit) { return symb_i8_queries_per_blk(rsplit); },
        py::arg("rsplit") = 2);
  m.def("i8_config", [](int tile_rows, int waves) { check(symb_i8_config(tile_rows, waves), "i8_config"); },
        py::arg("tile_rows"), py::arg("waves") = 8);
  m.def("i8_tile_rows", [](int dim, int heavy) { return symb_i8_tile_rows_for(dim, heavy); },
        py::arg("dim") = 384, py::arg("heavy") = 0);
  m.def("mx4_config", [](int tile_rows) { check(symb_mx4_config(tile_rows), "mx4_config"); },
        py::arg("tile_rows"));
  m.def("mx4_tile_rows", []() { return symb_mx4_tile_rows(); });
  m.def("i8_split_queries_per_blk", [](int rsplit) { return symb_i8_split_queries_per_blk(rsplit); },
        py::arg("rsplit") = 2);
  m.def("quant_rows_split", [](uptr X, int n, int dim, uptr X8, uptr sx, uptr bounds, uptr margin,
                               uptr st) {
    check(symb_quant_rows_split(P<const float>(X), n, dim, P<void>(X8), P<float>(sx),
                                P<float>(bounds), P<float>(margin), S(st)),
          "quant_rows_split");
  }, py::arg("X"), py::arg("n"), py::arg("dim"), py::arg("X8"), py::arg("sx"), py::arg("bounds"),
     py::arg("margin"), py::arg("stream"));
  m.def("i8_wgs_per_cu", []() { return symb_i8_wgs_per_cu(); });
  m.def("index_scan_i8", [](uptr X8, uptr sx, int n_valid, int alloc_rows, int rows_per_blk,
                            int n_rblk, uptr Q8, int NQ, uptr thr, uptr cand_s, uptr cand_i,
                            uptr cand_n, int cap, int xcd, uptr st, int rsplit, uptr skip, int dim,
                            int heavy, uptr sq, int form, uptr gate, int gate_want) {
    check(symb_index_scan_i8(P<void>(X8), P<const float>(sx), n_valid, alloc_rows, rows_per_blk,
                             n_rblk,
                             P<void>(Q8), NQ, P<const float>(thr), P<float>(cand_s), P<int>(cand_i),
                             P<int>(cand_n), cap, xcd, S(st), rsplit, P<const int>(skip), dim,
                             heavy, P<const float>(sq), form, P<const int>(gate), gate_want),
          "index_scan_i8");
  }, py::arg("X8"), py::arg("sx"), py::arg("n_valid"), py::arg("alloc_rows"),
     py::arg("rows_per_blk"), py::arg("n_rblk"), py::arg("Q8"), py::arg("NQ"), py::arg("thr"),
     py::arg("cand_s"), py::arg("cand_i"), py::arg("cand_n"), py::arg("cap"), py::arg("xcd"),
     py::arg("stream"), py::arg("rsplit"), py::arg("skip") = 0, py::arg("dim") = 384,
     py::arg("heavy") = 0, py::arg("sq") = 0, py::arg("form") = 0, py::arg("gate") = 0,
     py::arg("gate_want") = 0);
  m.def("stream_rec_bytes", [](int dim, int form) { return symb_stream_rec_bytes(dim, form); },
        py::arg("dim"), py::arg("form"));
  m.def("stream_config", [](int abl) { check(symb_stream_config(abl), "stream_config"); },
        py::arg("abl") = 0);
  m.def("stream_geometry", [](int dim, int form) {
    int qpb = 0, wpc = 0;
    check(symb_stream_geometry(dim, form, &qpb, &wpc), "stream_geometry");
    return py::make_tuple(qpb, wpc);
  }, py::arg("dim"), py::arg("form"));
  m.def("index_scan_stream", [](uptr img, int n_valid, int alloc_rows, int rows_per_blk, int n_rblk,
                                uptr Q, uptr qsc, int NQ, uptr thr, uptr cand_s, uptr cand_i,
                                uptr cand_n, int cap, int xcd, uptr st, uptr skip, int dim,
                                int form, uptr gate, int gate_want, int zero_cnt, uptr runs,
                                uptr cent4, uptr centqs, uptr centR, uptr bounds4) {
    check(symb_index_scan_stream(P<void>(img), n_valid, alloc_rows, rows_per_blk, n_rblk,
                                 P<void>(Q), P<void>(qsc), NQ, P<const float>(thr),
                                 P<float>(cand_s), P<int>(cand_i), P<int>(cand_n), cap, xcd, S(st),
                                 P<const int>(skip), dim, form, P<const int>(gate), gate_want,
                                 zero_cnt, P<int>(runs), P<void>(cent4), P<void>(centqs),
                                 P<const float>(centR), P<const float>(bounds4)),
          "index_scan_stream");
  }, py::arg("img"), py::arg("n_valid"), py::arg("alloc_rows"), py::arg("rows_per_blk"),
     py::arg("n_rblk"), py::arg("Q"), py::arg("qsc"), py::arg("NQ"), py::arg("thr"),
     py::arg("cand_s"), py::arg("cand_i"), py::arg("cand_n"), py::arg("cap"), py::arg("xcd"),
     py::arg("stream"), py::arg("skip") = 0, py::arg("dim") = 384, py::arg("form") = 0,
     py::arg("gate") = 0, py::arg("gate_want") = 0, py::arg("zero_cnt") = 1, py::arg("runs") = 0,
     py::arg("cent4") = 0, py::arg("centqs") = 0, py::arg("centR") = 0, py::arg("bounds4") = 0);
  m.def("mx4_centroids", [](uptr Xq, uptr QS, int NQ, int dim, uptr C4, uptr CS, uptr R, uptr st) {
    check(symb_mx4_centroids(P<void>(Xq), P<void>(QS), NQ, dim, P<void>(C4), P<void>(CS),
                             P<float>(R), S(st)),
          "mx4_centroids");
  }, py::arg("Xq"), py::arg("QS"), py::arg("NQ"), py::arg("dim"), py::arg("C4"), py::arg("CS"),
     py::arg("R"), py::arg("stream"));
  m.def("append_rows", [](uptr src, int n, int dim, uptr rows, int r0, uptr img8, uptr b8,
                          uptr img4, uptr b4, uptr st, uptr img6, uptr b6) {
    check(symb_append_rows(P<void>(src), n, dim, P<void>(rows), r0, P<void>(img8), P<float>(b8),
                           P<void>(img4), P<float>(b4), P<void>(img6), P<float>(b6), S(st)),
          "append_rows");
  }, py::arg("src"), py::arg("n"), py::arg("dim"), py::arg("rows"), py::arg("r0"),
     py::arg("img8"), py::arg("b8"), py::arg("img4"), py::arg("b4"), py::arg("stream"),
     py::arg("img6") = 0, py::arg("b6") = 0);
  m.def("dense_scores", [](uptr X, int dim, uptr rows, int n_list, int r_lo, int n_range, uptr Q,
                           int NQ, uptr out, int ld, uptr st, int ts, int div) {
    check(symb_dense_scores(P<void>(X), dim, P<const int>(rows), n_list, ts, div, r_lo, n_range,
                            P<void>(Q), NQ, P<float>(out), ld, S(st)),
          "dense_scores");
  }, py::arg("X"), py::arg("dim"), py::arg("rows"), py::arg("n_list"), py::arg("r_lo"),
     py::arg("n_range"), py::arg("Q"), py::arg("NQ"), py::arg("out"), py::arg("ld"),
     py::arg("stream"), py::arg("ts") = 0, py::arg("div") = 1);
  m.def("quant_stream_i8", [](uptr X, int r0, uptr rows, int n, int dim, uptr img, uptr bounds,
                              uptr st) {
    check(symb_quant_stream_i8(P<void>(X), r0, P<const int>(rows), n, dim, P<void>(img),
                               P<float>(bounds), S(st)),
          "quant_stream_i8");
  }, py::arg("X"), py::arg("r0"), py::arg("rows"), py::arg("n"), py::arg("dim"), py::arg("img"),
     py::arg("bounds"), py::arg("stream"));
  m.def("prefill_candidates", [](int NQ, int r_lo, int n, uptr cand_i, uptr cand_n, int cap,
                                 uptr st) {
    check(symb_prefill_candidates(NQ, r_lo, n, P<int>(cand_i), P<int>(cand_n), cap, S(st)),
          "prefill_candidates");
  }, py::arg("NQ"), py::arg("r_lo"), py::arg("n"), py::arg("cand_i"), py::arg("cand_n"),
     py::arg("cap"), py::arg("stream"));
  m.def("quant_stream_mx4", [](uptr X, int r0, uptr rows, int n, int dim, uptr img, uptr Xq,
                               uptr QS, uptr bounds, uptr margin, uptr st) {
    check(symb_quant_stream_mx4(P<void>(X), r0, P<const int>(rows), n, dim, P<void>(img),
                                P<void>(Xq), P<void>(QS), P<float>(bounds), P<float>(margin),
                                S(st)),
          "quant_stream_mx4");
  }, py::arg("X"), py::arg("r0"), py::arg("rows"), py::arg("n"), py::arg("dim"), py::arg("img"),
     py::arg("Xq"), py::arg("QS"), py::arg("bounds"), py::arg("margin"), py::arg("stream"));
  m.def("quant_stream_mx6", [](uptr X, int r0, uptr rows, int n, int dim, uptr img, uptr Xq,
                               uptr QS, uptr bounds, uptr margin, uptr st) {
    check(symb_quant_stream_mx6(P<void>(X), r0, P<const int>(rows), n, dim, P<void>(img),
                                P<void>(Xq), P<void>(QS), P<float>(bounds), P<float>(margin),
                                S(st)),
          "quant_stream_mx6");
  }, py::arg("X"), py::arg("r0"), py::arg("rows"), py::arg("n"), py::arg("dim"), py::arg("img"),
     py::arg("Xq"), py::arg("QS"), py::arg("bounds"), py::arg("margin"), py::arg("stream"));
  m.def("quant_rows_mx4", [](uptr X, int n, int dim, uptr X4, uptr SC, uptr bounds, uptr margin,
                             uptr st) {
    check(symb_quant_rows_mx4(P<void>(X), n, dim, P<void>(X4), P<void>(SC), P<float>(bounds),
                              P<float>(margin), S(st)),
          "quant_rows_mx4");
  }, py::arg("X"), py::arg("n"), py::arg("dim"), py::arg("X4"), py::arg("SC"), py::arg("bounds"),
     py::arg("margin"), py::arg("stream"));
  m.def("mx4_select", [](int NQ, uptr T, uptr margin4, uptr margin8, uptr probe_s, int n_cols,
                         float rate, uptr tail_cs, int tail_cap, float limit, uptr thr4, uptr nv,
                         uptr st, int ld, int tile_stride, int tail_ld, bool nv_zeroed, int stage,
                         float wa, float wb) {
    check(symb_mx4_select(NQ, P<const float>(T), P<const float>(margin4), P<const float>(margin8),
                          P<const float>(probe_s), n_cols, ld, tile_stride, rate,
                          P<const float>(tail_cs), tail_cap, tail_ld, limit, P<float>(thr4),
                          P<int>(nv), S(st), nv_zeroed ? 1 : 0, stage, wa, wb),
          "mx4_select");
  }, py::arg("NQ"), py::arg("T"), py::arg("margin4"), py::arg("margin8"), py::arg("probe_s"),
     py::arg("n_cols"), py::arg("rate"), py::arg("tail_cs"), py::arg("tail_cap"), py::arg("limit"),
     py::arg("thr4"), py::arg("nv"), py::arg("stream"), py::arg("ld") = 0,
     py::arg("tile_stride") = 1, py::arg("tail_ld") = 0, py::arg("nv_zeroed") = false,
     py::arg("stage") = 0, py::arg("wa") = 2.f, py::arg("wb") = 0.f);
  m.def("prune_qquant", [](uptr Q, int NQ, int dim, uptr bounds, uptr Q8, uptr sq, uptr margin,
                           uptr st, uptr zero, int zero_n) {
    check(symb_prune_qquant(P<void>(Q), NQ, dim, P<const float>(bounds), P<void>(Q8), P<float>(sq),
                            P<float>(margin), S(st), P<int>(zero), zero_n),
          "prune_qquant");
  }, py::arg("Q"), py::arg("NQ"), py::arg("dim"), py::arg("bounds"), py::arg("Q8"), py::arg("sq"),
     py::arg("margin"), py::arg("stream"), py::arg("zero") = 0, py::arg("zero_n") = 0);
  m.def("prune_route", [](int NQ, uptr pre_s, uptr tail_s, int k, float thr_margin, uptr sq,
                          uptr margin, uptr thr0, uptr cs_p, uptr ci_p, uptr cnt_p, int cap_p,
                          int tshift, int rows_per_blk, int n_rblk, float blk_limit, float limit,
                          int max_list, uptr T, uptr thr, uptr dense, uptr est, uptr blkmax,
                          uptr blk, uptr st, uptr tail_cs, uptr tail_ci, uptr tail_cnt,
                          int tail_cap, int tail_off, int tail_ld, bool zeroed) {
    check(symb_prune_route(NQ, P<const float>(pre_s), P<const float>(tail_s), k, thr_margin,
                           P<const float>(sq), P<const float>(margin), P<const float>(thr0),
                           P<const float>(cs_p), P<const int>(ci_p), P<const int>(cnt_p), cap_p,
                           tshift, rows_per_blk, n_rblk, blk_limit, limit, max_list, P<float>(T),
                           P<float>(thr), P<int>(dense), P<float>(est), P<int>(blkmax),
                           P<int>(blk), S(st), P<const float>(tail_cs), P<const int>(tail_ci),
                           P<const int>(tail_cnt), tail_cap, tail_off, tail_ld, zeroed ? 1 : 0),
          "prune_route");
  }, py::arg("NQ"), py::arg("pre_s"), py::arg("tail_s"), py::arg("k"), py::arg("thr_margin"),
     py::arg("sq"), py::arg("margin"), py::arg("thr0"), py::arg("cs_p"), py::arg("ci_p"),
     py::arg("cnt_p"), py::arg("cap_p"), py::arg("tshift"), py::arg("rows_per_blk"),
     py::arg("n_rblk"), py::arg("blk_limit"), py::arg("limit"), py::arg("max_list"), py::arg("T"),
     py::arg("thr"), py::arg("dense"), py::arg("est"), py::arg("blkmax"), py::arg("blk"),
     py::arg("stream"), py::arg("tail_cs") = 0, py::arg("tail_ci") = 0, py::arg("tail_cnt") = 0,
     py::arg("tail_cap") = 0, py::arg("tail_off") = 0, py::arg("tail_ld") = 0,
     py::arg("zeroed") = false);
  m.def("index_scan_i8_ablate", [](uptr X8, uptr sx, int n_valid, int alloc_rows,
                                   int rows_per_blk, int n_rblk, uptr Q8, int NQ, uptr thr,
                                   uptr cand_s, uptr cand_i, uptr cand_n, int cap, int xcd, uptr st,
                                   int abl) {
    check(symb_index_scan_i8_ablate(P<void>(X8), P<const float>(sx), n_valid, alloc_rows,
                                    rows_per_blk, n_rblk,
                                    P<void>(Q8), NQ, P<const float>(thr), P<float>(cand_s),
                                    P<int>(cand_i), P<int>(cand_n), cap, xcd, S(st), abl),
          "index_scan_i8_ablate");
  });
  m.def("rescore_bf16", [](uptr X, uptr Q, int NQ, int dim, uptr cand_i, uptr cand_n, int cap,
                           uptr cand_s, uptr st) {
    check(symb_rescore_bf16(P<void>(X), P<void>(Q), NQ, dim, P<const int>(cand_i),
                            P<const int>(cand_n), cap, P<float>(cand_s), S(st)),
          "rescore_bf16");
  });
  m.def("quant_rows_i8", [](uptr X, int n, int dim, uptr X8, uptr sx, uptr err, uptr xtn, uptr st,
                            uptr bounds) {
    check(symb_quant_rows_i8(P<void>(X), n, dim, P<void>(X8), P<float>(sx), P<float>(err),
                             P<float>(xtn), P<float>(bounds), S(st)),
          "quant_rows_i8");
  }, py::arg("X"), py::arg("n"), py::arg("dim"), py::arg("X8"), py::arg("sx"), py::arg("err"),
     py::arg("xtn"), py::arg("stream"), py::arg("bounds") = 0);
  m.def("prune_qprep", [](uptr Q, int NQ, int dim, uptr pre_s, uptr tail_s, int k, float margin,
                          uptr bounds, uptr Q8, uptr sq, uptr T, uptr thr, uptr st) {
    check(symb_prune_qprep(P<void>(Q), NQ, dim, P<float>(pre_s), P<float>(tail_s), k, margin,
                           P<float>(bounds), P<void>(Q8), P<float>(sq), P<float>(T), P<float>(thr),
                           S(st)),
          "prune_qprep");
  }, py::arg("Q"), py::arg("NQ"), py::arg("dim"), py::arg("pre_s"), py::arg("tail_s"),
     py::arg("k"), py::arg("thr_margin"), py::arg("bounds"), py::arg("Q8"), py::arg("sq"),
     py::arg("T"), py::arg("thr"), py::arg("stream"));
  m.def("mfma_f8f6f4_probe", [](uptr a, uptr b, uptr sa, uptr sb, uptr out, int fmt, uptr st) {
    check(symb_mfma_f8f6f4_probe(P<const int>(a), P<const int>(b), P<const int>(sa),
                                 P<const int>(sb), P<float>(out), fmt, S(st)),
          "mfma_f8f6f4_probe");
  });
  m.def("gemm_lt_config", [](int mode) { check(symb_gemm_lt_config(mode), "gemm_lt_config"); },
        py::arg("mode"));
  m.def("gemm_lt_plans", []() { return symb_gemm_lt_plans(); });
  m.def("mq_config", [](int aux) { check(symb_mq_config(aux), "mq_config"); }, py::arg("aux"));
  m.def("mq_queries_per_blk", [](int sets, int rsplit) { return symb_mq_queries_per_blk(sets, rsplit); },
        py::arg("sets") = 4, py::arg("rsplit") = 1);
  m.def("index_scan_mq", [](uptr X, int n_valid, int rows_per_blk, int n_rblk, uptr Q, int NQ,
                            uptr thr, uptr cand_s, uptr cand_i, uptr cand_n, int cap, int xcd,
                            uptr st, int sets, int tshift, int rsplit, uptr gate, uptr blist,
                            int list_tiles, bool zero_cnt, int dim) {
    check(symb_index_scan_mq(P<void>(X), n_valid, rows_per_blk, n_rblk, P<void>(Q), NQ,
                             P<const float>(thr), P<float>(cand_s), P<int>(cand_i), P<int>(cand_n),
                             cap, xcd, S(st), sets, tshift, rsplit, P<const int>(gate),
                             P<const int>(blist), list_tiles, zero_cnt ? 1 : 0, dim),
          "index_scan_mq");
  }, py::arg("X"), py::arg("n_valid"), py::arg("rows_per_blk"), py::arg("n_rblk"), py::arg("Q"),
     py::arg("NQ"), py::arg("thr"), py::arg("cand_s"), py::arg("cand_i"), py::arg("cand_n"),
     py::arg("cap"), py::arg("xcd"), py::arg("stream"), py::arg("sets") = 4,
     py::arg("tshift") = 0, py::arg("rsplit") = 1, py::arg("gate") = 0, py::arg("blist") = 0,
     py::arg("list_tiles") = 0, py::arg("zero_cnt") = true, py::arg("dim") = 384);
  m.def("mq_max_sets", [](int dim) { return symb_mq_max_sets(dim); }, py::arg("dim"));
  m.def("index_scan_mq_ablate", [](uptr X, int n_valid, int rows_per_blk, int n_rblk, uptr Q,
                                   int NQ, uptr thr, uptr cand_s, uptr cand_i, uptr cand_n,
                                   int cap, int xcd, uptr st, int abl, int sets, int rsplit) {
    check(symb_index_scan_mq_ablate(P<void>(X), n_valid, rows_per_blk, n_rblk, P<void>(Q), NQ,
                                    P<const float>(thr), P<float>(cand_s), P<int>(cand_i),
                                    P<int>(cand_n), cap, xcd, S(st), abl, sets, rsplit),
          "index_scan_mq_ablate");
  }, py::arg("X"), py::arg("n_valid"), py::arg("rows_per_blk"), py::arg("n_rblk"), py::arg("Q"),
     py::arg("NQ"), py::arg("thr"), py::arg("cand_s"), py::arg("cand_i"), py::arg("cand_n"),
     py::arg("cap"), py::arg("xcd"), py::arg("stream"), py::arg("abl"), py::arg("sets") = 4,
     py::arg("rsplit") = 1);
  m.def("prune_stats", [](uptr ovf, uptr cnt, int NQ, uptr dense, uptr blk, uptr tot, uptr st) {
    check(symb_prune_stats(P<const int>(ovf), P<const int>(cnt), NQ, P<const int>(dense),
                           P<const int>(blk), P<int>(tot), S(st)),
          "prune_stats");
  }, py::arg("ovf"), py::arg("cnt"), py::arg("NQ"), py::arg("dense"), py::arg("blk"),
     py::arg("tot"), py::arg("stream"));
  m.def("topk_select_counted", [](uptr cand_s, uptr cand_i, uptr cand_n, int cap, int NQ,
                                  int kmax, int k, uptr out_s, uptr out_i, uptr ovf, uptr st,
                                  uptr gate, bool reset_ovf, int ld, uptr kth_out,
                                  float kth_margin, uptr seg2_s, int seg2_cap, uptr seg2_out_s,
                                  uptr seg2_out_i) {
    check(symb_topk_select_counted(P<const float>(cand_s), P<const int>(cand_i),
                                   P<const int>(cand_n), cap, NQ, kmax, k, P<float>(out_s),
                                   P<int>(out_i), P<int>(ovf), S(st), P<const int>(gate),
                                   reset_ovf ? 1 : 0, ld, P<float>(kth_out), kth_margin,
                                   P<const float>(seg2_s), seg2_cap, P<float>(seg2_out_s),
                                   P<int>(seg2_out_i)),
          "topk_select_counted");
  }, py::arg("cand_s"), py::arg("cand_i"), py::arg("cand_n"), py::arg("cap"), py::arg("NQ"),
     py::arg("kmax"), py::arg("k"), py::arg("out_s"), py::arg("out_i"), py::arg("ovf"),
     py::arg("stream"), py::arg("gate") = 0, py::arg("reset_ovf") = true, py::arg("ld") = 0,
     py::arg("kth_out") = 0, py::arg("kth_margin") = 0.f, py::arg("seg2_s") = 0,
     py::arg("seg2_cap") = 0, py::arg("seg2_out_s") = 0, py::arg("seg2_out_i") = 0);
  m.def("index_scan_ablate", [](uptr X, int n_valid, int rows_per_blk, int n_rblk, uptr Q, int NQ,
                                uptr cs, uptr ci, uptr st, int abl, uptr thr) {
    check(symb_index_scan_ablate(P<void>(X), n_valid, rows_per_blk, n_rblk, P<void>(Q), NQ,
                                 P<float>(cs), P<int>(ci), S(st), abl, P<const float>(thr)),
          "index_scan_ablate");
  }, py::arg("X"), py::arg("n_valid"), py::arg("rows_per_blk"), py::arg("n_rblk"), py::arg("Q"),
     py::arg("NQ"), py::arg("cs"), py::arg("ci"), py::arg("stream"), py::arg("abl"),
     py::arg("thr") = 0);
  m.def("attention_config", [](int waves, int kvt, int xcd) {
    check(symb_attention_config(waves, kvt, xcd), "attention_config");
  }, py::arg("waves") = 8, py::arg("kvt") = 64, py::arg("xcd") = 2);
  m.def("gemm_config", [](int resln_bm, int tile, int group_m) {
    check(symb_gemm_config(resln_bm, tile, group_m), "gemm_config");
  }, py::arg("resln_bm") = 128, py::arg("tile") = 3, py::arg("group_m") = 8);
  m.def("gemm_skinny_config", [](int max_m, int fuse) {
    check(symb_gemm_skinny_config(max_m, fuse), "gemm_skinny_config");
  }, py::arg("max_m") = 64, py::arg("fuse") = 1);
  m.def("gemm_skinny_max_m", []() { return symb_gemm_skinny_max_m(); });
  m.def("gemm_skinny_nw8", [](int max_kg, int min_wgs) {
    check(symb_gemm_skinny_nw8(max_kg, min_wgs), "gemm_skinny_nw8");
  }, py::arg("max_kg"), py::arg("min_wgs") = 128);
  m.def("gemm_resln_config", [](int waves) { check(symb_gemm_resln_config(waves), "gemm_resln_config"); },
        py::arg("waves") = 16);
  m.def("mlp_fused", [](uptr X, uptr W1, uptr b1, uptr W2, uptr b2, uptr g, uptr b, float eps,
                        uptr C, int M, int H, int FF, uptr st) {
    check(symb_mlp_fused(P<void>(X), P<void>(W1), P<float>(b1), P<void>(W2), P<float>(b2),
                         P<float>(g), P<float>(b), eps, symb_gemm_gelu_poly(), P<void>(C), M, H, FF,
                         S(st)),
          "mlp_fused");
  });
  m.def("mlp_fused_config", [](int mode) {   // 0: two GEMMs, 1: the fused FFN block (default)
    if (mode < 0 || mode > 1) throw std::invalid_argument("mlp_fused_config: mode 0 or 1");
    g_mlp_fused = mode;
  });
  m.def("gemm_gelu_config", [](int poly) { check(symb_gemm_gelu_config(poly), "gemm_gelu_config"); },
        py::arg("poly"));
  m.def("gemm_fp8_config", [](int waves, int big) {
    check(symb_gemm_fp8_config(waves, big), "gemm_fp8_config");
  }, py::arg("waves") = 8, py::arg("big") = 2);
  m.def("gemm_fp8", [](int epi, uptr A8, int lda, uptr W8, int ldw, uptr sa, uptr sw, uptr bias,
                       uptr R, int ldr, uptr C, int ldc, int M, int N, int K, uptr st,
                       uptr ascale, uptr cscale) {
    check(symb_gemm_fp8(epi, P<void>(A8), lda, P<void>(W8), ldw, P<float>(sa), P<float>(sw),
                        P<float>(bias), P<void>(R), ldr, P<void>(C), ldc, M, N, K, S(st),
                        P<void>(ascale), P<void>(cscale)),
          "gemm_fp8");
  }, py::arg("epi"), py::arg("A8"), py::arg("lda"), py::arg("W8"), py::arg("ldw"), py::arg("sa"),
     py::arg("sw"), py::arg("bias"), py::arg("R"), py::arg("ldr"), py::arg("C"), py::arg("ldc"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("st"), py::arg("ascale") = 0,
     py::arg("cscale") = 0);
  m.def("quant_rows_fp8", [](uptr x, int ldx, uptr out, int ldo, uptr scale, int M, int K, uptr st) {
    check(symb_quant_rows_fp8(P<void>(x), ldx, P<void>(out), ldo, P<float>(scale), M, K, S(st)),
          "quant_rows_fp8");
  });
  m.def("quant_fp8", [](uptr in, bool in_f32, int ld_in, uptr out, int ld_out, int n, int D,
                        float scale, bool normalize, uptr st) {
    check(symb_quant_fp8(P<void>(in), in_f32, ld_in, P<uint8_t>(out), ld_out, n, D, scale,
                         normalize, S(st)),
          "quant_fp8");
  });
  m.def("index_scan_fp8", [](uptr X, int n_valid, int D, int rows_per_blk, int n_rblk, uptr Q,
                             int NQ, int kmax, uptr cand_s, uptr cand_i, uptr st, int aux, uptr thr,
                             int variant, int xcd) {
    check(symb_index_scan_fp8(P<void>(X), n_valid, D, rows_per_blk, n_rblk, P<void>(Q), NQ, kmax,
                              P<float>(cand_s), P<int>(cand_i), S(st), aux, P<const float>(thr),
                              variant, xcd),
          "index_scan_fp8");
  }, py::arg("X"), py::arg("n_valid"), py::arg("D"), py::arg("rows_per_blk"), py::arg("n_rblk"),
     py::arg("Q"), py::arg("NQ"), py::arg("kmax"), py::arg("cand_s"), py::arg("cand_i"),
     py::arg("stream"), py::arg("aux") = -1, py::arg("thr_init") = 0, py::arg("variant") = 0,
     py::arg("xcd") = 1);
  m.def("topk_merge", [](uptr cand_s, uptr cand_i, int NQ, int n_cand, int kmax, int k,
                         uptr out_s, uptr out_i, int64_t id_offset, uptr out_id64, uptr st,
                         uptr gate) {
    check(symb_topk_merge(P<float>(cand_s), P<int>(cand_i), NQ, n_cand, kmax, k, P<float>(out_s),
                          P<int>(out_i), id_offset, P<int64_t>(out_id64), S(st),
                          P<const int>(gate)),
          "topk_merge");
  }, py::arg("cand_s"), py::arg("cand_i"), py::arg("NQ"), py::arg("n_cand"), py::arg("kmax"),
     py::arg("k"), py::arg("out_s"), py::arg("out_i"), py::arg("id_offset"), py::arg("out_id64"),
     py::arg("stream"), py::arg("gate") = 0);
  py::class_<EncoderRuntime>(m, "EncoderRuntime")
      .def(py::init<int, int, int, float, uptr, uptr, uptr, uptr, uptr>())
      .def("add_layer", &EncoderRuntime::add_layer)
      .def("add_layer_fp8", &EncoderRuntime::add_layer_fp8)
      .def("num_layers", &EncoderRuntime::num_layers)
      .def("skinny_ws_bytes", &EncoderRuntime::skinny_ws_bytes)
      .def("set_fold", &EncoderRuntime::set_fold)
      .def("set_deferred_ln", &EncoderRuntime::set_deferred_ln)
      .def("deferred_ln_ready", &EncoderRuntime::deferred_ln_ready)
      .def("forward", &EncoderRuntime::forward);
}
