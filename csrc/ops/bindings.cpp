// Python bindings for the CDNA4 kernels in csrc/ops/*.hip.
// Every entry point validates shapes/dtypes/devices on the host (so a bad call
// fails loudly instead of faulting the GPU) and launches on the caller's
// current HIP stream, which keeps them hipGraph-capturable.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

extern "C" {
int pa_rmsnorm(void* out, const void* x, const void* w, int T, int D, float eps, hipStream_t st);
int pa_fused_add_rmsnorm(void* out, void* resid, const void* x, const void* w, int T, int D,
                         float eps, hipStream_t st);
int pa_rope_cache(void* q_out, void* k_cache, void* v_cache, const void* qkv, const int* positions,
                  const int* slot_mapping, const float* cos_sin, int T, int H, int KV, int ld,
                  int block_size, int apply_rope, hipStream_t st);
int pa_silu_mul(void* out, const void* in, int T, int F, hipStream_t st);
int pa_paged_attention(void* out, float* part_o, float* part_ml, const void* q, const void* k_cache,
                       const void* v_cache, const int* items, const int* n_items, int max_items,
                       const int* part_size, int* counters, const int* q_start,
                       const int* q_len, const int* ctx_len, const int* block_table,
                       int max_blocks, int H, int KV, float scale_log2, int waves, int* pf_counters,
                       hipStream_t st);
int pa_sample_workspace_floats(int rows, int V);
int pa_patch_pending_ids(int* ids, const int* sampled, int T, int n_sampled, hipStream_t st);
int pa_sample(int* out_tokens, float* out_keys, float* workspace, const void* logits, int rows,
              int V, int ld, int vocab_offset, const float* temperature, const int* mask_class,
              const uint32_t* class_masks, int mask_words, const int64_t* seeds,
              const int* offsets, const int* forced, const float* tau, hipStream_t st);
int pa_tp_topkp_phase(int phase, float* tau, float* ws, const void* logits, int rows, int v_local, int ld,
                      int vocab_offset, int V, const float* temperature, const int* top_k, const float* top_p,
                      const int* mask_class, const uint32_t* class_masks, int mask_words, hipStream_t st);
int pa_topkp_threshold(float* tau, const void* logits, int rows, int V, int ld, int shards,
                       long long shard_stride, const float* temperature, const int* top_k,
                       const float* top_p, const int* mask_class, const uint32_t* class_masks,
                       int mask_words, hipStream_t st);
void pa_skinny_set_variant(int v);
int pa_skinny_gemm(void* y, const void* x, const void* w, int M, int N, int K, int ldy, hipStream_t st);
void pa_decode_set_variant(int v);
void pa_handoff_set_acquire(int v);
void pa_handoff_set_modes(int gemm, int attn);
int pa_decode_gemm(void* y, const void* x, const void* wp, const void* resid, int M, int N, int K,
                   int ldx, int ldy, int ldr, int epi, int norm, float eps, int nt, int waves, int splits,
                   float* ws, long long ws_floats, int* counters, int n_counters, hipStream_t st);
int pa_decode_qkv_rope(const void* x, const void* wp, int M, int N, int K, int ldx, float eps, void* q_out,
                       void* k_cache, void* v_cache, const int* positions, const int* slots,
                       const float* cos_sin, int H, int KV, int nt, int waves, int splits, float* ws,
                       long long ws_floats, int* counters, int n_counters, hipStream_t st);
int pa_mid_gemm_plan(int M, int N, int K, int epi, int* fm, int* fn, int* S);
long long pa_mid_gemm_ws_floats(int M, int N, int K, int fm, int fn, int S);
int pa_mid_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws, long long ws_floats,
                int* counters, int n_counters, int M, int N, int K, int ldx, int ldy, int ldr, int epi,
                const float* ss_in, float* ss_out, float* ss_zero, float eps, int fm, int fn, int splits,
                void* q_out, void* k_cache, void* v_cache, const int* positions, const int* slots,
                const float* cos_sin, int H, int KV, hipStream_t st);
int pa_row_sumsq(float* out, const void* x, int M, int K, int ldx, hipStream_t st);
int pa_timeline_marker(int id, hipStream_t st);
int pa_store_test(void* dst, long long n16, int mode, int grid, hipStream_t st);
long long pa_stream_gemm_ws_floats(int M, int N, int K, int mg, int rg, int tpw, int wt, int wk, int S);
void pa_stream_gemm_plan(int M, int N, int K, int epi, int* plan);
int pa_stream_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws, long long ws_floats,
                   int* counters, int n_counters, int* err, int M, int N, int K, int ldx, int ldy, int ldr, int epi,
                   const float* ss_in, float* ss_out, float* ss_zero, float eps, const int* plan, void* q_out,
                   void* k_cache, void* v_cache, const int* positions, const int* slots, const float* cos_sin, int H,
                   int KV, int rel, unsigned long long* stamps, hipStream_t st);
void pa_prefill_gemm_plan(int M, int N, int K, int bn, int* full, int* S);
int pa_prefill_pick_bn(int M, int N);
void pa_prefill_set_variant(int v);
long long pa_prefill_gemm_ws_floats(int M, int N, int bn, int full, int S);
int pa_prefill_gemm(void* y, const void* x, const void* wp, const void* resid, float* ws, long long ws_floats,
                    int* counters, int n_counters, int M, int N, int K, int ldx, int ldy, int ldr, int epi,
                    const float* ss_in, float* ss_out, float* ss_zero, float eps, int full, int splits, int bn,
                    void* q_out, void* k_cache, void* v_cache, const int* positions, const int* slots,
                    const float* cos_sin, int H, int KV, int kernel_variant, hipStream_t st);
long long pa_cosine_topk_workspace_bytes(int Q, int N, int K);
int pa_cosine_topk(float* out_scores, int* out_rows, void* workspace, const void* queries,
                   const void* index, int Q, int N, int D, int K, const int* row_priority,
                   const uint64_t* row_tags, const float* row_expiry, const int* q_min_priority,
                   const uint64_t* q_tags, float now, int n_valid, hipStream_t st);
long long pa_q16_topk_workspace_bytes(int Q, int N);
int pa_q16_topk(float* out_scores, int* out_rows, int* unsafe, void* workspace, const void* queries_q,
                const float* qmeta, const void* hi, const void* lo, const float* rmeta, int Q, int N, int D, int K,
                const int* row_priority, const uint64_t* row_tags, const float* row_expiry,
                const int* q_min_priority, const uint64_t* q_tags, float now, int exact, hipStream_t st);
int pa_car_group();
long long pa_car_flag_bytes();
void* pa_car_alloc(long long bytes, void* handle_out);
void* pa_car_open(const void* handle);
int pa_car_close(void* p);
int pa_car_free(void* p);
int pa_car_collective(void* const* bases, int W, int rank0, int nranks_local, const void* const* ins,
                      void* const* outs, long long n4, long long cap_bytes, uint32_t* epochs, int* err, int op,
                      hipStream_t st);
int pa_car_all_reduce(void* const* bases, int W, int rank0, int nranks_local, const void* const* ins,
                      void* const* outs, long long nelem, long long cap_bytes, uint32_t* epochs, int* err,
                      int two_shot, const void* const* resids, float* const* ss, float* const* ss_zero,
                      int row_len, hipStream_t st);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_dtype(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " launch failed with code ", rc, " (",
              rc > 0 ? hipGetErrorString((hipError_t)rc) : "bad arguments", ")");
}

void rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, double eps) {
  check_gpu(out, "out"); check_gpu(x, "x"); check_gpu(w, "w");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(out, at::kBFloat16, "out");
  check_dtype(w, at::kBFloat16, "w");
  const int D = x.size(-1);
  const int T = x.numel() / D;
  TORCH_CHECK(w.numel() == D && out.numel() == x.numel(), "rmsnorm shape mismatch");
  check_rc(pa_rmsnorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), T, D, (float)eps, cur_stream()),
           "rmsnorm");
}

void fused_add_rmsnorm(at::Tensor out, at::Tensor resid, at::Tensor x, at::Tensor w, double eps) {
  check_gpu(out, "out"); check_gpu(resid, "resid"); check_gpu(x, "x"); check_gpu(w, "w");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(resid, at::kBFloat16, "resid");
  check_dtype(out, at::kBFloat16, "out"); check_dtype(w, at::kBFloat16, "w");
  const int D = x.size(-1);
  const int T = x.numel() / D;
  TORCH_CHECK(w.numel() == D && out.numel() == x.numel() && resid.numel() == x.numel(),
              "fused_add_rmsnorm shape mismatch");
  check_rc(pa_fused_add_rmsnorm(out.data_ptr(), resid.data_ptr(), x.data_ptr(), w.data_ptr(), T,
                                D, (float)eps, cur_stream()),
           "fused_add_rmsnorm");
}

void rope_cache(at::Tensor q_out, at::Tensor k_cache, at::Tensor v_cache, at::Tensor qkv,
                at::Tensor positions, at::Tensor slot_mapping, at::Tensor cos_sin, int64_t H,
                int64_t KV, bool apply_rope) {
  check_gpu(q_out, "q_out"); check_gpu(k_cache, "k_cache"); check_gpu(v_cache, "v_cache");
  check_gpu(positions, "positions"); check_gpu(slot_mapping, "slot_mapping");
  check_gpu(cos_sin, "cos_sin");
  TORCH_CHECK(qkv.is_cuda() && qkv.stride(-1) == 1, "qkv must be a GPU tensor with unit inner stride");
  check_dtype(qkv, at::kBFloat16, "qkv"); check_dtype(q_out, at::kBFloat16, "q_out");
  check_dtype(k_cache, at::kBFloat16, "k_cache"); check_dtype(v_cache, at::kBFloat16, "v_cache");
  check_dtype(positions, at::kInt, "positions"); check_dtype(slot_mapping, at::kInt, "slot_mapping");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  const int T = qkv.size(0);
  TORCH_CHECK(qkv.size(1) >= (H + 2 * KV) * 128, "qkv too narrow");
  TORCH_CHECK(positions.numel() >= T && slot_mapping.numel() >= T, "positions/slots too short");
  TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(1) == KV && k_cache.size(2) == 16 && k_cache.size(4) == 8,
              "k_cache must be [blocks, KV, 16, block, 8]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == KV && v_cache.size(2) == 128,
              "v_cache must be [blocks, KV, 128, block]");
  TORCH_CHECK(cos_sin.size(1) == 128, "cos_sin must be [max_pos, 128]");
  const int block = k_cache.size(3);
  check_rc(pa_rope_cache(q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), qkv.data_ptr(),
                         positions.data_ptr<int>(), slot_mapping.data_ptr<int>(),
                         cos_sin.data_ptr<float>(), T, H, KV, qkv.stride(0), block,
                         apply_rope ? 1 : 0, cur_stream()),
           "rope_cache");
}

void silu_mul(at::Tensor out, at::Tensor in) {
  check_gpu(out, "out"); check_gpu(in, "in");
  check_dtype(out, at::kBFloat16, "out"); check_dtype(in, at::kBFloat16, "in");
  const int F = out.size(-1);
  const int T = out.numel() / F;
  TORCH_CHECK(in.size(-1) == 2 * F && in.numel() == 2 * out.numel(), "silu_mul shape mismatch");
  check_rc(pa_silu_mul(out.data_ptr(), in.data_ptr(), T, F, cur_stream()), "silu_mul");
}

void paged_attention(at::Tensor out, at::Tensor part_o, at::Tensor part_ml, at::Tensor q,
                     at::Tensor k_cache, at::Tensor v_cache, at::Tensor items, at::Tensor n_items,
                     at::Tensor counters, at::Tensor q_start, at::Tensor q_len,
                     at::Tensor ctx_len, at::Tensor block_table, double scale,
                     c10::optional<at::Tensor> part_size, int64_t waves) {
  for (auto* t : {&out, &part_o, &part_ml, &q, &k_cache, &v_cache, &items, &n_items, &counters,
                  &q_start, &q_len, &ctx_len, &block_table})
    check_gpu(*t, "paged_attention arg");
  check_dtype(q, at::kBFloat16, "q"); check_dtype(out, at::kBFloat16, "out");
  check_dtype(k_cache, at::kBFloat16, "k_cache"); check_dtype(v_cache, at::kBFloat16, "v_cache");
  check_dtype(part_o, at::kFloat, "part_o"); check_dtype(part_ml, at::kFloat, "part_ml");
  for (auto* t : {&items, &n_items, &counters, &q_start, &q_len, &ctx_len, &block_table})
    check_dtype(*t, at::kInt, "paged_attention int arg");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [T, H, 128]");
  TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(2) == 16 && k_cache.size(3) == 16 && k_cache.size(4) == 8,
              "k_cache must be [blocks, KV, 16, 16, 8]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(2) == 128 && v_cache.size(3) == 16,
              "v_cache must be [blocks, KV, 128, 16]");
  const int H = q.size(1), KV = k_cache.size(1);
  TORCH_CHECK(items.dim() == 2 && items.size(1) == 4, "items must be [max_items, 4]");
  TORCH_CHECK(block_table.dim() == 2, "block_table must be [seqs, max_blocks]");
  const int max_items = items.size(0);
  TORCH_CHECK(part_o.numel() >= (int64_t)max_items * KV * 16 * 128, "part_o workspace too small");
  TORCH_CHECK(part_ml.numel() >= (int64_t)max_items * KV * 16 * 2, "part_ml workspace too small");
  TORCH_CHECK(counters.numel() >= block_table.size(0) * KV,
              "counters must hold one zero-initialised int per (sequence, KV head)");
  // split prefill items (attention.hip prefill_item_wg) take their tickets after the per-sequence
  // counters: one per (partial slot, KV head); without that room a split item computes its whole
  // key range (correct, only slower)
  int* pf_counters = counters.numel() >= (block_table.size(0) + (int64_t)max_items) * KV
                         ? counters.data_ptr<int>() + block_table.size(0) * KV
                         : nullptr;
  const float scale_log2 = (float)(scale * 1.4426950408889634);
  check_rc(pa_paged_attention(out.data_ptr(), part_o.data_ptr<float>(), part_ml.data_ptr<float>(),
                              q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                              items.data_ptr<int>(), n_items.data_ptr<int>(), max_items,
                              part_size.has_value() ? part_size->data_ptr<int>() : nullptr,
                              counters.data_ptr<int>(),
                              q_start.data_ptr<int>(), q_len.data_ptr<int>(),
                              ctx_len.data_ptr<int>(), block_table.data_ptr<int>(),
                              block_table.size(1), H, KV, scale_log2, (int)waves, pf_counters, cur_stream()),
           "paged_attention");
}

// y[M, N] = x[M, K] . w[N, K]^T for M <= 128; returns false if the shape is not handled.
bool skinny_gemm(at::Tensor y, at::Tensor x, at::Tensor w) {
  check_gpu(x, "x"); check_gpu(w, "w");
  TORCH_CHECK(y.is_cuda() && y.stride(-1) == 1, "y must be a GPU tensor with unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(w, at::kBFloat16, "w"); check_dtype(y, at::kBFloat16, "y");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "skinny_gemm expects 2-D tensors");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && y.size(0) == M && y.size(1) == N, "skinny_gemm shape mismatch");
  const int rc = pa_skinny_gemm(y.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K, y.stride(0), cur_stream());
  TORCH_CHECK(rc >= 0, "skinny_gemm launch failed");
  return rc == 0;
}

// y = epi(rownorm(x) . W^T) on fragment-major packed weights wp [N/16, K/32, 64, 8]
// (csrc/ops/gemm_decode.hip). epi 0 plain, 1 silu(gate)*up (y has N/2 columns),
// 2 y = resid + acc. Returns false if the shape is not handled.
bool decode_gemm(at::Tensor y, at::Tensor x, at::Tensor wp, c10::optional<at::Tensor> resid, int64_t epi,
                 bool norm, double eps, int64_t nt, int64_t waves, int64_t splits, c10::optional<at::Tensor> ws,
                 c10::optional<at::Tensor> counters) {
  check_gpu(wp, "wp");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1, "y must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp"); check_dtype(y, at::kBFloat16, "y");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K ", wp.size(1) * 32, " != x K ", K);
  TORCH_CHECK(x.stride(0) % 8 == 0 && K % 8 == 0, "x rows must be 16-byte aligned");
  const int NO = epi == 1 ? N / 2 : N;
  TORCH_CHECK(y.size(0) == M && y.size(1) == NO, "y shape [", y.size(0), ", ", y.size(1), "] != [", M, ", ", NO, "]");
  const void* rp = nullptr;
  int ldr = 0;
  if (epi == 2) {
    TORCH_CHECK(resid.has_value(), "epi=2 needs resid");
    const auto& r = *resid;
    TORCH_CHECK(r.is_cuda() && r.dim() == 2 && r.stride(1) == 1 && r.size(0) == M && r.size(1) == N,
                "resid must be [M, N] with unit inner stride");
    check_dtype(r, at::kBFloat16, "resid");
    rp = r.data_ptr();
    ldr = r.stride(0);
  }
  float* wsp = nullptr;
  long long wsn = 0;
  int* cp = nullptr;
  int cn = 0;
  if (ws.has_value() && counters.has_value()) {
    check_gpu(*ws, "ws"); check_gpu(*counters, "counters");
    check_dtype(*ws, at::kFloat, "ws"); check_dtype(*counters, at::kInt, "counters");
    wsp = ws->data_ptr<float>(); wsn = ws->numel(); cp = counters->data_ptr<int>(); cn = counters->numel();
  }
  const int rc = pa_decode_gemm(y.data_ptr(), x.data_ptr(), wp.data_ptr(), rp, M, N, K, x.stride(0), y.stride(0),
                                ldr, (int)epi, norm ? 1 : 0, (float)eps, (int)nt, (int)waves, (int)splits, wsp, wsn,
                                cp, cn, cur_stream());
  TORCH_CHECK(rc >= 0, "decode_gemm launch failed");
  return rc == 0;
}

// Decode QKV projection + RoPE + paged KV write (csrc/ops/gemm_decode.hip, EPI_ROPE).
void decode_qkv_rope(at::Tensor x, at::Tensor wp, double eps, at::Tensor q_out, at::Tensor k_cache,
                     at::Tensor v_cache, at::Tensor positions, at::Tensor slots, at::Tensor cos_sin, int64_t H,
                     int64_t KV, int64_t splits, c10::optional<at::Tensor> ws, c10::optional<at::Tensor> counters) {
  check_gpu(wp, "wp"); check_gpu(q_out, "q_out"); check_gpu(k_cache, "k_cache"); check_gpu(v_cache, "v_cache");
  check_gpu(positions, "positions"); check_gpu(slots, "slots"); check_gpu(cos_sin, "cos_sin");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp"); check_dtype(q_out, at::kBFloat16, "q_out");
  check_dtype(k_cache, at::kBFloat16, "k_cache"); check_dtype(v_cache, at::kBFloat16, "v_cache");
  check_dtype(positions, at::kInt, "positions"); check_dtype(slots, at::kInt, "slots");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K mismatch");
  TORCH_CHECK(N == (H + 2 * KV) * 128, "packed QKV has ", N, " columns, expected (H + 2 KV) * 128");
  TORCH_CHECK(q_out.numel() >= (int64_t)M * H * 128, "q_out too small");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M, "positions/slots shorter than x");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == 128, "cos_sin must be [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(1) == KV && k_cache.size(2) == 16 && k_cache.size(3) == 16 &&
                  k_cache.size(4) == 8, "k_cache must be [NB, KV, 16, 16, 8]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == KV && v_cache.size(2) == 128 && v_cache.size(3) == 16,
              "v_cache must be [NB, KV, 128, 16]");
  float* wsp = nullptr;
  long long wsn = 0;
  int* cp = nullptr;
  int cn = 0;
  if (ws.has_value() && counters.has_value()) {
    check_gpu(*ws, "ws"); check_gpu(*counters, "counters");
    check_dtype(*ws, at::kFloat, "ws"); check_dtype(*counters, at::kInt, "counters");
    wsp = ws->data_ptr<float>(); wsn = ws->numel(); cp = counters->data_ptr<int>(); cn = counters->numel();
  }
  const int rc = pa_decode_qkv_rope(x.data_ptr(), wp.data_ptr(), M, N, K, x.stride(0), (float)eps, q_out.data_ptr(),
                                    k_cache.data_ptr(), v_cache.data_ptr(), positions.data_ptr<int>(),
                                    slots.data_ptr<int>(), cos_sin.data_ptr<float>(), (int)H, (int)KV, 0, 0,
                                    (int)splits, wsp, wsn, cp, cn, cur_stream());
  check_rc(rc < 0 ? rc : (rc > 0 ? -1 : 0), "decode_qkv_rope");
}

const float* opt_rows(const c10::optional<at::Tensor>& t, int M, const char* name) {
  if (!t.has_value()) return nullptr;
  check_gpu(*t, name);
  check_dtype(*t, at::kFloat, name);
  TORCH_CHECK(t->numel() >= M, name, " must hold >= M floats");
  return t->data_ptr<float>();
}

// y = epi(rowscale(x) . W^T) for mid-size token counts on packed weights (csrc/ops/gemm_mid.hip).
// epi 0 plain, 1 silu(gate)*up (y has N/2 columns), 2 resid + acc, 3 plain with the RoPE tile
// permutation undone. ss_in: [M] fp32 row sums of x^2 -> rows scaled by rsqrt(ss/K + eps) (the
// RMSNorm weight folded into W). ss_out (epi 2): [M] += row sums of y^2. ss_zero: [M] zeroed.
// Returns false if the shape/config is not handled.
bool mid_gemm(at::Tensor y, at::Tensor x, at::Tensor wp, c10::optional<at::Tensor> resid, at::Tensor ws,
              at::Tensor counters, int64_t epi, c10::optional<at::Tensor> ss_in, c10::optional<at::Tensor> ss_out,
              c10::optional<at::Tensor> ss_zero, double eps, int64_t fm, int64_t fn, int64_t splits) {
  check_gpu(wp, "wp"); check_gpu(ws, "ws"); check_gpu(counters, "counters");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1, "y must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp"); check_dtype(y, at::kBFloat16, "y");
  check_dtype(ws, at::kFloat, "ws"); check_dtype(counters, at::kInt, "counters");
  TORCH_CHECK(epi >= 0 && epi <= 3, "mid_gemm epi must be 0..3 (RoPE + KV write: mid_qkv_rope)");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0 && y.stride(0) % 4 == 0, "x rows must be 16-byte, y rows 8-byte aligned");
  // the non-pair epilogues (plain, residual) of the ping-pong kernels store -- and read the
  // residual -- 16 B per lane (packed_epi.h store_pair_wide): y and resid rows 16-byte aligned
  const bool wide = epi == 0 || epi == 2;
  auto rows16 = [](const at::Tensor& t) { return t.stride(0) % 8 == 0 && ((uintptr_t)t.data_ptr() & 15) == 0; };
  TORCH_CHECK(!wide || rows16(y), "y rows must be 16-byte aligned for the plain / residual epilogue");
  TORCH_CHECK(((uintptr_t)y.data_ptr() & 7) == 0, "y must be 8-byte aligned");
  const int NO = epi == 1 ? N / 2 : N;
  TORCH_CHECK(y.size(0) == M && y.size(1) == NO, "y shape mismatch");
  const void* rp = nullptr;
  int ldr = 0;
  if (epi == 2) {
    TORCH_CHECK(resid.has_value(), "epi=2 needs resid");
    const auto& r = *resid;
    TORCH_CHECK(r.is_cuda() && r.dim() == 2 && r.stride(1) == 1 && r.size(0) == M && r.size(1) == N && rows16(r),
                "resid must be [M, N] with unit inner stride and 16-byte aligned rows");
    check_dtype(r, at::kBFloat16, "resid");
    rp = r.data_ptr();
    ldr = r.stride(0);
  }
  const int rc = pa_mid_gemm(y.data_ptr(), x.data_ptr(), wp.data_ptr(), rp, ws.data_ptr<float>(), ws.numel(),
                             counters.data_ptr<int>(), counters.numel(), M, N, K, x.stride(0), y.stride(0), ldr,
                             (int)epi, opt_rows(ss_in, M, "ss_in"), const_cast<float*>(opt_rows(ss_out, M, "ss_out")),
                             const_cast<float*>(opt_rows(ss_zero, M, "ss_zero")), (float)eps, (int)fm, (int)fn,
                             (int)splits, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, cur_stream());
  TORCH_CHECK(rc >= 0, "mid_gemm launch failed");
  return rc == 0;
}

// Mid-size QKV projection (RMSNorm folded into the rope-packed weights, row statistics
// ss_in) with RoPE and the paged KV write in the epilogue (csrc/ops/gemm_mid.hip, EP_ROPEKV).
bool mid_qkv_rope(at::Tensor x, at::Tensor wp, at::Tensor ss_in, double eps, at::Tensor q_out, at::Tensor k_cache,
                  at::Tensor v_cache, at::Tensor positions, at::Tensor slots, at::Tensor cos_sin, int64_t H,
                  int64_t KV, at::Tensor ws, at::Tensor counters, int64_t fm, int64_t fn, int64_t splits) {
  check_gpu(wp, "wp"); check_gpu(q_out, "q_out"); check_gpu(k_cache, "k_cache"); check_gpu(v_cache, "v_cache");
  check_gpu(positions, "positions"); check_gpu(slots, "slots"); check_gpu(cos_sin, "cos_sin");
  check_gpu(ws, "ws"); check_gpu(counters, "counters");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp"); check_dtype(q_out, at::kBFloat16, "q_out");
  check_dtype(k_cache, at::kBFloat16, "k_cache"); check_dtype(v_cache, at::kBFloat16, "v_cache");
  check_dtype(positions, at::kInt, "positions"); check_dtype(slots, at::kInt, "slots");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  check_dtype(ws, at::kFloat, "ws"); check_dtype(counters, at::kInt, "counters");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0, "x rows must be 16-byte aligned");
  TORCH_CHECK(N == (H + 2 * KV) * 128, "packed QKV has ", N, " columns, expected (H + 2 KV) * 128");
  TORCH_CHECK(q_out.numel() >= (int64_t)M * H * 128, "q_out too small");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M, "positions/slots shorter than x");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == 128, "cos_sin must be [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(1) == KV && k_cache.size(2) == 16 && k_cache.size(3) == 16 &&
                  k_cache.size(4) == 8, "k_cache must be [NB, KV, 16, 16, 8]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == KV && v_cache.size(2) == 128 && v_cache.size(3) == 16,
              "v_cache must be [NB, KV, 128, 16]");
  const float* ssp = opt_rows(c10::optional<at::Tensor>(ss_in), M, "ss_in");
  const int rc = pa_mid_gemm(nullptr, x.data_ptr(), wp.data_ptr(), nullptr, ws.data_ptr<float>(), ws.numel(),
                             counters.data_ptr<int>(), counters.numel(), M, N, K, x.stride(0), 0, 0, 4, ssp, nullptr,
                             nullptr, (float)eps, (int)fm, (int)fn, (int)splits, q_out.data_ptr(), k_cache.data_ptr(),
                             v_cache.data_ptr(), positions.data_ptr<int>(), slots.data_ptr<int>(),
                             cos_sin.data_ptr<float>(), (int)H, (int)KV, cur_stream());
  TORCH_CHECK(rc >= 0, "mid_qkv_rope launch failed");
  return rc == 0;
}

// Weight-streaming projections for 16 < M <= 256 (csrc/ops/gemm_stream.hip): every epilogue
// (0 plain, 1 SwiGLU, 2 residual, 3 rope-perm, 4 RoPE + paged KV write). plan: 7 ints
// (mg, rg, tpw, wt, wk, S, D) or empty for the default decomposition.
bool stream_gemm(c10::optional<at::Tensor> y, at::Tensor x, at::Tensor wp, c10::optional<at::Tensor> resid,
                 at::Tensor ws, at::Tensor counters, at::Tensor err, int64_t epi, c10::optional<at::Tensor> ss_in,
                 c10::optional<at::Tensor> ss_out, c10::optional<at::Tensor> ss_zero, double eps,
                 std::vector<int64_t> plan, c10::optional<at::Tensor> q_out, c10::optional<at::Tensor> k_cache,
                 c10::optional<at::Tensor> v_cache, c10::optional<at::Tensor> positions,
                 c10::optional<at::Tensor> slots, c10::optional<at::Tensor> cos_sin, int64_t H, int64_t KV,
                 int64_t rel, c10::optional<at::Tensor> stamps) {
  check_gpu(wp, "wp"); check_gpu(ws, "ws"); check_gpu(counters, "counters"); check_gpu(err, "err");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp");
  check_dtype(ws, at::kFloat, "ws"); check_dtype(counters, at::kInt, "counters"); check_dtype(err, at::kInt, "err");
  TORCH_CHECK(epi >= 0 && epi <= 4, "stream_gemm epi must be 0..4");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0 && ((uintptr_t)x.data_ptr() & 15) == 0, "x rows must be 16-byte aligned");
  void* yp = nullptr;
  int ldy = 0;
  if (epi != 4) {
    TORCH_CHECK(y.has_value(), "stream_gemm needs y for epi ", epi);
    const auto& t = *y;
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1, "y must be a 2-D GPU tensor, unit inner stride");
    check_dtype(t, at::kBFloat16, "y");
    const int NO = epi == 1 ? N / 2 : N;
    TORCH_CHECK(t.size(0) == M && t.size(1) == NO, "y shape mismatch");
    TORCH_CHECK(t.stride(0) % 4 == 0 && ((uintptr_t)t.data_ptr() & 7) == 0, "y rows must be 8-byte aligned");
    yp = t.data_ptr();
    ldy = t.stride(0);
  }
  const void* rp = nullptr;
  int ldr = 0;
  if (epi == 2) {
    TORCH_CHECK(resid.has_value(), "epi=2 needs resid");
    const auto& r = *resid;
    TORCH_CHECK(r.is_cuda() && r.dim() == 2 && r.stride(1) == 1 && r.size(0) == M && r.size(1) == N &&
                    r.stride(0) % 4 == 0 && ((uintptr_t)r.data_ptr() & 7) == 0,
                "resid must be [M, N] with unit inner stride, 8-byte aligned rows");
    check_dtype(r, at::kBFloat16, "resid");
    rp = r.data_ptr();
    ldr = r.stride(0);
  }
  void *qp = nullptr, *kp = nullptr, *vp = nullptr;
  const int *pp = nullptr, *sp = nullptr;
  const float* cp = nullptr;
  if (epi == 4) {
    TORCH_CHECK(q_out && k_cache && v_cache && positions && slots && cos_sin, "epi=4 needs the RoPE / cache tensors");
    check_gpu(*q_out, "q_out"); check_gpu(*k_cache, "k_cache"); check_gpu(*v_cache, "v_cache");
    check_gpu(*positions, "positions"); check_gpu(*slots, "slots"); check_gpu(*cos_sin, "cos_sin");
    check_dtype(*q_out, at::kBFloat16, "q_out"); check_dtype(*k_cache, at::kBFloat16, "k_cache");
    check_dtype(*v_cache, at::kBFloat16, "v_cache"); check_dtype(*positions, at::kInt, "positions");
    check_dtype(*slots, at::kInt, "slots"); check_dtype(*cos_sin, at::kFloat, "cos_sin");
    TORCH_CHECK(N == (H + 2 * KV) * 128, "packed QKV has ", N, " columns, expected (H + 2 KV) * 128");
    TORCH_CHECK(q_out->numel() >= (int64_t)M * H * 128, "q_out too small");
    TORCH_CHECK(positions->numel() >= M && slots->numel() >= M, "positions/slots shorter than x");
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == 128, "cos_sin must be [max_pos, 128]");
    TORCH_CHECK(k_cache->dim() == 5 && k_cache->size(1) == KV && k_cache->size(2) == 16 && k_cache->size(3) == 16 &&
                    k_cache->size(4) == 8, "k_cache must be [NB, KV, 16, 16, 8]");
    TORCH_CHECK(v_cache->dim() == 4 && v_cache->size(1) == KV && v_cache->size(2) == 128 && v_cache->size(3) == 16,
                "v_cache must be [NB, KV, 128, 16]");
    qp = q_out->data_ptr(); kp = k_cache->data_ptr(); vp = v_cache->data_ptr();
    pp = positions->data_ptr<int>(); sp = slots->data_ptr<int>(); cp = cos_sin->data_ptr<float>();
  }
  int pl[7] = {0, 0, 0, 0, 0, 0, 0};
  if (!plan.empty()) {
    TORCH_CHECK(plan.size() == 7, "plan must be 7 ints (mg, rg, tpw, wt, wk, S, D)");
    for (int i = 0; i < 7; ++i) pl[i] = (int)plan[i];
  }
  const int rc = pa_stream_gemm(yp, x.data_ptr(), wp.data_ptr(), rp, ws.data_ptr<float>(), ws.numel(),
                                counters.data_ptr<int>(), counters.numel(), err.data_ptr<int>(), M, N, K, x.stride(0),
                                ldy, ldr, (int)epi, opt_rows(ss_in, M, "ss_in"),
                                const_cast<float*>(opt_rows(ss_out, M, "ss_out")),
                                const_cast<float*>(opt_rows(ss_zero, M, "ss_zero")), (float)eps, pl, qp, kp, vp, pp,
                                sp, cp, (int)H, (int)KV, (int)rel,
                                stamps ? reinterpret_cast<unsigned long long*>(stamps->data_ptr<int64_t>()) : nullptr,
                                cur_stream());
  TORCH_CHECK(rc >= 0, "stream_gemm launch failed");
  return rc == 0;
}

std::vector<int64_t> stream_gemm_plan(int64_t M, int64_t N, int64_t K, int64_t epi) {
  int p[7];
  pa_stream_gemm_plan((int)M, (int)N, (int)K, (int)epi, p);
  const long long ws = pa_stream_gemm_ws_floats((int)M, (int)N, (int)K, p[0], p[1], p[2], p[3], p[4], p[5]);
  return {p[0], p[1], p[2], p[3], p[4], p[5], p[6], (int64_t)ws};
}

// Large-M projections (csrc/ops/gemm_prefill.hip): 256x256 MFMA tiles on the packed
// weights with the same epilogues as mid_gemm (0 plain, 1 SwiGLU, 2 residual, 3 rope-perm).
bool prefill_gemm(at::Tensor y, at::Tensor x, at::Tensor wp, c10::optional<at::Tensor> resid, at::Tensor ws,
                  at::Tensor counters, int64_t epi, c10::optional<at::Tensor> ss_in, c10::optional<at::Tensor> ss_out,
                  c10::optional<at::Tensor> ss_zero, double eps, int64_t full, int64_t splits, int64_t bn,
                  int64_t variant) {
  check_gpu(wp, "wp"); check_gpu(ws, "ws"); check_gpu(counters, "counters");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1, "y must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp"); check_dtype(y, at::kBFloat16, "y");
  check_dtype(ws, at::kFloat, "ws"); check_dtype(counters, at::kInt, "counters");
  TORCH_CHECK(epi >= 0 && epi <= 3, "prefill_gemm epi must be 0..3 (RoPE + KV write: prefill_qkv_rope)");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0 && y.stride(0) % 4 == 0, "x rows must be 16-byte, y rows 8-byte aligned");
  // the non-pair epilogues (plain, residual) of the ping-pong kernels store -- and read the
  // residual -- 16 B per lane (packed_epi.h store_pair_wide): y and resid rows 16-byte aligned
  const bool wide = epi == 0 || epi == 2;
  auto rows16 = [](const at::Tensor& t) { return t.stride(0) % 8 == 0 && ((uintptr_t)t.data_ptr() & 15) == 0; };
  TORCH_CHECK(!wide || rows16(y), "y rows must be 16-byte aligned for the plain / residual epilogue");
  TORCH_CHECK(((uintptr_t)y.data_ptr() & 7) == 0, "y must be 8-byte aligned");
  const int NO = epi == 1 ? N / 2 : N;
  TORCH_CHECK(y.size(0) == M && y.size(1) == NO, "y shape mismatch");
  const void* rp = nullptr;
  int ldr = 0;
  if (epi == 2) {
    TORCH_CHECK(resid.has_value(), "epi=2 needs resid");
    const auto& r = *resid;
    TORCH_CHECK(r.is_cuda() && r.dim() == 2 && r.stride(1) == 1 && r.size(0) == M && r.size(1) == N && rows16(r),
                "resid must be [M, N] with unit inner stride and 16-byte aligned rows");
    check_dtype(r, at::kBFloat16, "resid");
    rp = r.data_ptr();
    ldr = r.stride(0);
  }
  const int rc = pa_prefill_gemm(y.data_ptr(), x.data_ptr(), wp.data_ptr(), rp, ws.data_ptr<float>(), ws.numel(),
                                 counters.data_ptr<int>(), counters.numel(), M, N, K, x.stride(0), y.stride(0), ldr,
                                 (int)epi, opt_rows(ss_in, M, "ss_in"), const_cast<float*>(opt_rows(ss_out, M, "ss_out")),
                                 const_cast<float*>(opt_rows(ss_zero, M, "ss_zero")), (float)eps, (int)full,
                                 (int)splits, (int)bn, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0,
                                 (int)variant, cur_stream());
  TORCH_CHECK(rc >= 0, "prefill_gemm launch failed");
  return rc == 0;
}

bool prefill_qkv_rope(at::Tensor x, at::Tensor wp, at::Tensor ss_in, double eps, at::Tensor q_out, at::Tensor k_cache,
                      at::Tensor v_cache, at::Tensor positions, at::Tensor slots, at::Tensor cos_sin, int64_t H,
                      int64_t KV, at::Tensor ws, at::Tensor counters, int64_t full, int64_t splits, int64_t bn,
                      int64_t variant) {
  check_gpu(wp, "wp"); check_gpu(q_out, "q_out"); check_gpu(k_cache, "k_cache"); check_gpu(v_cache, "v_cache");
  check_gpu(positions, "positions"); check_gpu(slots, "slots"); check_gpu(cos_sin, "cos_sin");
  check_gpu(ws, "ws"); check_gpu(counters, "counters");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(wp, at::kBFloat16, "wp"); check_dtype(q_out, at::kBFloat16, "q_out");
  check_dtype(k_cache, at::kBFloat16, "k_cache"); check_dtype(v_cache, at::kBFloat16, "v_cache");
  check_dtype(positions, at::kInt, "positions"); check_dtype(slots, at::kInt, "slots");
  check_dtype(cos_sin, at::kFloat, "cos_sin");
  check_dtype(ws, at::kFloat, "ws"); check_dtype(counters, at::kInt, "counters");
  TORCH_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8, "wp must be packed [N/16, K/32, 64, 8]");
  const int M = x.size(0), K = x.size(1), N = wp.size(0) * 16;
  TORCH_CHECK(wp.size(1) * 32 == K, "packed weight K mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0, "x rows must be 16-byte aligned");
  TORCH_CHECK(N == (H + 2 * KV) * 128, "QKV width must be (H + 2 KV) * 128");
  TORCH_CHECK(q_out.numel() >= (int64_t)M * H * 128, "q_out too small");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M, "positions/slots shorter than x");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == 128, "cos_sin must be [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(1) == KV && k_cache.size(2) == 16 && k_cache.size(3) == 16 &&
                  k_cache.size(4) == 8, "k_cache must be [NB, KV, 16, 16, 8]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == KV && v_cache.size(2) == 128 && v_cache.size(3) == 16,
              "v_cache must be [NB, KV, 128, 16]");
  TORCH_CHECK(ss_in.is_cuda() && ss_in.numel() >= M, "ss_in must hold M row statistics");
  check_dtype(ss_in, at::kFloat, "ss_in");
  const int rc = pa_prefill_gemm(nullptr, x.data_ptr(), wp.data_ptr(), nullptr, ws.data_ptr<float>(), ws.numel(),
                                 counters.data_ptr<int>(), counters.numel(), M, N, K, x.stride(0), 0, 0, 4,
                                 ss_in.data_ptr<float>(), nullptr, nullptr, (float)eps, (int)full, (int)splits,
                                 (int)bn, q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), positions.data_ptr<int>(),
                                 slots.data_ptr<int>(), cos_sin.data_ptr<float>(), (int)H, (int)KV, (int)variant,
                                 cur_stream());
  TORCH_CHECK(rc >= 0, "prefill_qkv_rope launch failed");
  return rc == 0;
}

std::vector<int64_t> prefill_gemm_plan(int64_t M, int64_t N, int64_t K, int64_t bn) {
  int full, S;
  if (bn <= 0) bn = pa_prefill_pick_bn((int)M, (int)N);
  pa_prefill_gemm_plan((int)M, (int)N, (int)K, (int)bn, &full, &S);
  return {full, S, pa_prefill_gemm_ws_floats((int)M, (int)N, (int)bn, full, S), bn};
}

// out[m] = sum_k x[m, k]^2 (fp32)
void row_sumsq(at::Tensor out, at::Tensor x) {
  check_gpu(out, "out");
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x must be a 2-D GPU tensor, unit inner stride");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(out.numel() >= x.size(0), "out shorter than x");
  check_rc(pa_row_sumsq(out.data_ptr<float>(), x.data_ptr(), x.size(0), x.size(1), x.stride(0), cur_stream()),
           "row_sumsq");
}

std::vector<int64_t> mid_gemm_plan(int64_t M, int64_t N, int64_t K, int64_t epi) {
  int fm, fn, S;
  pa_mid_gemm_plan((int)M, (int)N, (int)K, (int)epi, &fm, &fn, &S);
  return {fm, fn, S, pa_mid_gemm_ws_floats((int)M, (int)N, (int)K, fm, fn, S)};
}

int64_t sample_workspace_floats(int64_t rows, int64_t V) {
  return pa_sample_workspace_floats(rows, V);
}

void patch_pending_ids(at::Tensor ids, at::Tensor sampled) {
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kInt && ids.is_contiguous(), "ids: int32 device tensor");
  TORCH_CHECK(sampled.is_cuda() && sampled.scalar_type() == at::kInt && sampled.is_contiguous(),
              "sampled: int32 device tensor");
  check_rc(pa_patch_pending_ids(ids.data_ptr<int>(), sampled.data_ptr<int>(), (int)ids.numel(),
                                (int)sampled.numel(), cur_stream()),
           "patch_pending_ids");
}

void sample(at::Tensor out_tokens, c10::optional<at::Tensor> out_keys, at::Tensor workspace,
            at::Tensor logits, int64_t vocab_offset, at::Tensor temperature, at::Tensor mask_class,
            at::Tensor class_masks, at::Tensor seeds, at::Tensor offsets,
            c10::optional<at::Tensor> forced, c10::optional<at::Tensor> tau) {
  check_gpu(out_tokens, "out_tokens"); check_gpu(workspace, "workspace");
  check_gpu(temperature, "temperature"); check_gpu(mask_class, "mask_class");
  check_gpu(class_masks, "class_masks"); check_gpu(seeds, "seeds"); check_gpu(offsets, "offsets");
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1,
              "logits must be a 2-D GPU tensor with unit inner stride");
  check_dtype(logits, at::kBFloat16, "logits"); check_dtype(out_tokens, at::kInt, "out_tokens");
  check_dtype(workspace, at::kFloat, "workspace"); check_dtype(temperature, at::kFloat, "temperature");
  check_dtype(mask_class, at::kInt, "mask_class"); check_dtype(class_masks, at::kInt, "class_masks");
  check_dtype(seeds, at::kLong, "seeds"); check_dtype(offsets, at::kInt, "offsets");
  const int rows = logits.size(0), V = logits.size(1);
  TORCH_CHECK(out_tokens.numel() >= rows && temperature.numel() >= rows &&
                  mask_class.numel() >= rows && seeds.numel() >= rows && offsets.numel() >= rows,
              "per-row sampling parameter tensors too short");
  TORCH_CHECK(workspace.numel() >= pa_sample_workspace_floats(rows, V), "sample workspace too small");
  TORCH_CHECK(class_masks.dim() == 2, "class_masks must be [classes, words]");
  TORCH_CHECK(class_masks.size(1) * 32 >= vocab_offset + V, "class_masks too narrow for vocab");
  float* keys = nullptr;
  if (out_keys.has_value()) {
    check_gpu(*out_keys, "out_keys"); check_dtype(*out_keys, at::kFloat, "out_keys");
    keys = out_keys->data_ptr<float>();
  }
  const int* fp = nullptr;
  if (forced.has_value()) {
    check_gpu(*forced, "forced"); check_dtype(*forced, at::kInt, "forced");
    fp = forced->data_ptr<int>();
  }
  const float* tp = nullptr;
  if (tau.has_value()) {
    check_gpu(*tau, "tau"); check_dtype(*tau, at::kFloat, "tau");
    TORCH_CHECK(tau->numel() >= rows, "tau too short");
    tp = tau->data_ptr<float>();
  }
  check_rc(pa_sample(out_tokens.data_ptr<int>(), keys, workspace.data_ptr<float>(),
                     logits.data_ptr(), rows, V, logits.stride(0), vocab_offset,
                     temperature.data_ptr<float>(), mask_class.data_ptr<int>(),
                     reinterpret_cast<const uint32_t*>(class_masks.data_ptr<int>()),
                     class_masks.size(1), seeds.data_ptr<int64_t>(), offsets.data_ptr<int>(), fp,
                     tp, cur_stream()),
           "sample");
}

int64_t cosine_topk_workspace_bytes(int64_t Q, int64_t N, int64_t K) {
  return pa_cosine_topk_workspace_bytes(Q, N, K);
}

void cosine_topk(at::Tensor out_scores, at::Tensor out_rows, at::Tensor workspace,
                 at::Tensor queries, at::Tensor index, int64_t n_valid, int64_t K,
                 at::Tensor row_priority, at::Tensor row_tags, at::Tensor row_expiry,
                 at::Tensor q_min_priority, at::Tensor q_tags, double now) {
  for (auto* t : {&out_scores, &out_rows, &workspace, &queries, &index, &row_priority, &row_tags,
                  &row_expiry, &q_min_priority, &q_tags})
    check_gpu(*t, "cosine_topk arg");
  check_dtype(queries, at::kBFloat16, "queries"); check_dtype(index, at::kBFloat16, "index");
  check_dtype(out_scores, at::kFloat, "out_scores"); check_dtype(out_rows, at::kInt, "out_rows");
  check_dtype(row_priority, at::kInt, "row_priority"); check_dtype(row_tags, at::kLong, "row_tags");
  check_dtype(row_expiry, at::kFloat, "row_expiry");
  check_dtype(q_min_priority, at::kInt, "q_min_priority"); check_dtype(q_tags, at::kLong, "q_tags");
  TORCH_CHECK(index.dim() == 4 && index.size(2) == 64 && index.size(3) == 8,
              "index must be packed in 16-row tiles [N/16, D/32, 64, 8] (memory/semantic_index.py)");
  const int Q = queries.size(0), N = index.size(0) * 16, D = index.size(1) * 32;
  TORCH_CHECK(queries.dim() == 2 && queries.size(1) == D, "queries [Q, D] and the index must agree on D");
  TORCH_CHECK(Q <= 64, "cosine_topk takes at most 64 queries per call (ops.cosine_topk chunks larger batches)");
  TORCH_CHECK(n_valid <= N, "n_valid exceeds index rows");
  TORCH_CHECK(row_priority.numel() >= n_valid && row_tags.numel() >= n_valid && row_expiry.numel() >= n_valid,
              "row metadata shorter than n_valid");
  TORCH_CHECK(queries.is_contiguous(), "queries must be contiguous");
  TORCH_CHECK(out_scores.numel() >= (int64_t)Q * K && out_rows.numel() >= (int64_t)Q * K,
              "output too small");
  TORCH_CHECK(workspace.numel() * workspace.element_size() >=
                  pa_cosine_topk_workspace_bytes(Q, n_valid, K),
              "cosine_topk workspace too small");
  check_rc(pa_cosine_topk(out_scores.data_ptr<float>(), out_rows.data_ptr<int>(),
                          workspace.data_ptr(), queries.data_ptr(), index.data_ptr(), Q,
                          (int)n_valid, D, K, row_priority.data_ptr<int>(),
                          reinterpret_cast<const uint64_t*>(row_tags.data_ptr<int64_t>()),
                          row_expiry.data_ptr<float>(), q_min_priority.data_ptr<int>(),
                          reinterpret_cast<const uint64_t*>(q_tags.data_ptr<int64_t>()),
                          (float)now, (int)n_valid, cur_stream()),
           "cosine_topk");
}

int64_t q16_topk_workspace_bytes(int64_t Q, int64_t N) { return pa_q16_topk_workspace_bytes(Q, N); }

// Two-stage exact top-k over the 16-bit fixed-point index (csrc/ops/similarity_q16.hip).
void q16_topk(at::Tensor out_scores, at::Tensor out_rows, at::Tensor unsafe, at::Tensor workspace,
              at::Tensor queries_q, at::Tensor qmeta, at::Tensor hi, at::Tensor lo, at::Tensor rmeta, int64_t n_valid,
              int64_t K, at::Tensor row_priority, at::Tensor row_tags, at::Tensor row_expiry,
              at::Tensor q_min_priority, at::Tensor q_tags, double now, int64_t exact) {
  for (auto* t : {&out_scores, &out_rows, &unsafe, &workspace, &queries_q, &qmeta, &hi, &lo, &rmeta, &row_priority,
                  &row_tags, &row_expiry, &q_min_priority, &q_tags})
    check_gpu(*t, "q16_topk arg");
  check_dtype(queries_q, at::kChar, "queries_q"); check_dtype(hi, at::kChar, "hi"); check_dtype(lo, at::kChar, "lo");
  check_dtype(qmeta, at::kFloat, "qmeta"); check_dtype(rmeta, at::kFloat, "rmeta");
  check_dtype(out_scores, at::kFloat, "out_scores"); check_dtype(out_rows, at::kInt, "out_rows");
  check_dtype(unsafe, at::kInt, "unsafe");
  check_dtype(row_priority, at::kInt, "row_priority"); check_dtype(row_tags, at::kLong, "row_tags");
  check_dtype(row_expiry, at::kFloat, "row_expiry");
  check_dtype(q_min_priority, at::kInt, "q_min_priority"); check_dtype(q_tags, at::kLong, "q_tags");
  TORCH_CHECK(hi.dim() == 4 && hi.size(2) == 64 && hi.size(3) == 16 && lo.sizes() == hi.sizes(),
              "hi / lo must be int8 planes [N/16, D/64, 64, 16] (memory/semantic_index.py storage='q16')");
  const int64_t N = hi.size(0) * 16, D = hi.size(1) * 64;
  const int64_t Q = queries_q.size(0);
  TORCH_CHECK(queries_q.dim() == 3 && queries_q.size(1) == 2 && queries_q.size(2) == D, "queries_q [Q, 2, D]");
  TORCH_CHECK(Q <= 64, "q16_topk takes at most 64 queries per call");
  TORCH_CHECK(qmeta.numel() >= 2 * Q && rmeta.numel() >= 2 * n_valid, "qmeta [Q, 2] / rmeta [N, 2] too short");
  TORCH_CHECK(n_valid <= N, "n_valid exceeds index rows");
  TORCH_CHECK(row_priority.numel() >= n_valid && row_tags.numel() >= n_valid && row_expiry.numel() >= n_valid,
              "row metadata shorter than n_valid");
  TORCH_CHECK(out_scores.numel() >= Q * K && out_rows.numel() >= Q * K && unsafe.numel() >= Q, "output too small");
  TORCH_CHECK(workspace.numel() * workspace.element_size() >= pa_q16_topk_workspace_bytes(Q, n_valid),
              "q16_topk workspace too small");
  check_rc(pa_q16_topk(out_scores.data_ptr<float>(), out_rows.data_ptr<int>(), unsafe.data_ptr<int>(),
                       workspace.data_ptr(), queries_q.data_ptr(), qmeta.data_ptr<float>(), hi.data_ptr(),
                       lo.data_ptr(), rmeta.data_ptr<float>(), (int)Q, (int)n_valid, (int)D, (int)K,
                       row_priority.data_ptr<int>(), reinterpret_cast<const uint64_t*>(row_tags.data_ptr<int64_t>()),
                       row_expiry.data_ptr<float>(), q_min_priority.data_ptr<int>(),
                       reinterpret_cast<const uint64_t*>(q_tags.data_ptr<int64_t>()), (float)now, (int)exact,
                       cur_stream()),
           "q16_topk");
}

}  // namespace

// One phase of the vocab-parallel top-k / top-p threshold (sampling.hip tp_topkp_kernel):
// logits [rows, v_local] is this rank's slice; ws [ceil4(rows) + rows * 1028] fp32 holds
// mx | h0 | h1 | st.
void tp_topkp_phase(int64_t phase, at::Tensor tau, at::Tensor ws, at::Tensor logits, int64_t vocab_offset,
                    int64_t V, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p, at::Tensor mask_class,
                    at::Tensor class_masks) {
  for (auto* t : {&tau, &ws, &temperature, &top_k, &top_p, &mask_class, &class_masks})
    check_gpu(*t, "tp_topkp_phase arg");
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits: [rows, v_local] GPU");
  check_dtype(tau, at::kFloat, "tau"); check_dtype(ws, at::kFloat, "ws"); check_dtype(logits, at::kBFloat16, "logits");
  check_dtype(temperature, at::kFloat, "temperature"); check_dtype(top_k, at::kInt, "top_k");
  check_dtype(top_p, at::kFloat, "top_p"); check_dtype(mask_class, at::kInt, "mask_class");
  check_dtype(class_masks, at::kInt, "class_masks");
  const int rows = logits.size(0), vl = logits.size(1);
  TORCH_CHECK(ws.numel() >= (int64_t)((rows + 3) & ~3) + (int64_t)rows * 1028,
              "ws must hold ceil4(rows) + rows * 1028 floats");
  TORCH_CHECK(tau.numel() >= rows && temperature.numel() >= rows && top_k.numel() >= rows &&
                  top_p.numel() >= rows && mask_class.numel() >= rows, "per-row tensors too short");
  TORCH_CHECK(class_masks.dim() == 2 && class_masks.size(1) * 32 >= V && vocab_offset + vl <= V,
              "class_masks / vocab slice");
  check_rc(pa_tp_topkp_phase((int)phase, tau.data_ptr<float>(), ws.data_ptr<float>(), logits.data_ptr(), rows, vl,
                             logits.stride(0), (int)vocab_offset, (int)V, temperature.data_ptr<float>(),
                             top_k.data_ptr<int>(), top_p.data_ptr<float>(), mask_class.data_ptr<int>(),
                             reinterpret_cast<const uint32_t*>(class_masks.data_ptr<int>()), class_masks.size(1),
                             cur_stream()),
           "tp_topkp_phase");
}

// tau[r] = top-k / top-p logit threshold of row r. `logits` is [rows, V] or a TP
// all-gather [shards, rows, V/shards] (then V is the full vocabulary).
void topkp_threshold(at::Tensor tau, at::Tensor logits, int64_t V, at::Tensor temperature,
                     at::Tensor top_k, at::Tensor top_p, at::Tensor mask_class, at::Tensor class_masks) {
  for (auto* t : {&tau, &logits, &temperature, &top_k, &top_p, &mask_class, &class_masks})
    check_gpu(*t, "topkp_threshold arg");
  check_dtype(tau, at::kFloat, "tau"); check_dtype(logits, at::kBFloat16, "logits");
  check_dtype(temperature, at::kFloat, "temperature"); check_dtype(top_k, at::kInt, "top_k");
  check_dtype(top_p, at::kFloat, "top_p"); check_dtype(mask_class, at::kInt, "mask_class");
  check_dtype(class_masks, at::kInt, "class_masks");
  int shards = 1, rows, ld;
  long long sstride = 0;
  if (logits.dim() == 3) {
    shards = logits.size(0); rows = logits.size(1); ld = logits.stride(1); sstride = logits.stride(0);
    TORCH_CHECK(logits.size(2) * shards == V, "gathered logits do not cover the vocabulary");
  } else {
    TORCH_CHECK(logits.dim() == 2 && logits.size(1) == V, "logits must be [rows, V]");
    rows = logits.size(0); ld = logits.stride(0);
  }
  TORCH_CHECK(logits.stride(-1) == 1, "logits need unit inner stride");
  TORCH_CHECK(tau.numel() >= rows && temperature.numel() >= rows && top_k.numel() >= rows &&
                  top_p.numel() >= rows && mask_class.numel() >= rows, "per-row tensors too short");
  TORCH_CHECK(class_masks.dim() == 2 && class_masks.size(1) * 32 >= V, "class_masks too narrow");
  check_rc(pa_topkp_threshold(tau.data_ptr<float>(), logits.data_ptr(), rows, V, ld, shards, sstride,
                              temperature.data_ptr<float>(), top_k.data_ptr<int>(), top_p.data_ptr<float>(),
                              mask_class.data_ptr<int>(),
                              reinterpret_cast<const uint32_t*>(class_masks.data_ptr<int>()),
                              class_masks.size(1), cur_stream()),
           "topkp_threshold");
}

// ---- custom P2P all-reduce (csrc/ops/custom_ar.hip) ----
py::tuple car_alloc(int64_t bytes) {
  char h[64];
  void* p = pa_car_alloc(bytes, h);
  TORCH_CHECK(p != nullptr, "car_alloc: uncached IPC allocation of ", bytes, " bytes failed");
  return py::make_tuple((int64_t)(uintptr_t)p, py::bytes(h, 64));
}

int64_t car_open(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK(h.size() == 64, "car_open: IPC handle must be 64 bytes");
  void* p = pa_car_open(h.data());
  TORCH_CHECK(p != nullptr, "car_open: hipIpcOpenMemHandle failed");
  return (int64_t)(uintptr_t)p;
}

void car_all_reduce(std::vector<int64_t> bases, int64_t rank0, std::vector<at::Tensor> ins,
                    std::vector<at::Tensor> outs, int64_t cap_bytes, at::Tensor epochs, at::Tensor err,
                    bool two_shot, std::vector<at::Tensor> resids, std::vector<at::Tensor> ss,
                    std::vector<at::Tensor> ss_zero, int64_t row_len) {
  const int W = (int)bases.size();
  const int nl = (int)ins.size();
  TORCH_CHECK(W >= 2 && W <= 8, "custom all-reduce supports 2..8 ranks");
  TORCH_CHECK(nl >= 1 && (int)outs.size() == nl && rank0 >= 0 && rank0 + nl <= W, "bad rank range");
  const int64_t n = ins[0].numel();
  std::vector<void*> b(W), ip(nl), op(nl);
  for (int i = 0; i < W; ++i) b[i] = (void*)(uintptr_t)bases[i];
  for (int i = 0; i < nl; ++i) {
    check_gpu(ins[i], "in"); check_gpu(outs[i], "out");
    check_dtype(ins[i], at::kBFloat16, "in"); check_dtype(outs[i], at::kBFloat16, "out");
    TORCH_CHECK(ins[i].numel() == n && outs[i].numel() == n, "all-reduce tensors differ in size");
    TORCH_CHECK(((uintptr_t)ins[i].data_ptr() & 15) == 0 && ((uintptr_t)outs[i].data_ptr() & 15) == 0,
                "all-reduce tensors must be 16-byte aligned");
    ip[i] = ins[i].data_ptr(); op[i] = outs[i].data_ptr();
  }
  TORCH_CHECK(n % 8 == 0 && n * 2 <= cap_bytes, "message of ", n, " bf16 does not fit the custom all-reduce");
  check_gpu(epochs, "epochs"); check_dtype(epochs, at::kInt, "epochs");
  TORCH_CHECK(epochs.numel() >= (int64_t)nl * pa_car_group(), "epochs too short");
  check_gpu(err, "err"); check_dtype(err, at::kInt, "err");
  // fused residual epilogue: out = resid + sum, ss[row] += sum(out^2), ss_zero <- 0
  std::vector<const void*> rp;
  std::vector<float*> sp, zp;
  const bool fused = !resids.empty();
  if (fused) {
    TORCH_CHECK((int)resids.size() == nl, "one resid per local rank");
    TORCH_CHECK(row_len > 0 && n % row_len == 0 && (row_len / 8) % 256 == 0 && row_len % 8 == 0,
                "fused all-reduce needs whole rows of a multiple of 2048 elements");
    const int64_t rows = n / row_len;
    for (int i = 0; i < nl; ++i) {
      check_gpu(resids[i], "resid"); check_dtype(resids[i], at::kBFloat16, "resid");
      TORCH_CHECK(resids[i].numel() == n && resids[i].is_contiguous() && ((uintptr_t)resids[i].data_ptr() & 15) == 0,
                  "resid must match the message, contiguous and 16-byte aligned");
      rp.push_back(resids[i].data_ptr());
    }
    TORCH_CHECK(ss.empty() || (int)ss.size() == nl, "one ss per local rank");
    TORCH_CHECK(ss_zero.empty() || (int)ss_zero.size() == nl, "one ss_zero per local rank");
    for (auto& t : ss) {
      check_gpu(t, "ss"); check_dtype(t, at::kFloat, "ss");
      TORCH_CHECK(t.numel() >= rows, "ss shorter than the message's rows");
      sp.push_back(t.data_ptr<float>());
    }
    for (auto& t : ss_zero) {
      check_gpu(t, "ss_zero"); check_dtype(t, at::kFloat, "ss_zero");
      TORCH_CHECK(t.numel() >= rows, "ss_zero shorter than the message's rows");
      zp.push_back(t.data_ptr<float>());
    }
  }
  check_rc(pa_car_all_reduce(b.data(), W, (int)rank0, nl, ip.data(), op.data(), n, cap_bytes,
                             reinterpret_cast<uint32_t*>(epochs.data_ptr<int>()), err.data_ptr<int>(),
                             two_shot ? 1 : 0, fused ? rp.data() : nullptr, sp.empty() ? nullptr : sp.data(),
                             zp.empty() ? nullptr : zp.data(), (int)row_len, cur_stream()),
           "custom all-reduce");
}

// Small collectives over the custom all-reduce buffers (custom_ar.hip co_kernel): op 0 = SUM
// and 1 = MAX of fp32 (outs may alias ins), 2 = all-gather of any 4-byte dtype (outs[i] holds
// W x n elements, rank-major). n % 4 == 0, 16-byte aligned tensors.
void car_collective(std::vector<int64_t> bases, int64_t rank0, std::vector<at::Tensor> ins,
                    std::vector<at::Tensor> outs, int64_t cap_bytes, at::Tensor epochs, at::Tensor err, int64_t op) {
  const int W = (int)bases.size();
  const int nl = (int)ins.size();
  TORCH_CHECK(W >= 2 && W <= 8, "custom collectives support 2..8 ranks");
  TORCH_CHECK(nl >= 1 && (int)outs.size() == nl && rank0 >= 0 && rank0 + nl <= W, "bad rank range");
  TORCH_CHECK(op >= 0 && op <= 2, "op: 0 sum, 1 max, 2 gather");
  const int64_t n = ins[0].numel();
  std::vector<void*> b(W), ip(nl), opp(nl);
  for (int i = 0; i < W; ++i) b[i] = (void*)(uintptr_t)bases[i];
  for (int i = 0; i < nl; ++i) {
    check_gpu(ins[i], "in"); check_gpu(outs[i], "out");
    TORCH_CHECK(ins[i].element_size() == 4 && outs[i].element_size() == 4, "4-byte elements");
    if (op < 2) {
      check_dtype(ins[i], at::kFloat, "in"); check_dtype(outs[i], at::kFloat, "out");
    }
    TORCH_CHECK(ins[i].numel() == n && outs[i].numel() == (op == 2 ? n * W : n), "collective tensor sizes");
    TORCH_CHECK(((uintptr_t)ins[i].data_ptr() & 15) == 0 && ((uintptr_t)outs[i].data_ptr() & 15) == 0,
                "collective tensors must be 16-byte aligned");
    ip[i] = ins[i].data_ptr(); opp[i] = outs[i].data_ptr();
  }
  TORCH_CHECK(n % 4 == 0 && n * 4 <= cap_bytes, "message of ", n, " x 4 B does not fit the custom buffers");
  check_gpu(epochs, "epochs"); check_dtype(epochs, at::kInt, "epochs");
  TORCH_CHECK(epochs.numel() >= (int64_t)nl * pa_car_group(), "epochs too short");
  check_gpu(err, "err"); check_dtype(err, at::kInt, "err");
  check_rc(pa_car_collective(b.data(), W, (int)rank0, nl, ip.data(), opp.data(), n, cap_bytes,
                             reinterpret_cast<uint32_t*>(epochs.data_ptr<int>()), err.data_ptr<int>(), (int)op,
                             cur_stream()),
           "custom collective");
}

// ---- uncached device memory (in-launch hand-off workspaces) ----
// Split-K slabs and attention partials are written by one workgroup and read by another
// inside the same launch. In uncached memory (MTYPE UC: no L1/L2 copy of any line) a reader
// can never see a stale copy held by its own CU or XCD, whatever the placement, so the
// hand-off needs no L2 write-back on the producer side.
at::Tensor empty_uncached(int64_t numel, at::ScalarType dtype, int64_t device) {
  TORCH_CHECK(numel > 0, "empty_uncached: numel must be positive");
  const int64_t bytes = numel * (int64_t)c10::elementSize(dtype);
  int prev = 0;
  TORCH_CHECK(hipGetDevice(&prev) == hipSuccess, "hipGetDevice failed");
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "hipSetDevice failed");
  void* p = nullptr;
  const hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) (void)hipMemset(p, 0, (size_t)bytes);
  (void)hipSetDevice(prev);
  TORCH_CHECK(e == hipSuccess && p != nullptr, "empty_uncached: hipExtMallocWithFlags(", bytes,
              " bytes, uncached) failed");
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "empty_uncached: memset failed");
  auto opts = at::TensorOptions().dtype(dtype).device(at::Device(at::kCUDA, (int)device));
  return torch::from_blob(p, {numel}, [](void* q) { (void)hipFree(q); }, opts);
}

PYBIND11_MODULE(_C, m) {
  m.def("store_test", [](at::Tensor dst, int64_t mode, int64_t grid) {
    check_gpu(dst, "dst");
    TORCH_CHECK(dst.is_contiguous() && dst.nbytes() % 16 == 0, "dst: contiguous, a multiple of 16 bytes");
    check_rc(pa_store_test(dst.data_ptr(), (long long)(dst.nbytes() / 16), (int)mode, (int)grid, cur_stream()),
             "store_test");
  }, py::arg("dst"), py::arg("mode"), py::arg("grid") = 256, "diagnostics: fill dst with one store form");
  m.def("timeline_marker", [](int64_t id) { check_rc(pa_timeline_marker((int)id, cur_stream()), "timeline_marker"); },
        "empty marker kernel (0 = begin, 1 = end of a timed region) for profile cutting");
  m.def("empty_uncached", &empty_uncached, py::arg("numel"), py::arg("dtype"), py::arg("device"),
        "zero-filled device tensor in uncached memory (hipDeviceMallocUncached)");
  m.doc() = "pilottai_amd CDNA4 (gfx950) HIP kernels";
  m.def("rmsnorm", &rmsnorm);
  m.def("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.def("rope_cache", &rope_cache);
  m.def("silu_mul", &silu_mul);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("skinny_set_variant", [](int v) { pa_skinny_set_variant(v); });
  m.def("decode_set_variant", [](int v) { pa_decode_set_variant(v); });
  m.def("handoff_set_acquire", [](int v) { pa_handoff_set_acquire(v); },
        "protocol of every in-launch hand-off (diagnostics): 0 sc1 only, 1 acquire, 2 release + acquire");
  m.def("handoff_set_modes", [](int gemm, int attn) { pa_handoff_set_modes(gemm, attn); },
        "hand-off protocols of the GEMM split-K slabs and of the attention merge (defaults 2, 1)");
  m.def("decode_gemm", &decode_gemm, py::arg("y"), py::arg("x"), py::arg("wp"), py::arg("resid") = py::none(),
        py::arg("epi") = 0, py::arg("norm") = false, py::arg("eps") = 1e-5, py::arg("nt") = 0,
        py::arg("waves") = 0, py::arg("splits") = 0, py::arg("ws") = py::none(), py::arg("counters") = py::none());
  m.def("decode_qkv_rope", &decode_qkv_rope, py::arg("x"), py::arg("wp"), py::arg("eps"), py::arg("q_out"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("positions"), py::arg("slots"), py::arg("cos_sin"),
        py::arg("H"), py::arg("KV"), py::arg("splits") = 0, py::arg("ws") = py::none(),
        py::arg("counters") = py::none());
  m.def("mid_gemm", &mid_gemm, py::arg("y"), py::arg("x"), py::arg("wp"), py::arg("resid"), py::arg("ws"),
        py::arg("counters"), py::arg("epi") = 0, py::arg("ss_in") = py::none(), py::arg("ss_out") = py::none(),
        py::arg("ss_zero") = py::none(), py::arg("eps") = 1e-5, py::arg("fm") = 0, py::arg("fn") = 0,
        py::arg("splits") = 0);
  m.def("mid_qkv_rope", &mid_qkv_rope, py::arg("x"), py::arg("wp"), py::arg("ss_in"), py::arg("eps"),
        py::arg("q_out"), py::arg("k_cache"), py::arg("v_cache"), py::arg("positions"), py::arg("slots"),
        py::arg("cos_sin"), py::arg("H"), py::arg("KV"), py::arg("ws"), py::arg("counters"), py::arg("fm") = 0,
        py::arg("fn") = 0, py::arg("splits") = 0);
  m.def("prefill_gemm", &prefill_gemm, py::arg("y"), py::arg("x"), py::arg("wp"), py::arg("resid"), py::arg("ws"),
        py::arg("counters"), py::arg("epi") = 0, py::arg("ss_in") = py::none(), py::arg("ss_out") = py::none(),
        py::arg("ss_zero") = py::none(), py::arg("eps") = 1e-5, py::arg("full") = -1, py::arg("splits") = 0,
        py::arg("bn") = 0, py::arg("variant") = -1);
  m.def("prefill_qkv_rope", &prefill_qkv_rope, py::arg("x"), py::arg("wp"), py::arg("ss_in"), py::arg("eps"),
        py::arg("q_out"), py::arg("k_cache"), py::arg("v_cache"), py::arg("positions"), py::arg("slots"),
        py::arg("cos_sin"), py::arg("H"), py::arg("KV"), py::arg("ws"), py::arg("counters"), py::arg("full") = -1,
        py::arg("splits") = 0, py::arg("bn") = 0, py::arg("variant") = -1);
  m.def("prefill_set_variant", [](int v) { pa_prefill_set_variant(v); });
  m.def("prefill_gemm_plan", &prefill_gemm_plan, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("bn") = 0,
        "default (full tiles, splits, workspace floats, tile width) of prefill_gemm");
  m.def("row_sumsq", &row_sumsq, py::arg("out"), py::arg("x"));
  m.def("stream_gemm", &stream_gemm, py::arg("y"), py::arg("x"), py::arg("wp"), py::arg("resid"), py::arg("ws"),
        py::arg("counters"), py::arg("err"), py::arg("epi"), py::arg("ss_in"), py::arg("ss_out"), py::arg("ss_zero"),
        py::arg("eps"), py::arg("plan"), py::arg("q_out") = py::none(), py::arg("k_cache") = py::none(),
        py::arg("v_cache") = py::none(), py::arg("positions") = py::none(), py::arg("slots") = py::none(),
        py::arg("cos_sin") = py::none(), py::arg("H") = 0, py::arg("KV") = 0, py::arg("rel") = 0,
        py::arg("stamps") = py::none());
  m.def("stream_gemm_plan", &stream_gemm_plan,
        "default (mg, rg, tpw, wt, wk, S, D, workspace floats) of stream_gemm");
  m.def("mid_gemm_plan", &mid_gemm_plan, "default (fm, fn, splits, workspace floats) of mid_gemm");
  m.def("paged_attention", &paged_attention, py::arg("out"), py::arg("part_o"), py::arg("part_ml"), py::arg("q"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("items"), py::arg("n_items"), py::arg("counters"),
        py::arg("q_start"), py::arg("q_len"), py::arg("ctx_len"), py::arg("block_table"), py::arg("scale"),
        py::arg("part_size") = py::none(), py::arg("waves") = 4);
  m.def("sample_workspace_floats", &sample_workspace_floats);
  m.def("patch_pending_ids", &patch_pending_ids);
  m.def("sample", &sample, py::arg("out_tokens"), py::arg("out_keys"), py::arg("workspace"),
        py::arg("logits"), py::arg("vocab_offset"), py::arg("temperature"), py::arg("mask_class"),
        py::arg("class_masks"), py::arg("seeds"), py::arg("offsets"), py::arg("forced"),
        py::arg("tau") = py::none());
  m.def("topkp_threshold", &topkp_threshold);
  m.def("tp_topkp_phase", &tp_topkp_phase);
  m.def("cosine_topk_workspace_bytes", &cosine_topk_workspace_bytes);
  m.def("cosine_topk", &cosine_topk);
  m.def("q16_topk_workspace_bytes", &q16_topk_workspace_bytes);
  m.def("q16_topk", &q16_topk);
  m.def("car_alloc", &car_alloc);
  m.def("car_open", &car_open);
  m.def("car_close", [](int64_t p) { return pa_car_close((void*)(uintptr_t)p); });
  m.def("car_free", [](int64_t p) { return pa_car_free((void*)(uintptr_t)p); });
  m.def("car_all_reduce", &car_all_reduce, py::arg("bases"), py::arg("rank0"), py::arg("ins"), py::arg("outs"),
        py::arg("cap_bytes"), py::arg("epochs"), py::arg("err"), py::arg("two_shot"),
        py::arg("resids") = std::vector<at::Tensor>(), py::arg("ss") = std::vector<at::Tensor>(),
        py::arg("ss_zero") = std::vector<at::Tensor>(), py::arg("row_len") = 0);
  m.def("car_collective", &car_collective, py::arg("bases"), py::arg("rank0"), py::arg("ins"), py::arg("outs"),
        py::arg("cap_bytes"), py::arg("epochs"), py::arg("err"), py::arg("op"));
  m.def("car_group", &pa_car_group);
  m.def("car_flag_bytes", &pa_car_flag_bytes);
  m.attr("ATT_PART") = 512;
  m.attr("SAMPLE_CHUNK") = 4096;
}
