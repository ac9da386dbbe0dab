// PyTorch bindings of the gfx950 kernel library (pybind11 + ATen).
// Shape / dtype / device checks live here so the .hip launchers stay raw and
// graph-capturable; every op runs on the current HIP stream of the tensor's
// device.
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <ATen/hip/HIPContext.h>

#include "kernels.h"

namespace {

inline hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

// Launch-error check after every kernel launch: hipGetLastError is a host-side
// query (no sync), so it is always on.  MCP_CHECK_LAUNCH=1 (the GPU tests set
// it) additionally synchronises the stream outside graph capture, so an
// asynchronous fault is reported by the op that caused it.
bool sync_check() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("MCP_CHECK_LAUNCH");
    on = e && e[0] == '1';
  }
  return on == 1;
}

void check_launch(const char* op) {
  hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, op, ": kernel launch failed: ", hipGetErrorString(e));
  if (!sync_check()) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream(), &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  e = hipStreamSynchronize(stream());
  TORCH_CHECK(e == hipSuccess, op, ": kernel failed: ", hipGetErrorString(e));
}

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_BF16_TENSOR(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_BF16(t)
#define CHECK_I32_TENSOR(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_I32(t)

// fused RMSNorm operands (kernels.h NormEpi): ss_out [M] int64 += the rows'
// sums of squares (residual GEMMs); ss_in [M] int64: rows scaled by
// rsqrt(ss_in / K + eps) (the GEMMs consuming the normed rows)
NormEpi make_norm_epi(int M, int K, const c10::optional<at::Tensor>& ss_out,
                      const c10::optional<at::Tensor>& ss_in, double eps) {
  NormEpi ne;
  for (const auto* t : {&ss_out, &ss_in}) {
    if (!t->has_value()) continue;
    CHECK_DEV((**t)); CHECK_CONTIG((**t));
    TORCH_CHECK((*t)->scalar_type() == at::kLong && (*t)->numel() >= M, "ss buffers: int64 [M]");
  }
  if (ss_out.has_value()) ne.ss_out = reinterpret_cast<unsigned long long*>(ss_out->data_ptr<int64_t>());
  if (ss_in.has_value()) ne.ss_in = reinterpret_cast<const unsigned long long*>(ss_in->data_ptr<int64_t>());
  ne.inv_h = 1.f / (float)K;
  ne.eps = (float)eps;
  return ne;
}

void rmsnorm(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, double eps) {
  CHECK_BF16_TENSOR(x); CHECK_BF16_TENSOR(w); CHECK_BF16_TENSOR(out);
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && w.numel() == H && out.sizes() == x.sizes(), "rmsnorm shapes");
  launch_rmsnorm(x.data_ptr(), w.data_ptr(), out.data_ptr(), x.numel() / H, H, (float)eps, stream());
  check_launch("rmsnorm");
}

void add_rmsnorm(const at::Tensor& x, at::Tensor& residual, const at::Tensor& w, at::Tensor& out,
                 double eps) {
  CHECK_BF16_TENSOR(x); CHECK_BF16_TENSOR(residual); CHECK_BF16_TENSOR(w); CHECK_BF16_TENSOR(out);
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && w.numel() == H && residual.sizes() == x.sizes() &&
              out.sizes() == x.sizes(), "add_rmsnorm shapes");
  launch_add_rmsnorm(x.data_ptr(), residual.data_ptr(), w.data_ptr(), out.data_ptr(),
                     x.numel() / H, H, (float)eps, stream());
  check_launch("add_rmsnorm");
}

void silu_mul(const at::Tensor& x, at::Tensor& y) {
  CHECK_BF16_TENSOR(x); CHECK_BF16_TENSOR(y);
  const int F = y.size(-1);
  TORCH_CHECK(F % 8 == 0 && x.size(-1) == 2 * F && x.numel() == 2 * y.numel(), "silu_mul shapes");
  launch_silu_mul(x.data_ptr(), y.data_ptr(), y.numel() / F, F, stream());
  check_launch("silu_mul");
}

void embedding(const at::Tensor& ids, const at::Tensor& table, at::Tensor& out) {
  CHECK_I32_TENSOR(ids); CHECK_BF16_TENSOR(table); CHECK_BF16_TENSOR(out);
  const int H = table.size(1);
  TORCH_CHECK(H % 8 == 0 && out.size(-1) == H && out.numel() == ids.numel() * H, "embedding shapes");
  launch_embedding(ids.data_ptr<int>(), table.data_ptr(), out.data_ptr(), ids.numel(), H, stream());
  check_launch("embedding");
}

void rope_kv(const at::Tensor& qkv, const at::Tensor& pos, const at::Tensor& slots,
             const at::Tensor& cos_sin, at::Tensor& q_out, at::Tensor& k_cache,
             at::Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t D) {
  CHECK_BF16_TENSOR(qkv); CHECK_I32_TENSOR(pos); CHECK_I32_TENSOR(slots);
  CHECK_BF16_TENSOR(q_out); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache);
  CHECK_DEV(cos_sin); CHECK_CONTIG(cos_sin);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.dim() == 3 &&
              cos_sin.size(1) == D / 2 && cos_sin.size(2) == 2, "cos_sin [P, D/2, 2] f32");
  const int T = pos.numel();
  TORCH_CHECK(qkv.numel() == (int64_t)T * (Hq + 2 * Hkv) * D, "qkv shape");
  TORCH_CHECK(q_out.numel() == (int64_t)T * Hq * D, "q_out shape");
  TORCH_CHECK(slots.numel() == T, "slots shape");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D, "cache [nb, Hkv, BS, D]");
  TORCH_CHECK(D == 128 || D == 64, "head_dim must be 64 or 128");
  launch_rope_kv(qkv.data_ptr(), pos.data_ptr<int>(), slots.data_ptr<int>(), cos_sin.data_ptr(),
                 q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), T, Hq, Hkv, D,
                 k_cache.size(2), stream());
  check_launch("rope_kv");
}

// QKV projection + RoPE + paged K/V write: fused in the GEMM epilogue when the
// AGPR kernel serves the shape, else GEMM into ``qkv`` (scratch) + rope_kv
int64_t qkv_rope_impl(const at::Tensor& X, const at::Tensor& W, at::Tensor& qkv, const at::Tensor& pos,
                      const at::Tensor& slots, const at::Tensor& cos_sin, at::Tensor& q_out,
                      at::Tensor& k_cache, at::Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t D,
                      const c10::optional<at::Tensor>& ss_in, double norm_eps, int64_t algo) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(qkv);
  CHECK_I32_TENSOR(pos); CHECK_I32_TENSOR(slots);
  CHECK_BF16_TENSOR(q_out); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache);
  CHECK_DEV(cos_sin); CHECK_CONTIG(cos_sin);
  const int K = X.size(-1), M = X.numel() / K, N = W.size(0);
  TORCH_CHECK(W.dim() == 2 && W.size(1) == K, "W must be [N, K]");
  TORCH_CHECK(N == (Hq + 2 * Hkv) * D, "W rows must be (Hq + 2 Hkv) * D");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.dim() == 3 &&
              cos_sin.size(1) == D / 2 && cos_sin.size(2) == 2, "cos_sin [P, D/2, 2] f32");
  TORCH_CHECK(pos.numel() == M && slots.numel() == M, "pos / slots: one per row of X");
  TORCH_CHECK(qkv.numel() == (int64_t)M * N, "qkv scratch [M, N]");
  TORCH_CHECK(q_out.numel() == (int64_t)M * Hq * D, "q_out shape");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D &&
              v_cache.sizes() == k_cache.sizes(), "cache [nb, Hkv, BS, D]");
  TORCH_CHECK(D == 128 || D == 64, "head_dim must be 64 or 128");
  TORCH_CHECK(gemm_tn_check(M, N, K) == 0, "qkv_rope: unsupported GEMM shape");
  RopeArgs ra{pos.data_ptr<int>(), slots.data_ptr<int>(), cos_sin.data_ptr<float>(),
              q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), (int)Hq, (int)Hkv,
              (int)k_cache.size(2)};
  NormEpiScope scope(make_norm_epi(M, K, c10::nullopt, ss_in, norm_eps));
  if (algo >= 0) {             // tuning / tests: one path by code, nonzero = not taken
    const int rc = launch_qkv_rope_algo(X.data_ptr(), W.data_ptr(), qkv.data_ptr(), M, N, K, (int)D,
                                        ra, (int)algo, stream());
    if (rc == 0) check_launch("qkv_rope_algo");
    return rc;
  }
  launch_qkv_rope(X.data_ptr(), W.data_ptr(), qkv.data_ptr(), M, N, K, (int)D, ra, stream());
  check_launch("qkv_rope");
  return 0;
}

void qkv_rope(const at::Tensor& X, const at::Tensor& W, at::Tensor& qkv, const at::Tensor& pos,
              const at::Tensor& slots, const at::Tensor& cos_sin, at::Tensor& q_out,
              at::Tensor& k_cache, at::Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t D,
              const c10::optional<at::Tensor>& ss_in, double norm_eps) {
  qkv_rope_impl(X, W, qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D, ss_in,
                norm_eps, -1);
}

int64_t qkv_rope_algo(const at::Tensor& X, const at::Tensor& W, at::Tensor& qkv,
                      const at::Tensor& pos, const at::Tensor& slots, const at::Tensor& cos_sin,
                      at::Tensor& q_out, at::Tensor& k_cache, at::Tensor& v_cache, int64_t Hq,
                      int64_t Hkv, int64_t D, int64_t algo, const c10::optional<at::Tensor>& ss_in,
                      double norm_eps) {
  TORCH_CHECK(algo >= 0, "qkv_rope_algo: algo >= 0");
  return qkv_rope_impl(X, W, qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D, ss_in,
                       norm_eps, algo);
}

void gemm_plan_set_rope_py(int64_t N, int64_t K, const std::vector<int64_t>& codes) {
  std::vector<int> c(codes.begin(), codes.end());
  for (int v : c)
    TORCH_CHECK(v == -1 || (v >= 1 && v <= 5) || v == 200 || v == 500 ||
                    (v >= 1000 && v < 1000 + 16 * 16),
                "gemm plan rope: -1 or a launch_qkv_rope_algo code");
  gemm_plan_set_rope((int)N, (int)K, c.data(), (int)c.size());
}

void row_sumsq(const at::Tensor& x, at::Tensor& ss) {
  CHECK_BF16_TENSOR(x); CHECK_DEV(ss); CHECK_CONTIG(ss);
  const int H = x.size(-1), T = x.numel() / H;
  TORCH_CHECK(H % 8 == 0 && ss.scalar_type() == at::kLong && ss.numel() >= T, "row_sumsq shapes");
  launch_row_sumsq(x.data_ptr(), reinterpret_cast<unsigned long long*>(ss.data_ptr<int64_t>()), T, H,
                   stream());
  check_launch("row_sumsq");
}

void gemm(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y, const c10::optional<at::Tensor>& R,
          int64_t algo, const c10::optional<at::Tensor>& ss_out) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(Y);
  const int K = X.size(-1);
  const int M = X.numel() / K;
  const int N = W.size(0);
  TORCH_CHECK(W.dim() == 2 && W.size(1) == K, "W must be [N, K]");
  TORCH_CHECK(Y.numel() == (int64_t)M * N && Y.size(-1) == N, "Y must be [M, N]");
  const int rc = gemm_tn_check(M, N, K);
  TORCH_CHECK(rc == 0, "gemm: unsupported shape M=", M, " N=", N, " K=", K, " (code ", rc, ")");
  const void* rp = nullptr;
  if (R.has_value()) {
    CHECK_BF16_TENSOR((*R));
    TORCH_CHECK(R->numel() == Y.numel(), "R shape");
    rp = R->data_ptr();
  }
  TORCH_CHECK(!ss_out.has_value() || rp, "ss_out (fused RMSNorm statistic) needs the residual R");
  NormEpiScope scope(make_norm_epi(M, K, ss_out, c10::nullopt, 0.0));
  launch_gemm_tn_algo(X.data_ptr(), W.data_ptr(), Y.data_ptr(), rp, M, N, K, (int)algo, stream());
  check_launch("gemm");
}

// read up to `nbytes` of W once on the current stream (MALL warm-up, prefetch.hip)
void weight_prefetch(const at::Tensor& W, int64_t nbytes, int64_t wgs, at::Tensor& sink) {
  TORCH_CHECK(W.is_cuda() && W.is_contiguous() && sink.is_cuda() && sink.dtype() == at::kInt &&
              sink.numel() >= 256, "weight_prefetch: contiguous device tensor and an int32 sink of >= 256");
  const int64_t total = W.numel() * W.element_size();
  const int64_t n = nbytes < 0 || nbytes > total ? total : nbytes;
  launch_prefetch(W.data_ptr(), (size_t)n, (int)wgs, sink.data_ptr<int>(), stream());
  check_launch("weight_prefetch");
}

void gemm_silu(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y,
               const c10::optional<at::Tensor>& ss_in, double norm_eps) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(Y);
  const int K = X.size(-1), M = X.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K && N % 64 == 0, "gemm_silu: W [N, K], N % 64 == 0");
  TORCH_CHECK(Y.numel() == (int64_t)M * (N / 2), "gemm_silu: Y [M, N/2]");
  TORCH_CHECK(gemm_tn_check(M, N, K) == 0, "gemm_silu: unsupported shape");
  NormEpiScope scope(make_norm_epi(M, K, c10::nullopt, ss_in, norm_eps));
  TORCH_CHECK(launch_gemm_silu(X.data_ptr(), W.data_ptr(), Y.data_ptr(), M, N, K, stream()) == 0,
              "gemm_silu failed");
  check_launch("gemm_silu");
}

// tuning / tests: one SwiGLU path by code (launch_gemm_silu_algo); returns
// nonzero (nothing launched) where the path does not take the shape
int64_t gemm_silu_algo(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y, int64_t algo,
                       const c10::optional<at::Tensor>& ss_in, double norm_eps) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(Y);
  const int K = X.size(-1), M = X.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K && N % 64 == 0, "gemm_silu_algo: W [N, K], N % 64 == 0");
  TORCH_CHECK(Y.numel() == (int64_t)M * (N / 2), "gemm_silu_algo: Y [M, N/2]");
  TORCH_CHECK(gemm_tn_check(M, N, K) == 0, "gemm_silu_algo: unsupported shape");
  NormEpiScope scope(make_norm_epi(M, K, c10::nullopt, ss_in, norm_eps));
  const int rc = launch_gemm_silu_algo(X.data_ptr(), W.data_ptr(), Y.data_ptr(), M, N, K, (int)algo,
                                       stream());
  if (rc == 0) check_launch("gemm_silu_algo");
  return rc;
}

void gemm_plan_set_silu_py(int64_t N, int64_t K, const std::vector<int64_t>& codes) {
  std::vector<int> c(codes.begin(), codes.end());
  for (int v : c)
    TORCH_CHECK(v == -1 || (v >= 1 && v <= 5) || (v >= 101 && v <= 116) || v == 200 ||
                    (v >= 300 && v < 364) || (v >= 400 && v <= 405) || (v >= 1000 && v < 1000 + 16 * 16),
                "gemm plan silu: -1 or a launch_gemm_silu_algo code");
  gemm_plan_set_silu((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_variant(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y, int64_t v) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(Y);
  const int K = X.size(-1), M = X.numel() / K, N = W.size(0);
  TORCH_CHECK(gemm_tn_check(M, N, K) == 0, "gemm_variant: unsupported shape");
  TORCH_CHECK(launch_gemm_tn_256_variant(X.data_ptr(), W.data_ptr(), Y.data_ptr(), M, N, K, v,
                                         stream()) == 0, "bad variant");
  check_launch("gemm_variant");
}

void gemm_plan_set_py(int64_t N, int64_t K, const std::vector<int64_t>& codes) {
  std::vector<int> c(codes.begin(), codes.end());
  for (int v : c) TORCH_CHECK(v >= -1 && v <= 5, "gemm plan code must be -1..5");
  gemm_plan_set((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_plan_set_splits_py(int64_t N, int64_t K, const std::vector<int64_t>& splits) {
  std::vector<int> c(splits.begin(), splits.end());
  for (int v : c) TORCH_CHECK(v >= 0 && v <= 16, "gemm plan split must be 0..16");
  gemm_plan_set_splits((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_plan_set_flex_py(int64_t N, int64_t K, const std::vector<int64_t>& flex) {
  std::vector<int> c(flex.begin(), flex.end());
  for (int v : c)
    TORCH_CHECK(v == -1 || (v & 31) < gemm_flex_count(), "gemm plan flex must be -1 or a candidate");
  gemm_plan_set_flex((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_plan_set_fsplit_py(int64_t N, int64_t K, const std::vector<int64_t>& fs) {
  std::vector<int> c(fs.begin(), fs.end());
  for (int v : c)
    TORCH_CHECK(v == -1 || (v >= 0 && v / 16 < 14 && v % 16 >= 2),
                "gemm plan fsplit must be -1 or 16 cand + S (cand < 14, S >= 2)");
  gemm_plan_set_fsplit((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_plan_set_group_py(int64_t N, int64_t K, const std::vector<int64_t>& group) {
  std::vector<int> c(group.begin(), group.end());
  for (int v : c) TORCH_CHECK(v >= 0 && v <= 64, "gemm plan group must be 0..64");
  gemm_plan_set_group((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_plan_set_persist_py(int64_t N, int64_t K, const std::vector<int64_t>& persist) {
  std::vector<int> c(persist.begin(), persist.end());
  for (int v : c) TORCH_CHECK(v == 0 || v == 1, "gemm plan persist must be 0 or 1");
  gemm_plan_set_persist((int)N, (int)K, c.data(), (int)c.size());
}

void gemm_f32out(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_DEV(Y); CHECK_CONTIG(Y);
  TORCH_CHECK(Y.scalar_type() == at::kFloat, "Y must be f32");
  const int K = X.size(-1), M = X.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K && Y.numel() == (int64_t)M * N, "gemm_f32out shapes");
  TORCH_CHECK(gemm_tn_check(M, N, K) == 0, "gemm_f32out: unsupported shape");
  launch_gemm_tn_f32out(X.data_ptr(), W.data_ptr(), Y.data_ptr<float>(), M, N, K, stream());
  check_launch("gemm_f32out");
}

void l2norm_rows(at::Tensor& x) {
  CHECK_BF16_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 8 == 0, "l2norm_rows: [N, D], D % 8 == 0");
  launch_l2norm_rows(x.data_ptr(), x.size(0), x.size(1), stream());
  check_launch("l2norm_rows");
}

void segment_topk(const at::Tensor& vals, const c10::optional<at::Tensor>& idx, int64_t seg_len,
                  int64_t k, at::Tensor& out_v, at::Tensor& out_i) {
  CHECK_DEV(vals); CHECK_CONTIG(vals);
  TORCH_CHECK(vals.scalar_type() == at::kFloat && vals.dim() == 2, "vals [B, L] f32");
  const int B = vals.size(0), L = vals.size(1);
  const int nseg = (L + seg_len - 1) / seg_len;
  TORCH_CHECK(out_v.numel() == (int64_t)B * nseg * k && out_i.numel() == out_v.numel(), "topk out shapes");
  const int* ip = nullptr;
  if (idx.has_value()) { CHECK_I32_TENSOR((*idx)); TORCH_CHECK(idx->numel() == vals.numel(), "idx shape"); ip = idx->data_ptr<int>(); }
  const int rc = launch_segment_topk(vals.data_ptr<float>(), ip, B, L, seg_len, k,
                                     out_v.data_ptr<float>(), out_i.data_ptr<int>(), stream());
  TORCH_CHECK(rc == 0, "segment_topk: seg_len <= 4096 and 0 < k <= seg_len");
  check_launch("segment_topk");
}

void topk_fused(const at::Tensor& Q, const at::Tensor& E, int64_t k, at::Tensor& cand_v,
                at::Tensor& cand_i) {
  CHECK_BF16_TENSOR(Q); CHECK_BF16_TENSOR(E);
  TORCH_CHECK(Q.dim() == 2 && E.dim() == 2 && Q.size(1) == E.size(1), "Q [B, D], E [N, D]");
  const int B = Q.size(0), N = E.size(0), D = Q.size(1);
  const int nseg = topk_fused_segments(N, B);
  TORCH_CHECK(cand_v.scalar_type() == at::kFloat && cand_v.is_contiguous() &&
              cand_v.numel() == (int64_t)B * nseg * k, "cand_v [B, nseg, k] f32");
  CHECK_I32_TENSOR(cand_i);
  TORCH_CHECK(cand_i.numel() == cand_v.numel(), "cand_i shape");
  const int rc = launch_topk_fused(Q.data_ptr(), E.data_ptr(), B, N, D, (int)k,
                                   cand_v.data_ptr<float>(), cand_i.data_ptr<int>(), stream());
  TORCH_CHECK(rc == 0, "topk_fused: B <= 64, k <= 64, D in {512, 1024} (code ", rc, ")");
  check_launch("topk_fused");
}

void paged_attention(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                     at::Tensor& out, const at::Tensor& q_start, const at::Tensor& q_len,
                     const at::Tensor& ctx_len, const at::Tensor& block_table,
                     const at::Tensor& work_seq, const at::Tensor& work_q0, int64_t nw,
                     double scale, const c10::optional<at::Tensor>& kv_begin,
                     const c10::optional<at::Tensor>& pre_o,
                     const c10::optional<at::Tensor>& pre_lse, int64_t nsplit,
                     const c10::optional<at::Tensor>& split_o,
                     const c10::optional<at::Tensor>& split_lse,
                     const c10::optional<at::Tensor>& own_lse) {
  CHECK_BF16_TENSOR(q); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache); CHECK_BF16_TENSOR(out);
  CHECK_I32_TENSOR(q_start); CHECK_I32_TENSOR(q_len); CHECK_I32_TENSOR(ctx_len);
  CHECK_I32_TENSOR(block_table); CHECK_I32_TENSOR(work_seq); CHECK_I32_TENSOR(work_q0);
  TORCH_CHECK(q.dim() == 3, "q must be [T, Hq, D]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 64, "cache block size must be 64");
  const int Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape");
  TORCH_CHECK(block_table.dim() == 2, "block_table [S, max_blocks]");
  TORCH_CHECK(work_seq.numel() == work_q0.numel(), "work list");
  if (nsplit > 1) {
    TORCH_CHECK(nw == 1 || nw == 4, "split-KV serves 1- and 4-wave items");
    TORCH_CHECK(split_o.has_value() && split_lse.has_value(), "split-KV needs split_o / split_lse");
    TORCH_CHECK(split_o->scalar_type() == at::kFloat && split_o->is_contiguous() &&
                split_o->numel() >= nsplit * q.numel(), "split_o [nsplit, T, Hq, D] f32");
    TORCH_CHECK(split_lse->scalar_type() == at::kFloat && split_lse->is_contiguous() &&
                split_lse->numel() >= nsplit * q.size(0) * Hq, "split_lse [nsplit, T, Hq] f32");
  }
  const int* kb = nullptr;
  const void* po = nullptr;
  const float* pl = nullptr;
  float* ol = nullptr;
  if (kv_begin.has_value()) {
    CHECK_I32_TENSOR((*kv_begin));
    TORCH_CHECK(kv_begin->numel() == q_len.numel(), "kv_begin [S]");
    kb = kv_begin->data_ptr<int>();
    if (own_lse.has_value()) {
      // concurrent cascade: own-key partial + its LSE, merged later (cascade_merge)
      TORCH_CHECK(own_lse->scalar_type() == at::kFloat && own_lse->is_contiguous() &&
                      own_lse->numel() == q.size(0) * Hq, "own_lse [T, Hq] f32");
      ol = own_lse->data_ptr<float>();
    } else {
      TORCH_CHECK(pre_o.has_value() && pre_lse.has_value(), "kv_begin needs pre_o / pre_lse or own_lse");
      CHECK_BF16_TENSOR((*pre_o));
      TORCH_CHECK(pre_o->sizes() == q.sizes(), "pre_o shape");
      TORCH_CHECK(pre_lse->scalar_type() == at::kFloat && pre_lse->numel() == q.size(0) * Hq, "pre_lse [T, Hq]");
      po = pre_o->data_ptr();
      pl = pre_lse->data_ptr<float>();
    }
  }
  const int rc = launch_paged_attention(
      q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), out.data_ptr(), q_start.data_ptr<int>(),
      q_len.data_ptr<int>(), ctx_len.data_ptr<int>(), block_table.data_ptr<int>(),
      block_table.size(1), work_seq.data_ptr<int>(), work_q0.data_ptr<int>(), work_seq.numel(), nw,
      Hq, Hkv, D, (float)scale, kb, po, pl, stream(), (int)nsplit,
      nsplit > 1 ? split_o->data_ptr<float>() : nullptr,
      nsplit > 1 ? split_lse->data_ptr<float>() : nullptr, (int)(q.size(0) * Hq), ol);
  TORCH_CHECK(rc == 0, "paged_attention: unsupported config (code ", rc, ")");
  check_launch("paged_attention");
}

// split-KV step as ONE launch (both work lists, combine fused); false = not
// launched (ticket / range limits), the caller runs the per-list path
bool paged_attention_mixed(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                           at::Tensor& out, const at::Tensor& q_start, const at::Tensor& q_len,
                           const at::Tensor& ctx_len, const at::Tensor& block_table,
                           const at::Tensor& work_seq4, const at::Tensor& work_q04,
                           const at::Tensor& work_seq1, const at::Tensor& work_q01, double scale,
                           int64_t nsplit, at::Tensor& split_o, at::Tensor& split_lse,
                           const c10::optional<at::Tensor>& kv_begin,
                           const c10::optional<at::Tensor>& pre_o,
                           const c10::optional<at::Tensor>& pre_lse,
                           const c10::optional<at::Tensor>& own_lse) {
  CHECK_BF16_TENSOR(q); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache); CHECK_BF16_TENSOR(out);
  CHECK_I32_TENSOR(q_start); CHECK_I32_TENSOR(q_len); CHECK_I32_TENSOR(ctx_len);
  CHECK_I32_TENSOR(block_table); CHECK_I32_TENSOR(work_seq4); CHECK_I32_TENSOR(work_q04);
  CHECK_I32_TENSOR(work_seq1); CHECK_I32_TENSOR(work_q01);
  TORCH_CHECK(q.dim() == 3, "q must be [T, Hq, D]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 64, "cache block size must be 64");
  const int Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape");
  TORCH_CHECK(block_table.dim() == 2, "block_table [S, max_blocks]");
  TORCH_CHECK(work_seq4.numel() == work_q04.numel() && work_seq1.numel() == work_q01.numel(),
              "work lists");
  TORCH_CHECK(nsplit >= 2, "mixed launch is the split-KV path");
  TORCH_CHECK(split_o.scalar_type() == at::kFloat && split_o.is_contiguous() &&
              split_o.numel() >= nsplit * q.numel(), "split_o [nsplit, T, Hq, D] f32");
  TORCH_CHECK(split_lse.scalar_type() == at::kFloat && split_lse.is_contiguous() &&
              split_lse.numel() >= nsplit * q.size(0) * Hq, "split_lse [nsplit, T, Hq] f32");
  const int* kb = nullptr;
  const void* po = nullptr;
  const float* pl = nullptr;
  float* ol = nullptr;
  if (kv_begin.has_value()) {
    CHECK_I32_TENSOR((*kv_begin));
    TORCH_CHECK(kv_begin->numel() == q_len.numel(), "kv_begin [S]");
    kb = kv_begin->data_ptr<int>();
    if (own_lse.has_value()) {
      TORCH_CHECK(own_lse->scalar_type() == at::kFloat && own_lse->is_contiguous() &&
                      own_lse->numel() == q.size(0) * Hq, "own_lse [T, Hq] f32");
      ol = own_lse->data_ptr<float>();
    } else {
      TORCH_CHECK(pre_o.has_value() && pre_lse.has_value(), "kv_begin needs pre_o / pre_lse or own_lse");
      CHECK_BF16_TENSOR((*pre_o));
      TORCH_CHECK(pre_o->sizes() == q.sizes(), "pre_o shape");
      TORCH_CHECK(pre_lse->scalar_type() == at::kFloat && pre_lse->numel() == q.size(0) * Hq, "pre_lse [T, Hq]");
      po = pre_o->data_ptr();
      pl = pre_lse->data_ptr<float>();
    }
  }
  const int rc = launch_paged_attention_mixed(
      q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), out.data_ptr(), q_start.data_ptr<int>(),
      q_len.data_ptr<int>(), ctx_len.data_ptr<int>(), block_table.data_ptr<int>(),
      block_table.size(1), work_seq4.data_ptr<int>(), work_q04.data_ptr<int>(), work_seq4.numel(),
      work_seq1.data_ptr<int>(), work_q01.data_ptr<int>(), work_seq1.numel(), Hq, Hkv, D,
      (float)scale, kb, po, pl, stream(), (int)nsplit, split_o.data_ptr<float>(),
      split_lse.data_ptr<float>(), (int)(q.size(0) * Hq), ol);
  TORCH_CHECK(rc != 1 && rc != 3 && rc != 4, "paged_attention_mixed: unsupported config (code ", rc, ")");
  if (rc != 0) return false;
  check_launch("paged_attention_mixed");
  return true;
}

// decode-sized split-KV step (attention_decode.hip); false = not launched
// (the caller takes the work-list split path)
bool paged_attention_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                            at::Tensor& out, const at::Tensor& q_start, const at::Tensor& q_len,
                            const at::Tensor& ctx_len, const at::Tensor& block_table,
                            const at::Tensor& work_seq4, const at::Tensor& work_q04,
                            const at::Tensor& work_seq1, const at::Tensor& work_q01, double scale,
                            int64_t nz, at::Tensor& split_o, at::Tensor& split_lse,
                            const c10::optional<at::Tensor>& kv_begin,
                            const c10::optional<at::Tensor>& pre_o,
                            const c10::optional<at::Tensor>& pre_lse, int64_t own_tiles) {
  CHECK_BF16_TENSOR(q); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache); CHECK_BF16_TENSOR(out);
  CHECK_I32_TENSOR(q_start); CHECK_I32_TENSOR(q_len); CHECK_I32_TENSOR(ctx_len);
  CHECK_I32_TENSOR(block_table); CHECK_I32_TENSOR(work_seq4); CHECK_I32_TENSOR(work_q04);
  CHECK_I32_TENSOR(work_seq1); CHECK_I32_TENSOR(work_q01);
  TORCH_CHECK(q.dim() == 3, "q must be [T, Hq, D]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 64, "cache block size must be 64");
  const int Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape");
  TORCH_CHECK(block_table.dim() == 2 && block_table.size(0) == q_len.numel(), "block_table [S, max_blocks]");
  TORCH_CHECK(work_seq4.numel() == work_q04.numel() && work_seq1.numel() == work_q01.numel(),
              "work lists");
  TORCH_CHECK(own_tiles >= 0 && own_tiles <= block_table.size(1), "own_tiles in [0, max_blocks]");
  TORCH_CHECK(nz == (own_tiles > 0 ? attn_decode_rel_blocks((int)own_tiles)
                                   : attn_decode_blocks(block_table.size(1))),
              "nz must be attn_decode_blocks(max_blocks), or attn_decode_rel_blocks(own_tiles)");
  TORCH_CHECK(split_o.scalar_type() == at::kFloat && split_o.is_contiguous() &&
              (nz == 1 || split_o.numel() >= nz * q.numel()), "split_o [nz, T, Hq, D] f32");
  TORCH_CHECK(split_lse.scalar_type() == at::kFloat && split_lse.is_contiguous() &&
              (nz == 1 || split_lse.numel() >= nz * q.size(0) * Hq), "split_lse [nz, T, Hq] f32");
  const int* kb = nullptr;
  const void* po = nullptr;
  const float* pl = nullptr;
  if (kv_begin.has_value()) {
    CHECK_I32_TENSOR((*kv_begin));
    TORCH_CHECK(kv_begin->numel() == q_len.numel(), "kv_begin [S]");
    TORCH_CHECK(pre_o.has_value() && pre_lse.has_value(), "kv_begin needs pre_o / pre_lse");
    CHECK_BF16_TENSOR((*pre_o));
    TORCH_CHECK(pre_o->sizes() == q.sizes(), "pre_o shape");
    TORCH_CHECK(pre_lse->scalar_type() == at::kFloat && pre_lse->numel() == q.size(0) * Hq, "pre_lse [T, Hq]");
    kb = kv_begin->data_ptr<int>();
    po = pre_o->data_ptr();
    pl = pre_lse->data_ptr<float>();
  }
  const int rc = launch_attn_decode(
      q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), out.data_ptr(), q_start.data_ptr<int>(),
      q_len.data_ptr<int>(), ctx_len.data_ptr<int>(), block_table.data_ptr<int>(),
      block_table.size(1), work_seq4.data_ptr<int>(), work_q04.data_ptr<int>(), work_seq4.numel(),
      work_seq1.data_ptr<int>(), work_q01.data_ptr<int>(), work_seq1.numel(), Hq, Hkv, D,
      (float)scale, kb, po, pl, split_o.data_ptr<float>(), split_lse.data_ptr<float>(),
      (int)(q.size(0) * Hq), (int)nz, stream(), (int)own_tiles);
  TORCH_CHECK(rc != 1 && rc != 3 && rc != 4, "paged_attention_decode: unsupported config (code ", rc, ")");
  if (rc != 0) return false;
  check_launch("paged_attention_decode");
  return true;
}

// K-half split AGPR GEMM (gemm256d.hip SPLIT 2), plain (R none) or + residual
// R; tests / tuning.  Returns the launcher's code (0 = launched)
int64_t gemm_split2(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y,
                    const c10::optional<at::Tensor>& R, int64_t bm) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(Y);
  const int M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K && Y.size(0) == M && Y.size(1) == N, "gemm_split2: X [M, K], W [N, K], Y [M, N]");
  if (R) {
    CHECK_BF16_TENSOR((*R));
    TORCH_CHECK(R->size(0) == M && R->size(1) == N, "gemm_split2: R [M, N]");
  }
  const int rc = launch_gemm_tn_256d_split2(X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                            R ? R->data_ptr() : nullptr, M, N, K, R ? 1 : 0, (int)bm,
                                            stream());
  if (rc == 0) check_launch("gemm_split2");
  return rc;
}

// GEMM power ladder rung (gemm256d.hip PROBE): Y [M, N] (epi 0) or [M, N/2] (epi 2)
void gemm_probe(const at::Tensor& X, const at::Tensor& W, at::Tensor& Y, int64_t epi, int64_t probe) {
  CHECK_BF16_TENSOR(X); CHECK_BF16_TENSOR(W); CHECK_BF16_TENSOR(Y);
  const int M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "W [N, K]");
  TORCH_CHECK(Y.size(0) == M && Y.size(1) == (epi == 2 ? N / 2 : N), "Y shape");
  const int rc = launch_gemm_probe(X.data_ptr(), W.data_ptr(), Y.data_ptr(), M, N, K, (int)epi,
                                   (int)probe, stream());
  TORCH_CHECK(rc == 0, "gemm_probe: M % 256, N % 256, K % 128, epi 0 / 2, probe 0-3");
  check_launch("gemm_probe");
}

// decode attention + o-projection in one launch (attention_decode.hip
// attn_oproj_kernel): out = attention, x += out Wo^T (in place) with the rows'
// fused-norm statistic added to ss_out; false = not launched (the caller runs
// paged_attention_decode and the GEMM apart)
bool paged_attention_decode_oproj(const at::Tensor& q, const at::Tensor& k_cache,
                                  const at::Tensor& v_cache, at::Tensor& out,
                                  const at::Tensor& q_start, const at::Tensor& q_len,
                                  const at::Tensor& ctx_len, const at::Tensor& block_table,
                                  const at::Tensor& work_seq4, const at::Tensor& work_q04,
                                  const at::Tensor& work_seq1, const at::Tensor& work_q01,
                                  double scale, int64_t nz, at::Tensor& split_o,
                                  at::Tensor& split_lse, const at::Tensor& wo, at::Tensor& x,
                                  const c10::optional<at::Tensor>& ss_out) {
  CHECK_BF16_TENSOR(q); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache); CHECK_BF16_TENSOR(out);
  CHECK_BF16_TENSOR(wo); CHECK_BF16_TENSOR(x);
  CHECK_I32_TENSOR(q_start); CHECK_I32_TENSOR(q_len); CHECK_I32_TENSOR(ctx_len);
  CHECK_I32_TENSOR(block_table); CHECK_I32_TENSOR(work_seq4); CHECK_I32_TENSOR(work_q04);
  CHECK_I32_TENSOR(work_seq1); CHECK_I32_TENSOR(work_q01);
  TORCH_CHECK(q.dim() == 3, "q must be [T, Hq, D]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 64, "cache block size must be 64");
  const int Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1);
  const int T = q.size(0);
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape");
  TORCH_CHECK(block_table.dim() == 2 && block_table.size(0) == q_len.numel(), "block_table [S, max_blocks]");
  TORCH_CHECK(work_seq4.numel() == work_q04.numel() && work_seq1.numel() == work_q01.numel(),
              "work lists");
  TORCH_CHECK(nz == attn_decode_blocks(block_table.size(1)), "nz must be attn_decode_blocks(max_blocks)");
  TORCH_CHECK(split_o.scalar_type() == at::kFloat && split_o.is_contiguous() &&
              (nz == 1 || split_o.numel() >= nz * q.numel()), "split_o [nz, T, Hq, D] f32");
  TORCH_CHECK(split_lse.scalar_type() == at::kFloat && split_lse.is_contiguous() &&
              (nz == 1 || split_lse.numel() >= nz * T * Hq), "split_lse [nz, T, Hq] f32");
  TORCH_CHECK(wo.dim() == 2 && wo.size(1) == (int64_t)Hq * D, "wo [N, Hq * D]");
  TORCH_CHECK(x.dim() == 2 && x.size(0) == T && x.size(1) == wo.size(0), "x [T, N]");
  unsigned long long* ss = nullptr;
  if (ss_out.has_value()) {
    TORCH_CHECK(ss_out->scalar_type() == at::kLong && ss_out->is_contiguous() && ss_out->numel() >= T,
                "ss_out int64 [>= T]");
    ss = reinterpret_cast<unsigned long long*>(ss_out->data_ptr<int64_t>());
  }
  const int rc = launch_attn_decode_oproj(
      q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), out.data_ptr(), q_start.data_ptr<int>(),
      q_len.data_ptr<int>(), ctx_len.data_ptr<int>(), block_table.data_ptr<int>(),
      block_table.size(1), work_seq4.data_ptr<int>(), work_q04.data_ptr<int>(), work_seq4.numel(),
      work_seq1.data_ptr<int>(), work_q01.data_ptr<int>(), work_seq1.numel(), Hq, Hkv, D,
      (float)scale, split_o.data_ptr<float>(), split_lse.data_ptr<float>(), T * Hq, (int)nz,
      wo.data_ptr(), x.data_ptr(), T, (int)wo.size(0), (int)wo.size(1), ss, stream());
  TORCH_CHECK(rc != 1 && rc != 3 && rc != 4, "paged_attention_decode_oproj: unsupported config (code ", rc, ")");
  if (rc != 0) return false;
  check_launch("paged_attention_decode_oproj");
  return true;
}

void cascade_merge(at::Tensor& out, const at::Tensor& own_lse, const at::Tensor& pre_o,
                   const at::Tensor& pre_lse, int64_t pre_tokens,
                   const c10::optional<at::Tensor>& pre_dims) {
  CHECK_BF16_TENSOR(out); CHECK_BF16_TENSOR(pre_o);
  TORCH_CHECK(out.dim() == 3 && pre_o.sizes() == out.sizes(), "out / pre_o [T, Hq, D]");
  const int Hq = out.size(1), D = out.size(2);
  TORCH_CHECK(own_lse.scalar_type() == at::kFloat && pre_lse.scalar_type() == at::kFloat &&
                  own_lse.numel() == out.size(0) * Hq && pre_lse.numel() == out.size(0) * Hq,
              "own_lse / pre_lse [T, Hq] f32");
  TORCH_CHECK(pre_tokens <= out.size(0), "pre_tokens");
  const int* dims = nullptr;
  if (pre_dims.has_value()) {
    CHECK_I32_TENSOR((*pre_dims));
    dims = pre_dims->data_ptr<int>();
  }
  const int rc = launch_cascade_merge(out.data_ptr(), own_lse.data_ptr<float>(), pre_o.data_ptr(),
                                      pre_lse.data_ptr<float>(), (int)pre_tokens, dims, Hq, D,
                                      stream());
  TORCH_CHECK(rc == 0, "cascade_merge: unsupported config (code ", rc, ")");
  check_launch("cascade_merge");
}

void prefix_attention(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                      at::Tensor& out, at::Tensor& lse, const at::Tensor& pre_bt, int64_t pre_keys,
                      int64_t pre_tokens, double scale,
                      const c10::optional<at::Tensor>& pre_dims, int64_t nsplit,
                      const c10::optional<at::Tensor>& split_o,
                      const c10::optional<at::Tensor>& split_lse) {
  CHECK_BF16_TENSOR(q); CHECK_BF16_TENSOR(k_cache); CHECK_BF16_TENSOR(v_cache); CHECK_BF16_TENSOR(out);
  CHECK_I32_TENSOR(pre_bt); CHECK_DEV(lse); CHECK_CONTIG(lse);
  TORCH_CHECK(lse.scalar_type() == at::kFloat, "lse f32");
  const int Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1);
  TORCH_CHECK(out.sizes() == q.sizes() && lse.numel() == q.size(0) * Hq, "prefix attention shapes");
  TORCH_CHECK(pre_tokens <= q.size(0) && pre_bt.numel() * 64 >= pre_keys, "prefix ranges");
  const int* dims = nullptr;
  if (pre_dims.has_value()) {
    // device-side [pre_tokens, pre_keys]: the kernel trusts pre_keys <= 64 *
    // pre_bt.numel(); the graph packer (engine/graphs.py) guarantees it
    CHECK_I32_TENSOR((*pre_dims));
    TORCH_CHECK(pre_dims->numel() == 2, "pre_dims [2]");
    dims = pre_dims->data_ptr<int>();
  }
  float* so = nullptr;
  float* sl = nullptr;
  if (nsplit > 1) {
    // fp32 partials [nsplit][pre_tokens][Hq][D] and LSE [nsplit][pre_tokens][Hq]
    TORCH_CHECK(split_o.has_value() && split_lse.has_value(), "split prefix needs split_o / split_lse");
    TORCH_CHECK(split_o->scalar_type() == at::kFloat && split_lse->scalar_type() == at::kFloat &&
                    split_o->is_contiguous() && split_lse->is_contiguous(), "split buffers f32");
    TORCH_CHECK(split_o->numel() >= nsplit * pre_tokens * Hq * D &&
                    split_lse->numel() >= nsplit * pre_tokens * Hq, "split buffer sizes");
    so = split_o->data_ptr<float>();
    sl = split_lse->data_ptr<float>();
  }
  const int rc = launch_prefix_attention(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                         out.data_ptr(), lse.data_ptr<float>(),
                                         pre_bt.data_ptr<int>(), pre_keys, pre_tokens, Hq, Hkv, D,
                                         (float)scale, stream(), dims, (int)nsplit, so, sl);
  TORCH_CHECK(rc == 0, "prefix_attention: unsupported config (code ", rc, ")");
  check_launch("prefix_attention");
}

void sample_allowed(const at::Tensor& hidden, const at::Tensor& W, const at::Tensor& allow_ptr,
                    const at::Tensor& allow_ids, const at::Tensor& ctr, double temperature,
                    int64_t seed, at::Tensor& out_tok, const c10::optional<at::Tensor>& out_logit) {
  CHECK_BF16_TENSOR(hidden); CHECK_BF16_TENSOR(W);
  CHECK_I32_TENSOR(allow_ptr); CHECK_I32_TENSOR(allow_ids); CHECK_I32_TENSOR(out_tok);
  CHECK_I32_TENSOR(ctr);
  const int S = hidden.size(0), H = hidden.size(1);
  TORCH_CHECK(W.size(1) == H && H % 8 == 0, "W [V, H]");
  TORCH_CHECK(allow_ptr.numel() == S + 1 && out_tok.numel() == S && ctr.numel() == S, "sample shapes");
  float* lp = nullptr;
  if (out_logit.has_value()) lp = out_logit->data_ptr<float>();
  launch_sample_allowed(hidden.data_ptr(), W.data_ptr(), allow_ptr.data_ptr<int>(),
                        allow_ids.data_ptr<int>(), ctr.data_ptr<int>(),
                        (float)temperature, (unsigned long long)seed, S, H,
                        out_tok.data_ptr<int>(), lp, stream());
  check_launch("sample_allowed");
}

void sample_dense(const at::Tensor& logits, const at::Tensor& ctr, double temperature,
                  int64_t seed, at::Tensor& out_tok) {
  CHECK_BF16_TENSOR(logits); CHECK_I32_TENSOR(out_tok);
  CHECK_I32_TENSOR(ctr);
  launch_sample_dense(logits.data_ptr(), logits.size(0), logits.size(1),
                      ctr.data_ptr<int>(), (float)temperature,
                      (unsigned long long)seed, out_tok.data_ptr<int>(), stream());
  check_launch("sample_dense");
}

// decision lookahead: the sampled outcome's tokens / sizes / allowed set into
// the next step's device views (sampling.hip).  The caller (engine
// _launch_branch) bounds every offset of ``tab`` against these views on the host.
void branch_select(const at::Tensor& prev_tok, const at::Tensor& tab, int64_t n, at::Tensor& ids,
                   at::Tensor& slots, at::Tensor& q_len, at::Tensor& ctx_len, at::Tensor& rows, at::Tensor& aptr,
                   at::Tensor& aids, at::Tensor& err) {
  CHECK_I32_TENSOR(prev_tok); CHECK_I32_TENSOR(tab); CHECK_I32_TENSOR(ids); CHECK_I32_TENSOR(slots);
  TORCH_CHECK(slots.numel() == ids.numel(), "branch_select: slots / ids");
  CHECK_I32_TENSOR(q_len); CHECK_I32_TENSOR(ctx_len); CHECK_I32_TENSOR(rows);
  CHECK_I32_TENSOR(aptr); CHECK_I32_TENSOR(aids); CHECK_I32_TENSOR(err);
  TORCH_CHECK(n >= 0 && q_len.numel() >= n && ctx_len.numel() >= n && rows.numel() >= n &&
              aptr.numel() >= n + 1 && tab.numel() >= 2 + 6 * n, "branch_select sizes");
  const int rc = launch_branch_select(prev_tok.data_ptr<int>(), tab.data_ptr<int>(), (int)n,
                                      ids.data_ptr<int>(), slots.data_ptr<int>(), q_len.data_ptr<int>(),
                                      ctx_len.data_ptr<int>(), rows.data_ptr<int>(),
                                      aptr.data_ptr<int>(), (int)aptr.numel(),
                                      aids.data_ptr<int>(), err.data_ptr<int>(), stream());
  TORCH_CHECK(rc == 0, "branch_select: too many sequences");
  check_launch("branch_select");
}

void copy_blocks(at::Tensor& data, const at::Tensor& src, const at::Tensor& dst) {
  CHECK_BF16_TENSOR(data); CHECK_I32_TENSOR(src); CHECK_I32_TENSOR(dst);
  TORCH_CHECK(data.dim() == 6, "kv data [L, 2, nb, Hkv, BS, D]");
  TORCH_CHECK(src.numel() == dst.numel(), "pairs");
  const int64_t block_elems = data.size(3) * data.size(4) * data.size(5);
  launch_copy_blocks(data.data_ptr(), src.data_ptr<int>(), dst.data_ptr<int>(), src.numel(),
                     data.size(0) * 2, data.size(2), block_elems, stream());
  check_launch("copy_blocks");
}

void add_inplace(at::Tensor& y, const at::Tensor& x) {
  CHECK_BF16_TENSOR(y); CHECK_BF16_TENSOR(x);
  TORCH_CHECK(y.numel() == x.numel() && y.numel() % 8 == 0, "add_inplace shapes");
  launch_add_inplace(y.data_ptr(), x.data_ptr(), y.numel(), stream());
  check_launch("add_inplace");
}

// ---- K12 custom all-reduce: the state is an opaque int64 handle on the Python side
int64_t car_init(int64_t rank, int64_t world, int64_t buf_bytes, at::Tensor& handles_out) {
  TORCH_CHECK(handles_out.device().is_cpu() && handles_out.scalar_type() == at::kByte &&
              handles_out.numel() == (int64_t)car_handle_bytes(), "handles_out: uint8 cpu");
  void* st = car_create(rank, world, buf_bytes, handles_out.data_ptr());
  TORCH_CHECK(st != nullptr, "custom all-reduce: allocation / IPC export failed");
  return (int64_t)(intptr_t)st;
}

void car_connect(int64_t h, const at::Tensor& all_handles) {
  TORCH_CHECK(all_handles.device().is_cpu() && all_handles.scalar_type() == at::kByte &&
              all_handles.is_contiguous(), "all_handles: uint8 cpu [world, handle_bytes]");
  const int rc = car_open((void*)(intptr_t)h, all_handles.data_ptr());
  TORCH_CHECK(rc == 0, "custom all-reduce: hipIpcOpenMemHandle failed (", rc, ")");
}

// ss (optional, int64 [>= rows]): also add each output row's fixed-point sum
// of squares (the fused RMSNorm statistic of the next layer); rows are the
// last dimension of inp
void comm_emulate(double us, int64_t nbytes, int64_t max_blocks) {
  TORCH_CHECK(launch_comm_emulate(us, nbytes, (int)max_blocks, stream()) == 0, "comm_emulate failed");
}

void car_run(int64_t h, const at::Tensor& inp, at::Tensor& out, int64_t mode, int64_t blocks,
             const c10::optional<at::Tensor>& ss) {
  CHECK_BF16_TENSOR(inp); CHECK_BF16_TENSOR(out);
  TORCH_CHECK(inp.numel() == out.numel(), "all-reduce shapes");
  unsigned long long* ssp = nullptr;
  int row_len = 0;
  if (ss && ss->defined()) {
    TORCH_CHECK(ss->is_cuda() && ss->scalar_type() == at::kLong && ss->is_contiguous(),
                "ss: int64 cuda contiguous");
    row_len = (int)inp.size(-1);
    TORCH_CHECK(ss->numel() >= inp.numel() / row_len, "ss: one entry per row");
    ssp = (unsigned long long*)ss->data_ptr();
  }
  const int rc = car_allreduce((void*)(intptr_t)h, inp.data_ptr(), out.data_ptr(), inp.numel(),
                               (int)mode, (int)blocks, stream(), ssp, row_len);
  TORCH_CHECK(rc == 0, "custom all-reduce launch failed (", rc, ")");
  check_launch("car_run");
}

// ---- K13 direct RCCL communicator: opaque int64 handle on the Python side
int rccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return 0;
    case at::kFloat: return 1;
    case at::kInt: return 2;
    case at::kHalf: return 3;
    default: TORCH_CHECK(false, "rccl: unsupported dtype");
  }
  return -1;
}

at::Tensor nccl_unique_id() {
  auto t = at::empty({(int64_t)rccl_unique_id_bytes()}, at::TensorOptions().dtype(at::kByte));
  TORCH_CHECK(rccl_get_unique_id(t.data_ptr()) == 0, "ncclGetUniqueId failed");
  return t;
}

int64_t nccl_init(int64_t world, int64_t rank, const at::Tensor& uid) {
  TORCH_CHECK(uid.device().is_cpu() && uid.numel() == (int64_t)rccl_unique_id_bytes(), "uid");
  void* c = rccl_init(world, rank, uid.data_ptr());
  TORCH_CHECK(c != nullptr, "ncclCommInitRank failed");
  return (int64_t)(intptr_t)c;
}

void nccl_all_reduce(int64_t comm, at::Tensor& t, int64_t op) {
  CHECK_DEV(t); CHECK_CONTIG(t);
  TORCH_CHECK(rccl_all_reduce((void*)(intptr_t)comm, t.data_ptr(), t.data_ptr(), t.numel(),
                              rccl_dtype(t), op, stream()) == 0,
              "ncclAllReduce: ", rccl_last_error((void*)(intptr_t)comm));
  check_launch("nccl_all_reduce");
}

void nccl_all_gather(int64_t comm, const at::Tensor& in, at::Tensor& out) {
  CHECK_DEV(in); CHECK_CONTIG(in); CHECK_DEV(out); CHECK_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && out.numel() % in.numel() == 0, "shapes");
  TORCH_CHECK(rccl_all_gather((void*)(intptr_t)comm, in.data_ptr(), out.data_ptr(), in.numel(),
                              rccl_dtype(in), stream()) == 0,
              "ncclAllGather: ", rccl_last_error((void*)(intptr_t)comm));
  check_launch("nccl_all_gather");
}

void nccl_reduce_scatter(int64_t comm, const at::Tensor& in, at::Tensor& out, int64_t op) {
  CHECK_DEV(in); CHECK_CONTIG(in); CHECK_DEV(out); CHECK_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && in.numel() % out.numel() == 0, "shapes");
  TORCH_CHECK(rccl_reduce_scatter((void*)(intptr_t)comm, in.data_ptr(), out.data_ptr(),
                                  out.numel(), rccl_dtype(in), op, stream()) == 0,
              "ncclReduceScatter: ", rccl_last_error((void*)(intptr_t)comm));
  check_launch("nccl_reduce_scatter");
}

void nccl_broadcast(int64_t comm, at::Tensor& t, int64_t root) {
  CHECK_DEV(t); CHECK_CONTIG(t);
  TORCH_CHECK(rccl_broadcast((void*)(intptr_t)comm, t.data_ptr(), t.numel(), rccl_dtype(t), root,
                             stream()) == 0,
              "ncclBroadcast: ", rccl_last_error((void*)(intptr_t)comm));
  check_launch("nccl_broadcast");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for the MCP planner engine";
  m.def("rmsnorm", &rmsnorm);
  m.def("add_rmsnorm", &add_rmsnorm);
  m.def("silu_mul", &silu_mul);
  m.def("embedding", &embedding);
  m.def("rope_kv", &rope_kv);
  m.def("gemm", &gemm, py::arg("X"), py::arg("W"), py::arg("Y"), py::arg("R") = py::none(),
        py::arg("algo") = -1, py::arg("ss_out") = py::none());
  m.def("row_sumsq", &row_sumsq, "per-row sum of squares, int64 fixed point (fused RMSNorm statistic)");
  m.def("gemm_select", &gemm_select);
  m.def("qkv_rope", &qkv_rope, py::arg("X"), py::arg("W"), py::arg("qkv"), py::arg("pos"),
        py::arg("slots"), py::arg("cos_sin"), py::arg("q_out"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"),
        py::arg("ss_in") = py::none(), py::arg("norm_eps") = 0.0);
  m.def("gemm_variant", &gemm_variant);
  m.def("gemm_plan_set", &gemm_plan_set_py, "measured tile plan for one (N, K): a code per 64-row M bucket");
  m.def("qkv_rope_algo", &qkv_rope_algo, "one QKV + RoPE path by code (tuning / tests)",
        py::arg("X"), py::arg("W"), py::arg("qkv"), py::arg("pos"), py::arg("slots"),
        py::arg("cos_sin"), py::arg("q_out"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("Hq"), py::arg("Hkv"), py::arg("D"), py::arg("algo"),
        py::arg("ss_in") = py::none(), py::arg("norm_eps") = 0.0);
  m.def("gemm_plan_set_rope", &gemm_plan_set_rope_py,
        "measured QKV + RoPE path per 64-row M bucket for one qkv (N, K) (-1: the rule)");
  m.def("gemm_plan_set_silu", &gemm_plan_set_silu_py,
        "measured SwiGLU path per 64-row M bucket for one gate|up (N, K) (-1: the rule)");
  m.def("gemm_silu_algo", &gemm_silu_algo, "one SwiGLU GEMM path by code (tuning / tests)",
        py::arg("X"), py::arg("W"), py::arg("Y"), py::arg("algo"), py::arg("ss_in") = py::none(),
        py::arg("norm_eps") = 0.0);
  m.def("gemm_plan_set_splits", &gemm_plan_set_splits_py,
        "measured split-K of the 128^2 path for one (N, K): a count per 64-row M bucket (0 = rule)");
  m.def("gemm_plan_split", &gemm_plan_split);
  m.def("gemm_plan_set_fsplit", &gemm_plan_set_fsplit_py,
        "measured flex tile with split-K per 64-row M bucket for one (N, K) (16 cand + S; -1 = none)");
  m.def("gemm_plan_fsplit", &gemm_plan_fsplit);
  m.def("gemm_plan_set_flex", &gemm_plan_set_flex_py,
        "measured flex tile per 64-row M bucket for one (N, K) (-1 = none; +32 = 4-stage form)");
  m.def("gemm_plan_flex", &gemm_plan_flex);
  m.def("gemm_plan_set_group", &gemm_plan_set_group_py,
        "measured tile group of the AGPR kernel per 64-row M bucket for one (N, K) (0 = default)");
  m.def("gemm_plan_group", &gemm_plan_group);
  m.def("gemm_group_force", &gemm_group_force, "AGPR kernel tile group: 0 = plan / default 4");
  m.def("gemm256d_group", &gemm256d_group);
  m.def("gemm_plan_set_persist", &gemm_plan_set_persist_py,
        "per 64-row M bucket for one (N, K): 1 = the persistent AGPR kernel measured faster");
  m.def("gemm_plan_persist", &gemm_plan_persist);
  m.def("gemm256d_persist", &gemm256d_persist,
        "1 if an AGPR GEMM of this shape and tile count runs the persistent form");
  m.def("gemm_persist_force", &gemm_persist_force,
        "persistent AGPR GEMM: -1 plan / MCP_GEMM_PERSIST, 0 off, 1 when tiles > CUs, 2 always");
  m.def("gemm_wide_force", &gemm_wide_force,
        "AGPR GEMM epilogue: -1 MCP_GEMM_WIDE_EPI, 0 LDS-staged, 1 wide direct (permlane16 + 16-B stores)");
  m.def("gemm_plan_clear", &gemm_plan_clear);
  m.def("gemm_flex_count", &gemm_flex_count, "flex tile candidates (gemm(..., algo=16 + i))");
  m.def("gemm_flex_silu_ok", &gemm_flex_silu_ok, "1 if flex candidate i has the SwiGLU epilogue");
  m.def("gemm_flex_tiles", &gemm_flex_tiles, py::arg("cand"), py::arg("M"), py::arg("N"));
  m.def("gemm_plan_lookup", &gemm_plan_lookup);
  m.def("gemm_splitk_init", [](int64_t bytes) { return gemm_splitk_init((size_t)bytes); },
        "allocate the split-K fp32 workspace (call outside graph capture)");
  m.def("gemm128_splits", &gemm128_splits);
  m.def("gemm_stream_force_splits", &gemm_stream_force_splits, "split count of the K2 stream kernel: 0 auto");
  m.def("gemm_stream_splits", &gemm_stream_splits);
  m.def("gemm_splitk_force", &gemm_splitk_force, "split-K count of the 128^2 path: -1 auto, <= 1 off, S forced");
  m.def("gemm_skinny_half", &gemm_skinny_half, "SwiGLU skinny form: 8 gate + 8 up rows per block at M <= 4 (1, default), always (2), never (0: 32-row blocks)");
  m.def("weight_prefetch", &weight_prefetch, py::arg("W"), py::arg("nbytes"), py::arg("wgs"), py::arg("sink"),
        "read up to nbytes of W once on the current stream (Infinity Cache warm-up)");
  m.def("gemm_silu", &gemm_silu, py::arg("X"), py::arg("W"), py::arg("Y"),
        py::arg("ss_in") = py::none(), py::arg("norm_eps") = 0.0);
  m.def("gemm_f32out", &gemm_f32out);
  m.def("l2norm_rows", &l2norm_rows);
  m.def("topk_fused", &topk_fused, py::arg("Q"), py::arg("E"), py::arg("k"), py::arg("cand_v"),
        py::arg("cand_i"));
  m.def("topk_fused_segments", &topk_fused_segments, py::arg("N"), py::arg("B") = 1);
  m.def("segment_topk", &segment_topk, py::arg("vals"), py::arg("idx"), py::arg("seg_len"),
        py::arg("k"), py::arg("out_v"), py::arg("out_i"));
  m.def("paged_attention", &paged_attention, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("out"), py::arg("q_start"), py::arg("q_len"), py::arg("ctx_len"),
        py::arg("block_table"), py::arg("work_seq"), py::arg("work_q0"), py::arg("nw"),
        py::arg("scale"), py::arg("kv_begin") = py::none(), py::arg("pre_o") = py::none(),
        py::arg("pre_lse") = py::none(), py::arg("nsplit") = 1, py::arg("split_o") = py::none(),
        py::arg("split_lse") = py::none(), py::arg("own_lse") = py::none());
  m.def("paged_attention_mixed", &paged_attention_mixed, py::arg("q"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("out"), py::arg("q_start"), py::arg("q_len"), py::arg("ctx_len"),
        py::arg("block_table"), py::arg("work_seq4"), py::arg("work_q04"), py::arg("work_seq1"),
        py::arg("work_q01"), py::arg("scale"), py::arg("nsplit"), py::arg("split_o"),
        py::arg("split_lse"), py::arg("kv_begin") = py::none(), py::arg("pre_o") = py::none(),
        py::arg("pre_lse") = py::none(), py::arg("own_lse") = py::none(),
        "split-KV attention step in one launch (both work lists, combine fused); False = not launched");
  m.def("attn_split_init", &attn_split_init, "allocate the fused split-KV tickets (outside graph capture)");
  m.def("cascade_merge", &cascade_merge, py::arg("out"), py::arg("own_lse"), py::arg("pre_o"),
        py::arg("pre_lse"), py::arg("pre_tokens"), py::arg("pre_dims") = py::none());
  m.def("prefix_attention", &prefix_attention, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("out"), py::arg("lse"), py::arg("pre_bt"), py::arg("pre_keys"),
        py::arg("pre_tokens"), py::arg("scale"), py::arg("pre_dims") = py::none(),
        py::arg("nsplit") = 1, py::arg("split_o") = py::none(), py::arg("split_lse") = py::none());
  m.def("attn_tokens_per_item", &attn_tokens_per_item);
  m.def("sample_allowed", &sample_allowed, py::arg("hidden"), py::arg("W"), py::arg("allow_ptr"),
        py::arg("allow_ids"), py::arg("ctr"), py::arg("temperature"), py::arg("seed"),
        py::arg("out_tok"), py::arg("out_logit") = py::none());
  m.def("sample_dense", &sample_dense);
  m.def("branch_select", &branch_select);
  m.def("add_inplace", &add_inplace);
  m.def("paged_attention_decode_oproj", &paged_attention_decode_oproj,
        "decode attention + o-projection (x += out Wo^T, in place) in one launch; false: not launched",
        py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("out"), py::arg("q_start"),
        py::arg("q_len"), py::arg("ctx_len"), py::arg("block_table"), py::arg("work_seq4"),
        py::arg("work_q04"), py::arg("work_seq1"), py::arg("work_q01"), py::arg("scale"),
        py::arg("nz"), py::arg("split_o"), py::arg("split_lse"), py::arg("wo"), py::arg("x"),
        py::arg("ss_out") = py::none());
  m.def("attn_lazy_rescale", &attn_lazy_rescale, "shared-prefix attention: lazy max rescaling on / off");
  m.def("gemm_pf_force", &gemm_pf_force, "split-form W L2 fills ahead of the DMA: -1 = MCP_GEMM_PF, 0 off, 1 on");
  m.def("gemm_split2", &gemm_split2, "AGPR GEMM, K halves over two workgroups per tile (tests / tuning)",
        py::arg("X"), py::arg("W"), py::arg("Y"), py::arg("R") = py::none(), py::arg("bm") = 256);
  m.def("gemm_probe", &gemm_probe, "GEMM power-ladder rung (gemm256d.hip PROBE 0-3)");
  m.def("attn_oproj_error", &attn_oproj_error, "nonzero: a fused o-projection wait timed out");
  m.def("attn_decode_blocks", &attn_decode_blocks, "grid z of paged_attention_decode for a table width");
  m.def("paged_attention_decode", &paged_attention_decode, py::arg("q"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("out"), py::arg("q_start"), py::arg("q_len"), py::arg("ctx_len"),
        py::arg("block_table"), py::arg("work_seq4"), py::arg("work_q04"), py::arg("work_seq1"),
        py::arg("work_q01"), py::arg("scale"), py::arg("nz"), py::arg("split_o"),
        py::arg("split_lse"), py::arg("kv_begin") = py::none(), py::arg("pre_o") = py::none(),
        py::arg("pre_lse") = py::none(), py::arg("own_tiles") = 0);
  m.def("attn_decode_rel_blocks", &attn_decode_rel_blocks,
        "grid z of paged_attention_decode in own-span mode (own_tiles > 0)");
  m.def("copy_blocks", &copy_blocks);
  m.def("car_handle_bytes", []() { return (int64_t)car_handle_bytes(); });
  m.def("car_init", &car_init);
  m.def("car_connect", &car_connect);
  m.def("comm_emulate", &comm_emulate, "hold a K12 call's CUs for us microseconds (TP simulation)",
        py::arg("us"), py::arg("nbytes"), py::arg("max_blocks") = 0);
  m.def("car_run", &car_run, py::arg("h"), py::arg("inp"), py::arg("out"), py::arg("mode"),
        py::arg("blocks"), py::arg("ss") = py::none());
  m.def("car_error", [](int64_t h) { return car_error((void*)(intptr_t)h); });
  m.def("car_destroy", [](int64_t h) { car_destroy((void*)(intptr_t)h); });
  m.def("nccl_unique_id", &nccl_unique_id);
  m.def("nccl_init", &nccl_init);
  m.def("nccl_all_reduce", &nccl_all_reduce);
  m.def("nccl_all_gather", &nccl_all_gather);
  m.def("nccl_reduce_scatter", &nccl_reduce_scatter);
  m.def("nccl_broadcast", &nccl_broadcast);
  m.def("nccl_destroy", [](int64_t c) { rccl_destroy((void*)(intptr_t)c); });
}
