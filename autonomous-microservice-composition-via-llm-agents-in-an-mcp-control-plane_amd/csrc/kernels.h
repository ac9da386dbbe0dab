// Host-side launch API of the gfx950 kernel library.  Every launcher takes raw
// device pointers and a HIP stream, performs no allocation and no host sync,
// so all of them are safe inside hipGraph stream capture.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

// RMSNorm fused into the GEMM epilogues (TP = 1 forward, models/llama.py):
// the residual projections (EPI 1) add the sum of squares of every bf16 row
// they write to ss_out[row] (atomic), and the projections that consume a
// normed activation (SwiGLU EPI 2, QKV + RoPE EPI 3, rope_kv) scale each row
// of their fp32 accumulators by rsqrt(ss_in[row] * inv_h + eps) - the norm's
// per-column weight is folded into those weights once at load.  Set for the
// duration of one launcher call (NormEpiScope); every kernel launcher copies
// it into its kernel's arguments, so it is safe under hipGraph capture.
struct NormEpi {
  unsigned long long* ss_out = nullptr;     // [M] fixed point (common.h SS_FIX), zeroed by the caller
  const unsigned long long* ss_in = nullptr;
  float inv_h = 0.f, eps = 0.f;
};
NormEpi& norm_epi();                     // the current launch's (host, not thread-shared)
struct NormEpiScope {
  NormEpi saved;
  explicit NormEpiScope(const NormEpi& ne) : saved(norm_epi()) { norm_epi() = ne; }
  ~NormEpiScope() { norm_epi() = saved; }
};

// elementwise.hip
// per-row sum of squares (ss[t] = sum_h x[t, h]^2, NormEpi fixed point) of a bf16 [T, H] matrix
void launch_row_sumsq(const void* x, unsigned long long* ss, int T, int H, hipStream_t s);
void launch_rmsnorm(const void* x, const void* w, void* out, int T, int H, float eps,
                    hipStream_t s);
void launch_add_rmsnorm(const void* x, void* residual, const void* w, void* out, int T, int H,
                        float eps, hipStream_t s);
void launch_silu_mul(const void* x, void* y, int T, int F, hipStream_t s);
void launch_embedding(const int* ids, const void* table, void* out, int T, int H, hipStream_t s);
void launch_rope_kv(const void* qkv, const int* pos, const int* slots, const void* cos_sin,
                    void* q_out, void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D,
                    int BS, hipStream_t s);
void launch_add_inplace(void* y, const void* x, size_t n, hipStream_t s);

// QKV projection + RoPE + paged K/V write fused in the GEMM epilogue (K1+K4+K10)
// serving-size M: tile shape per (M, N) filling one wave of workgroups (gemm_flex.hip)
int launch_gemm_flex(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                     int cand, hipStream_t s);
int launch_gemm_flex_epi(const void* X, const void* W, void* Y, const void* R, int M, int N,
                         int K, int cand, int epi, hipStream_t s);   // epi 2: SwiGLU
int gemm_flex_silu_ok(int cand);
int gemm_flex_count();
void gemm_plan_set_flex(int N, int K, const int* flex, int n);
int gemm_plan_flex(int M, int N, int K);
void gemm_plan_set_group(int N, int K, const int* group, int n);
int gemm_plan_group(int M, int N, int K);   // 0 = none recorded
void gemm_group_force(int g);               // AGPR kernel tile group: 0 = plan / default
int gemm256d_group(int M, int N, int K);
void gemm_plan_set_persist(int N, int K, const int* persist, int n);
int gemm_plan_persist(int M, int N, int K);  // 1 = the persistent AGPR kernel measured faster
void gemm_wide_force(int w);                // AGPR kernel epilogue: -1 env, 0 staged, 1 wide direct
bool gemm_wide_on(int M, int N, int epi);   // that choice for one shape (EPI 0-2)
void gemm_persist_force(int p);             // -1 plan / env, 0 off, 1 multi-wave, 2 always
int gemm256d_persist(int M, int N, int K, int tiles);
struct RopeArgs;
// gemm256p.hip: persistent AGPR GEMM (grid = min(tiles, cus))
int launch_gemm_tn_256p(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        int epi, int bm, int cus, int group, const RopeArgs& ra, hipStream_t s);
int gemm_flex_tiles(int cand, int M, int N);
struct RopeArgs {
  const int* pos;          // [T] positions
  const int* slots;        // [T] KV-cache slots (-1: no write)
  const float* cos_sin;    // [P, D/2, 2]
  void* q_out;             // [T, Hq, D]
  void* k_cache;           // [nb, Hkv, BS, D]
  void* v_cache;
  int Hq, Hkv, BS;
};
// fused when the AGPR GEMM serves the shape (D = 128), else GEMM into qkv + rope_kv
void launch_qkv_rope(const void* X, const void* W, void* qkv, int M, int N, int K, int D,
                     const RopeArgs& ra, hipStream_t s);
void launch_copy_blocks(void* data, const int* src, const int* dst, int npairs, int layers2,
                        int nb, int block_elems, hipStream_t s);

// gemm_skinny.hip (K2): decode-sized M, weight-streaming; epi 0 plain, 1 +R, 2 SwiGLU
#define SKINNY_MAX_M 128
void gemm_skinny_half(int on);   // SwiGLU skinny form: 8+8-row blocks at M <= 4 (1), always (2), never (0)
int gemm_stream_rule();          // 1: round-4 stream split rule / skinny-first test, 0: round 3
int skinny_ok(int M, int N, int K, int epi);
int launch_gemm_skinny(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                       int epi, hipStream_t s);

// gemm_stream.hip (K2 proper): weight streaming for M <= 128, register-ring
// prefetch, fused split-K reduction; epi 0 plain, 1 +R, 2 SwiGLU, 3 QKV+RoPE+KV
#define GEMM_STREAM_MAX_M 128
int gemm_stream_ok(int M, int N, int K, int epi, int D, int Hq, int Hkv);
int gemm_stream_splits(int M, int N, int K, int epi);
void gemm_stream_force_splits(int S);   // 0 = auto
int launch_gemm_stream(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                       int epi, const RopeArgs& ra, hipStream_t s);
int gemm_stream_enabled();
// production routing: the measured (M, N, K, epi) range where it beats the
// 128^2 split-K path (profiles/gemm_stream_sweep.md)
bool gemm_stream_pick(int M, int N, int K, int epi);

// gemm.hip
int gemm256_num_cus();
// the split-K workspace (fp32 partial tiles) and per-tile tickets, allocated at
// library load; false when a launch would not fit
bool gemm_splitk_workspace(float** ws, int** tickets, size_t bytes, size_t tiles);
int gemm_tn_check(int M, int N, int K);
void launch_gemm_tn(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                    hipStream_t s);
void launch_gemm_tn_256(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        hipStream_t s);
// algo: -1 auto, 0 = 128x128 two-barrier kernel, 1 = 256x256 multi-phase kernel, 2 = skinny (K2)
int gemm_select(int M, int N, int K);
int gemm_plan_lookup(int M, int N, int K);
int gemm_splitk_init(size_t bytes);
int gemm128_splits(int M, int N, int K);
void gemm_splitk_force(int S);   // -1 auto, 0/1 off, S > 1 forced where admissible
void gemm_plan_set(int N, int K, const int* codes, int n);
void gemm_plan_set_splits(int N, int K, const int* splits, int n);
int gemm_plan_split(int M, int N, int K);
void gemm_plan_clear();
int gemm256d_ok(int M, int N, int K);
int gemm256d_code_height(int code);     // plan code 1..5 -> AGPR tile height (0: none)
// timing / power ladder of the 256-row AGPR kernel (tools/gemm_power_ladder.py):
// probe 0 production, 1 MFMA only, 2 + ds_read + barriers, 3 + LDS-DMA (no stores)
int launch_gemm_probe(const void* X, const void* W, void* Y, int M, int N, int K, int epi,
                      int probe, hipStream_t s);
// K-half split form (gemm256d.hip SPLIT 2): two workgroups per tile
void gemm_pf_force(int p);                           // W L2 fills in the split form: -1 env, 0 / 1
int launch_gemm_tn_256d_split2(const void* X, const void* W, void* Y, const void* R, int M, int N,
                               int K, int epi, int bm, hipStream_t s);
int launch_gemm_tn_256d_bm(const void* X, const void* W, void* Y, const void* R, int M, int N,
                           int K, int epi, int bm, hipStream_t s);
// Y[M, N/2] = silu(X W_g^T) * (X W_u^T), W rows interleaved [gate 16 | up 16]
int launch_gemm_silu(const void* X, const void* W, void* Y, int M, int N, int K, hipStream_t s);
// one SwiGLU path by code (gemm.hip: AGPR height, 128^2 x split, stream, flex, flex x split)
int launch_gemm_silu_algo(const void* X, const void* W, void* Y, int M, int N, int K, int algo,
                          hipStream_t s);
void gemm_plan_set_silu(int N, int K, const int* codes, int n);
int gemm_plan_silu(int M, int N, int K);
int launch_gemm_tn_256_variant(const void* X, const void* W, void* Y, int M, int N, int K, int v,
                               hipStream_t s);
void launch_gemm_tn_algo(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                         int algo, hipStream_t s);
void launch_gemm_tn_f32out(const void* X, const void* W, float* Y, int M, int N, int K,
                           hipStream_t s);

// topk.hip
void launch_l2norm_rows(void* x, int N, int D, hipStream_t s);
// fused scoring + per-segment top-k: cand [B, topk_fused_segments(N, B), k]
int topk_fused_segments(int N, int B = 1);
int launch_topk_fused(const void* Q, const void* E, int B, int N, int D, int k, float* cand_v,
                      int* cand_i, hipStream_t s);
int launch_segment_topk(const float* vals, const int* idx_in, int B, int L, int seg_len, int k,
                        float* out_v, int* out_i, hipStream_t s);

// attention.hip
int attn_tokens_per_item(int nw, int group);
int launch_paged_attention(const void* q, const void* k_cache, const void* v_cache, void* out,
                           const int* q_start, const int* q_len, const int* ctx_len,
                           const int* block_table, int max_blocks, const int* work_seq,
                           const int* work_q0, int nwork, int nw, int Hq, int Hkv, int head_dim,
                           float scale, const int* kv_begin, const void* pre_o,
                           const float* pre_lse, hipStream_t s, int nsplit = 1,
                           float* split_o = nullptr, float* split_lse = nullptr, int rows = 0,
                           float* own_lse = nullptr);
int attn_split_init();
void attn_lazy_rescale(int on);   // shared-prefix pass: lazy max rescaling (1) or exact (0)
// decode-sized split-KV steps (attention_decode.hip): grid (items, Hkv, nz),
// nz = attn_decode_blocks(max_blocks); nonzero = not launched
int attn_decode_blocks(int max_blocks);
int launch_attn_decode(const void* q, const void* k_cache, const void* v_cache, void* out,
                       const int* q_start, const int* q_len, const int* ctx_len,
                       const int* block_table, int max_blocks, const int* work_seq4,
                       const int* work_q04, int nwork4, const int* work_seq1, const int* work_q01,
                       int nwork1, int Hq, int Hkv, int head_dim, float scale, const int* kv_begin,
                       const void* pre_o, const float* pre_lse, float* split_o, float* split_lse,
                       int rows, int nz, hipStream_t s, int own_tiles = 0);
int attn_decode_rel_blocks(int own_tiles);   // grid z of the own-span mode
// the decode attention and the o-projection (x += out Wo^T, fused-norm
// statistic) in one launch; nonzero = not launched (shape outside the form)
int launch_attn_decode_oproj(const void* q, const void* k_cache, const void* v_cache, void* out,
                             const int* q_start, const int* q_len, const int* ctx_len,
                             const int* block_table, int max_blocks, const int* work_seq4,
                             const int* work_q04, int nwork4, const int* work_seq1,
                             const int* work_q01, int nwork1, int Hq, int Hkv, int head_dim,
                             float scale, float* split_o, float* split_lse, int rows, int nz,
                             const void* Wo, void* x, int M, int N, int K,
                             unsigned long long* ss_out, hipStream_t s);
int attn_oproj_error();
int launch_paged_attention_mixed(const void* q, const void* k_cache, const void* v_cache,
                                 void* out, const int* q_start, const int* q_len,
                                 const int* ctx_len, const int* block_table, int max_blocks,
                                 const int* work_seq4, const int* work_q04, int nwork4,
                                 const int* work_seq1, const int* work_q01, int nwork1, int Hq,
                                 int Hkv, int head_dim, float scale, const int* kv_begin,
                                 const void* pre_o, const float* pre_lse, hipStream_t s,
                                 int nsplit, float* split_o, float* split_lse, int rows,
                                 float* own_lse);
int launch_cascade_merge(void* out, const float* own_lse, const void* pre_o, const float* pre_lse,
                         int pre_tokens, const int* pre_dims, int Hq, int head_dim, hipStream_t s);
int launch_prefix_attention(const void* q, const void* k_cache, const void* v_cache, void* out,
                            float* lse_out, const int* pre_bt, int pre_keys, int pre_tokens,
                            int Hq, int Hkv, int head_dim, float scale, hipStream_t s,
                            const int* pre_dims = nullptr, int nsplit = 1,
                            float* split_o = nullptr, float* split_lse = nullptr);

// sampling.hip
void launch_sample_allowed(const void* hidden, const void* W, const int* allow_ptr,
                           const int* allow_ids, const int* ctr, float temperature,
                           unsigned long long seed, int S, int H, int* out_tok, float* out_logit,
                           hipStream_t s);
void launch_sample_dense(const void* logits, int S, int V, const int* ctr, float temperature,
                         unsigned long long seed, int* out_tok, hipStream_t s);
int launch_branch_select(const int* prev_tok, const int* tab, int n, int* ids, int* slots, int* q_len,
                         int* ctx_len, int* rows, int* aptr, int aptr_len, int* aids, int* err,
                         hipStream_t s);

// custom_allreduce.hip (K12): opaque state handle, IPC handles exchanged by the caller
size_t car_handle_bytes();
void* car_create(int rank, int world, size_t buf_bytes, void* handles_out);
int car_open(void* state, const void* all_handles);
// emulated K12 call: its block count, resident for ``us`` (bench_tp --emulate-comm)
int launch_comm_emulate(double us, long long nbytes, int max_blocks, hipStream_t s);
int car_allreduce(void* state, const void* inp, void* out, long long n_elems, int mode,
                  int blocks, hipStream_t s, unsigned long long* ss = nullptr, int row_len = 0);
int car_error(void* state);
void car_destroy(void* state);

// rccl_comm.hip (K13): direct rccl.h wrapper; dtype 0 bf16, 1 f32, 2 i32, 3 f16; op 0 sum, 1 max, 2 min
size_t rccl_unique_id_bytes();
int rccl_get_unique_id(void* out);
void* rccl_init(int world, int rank, const void* unique_id);
int rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                    hipStream_t s);
int rccl_all_gather(void* comm, const void* send, void* recv, size_t count, int dtype,
                    hipStream_t s);
int rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                        hipStream_t s);
int rccl_broadcast(void* comm, void* buf, size_t count, int dtype, int root, hipStream_t s);
const char* rccl_last_error(void* comm);
void rccl_destroy(void* comm);

// prefetch.hip: read a weight range once (MALL warm-up beside latency-bound work)
int launch_prefetch(const void* p, size_t bytes, int wgs, int* sink, hipStream_t s);
// gemm_flex.hip: fp32 split-K partials of a flex tile (candidates 0..11 as
// the flex list; 12 = 256 x 64, 13 = 192 x 64: split-only whole-M tiles)
int launch_gemm_flex_partials(const void* X, const void* W, float* ws, int M, int N, int K,
                              int cand, int S, hipStream_t s);
void gemm_plan_set_fsplit(int N, int K, const int* fs, int n);
int gemm_plan_fsplit(int M, int N, int K);
int launch_gemm_flex_split(const void* X, const void* W, void* Y, const void* R, int M, int N,
                           int K, int cand, int S, int epi, hipStream_t s);
int launch_qkv_rope_fsplit(const void* X, const void* W, int M, int N, int K, int D,
                           const RopeArgs& ra, hipStream_t s);
int launch_qkv_rope_flex_split(const void* X, const void* W, int M, int N, int K, int D,
                               const RopeArgs& ra, int cand, int S, hipStream_t s);
// one QKV + RoPE path by code (gemm256d.hip: AGPR height, stream, unfused, flex x split)
int launch_qkv_rope_algo(const void* X, const void* W, void* qkv, int M, int N, int K, int D,
                         const RopeArgs& ra, int algo, hipStream_t s);
void gemm_plan_set_rope(int N, int K, const int* codes, int n);
int gemm_plan_rope(int M, int N, int K);
