// K9: LM head + grammar mask + temperature sampling, fused.
//
// Constrained decoding only ever samples from a small allowed set per sequence
// (the DAG grammar's choice points, planner/grammar.py).  Masking the full
// 128,256-entry softmax to that set is mathematically identical to a softmax
// over the allowed tokens only, so this kernel computes the logits of the
// allowed rows of the LM head (one 8 KiB row dot-product per allowed token)
// and draws with Gumbel-max:  argmax_i (logit_i / T + g_i),  g_i ~ Gumbel(0,1)
// from a counter-based hash RNG (reproducible per (seed, sequence counter, token)).
// T <= 0 selects greedy decoding.
#include "common.h"
#include "kernels.h"

__global__ __launch_bounds__(256) void sample_allowed_kernel(
    const bf16* __restrict__ hidden, const bf16* __restrict__ W, const int* __restrict__ allow_ptr,
    const int* __restrict__ allow_ids, const int* __restrict__ ctr, float inv_temp,
    unsigned long long seed, int H, int* __restrict__ out_tok, float* __restrict__ out_logit) {
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a0 = allow_ptr[s], a1 = allow_ptr[s + 1];
  const bf16* h = hidden + (size_t)s * H;
  const int nvec = H >> 3;
  float best = -INFINITY, best_logit = 0.f;
  int best_tok = -1;
  for (int a = a0 + wave; a < a1; a += 4) {
    const int tok = allow_ids[a];
    const bf16* w = W + (size_t)tok * H;
    float acc = 0.f;
    for (int c = lane; c < nvec; c += 64) {
      const bf16x8 x = reinterpret_cast<const bf16x8*>(h)[c];
      const bf16x8 y = reinterpret_cast<const bf16x8*>(w)[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += (float)x[j] * (float)y[j];
    }
    acc = wave_sum(acc);
    float score = acc;
    if (inv_temp > 0.f) {
      const float u = uniform01(seed, (unsigned long long)(unsigned)ctr[s], (unsigned long long)tok);
      score = acc * inv_temp - __logf(-__logf(u));
    }
    if (score > best) {
      best = score;
      best_tok = tok;
      best_logit = acc;
    }
  }
  __shared__ float sb[4], sl[4];
  __shared__ int st[4];
  if (lane == 0) {
    sb[wave] = best;
    st[wave] = best_tok;
    sl[wave] = best_logit;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bi = 0;
    for (int i = 1; i < 4; ++i)
      if (st[i] >= 0 && (st[bi] < 0 || sb[i] > sb[bi])) bi = i;
    out_tok[s] = st[bi];
    if (out_logit) out_logit[s] = sl[bi];
  }
}

void launch_sample_allowed(const void* hidden, const void* W, const int* allow_ptr,
                           const int* allow_ids, const int* ctr, float temperature,
                           unsigned long long seed, int S, int H, int* out_tok, float* out_logit,
                           hipStream_t s) {
  if (S <= 0) return;
  const float inv_t = temperature > 0.f ? 1.f / temperature : 0.f;
  sample_allowed_kernel<<<S, 256, 0, s>>>((const bf16*)hidden, (const bf16*)W, allow_ptr,
                                          allow_ids, ctr, inv_t, seed, H, out_tok, out_logit);
}

// Dense variant: logits [S, V] (fp32 or bf16 via the GEMM), optional -inf mask
// folded in by the caller.  One block per row, Gumbel-max over the full vocab.
__global__ __launch_bounds__(256) void sample_dense_kernel(const bf16* __restrict__ logits, int V,
                                                           const int* __restrict__ ctr,
                                                           float inv_temp,
                                                           unsigned long long seed,
                                                           int* __restrict__ out_tok) {
  const int s = blockIdx.x;
  const bf16* row = logits + (size_t)s * V;
  float best = -INFINITY;
  int bt = 0;
  for (int i = threadIdx.x; i < V; i += 256) {
    const float l = (float)row[i];
    float sc = l;
    if (inv_temp > 0.f) sc = l * inv_temp - __logf(-__logf(uniform01(seed, (unsigned long long)(unsigned)ctr[s], (unsigned long long)i)));
    if (sc > best) { best = sc; bt = i; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int ot = __shfl_xor(bt, o, 64);
    if (ob > best || (ob == best && ot < bt)) { best = ob; bt = ot; }
  }
  __shared__ float sb[4];
  __shared__ int st[4];
  if ((threadIdx.x & 63) == 0) { sb[threadIdx.x >> 6] = best; st[threadIdx.x >> 6] = bt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bi = 0;
    for (int i = 1; i < 4; ++i) if (sb[i] > sb[bi]) bi = i;
    out_tok[s] = st[bi];
  }
}

void launch_sample_dense(const void* logits, int S, int V, const int* ctr, float temperature,
                         unsigned long long seed, int* out_tok, hipStream_t s) {
  if (S <= 0) return;
  const float inv_t = temperature > 0.f ? 1.f / temperature : 0.f;
  sample_dense_kernel<<<S, 256, 0, s>>>((const bf16*)logits, V, ctr, inv_t, seed, out_tok);
}

// Decision lookahead (engine MCP_LOOKAHEAD): the next forward was launched
// before the host read this step's sampled tokens, laid out for every outcome
// of each sequence's pending choice (engine._launch_branch).  This kernel runs
// between the step payload's H2D copy and the forward: per sequence it finds
// the record of the token the previous step sampled and writes that outcome's
// tokens (the token, then its jump-forward span), the sequence's new-token
// count and context length, its logit row and the allowed set of the choice
// after it into the step's device views.  The sequence's rows past the
// outcome's span get KV slot -1: their K/V are never written (they sit past
// the context, in the tile the next step's attention masks - a masked key
// still multiplies its V row by 0, and these rows' values are undefined).
//   tab[0] = n;  tab[1] = offset of the tail section (0: none);
//   tab[2 + 6 i ..] = {prev_row, q_start, start, Lmax, n_branches, rec_off}
//   record (4 + Lmax ints) = {token, q_len, allowed_off, allowed_len, ids[Lmax]}
//   tail = {nt, rel[nt + 1], pool[rel[nt]]}: the allowed sets of nt sampled
//   rows after the n lookahead rows (requests admitted into the step, their
//   tokens known), placed after the n rows' chosen sets
// One block: n <= 64 sequences, a few hundred ints of output.
constexpr int BRANCH_MAX_SEQS = 64;

__global__ __launch_bounds__(256) void branch_select_kernel(
    const int* __restrict__ prev_tok, const int* __restrict__ tab, int* __restrict__ ids,
    int* __restrict__ slots, int* __restrict__ q_len, int* __restrict__ ctx_len, int* __restrict__ rows,
    int* __restrict__ aptr, int aptr_len, int* __restrict__ aids, int* __restrict__ err) {
  __shared__ int s_rec[BRANCH_MAX_SEQS], s_aoff[BRANCH_MAX_SEQS + 1];
  const int n = tab[0];
  const int t = threadIdx.x;
  if (t < n) {
    const int* h = tab + 2 + 6 * t;
    const int tok = prev_tok[h[0]];
    const int L = h[3], nb = h[4];
    int rec = h[5];
    int found = -1;
    for (int b = 0; b < nb; ++b)
      if (tab[h[5] + b * (4 + L)] == tok) {
        found = b;
        break;
      }
    if (found < 0) {
      err[0] = 1 + t;                                  // the host checks it with the tokens
      found = 0;
    }
    rec += found * (4 + L);
    s_rec[t] = rec;
  }
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int i = 0; i < n; ++i) {
      s_aoff[i] = acc;
      acc += tab[s_rec[i] + 3];
    }
    s_aoff[n] = acc;
  }
  __syncthreads();
  if (t < n) {
    const int* h = tab + 2 + 6 * t;
    const int ql = tab[s_rec[t] + 1];
    q_len[t] = ql;
    ctx_len[t] = h[2] + ql;
    rows[t] = h[1] + ql - 1;
  }
  const int tail = tab[1];
  const int nt = tail ? tab[tail] : 0;
  const int total = s_aoff[n];
  for (int i = n + t; i < aptr_len; i += 256)
    aptr[i] = total + (tail ? tab[tail + 1 + min(i - n, nt)] : 0);
  if (t < n) aptr[t] = s_aoff[t];
  if (tail) {
    const int tl = tab[tail + 1 + nt];
    for (int j = t; j < tl; j += 256) aids[total + j] = tab[tail + 2 + nt + j];
  }
  for (int i = 0; i < n; ++i) {
    const int* h = tab + 2 + 6 * i;
    const int* rec = tab + s_rec[i];
    for (int j = t; j < h[3]; j += 256) {
      ids[h[1] + j] = rec[4 + j];
      if (j >= rec[1]) slots[h[1] + j] = -1;
    }
    for (int j = t; j < rec[3]; j += 256) aids[s_aoff[i] + j] = tab[rec[2] + j];
  }
}

int launch_branch_select(const int* prev_tok, const int* tab, int n, int* ids, int* slots, int* q_len,
                         int* ctx_len, int* rows, int* aptr, int aptr_len, int* aids, int* err,
                         hipStream_t s) {
  if (n <= 0) return 0;
  if (n > BRANCH_MAX_SEQS || aptr_len < n + 1) return 1;
  branch_select_kernel<<<1, 256, 0, s>>>(prev_tok, tab, ids, slots, q_len, ctx_len, rows, aptr, aptr_len,
                                         aids, err);
  return 0;
}
