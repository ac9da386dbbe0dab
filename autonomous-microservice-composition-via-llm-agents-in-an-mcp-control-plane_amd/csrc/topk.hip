// K11: HBM-resident top-k cosine retrieval (replaces the pgvector table of
// control_plane.py:51-55).  Scores come from the MFMA GEMM (fp32 output,
// gemm.hip: scores[Bq, N] = Qn . En^T over unit-norm rows); this file holds
//   * l2-normalisation of embedding rows (bf16, in place, one wave per row);
//   * segmented top-k selection: each (segment, query) block loads <= 4096
//     scores into LDS and extracts the k largest by repeated block argmax in
//     which only the owning thread of the last winner rescans its 16 values.
//     Applied hierarchically (N -> N/4096*k -> ... -> k) it handles 10^8 rows.
#include "common.h"
#include "kernels.h"

__global__ __launch_bounds__(64) void l2norm_rows_kernel(bf16* __restrict__ x, int D) {
  bf16* row = x + (size_t)blockIdx.x * D;
  float ss = 0.f;
  for (int c = threadIdx.x; c < D / 8; c += 64) {
    const bf16x8 v = reinterpret_cast<bf16x8*>(row)[c];
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += (float)v[j] * (float)v[j];
  }
  ss = wave_sum(ss);
  const float inv = ss > 0.f ? rsqrtf(ss) : 0.f;
  for (int c = threadIdx.x; c < D / 8; c += 64) {
    bf16x8 v = reinterpret_cast<bf16x8*>(row)[c];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] * inv);
    reinterpret_cast<bf16x8*>(row)[c] = v;
  }
}

void launch_l2norm_rows(void* x, int N, int D, hipStream_t s) {
  if (N > 0) l2norm_rows_kernel<<<N, 64, 0, s>>>((bf16*)x, D);
}

namespace {
constexpr int SEG = 4096, NT = 256, PER = SEG / NT;

DEV bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }
}  // namespace

__global__ __launch_bounds__(NT) void segment_topk_kernel(const float* __restrict__ vals,
                                                          const int* __restrict__ idx_in, int L,
                                                          int seg_len, int k,
                                                          float* __restrict__ out_v,
                                                          int* __restrict__ out_i) {
  __shared__ float sv[SEG];
  __shared__ int si[SEG];
  __shared__ float wv[NT / 64];
  __shared__ int wp[NT / 64];
  const int seg = blockIdx.x, q = blockIdx.y, nseg = gridDim.x;
  const int base = seg * seg_len;
  const int n = min(seg_len, L - base);
  const float* vrow = vals + (size_t)q * L + base;
  const int* irow = idx_in ? idx_in + (size_t)q * L + base : nullptr;
  for (int i = threadIdx.x; i < SEG; i += NT) {
    const bool ok = i < n;
    sv[i] = ok ? vrow[i] : -INFINITY;
    si[i] = ok ? (irow ? irow[i] : base + i) : 0x7fffffff;
  }
  __syncthreads();
  // thread t owns positions t, t+NT, ...
  auto local_best = [&](float& bv, int& bp) {
    bv = -INFINITY;
    bp = -1;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int p = threadIdx.x + j * NT;
      if (bp < 0 || better(sv[p], si[p], bv, si[bp])) {
        bv = sv[p];
        bp = p;
      }
    }
  };
  float bv;
  int bp;
  local_best(bv, bp);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* ov = out_v + ((size_t)q * nseg + seg) * k;
  int* oi = out_i + ((size_t)q * nseg + seg) * k;
  for (int r = 0; r < k; ++r) {
    float v = bv;
    int p = bp;
    int id = si[p];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov2 = __shfl_xor(v, o, 64);
      const int op = __shfl_xor(p, o, 64);
      const int oid = __shfl_xor(id, o, 64);
      if (better(ov2, oid, v, id)) {
        v = ov2;
        p = op;
        id = oid;
      }
    }
    if (lane == 0) {
      wv[wave] = v;
      wp[wave] = p;
    }
    __syncthreads();
    float best = wv[0];
    int bpos = wp[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w)
      if (better(wv[w], si[wp[w]], best, si[bpos])) {
        best = wv[w];
        bpos = wp[w];
      }
    if (threadIdx.x == 0) {
      ov[r] = best;
      oi[r] = si[bpos];
    }
    __syncthreads();
    if ((bpos % NT) == threadIdx.x) {
      sv[bpos] = -INFINITY;
      si[bpos] = 0x7fffffff;
      local_best(bv, bp);
    }
    __syncthreads();
  }
}

int launch_segment_topk(const float* vals, const int* idx_in, int B, int L, int seg_len, int k,
                        float* out_v, int* out_i, hipStream_t s) {
  if (seg_len > SEG || k > seg_len || k <= 0) return 1;
  const int nseg = (L + seg_len - 1) / seg_len;
  segment_topk_kernel<<<dim3(nseg, B), NT, 0, s>>>(vals, idx_in, L, seg_len, k, out_v, out_i);
  return 0;
}
