// K11: HBM-resident top-k cosine retrieval (replaces the pgvector table of
// control_plane.py:51-55).  Scores come from the MFMA GEMM (fp32 output,
// gemm.hip: scores[Bq, N] = Qn . En^T over unit-norm rows); this file holds
//   * l2-normalisation of embedding rows (bf16, in place, one wave per row);
//   * segmented top-k selection: each (segment, query) block loads <= 4096
//     scores into LDS and extracts the k largest by repeated block argmax in
//     which only the owning thread of the last winner rescans its 16 values.
//     Applied hierarchically (N -> N/4096*k -> ... -> k) it handles 10^8 rows.
#include <stdlib.h>

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

// ---------------------------------------------------------------------------
// Fused scoring + per-segment top-k (the production K11 path): scores never
// touch HBM.  Workgroup = ceil(B / 16) waves on one segment of SEGR corpus
// rows; wave w owns queries 16 w .. 16 w + 15, all waves stream the same
// rows (HBM once, the other reads hit L1/L2).
//  * S^T[row][query] per 16-row block by v_mfma_f32_16x16x32_bf16: corpus rows
//    are the A operand (a 16-step register ring of direct loads keeps ~16 KiB
//    per wave in flight), the wave's 16 query vectors stay in registers as the
//    B operand (D/32 fragments).  Lane (r, g) holds rows 4 g + i of query r.
//  * per query a candidate list in LDS (CAP entries) behind a running
//    threshold tau = the k-th best so far: scores >= tau are appended (LDS
//    atomic slot), and a list close to full is compacted by the whole wave to
//    its k best by exact rank (score desc, row index asc), which raises tau.
//    After the first few blocks almost nothing passes tau.
//  * the segment's top k per query (rank order) go to cand[B][nseg][k]; the
//    hierarchical segment_topk above merges the segments.
// Measured (profiles/config3_topk.md): 10M x 1024 rows in 3.9 / 4.2 / 10.0 ms
// for 1 / 16 / 64 queries.  At 64 queries the 4 waves of a workgroup each
// pull the same rows through L1/L2; a barrier per block to keep them in step
// was slower (11.7 ms).  Sharing the rows through an LDS ring is the next
// step for wide query batches.
namespace {
constexpr int FT_CAP = 128;
constexpr int FT_SEGR = 4096;

template <int NS>
__global__ __launch_bounds__(256) void topk_fused_kernel(const bf16* __restrict__ Q,
                                                          const bf16* __restrict__ E, int B,
                                                          int N, int k, float* __restrict__ cand_v,
                                                          int* __restrict__ cand_i) {
  constexpr int D = NS * 32;
  // per wave (dynamic LDS, so a 1-wave workgroup takes 16.5 KiB, not 66):
  // candidate values [16][CAP], indices [16][CAP], counts [16], thresholds [16]
  extern __shared__ __attribute__((aligned(16))) char ft_smem[];
  constexpr int WAVE_BYTES = 16 * FT_CAP * 8 + 16 * 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int seg = blockIdx.x, nseg = gridDim.x;
  const int row0 = seg * FT_SEGR;
  const int rows = min(FT_SEGR, N - row0);
  const int q = wave * 16 + r;                        // this lane's query
  char* wbase = ft_smem + wave * WAVE_BYTES;
  float (*BV)[FT_CAP] = reinterpret_cast<float (*)[FT_CAP]>(wbase);
  int (*BI)[FT_CAP] = reinterpret_cast<int (*)[FT_CAP]>(wbase + 16 * FT_CAP * 4);
  int* cntw = reinterpret_cast<int*>(wbase + 16 * FT_CAP * 8);
  float* tauw = reinterpret_cast<float*>(wbase + 16 * FT_CAP * 8 + 64);

  // query fragments: step s covers d = 32 s + {8 g .. 8 g + 7}
  bf16x8 qf[NS];
  {
    const bf16* qp = Q + (size_t)min(q, B - 1) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
  }
  if (lane < 16) {
    cntw[lane] = 0;
    tauw[lane] = -INFINITY;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  float tau = -INFINITY;

  // compaction of query qq's list to its k best (whole wave, uniform)
  auto compact = [&](int qq) {
    const int n = cntw[qq];
    float v0 = -INFINITY, v1 = -INFINITY;
    int i0 = 0x7fffffff, i1 = 0x7fffffff;
    if (lane < n) { v0 = BV[qq][lane]; i0 = BI[qq][lane]; }
    if (lane + 64 < n) { v1 = BV[qq][lane + 64]; i1 = BI[qq][lane + 64]; }
    int r0 = 0, r1 = 0;
    for (int j = 0; j < n; ++j) {
      const float vj = BV[qq][j];
      const int ij = BI[qq][j];
      r0 += (vj > v0 || (vj == v0 && ij < i0)) ? 1 : 0;
      r1 += (vj > v1 || (vj == v1 && ij < i1)) ? 1 : 0;
    }
    if (lane < n && r0 < k) { BV[qq][r0] = v0; BI[qq][r0] = i0; }
    if (lane + 64 < n && r1 < k) { BV[qq][r1] = v1; BI[qq][r1] = i1; }
    if (lane < n && r0 == k - 1) tauw[qq] = v0;
    if (lane + 64 < n && r1 == k - 1) tauw[qq] = v1;
    if (lane == 0) cntw[qq] = min(n, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  };

  const int nblk = (rows + 15) / 16;
  // A-operand ring: 16 d-steps in flight; step t = NS b + s, the loop is
  // unrolled by NS so that s (the query fragment) and the ring slot are static
  static_assert(NS % 16 == 0, "ring of 16 d-steps");
  bf16x8 ring[16];
  auto rowp = [&](int b) {                             // this lane's row of block b
    return E + (size_t)(row0 + min(16 * b + r, rows - 1)) * D + 8 * g;
  };
  {
    const bf16* p0 = rowp(0);
    const bf16* p1 = rowp(1);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      ring[j] = *reinterpret_cast<const bf16x8*>((j < NS ? p0 + 32 * j : p1 + 32 * (j - NS)));
  }
  for (int b = 0; b < nblk; ++b) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16* pc = rowp(b);
    const bf16* pn = rowp(min(b + 1, nblk - 1));      // past the end: re-read, unused
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      acc = mfma16x16x32(ring[s % 16], qf[s], acc);
      const int sn = s + 16;                         // prefetch 16 d-steps ahead
      ring[s % 16] = *reinterpret_cast<const bf16x8*>(sn < NS ? pc + 32 * sn : pn + 32 * (sn - NS));
    }
    // block b done: lane holds rows 4 g + i of query r
    if (q < B) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int lr = 16 * b + 4 * g + i;
        if (lr < rows && acc[i] >= tau) {
          const int pos = atomicAdd(&cntw[r], 1);
          BV[r][pos] = acc[i];
          BI[r][pos] = row0 + lr;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    // compact the lists that could overflow on the next block (<= 16 adds each)
    unsigned long long need = __ballot(lane < 16 && cntw[lane] > FT_CAP - 16);
    while (need) {
      const int qq = __ffsll((long long)need) - 1;
      need &= need - 1;
      compact(qq);
    }
    tau = tauw[r];
  }
  // final: every list to its k best, in rank order
  for (int qq = 0; qq < 16; ++qq) compact(qq);
  if (wave * 16 >= B) return;
  for (int qq = 0; qq < 16; ++qq) {
    const int qg = wave * 16 + qq;
    if (qg >= B) break;
    const int n = cntw[qq];
    float* ov = cand_v + ((size_t)qg * nseg + seg) * k;
    int* oi = cand_i + ((size_t)qg * nseg + seg) * k;
    for (int j = lane; j < k; j += 64) {
      ov[j] = j < n ? BV[qq][j] : -INFINITY;
      oi[j] = j < n ? BI[qq][j] : 0x7fffffff;
    }
  }
}
}  // namespace

int topk_fused_segments(int N) { return (N + FT_SEGR - 1) / FT_SEGR; }

// cand_v / cand_i: [B, topk_fused_segments(N), k]; returns nonzero if unsupported
int launch_topk_fused(const void* Q, const void* E, int B, int N, int D, int k, float* cand_v,
                      int* cand_i, hipStream_t s) {
  if (B <= 0 || B > 64 || N <= 0 || k <= 0 || k > 64) return 1;
  const int nseg = topk_fused_segments(N);
  const int waves = (B + 15) / 16;
  const size_t lds = (size_t)waves * (16 * FT_CAP * 8 + 16 * 8);
  switch (D) {
    case 1024: topk_fused_kernel<32><<<nseg, 64 * waves, lds, s>>>((const bf16*)Q, (const bf16*)E, B, N, k, cand_v, cand_i); return 0;
    case 512: topk_fused_kernel<16><<<nseg, 64 * waves, lds, s>>>((const bf16*)Q, (const bf16*)E, B, N, k, cand_v, cand_i); return 0;
    default: return 2;
  }
}
