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
// Measured (profiles/config3_topk.md): 10M x 1024 rows in 3.9 / 4.2 ms for 1
// / 16 queries.  Wider batches (17-64 queries, k <= 32) use
// topk_fused_dsplit_kernel below: the waves split the embedding dimension.
namespace {
constexpr int FT_CAP = 128;
constexpr int FT_SEGR = 4096;

// corpus rows per workgroup: 4096-row segments, several per workgroup once
// there are more segments than ~8 waves per CU can take (10M x 64 queries: 4).
// The candidate lists and their threshold carry over the segments of a
// workgroup, so each query admits ~k ln(rows / k) candidates per workgroup
// instead of per segment (the list compactions were the cost that grew with
// the query count), and fewer partial lists reach the merge.
__host__ __device__ inline int topk_seg_rows(int N, int B) {
  const int nseg1 = (N + FT_SEGR - 1) / FT_SEGR;
  const int waves = B > 16 ? 4 : 1;                  // 17-64 queries: 4-wave (d-split) workgroups
  const int slots = 2048 / waves;                    // resident workgroups (8 waves per CU)
  // multi-wave workgroups: ONE wave of workgroups (a 1.2-wave grid left 19 %
  // of it as a tail); 1-wave workgroups keep whole segments (5.2 TB/s)
  const int spw = waves > 1 ? (nseg1 + slots - 1) / slots : nseg1 / slots;
  return FT_SEGR * (spw > 1 ? spw : 1);
}

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
  const int segr = topk_seg_rows(N, B);
  const int row0 = seg * segr;
  const int rows = min(segr, N - row0);
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

// Wide query batches (17-64 queries, k <= 48): the 4 waves of a workgroup
// split the EMBEDDING DIMENSION instead of the queries.  Wave w streams the
// d-quarter [D/4 w, D/4 (w+1)) of every 16-row corpus block (register ring,
// direct loads, no row is read twice) against ALL query groups, and every
// block's partial scores are summed through LDS: wave w then owns query
// group w (queries 16 w .. 16 w + 15) and runs the candidate-list filter of
// the 1-16 query kernel above.  With the queries split instead (4 waves each
// streaming the same rows) the lagging waves miss L2 and 10M x 64 took 10.0
// ms vs 3.9 for one query; an LDS ring shared by query-split waves (one
// workgroup per CU, 64 KiB in flight) took 13.5 ms.
constexpr int FTD_W = 4, FTD_CAP = 64;

// 16-B global load the compiler does not track (the caller waits vmcnt itself)
DEV bf16x8 gload16(const bf16* p) {
  bf16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

DEV void raw_barrier_tk() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int NS, int NG>
__global__ __launch_bounds__(256, 2) void topk_fused_dsplit_kernel(const bf16* __restrict__ Q,
                                                                  const bf16* __restrict__ E,
                                                                  int B, int N, int k,
                                                                  float* __restrict__ cand_v,
                                                                  int* __restrict__ cand_i) {
  constexpr int D = NS * 32;
  constexpr int NQ = NS / FTD_W;                     // 32-d steps per wave per block
  constexpr int LIST_B = 16 * FTD_CAP * 8 + 16 * 8;  // one wave's candidate lists
  constexpr int XCH_F4 = FTD_W * 4 * 64;             // partial tiles [wave][group][lane]
  __shared__ __attribute__((aligned(16))) char sm[FTD_W * LIST_B + XCH_F4 * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int seg = blockIdx.x, nseg = gridDim.x;
  const int segr = topk_seg_rows(N, B);
  const int row0 = seg * segr;
  const int rows = min(segr, N - row0);
  char* wbase = sm + wave * LIST_B;
  float (*BV)[FTD_CAP] = reinterpret_cast<float (*)[FTD_CAP]>(wbase);
  int (*BI)[FTD_CAP] = reinterpret_cast<int (*)[FTD_CAP]>(wbase + 16 * FTD_CAP * 4);
  int* cntw = reinterpret_cast<int*>(wbase + 16 * FTD_CAP * 8);
  float* tauw = reinterpret_cast<float*>(wbase + 16 * FTD_CAP * 8 + 64);
  f32x4* xch = reinterpret_cast<f32x4*>(sm + FTD_W * LIST_B);
  const int q = wave * 16 + r;                       // this lane's query as a list owner
  const bool owner = wave < NG;                      // static group count: the MFMA loop
                                                     // has no branch (no vmcnt(0) per MFMA)

  // query fragments of every group for this wave's d-quarter
  bf16x8 qf[NG][NQ];
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const bf16* qp = Q + (size_t)min(16 * j + r, B - 1) * D + (D / FTD_W) * wave + 8 * g;
#pragma unroll
    for (int s = 0; s < NQ; ++s) qf[j][s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
  }
  // make hipcc retire the query loads HERE: a compiler-visible load still
  // pending at the loop would make it wait on its own count inside the loop,
  // which the hand-counted ring loads below would turn into a full drain
#pragma unroll
  for (int j = 0; j < NG; ++j)
#pragma unroll
    for (int s = 0; s < NQ; ++s) asm volatile("" :: "v"(qf[j][s]));
  if (lane < 16) {
    cntw[lane] = 0;
    tauw[lane] = -INFINITY;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  float tau = -INFINITY;

  auto compact = [&](int qq) {
    const int n = cntw[qq];
    float v0 = -INFINITY;
    int i0 = 0x7fffffff;
    if (lane < n) { v0 = BV[qq][lane]; i0 = BI[qq][lane]; }
    int r0 = 0;
    for (int jj = 0; jj < n; ++jj) {
      const float vj = BV[qq][jj];
      const int ij = BI[qq][jj];
      r0 += (vj > v0 || (vj == v0 && ij < i0)) ? 1 : 0;
    }
    if (lane < n && r0 < k) { BV[qq][r0] = v0; BI[qq][r0] = i0; }
    if (lane < n && r0 == k - 1) tauw[qq] = v0;
    if (lane == 0) cntw[qq] = min(n, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  };

  // register ring: two blocks of loads per lane (D = 1024: 16 x 16 B), block b
  // in slots (b & 1) NQ + s; the loop body covers a block pair so every slot
  // index is static, and block b + 2's loads are issued right after block b's
  // MFMAs while block b + 1's are still in flight
  constexpr int RING = 2 * NQ;
  const int nblk = (rows + 15) / 16;
  auto rowp = [&](int b) {
    return E + (size_t)(row0 + min(16 * min(b, nblk - 1) + r, rows - 1)) * D +
           (D / FTD_W) * wave + 8 * g;
  };
  // The ring loads are inline asm and counted by hand: with compiler-visible
  // loads hipcc merged the ring's loop-carried registers through copies and
  // waited vmcnt(0) at the top of every block pair (no load in flight while
  // computing).  Before block b's MFMAs: vmcnt(NQ) = block b's loads landed,
  // block b + 1's still in flight; the wait names the slots, so no MFMA that
  // reads them can be scheduled above it.
  static_assert(NQ == 8 || NQ == 4, "hand-counted ring");
  bf16x8 ring[RING];
#pragma unroll
  for (int t = 0; t < RING; ++t) ring[t] = gload16(rowp(t / NQ) + 32 * (t % NQ));

  for (int b0 = 0; b0 < nblk; b0 += 2) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int b = b0 + e;
      f32x4 acc[NG];
#pragma unroll
      for (int j = 0; j < NG; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const bf16* pn = rowp(b + 2);
      if constexpr (NQ == 8) {
        bf16x8* rr = ring + e * NQ;
        asm volatile("s_waitcnt vmcnt(8)" : "+v"(rr[0]), "+v"(rr[1]), "+v"(rr[2]), "+v"(rr[3]),
                     "+v"(rr[4]), "+v"(rr[5]), "+v"(rr[6]), "+v"(rr[7]));
      } else {
        bf16x8* rr = ring + e * NQ;
        asm volatile("s_waitcnt vmcnt(4)" : "+v"(rr[0]), "+v"(rr[1]), "+v"(rr[2]), "+v"(rr[3]));
      }
#pragma unroll
      for (int s = 0; s < NQ; ++s) {
        const bf16x8 a = ring[e * NQ + s];
#pragma unroll
        for (int j = 0; j < NG; ++j) acc[j] = mfma16x16x32(a, qf[j][s], acc[j]);
      }
#pragma unroll
      for (int s = 0; s < NQ; ++s) ring[e * NQ + s] = gload16(pn + 32 * s);
      // partials -> LDS; owner wave w sums group w over the 4 d-quarters
#pragma unroll
      for (int j = 0; j < NG; ++j) xch[(wave * 4 + j) * 64 + lane] = acc[j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier_tk();
      if (owner) {
        f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < FTD_W; ++w) sc += xch[(w * 4 + wave) * 64 + lane];
        if (q < B && b < nblk) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int lr = 16 * b + 4 * g + i;
            if (lr < rows && sc[i] >= tau) {
              const int pos = atomicAdd(&cntw[r], 1);
              BV[r][pos] = sc[i];
              BI[r][pos] = row0 + lr;
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier_tk();                              // xch free for the next block
      if (owner) {
        unsigned long long need = __ballot(lane < 16 && cntw[lane] > FTD_CAP - 16);
        while (need) {
          const int qq = __ffsll((long long)need) - 1;
          need &= need - 1;
          compact(qq);
        }
        tau = tauw[r];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing ring loads
  if (!owner) return;
  for (int qq = 0; qq < 16; ++qq) compact(qq);
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

int topk_fused_segments(int N, int B) {
  const int r = topk_seg_rows(N, B);
  return (N + r - 1) / r;
}

// cand_v / cand_i: [B, topk_fused_segments(N), k]; returns nonzero if unsupported
int launch_topk_fused(const void* Q, const void* E, int B, int N, int D, int k, float* cand_v,
                      int* cand_i, hipStream_t s) {
  if (B <= 0 || B > 64 || N <= 0 || k <= 0 || k > 64) return 1;
  const int nseg = topk_fused_segments(N, B);
  const int waves = (B + 15) / 16;
  static const int dsplit = getenv("MCP_TOPK_DSPLIT") ? atoi(getenv("MCP_TOPK_DSPLIT")) : 1;
  if (waves > 1 && dsplit && k <= FTD_CAP - 16) {
#define FTD_LAUNCH(NS_, NG_) \
  topk_fused_dsplit_kernel<NS_, NG_><<<nseg, 256, 0, s>>>((const bf16*)Q, (const bf16*)E, B, N, k, cand_v, cand_i)
    if (D != 1024 && D != 512) return 2;
    if (D == 1024) {
      if (waves == 2) FTD_LAUNCH(32, 2); else if (waves == 3) FTD_LAUNCH(32, 3); else FTD_LAUNCH(32, 4);
    } else {
      if (waves == 2) FTD_LAUNCH(16, 2); else if (waves == 3) FTD_LAUNCH(16, 3); else FTD_LAUNCH(16, 4);
    }
#undef FTD_LAUNCH
    return 0;
  }
  const size_t lds = (size_t)waves * (16 * FT_CAP * 8 + 16 * 8);
  switch (D) {
    case 1024: topk_fused_kernel<32><<<nseg, 64 * waves, lds, s>>>((const bf16*)Q, (const bf16*)E, B, N, k, cand_v, cand_i); return 0;
    case 512: topk_fused_kernel<16><<<nseg, 64 * waves, lds, s>>>((const bf16*)Q, (const bf16*)E, B, N, k, cand_v, cand_i); return 0;
    default: return 2;
  }
}
