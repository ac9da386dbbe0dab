// K2: weight-streaming GEMM for decode-sized steps (M <= 128 tokens).
//   Y[M,N] = X[M,K] . W[N,K]^T   epilogues: 0 plain, 1 + R, 2 SwiGLU
//   (interleaved gate|up rows), 3 QKV + RoPE + paged K/V write.
//
// At M <= 128 a projection is a weight stream (2 M flop per weight byte, far
// under the ~400 flop/B ridge), so the kernel's job is keeping ~6 TB/s of HBM
// reads in flight.  The 128^2 tile kernel (gemm.hip) at these M is latency
// bound: each workgroup has ~32 KiB in flight through a 2-stage LDS pipeline
// (measured 6-25 GB/s per workgroup, profiles/gemm_tuning.md).  Here:
//
//  * workgroup = 4 waves on one 16 NF-row weight panel (BN = 64 rows for
//    NF = 4) and a 1/S slice of K; the waves interleave 64-deep k-steps;
//  * no LDS staging: v_mfma_f32_16x16x32_bf16 takes W and X fragments
//    straight from registers.  Lane (r = l & 15, g = l >> 4) loads
//    W[row r][k0 + 32 h + 8 g .. +8) for h = 0, 1: each load instruction reads
//    64 contiguous bytes of 16 rows (the two cover the 128-byte row piece of
//    the step) and the X fragment uses the SAME k permutation (a dot product is
//    order-free): MFMA h consumes load h of every lane group;
//  * a DEPTH-deep register ring per wave keeps DEPTH k-steps of W and X in
//    flight (8-12 KiB per wave, ~64 KiB per CU at two workgroups per CU);
//  * the 4 waves' partial tiles are summed through LDS, each wave owning a
//    quarter of the tile's fragments; S > 1 splits publish their quarter
//    write-through (sc1) to the split-K workspace and take a ticket; the last
//    split of a tile adds the other S-1 partials (sc1 loads: the hand-off of
//    MI355X_MICROARCH.md "Valid forms", row 1) and runs the epilogue - no
//    second launch, and the reduction is spread over its 4 waves.
//
// EPI 3 reads W rows in a rotate-half order: tile t covers head t / 2, dims
// 32 (t & 1) + {0..31} in fragments 0 and 2 and the same dims + 64 in
// fragments 1 and 3, so a lane holds both halves of every RoPE pair.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int SW_WAVES = 4;
constexpr int SW_STEP = 64;

// weights are read once per launch: NT = non-temporal loads (MI355X_MICROARCH.md
// "nt-weights": once-read decode weight streams)
template <bool NT>
DEV bf16x8 wload(const bf16* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
  return *reinterpret_cast<const bf16x8*>(p);
}

template <int EPI, int MF, int NF, int DEPTH, int MH, bool NT>
__global__ __launch_bounds__(256 * MH, MH == 1 ? 2 : 1) void gemm_stream(const bf16* __restrict__ X,
                                                      const bf16* __restrict__ W,
                                                      bf16* __restrict__ Y,
                                                      const bf16* __restrict__ R, int M, int N,
                                                      int K, int S, float* __restrict__ ws,
                                                      int* __restrict__ tickets, const RopeArgs ra,
                                                      const NormEpi ne) {
  static_assert(NF % 2 == 0, "fragment pairs");
  constexpr int NQ = NF * MF;                        // fragments per tile
  constexpr int FPU = (EPI >= 2) ? 2 : 1;            // fragments per epilogue unit
  constexpr int NU = NQ / FPU;                       // units per tile
  constexpr int UPW = (NU + SW_WAVES - 1) / SW_WAVES;
  __shared__ f32x4 red[MH][SW_WAVES][NQ][64];
  __shared__ int s_last;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mh = wv / SW_WAVES;                      // row half (MH = 2: rows 64 mh ..)
  const int wave = wv % SW_WAVES;                    // k-step lane of the workgroup
  const int r = lane & 15, g = lane >> 4;
  const int bid = blockIdx.x;
  const int sp = bid % S, tile = bid / S;
  const int n0 = tile * 16 * NF;

  // ---- per-lane row pointers (k offset 16 g inside a step)
  const bf16* wrow[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    int row;
    if constexpr (EPI == 3) {
      const int head = tile >> 1, q = tile & 1;
      row = head * 128 + 32 * q + 16 * (f >> 1) + 64 * (f & 1) + r;
    } else {
      row = n0 + 16 * f + r;
    }
    wrow[f] = W + (size_t)row * K + 8 * g;
  }
  const bf16* xrow[MF];
#pragma unroll
  for (int mm = 0; mm < MF; ++mm)
    xrow[mm] = X + (size_t)min(16 * MF * mh + 16 * mm + r, M - 1) * K + 8 * g;

  // ---- this split's k-steps [s0, s1), wave w takes s0 + w, s0 + w + 4, ...
  const int nsteps = K / SW_STEP;
  const int s0 = (int)(((long long)sp * nsteps) / S), s1 = (int)(((long long)(sp + 1) * nsteps) / S);
  const int count = s1 - s0 > wave ? (s1 - s0 - wave + SW_WAVES - 1) / SW_WAVES : 0;

  f32x4 acc[NF][MF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int mm = 0; mm < MF; ++mm) acc[f][mm] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- the epilogue's per-row inputs, loaded before the weight stream: the
  //      fused-norm statistic (EPI 2 / 3), the RoPE position and cache slot
  //      (EPI 3), the residual piece (EPI 1).  Issued after the mainloop they
  //      cost the kernel's critical path one to three dependent round trips
  //      at its very end (decode steps: ~1 us each, 4 kernels per layer)
  constexpr int UPW_ = (NQ / ((EPI >= 2) ? 2 : 1) + SW_WAVES - 1) / SW_WAVES;
  constexpr int FPU_ = (EPI >= 2) ? 2 : 1;
  unsigned long long pre_ss[UPW_];
  int pre_pos[UPW_], pre_slot[UPW_];
  bf16x4 pre_rr[UPW_][FPU_];
#pragma unroll
  for (int a = 0; a < UPW_; ++a) {
    pre_ss[a] = 0;
    pre_pos[a] = 0;
    pre_slot[a] = -1;
  }
  {
#pragma unroll
    for (int a = 0; a < UPW_; ++a) {
      const int u = min(wave + a * SW_WAVES, NQ / FPU_ - 1);
      const int mm = u % MF;
      const int m = min(16 * MF * mh + 16 * mm + r, M - 1);
      if constexpr (EPI == 3) {
        pre_pos[a] = ra.pos[m];
        pre_slot[a] = ra.slots[m];
      }
      if constexpr (EPI == 1) {
        const int f0 = u / MF;
#pragma unroll
        for (int j = 0; j < FPU_; ++j)
          pre_rr[a][j] = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n0 + 16 * (f0 + j) + 4 * g);
      }
    }
    if (EPI >= 2 && ne.ss_in) {
#pragma unroll
      for (int a = 0; a < UPW_; ++a) {
        const int u = min(wave + a * SW_WAVES, NQ / FPU_ - 1);
        pre_ss[a] = ne.ss_in[min(16 * MF * mh + 16 * (u % MF) + r, M - 1)];
      }
    }
  }

  bf16x8 wr[DEPTH][NF][2], xr[DEPTH][MF][2];
  auto load = [&](int slot_i, int i) {
    const int k = (s0 + wave + i * SW_WAVES) * SW_STEP;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (d != slot_i) continue;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        wr[d][f][0] = wload<NT>(wrow[f] + k);
        wr[d][f][1] = wload<NT>(wrow[f] + k + 32);
      }
#pragma unroll
      for (int mm = 0; mm < MF; ++mm) {
        xr[d][mm][0] = *reinterpret_cast<const bf16x8*>(xrow[mm] + k);
        xr[d][mm][1] = *reinterpret_cast<const bf16x8*>(xrow[mm] + k + 32);
      }
    }
  };
  // Software pipeline: DEPTH steps in flight.  (Issuing the loads
  // unconditionally - clamped past the end - gives the compiler exact vmcnt
  // waits but measured 10-20 % slower: the clamped re-reads cost more than
  // the conservative waits of this form, profiles/gemm_stream_sweep.md.)
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < count) load(d, d);
  for (int i0 = 0; i0 < count; i0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int i = i0 + d;
      if (i < count) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int mm = 0; mm < MF; ++mm)
              acc[f][mm] = mfma16x16x32(wr[d][f][h], xr[d][mm][h], acc[f][mm]);
        if (i + DEPTH < count) load(d, i + DEPTH);
      }
    }
  }

  // ---- sum the 4 waves' partials; wave w owns units w, w + 4, ...
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int mm = 0; mm < MF; ++mm) red[mh][wave][f * MF + mm][lane] = acc[f][mm];
  __syncthreads();
  // unit u -> fragments: FPU 1: q = u; FPU 2: (f = 2 (u / MF), mm = u % MF) and f + 1
  auto unit_frag = [](int u, int j) -> int {
    if constexpr (FPU == 1) return u;
    return (2 * (u / MF) + j) * MF + u % MF;
  };
  f32x4 sum[UPW][FPU];
#pragma unroll
  for (int a = 0; a < UPW; ++a) {
    const int u = wave + a * SW_WAVES;
#pragma unroll
    for (int j = 0; j < FPU; ++j) {
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (u < NU) {
        const int q = unit_frag(u, j);
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) v += red[mh][w][q][lane];
      }
      sum[a][j] = v;
    }
  }

  if (S > 1) {
    constexpr int TILE_F = MH * NQ * 256;            // floats per partial tile
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(ws + (size_t)tile * S * TILE_F, (short)0,
                                                      S * TILE_F * 4, 0x00020000);
#pragma unroll
    for (int a = 0; a < UPW; ++a) {
      const int u = wave + a * SW_WAVES;
      if (u >= NU) continue;
#pragma unroll
      for (int j = 0; j < FPU; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sum[a][j]), rs,
                                               ((mh * NQ + unit_frag(u, j)) * 64 + lane) * 16,
                                               sp * TILE_F * 4, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(tickets + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) __hip_atomic_store(tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    // every split's partial (this one's too) summed in split order: the
    // output is bit-identical whichever split arrives last
#pragma unroll
    for (int a = 0; a < UPW; ++a)
#pragma unroll
      for (int j = 0; j < FPU; ++j) sum[a][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int js = 0; js < S; ++js) {
      f32x4 p[UPW][FPU];
#pragma unroll
      for (int a = 0; a < UPW; ++a) {
        const int u = wave + a * SW_WAVES;
#pragma unroll
        for (int j = 0; j < FPU; ++j)
          p[a][j] = u < NU ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                 rs, ((mh * NQ + unit_frag(u, j)) * 64 + lane) * 16, js * TILE_F * 4, 16))
                           : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int a = 0; a < UPW; ++a)
#pragma unroll
        for (int j = 0; j < FPU; ++j) sum[a][j] += p[a][j];
    }
  }

  // ---- epilogue: fragment (f, mm) lane holds rows n = 16 f + 4 g + i (i < 4)
  //      of token m = 16 mm + r.  Its row inputs were loaded at kernel entry;
  //      EPI 3's (cos, sin) pairs (they need the position) go out together here
  static_assert(UPW_ == UPW && FPU_ == FPU, "prefetch geometry");
  f32x4 pre_cs[EPI == 3 ? UPW : 1][2];
  if constexpr (EPI == 3) {
    if ((tile >> 1) < ra.Hq + ra.Hkv) {              // q / k heads rotate (v heads do not)
#pragma unroll
      for (int a = 0; a < UPW; ++a) {
        const int u = min(wave + a * SW_WAVES, NU - 1);
        const int d = 32 * (tile & 1) + 16 * ((2 * (u / MF)) >> 1) + 4 * g;
        const f32x4* cs = reinterpret_cast<const f32x4*>(ra.cos_sin) + (size_t)pre_pos[a] * 32 + d / 2;
        pre_cs[a][0] = cs[0];
        pre_cs[a][1] = cs[1];
      }
    }
  }
#pragma unroll
  for (int a = 0; a < UPW; ++a) {
    const int u = wave + a * SW_WAVES;
    if (u >= NU) continue;
    const int f0 = FPU == 1 ? u / MF : 2 * (u / MF);
    const int mm = u % MF;
    const int m = 16 * MF * mh + 16 * mm + r;
    if (m >= M) continue;                            // the four g lanes of token r together
    // fused RMSNorm of the input row (1 when none), from the entry prefetch
    const float rs = (EPI >= 2 && ne.ss_in)
                         ? rsqrtf((float)pre_ss[a] * (1.f / SS_FIX) * ne.inv_h + ne.eps) : 1.f;
    if constexpr (EPI == 2) {
      // gate fragment f0, up fragment f0 + 1: output features n0/2 + 8 f0 + 4 g + i
      const f32x4 gv = sum[a][0] * rs, uv = sum[a][1] * rs;
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (bf16)(gv[i] / (1.f + __expf(-gv[i])) * uv[i]);
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * (N >> 1) + (n0 >> 1) + 8 * f0 + 4 * g) = o;
    } else if constexpr (EPI == 3) {
      const int head = tile >> 1;
      const int d = 32 * (tile & 1) + 16 * (f0 >> 1) + 4 * g;       // first of 4 dims (< 64)
      const f32x4 x1 = sum[a][0] * rs, x2 = sum[a][1] * rs;
      bf16x4 o1, o2;
      const bool is_v = head >= ra.Hq + ra.Hkv;
      if (is_v) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o1[i] = (bf16)x1[i];
          o2[i] = (bf16)x2[i];
        }
      } else {
        const f32x4 c01 = pre_cs[EPI == 3 ? a : 0][0], c23 = pre_cs[EPI == 3 ? a : 0][1];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 cc = i < 2 ? c01 : c23;
          const float rc = cc[(i & 1) * 2], rsn = cc[(i & 1) * 2 + 1];
          o1[i] = (bf16)(x1[i] * rc - x2[i] * rsn);
          o2[i] = (bf16)(x2[i] * rc + x1[i] * rsn);
        }
      }
      bf16* dst;
      if (head < ra.Hq) {
        dst = reinterpret_cast<bf16*>(ra.q_out) + ((size_t)m * ra.Hq + head) * 128;
      } else {
        const int slot = pre_slot[a];
        if (slot < 0) continue;
        const int hk = head - ra.Hq - (is_v ? ra.Hkv : 0);
        dst = reinterpret_cast<bf16*>(is_v ? ra.v_cache : ra.k_cache) +
              (((size_t)(slot / ra.BS) * ra.Hkv + hk) * ra.BS + slot % ra.BS) * 128;
      }
      *reinterpret_cast<bf16x4*>(dst + d) = o1;
      *reinterpret_cast<bf16x4*>(dst + d + 64) = o2;
    } else {
#pragma unroll
      for (int j = 0; j < FPU; ++j) {
        const int n = n0 + 16 * (f0 + j) + 4 * g;
        f32x4 v = sum[a][j];
        if constexpr (EPI == 1) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] += (float)pre_rr[a][j][i];
        }
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)v[i];
        *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
        if (EPI == 1 && ne.ss_out) {
          // fused RMSNorm statistic: token r's 16 rows of this fragment sit in lanes r + 16 g
          float ss = sumsq_bf16x4(o);
          ss += __shfl_xor(ss, 16, 64);
          ss += __shfl_xor(ss, 32, 64);
          if (g == 0) ss_atomic_add(ne.ss_out + m, ss);
        }
      }
    }
  }
}

int g_stream_nt = -1;

template <int EPI, int MF, int NF, int DEPTH, int MH = 1>
void launch_v(const void* X, const void* W, void* Y, const void* R, int M, int N, int K, int S,
              float* ws, int* tk, const RopeArgs& ra, hipStream_t s) {
  const int tiles = N / (16 * NF);
  if (g_stream_nt < 0) {
    const char* e = getenv("MCP_GEMM_STREAM_NT");
    g_stream_nt = e ? atoi(e) : 0;
  }
  if (g_stream_nt)
    gemm_stream<EPI, MF, NF, DEPTH, MH, true><<<tiles * S, 256 * MH, 0, s>>>(
        (const bf16*)X, (const bf16*)W, (bf16*)Y, (const bf16*)R, M, N, K, S, ws, tk, ra,
        norm_epi());
  else
  gemm_stream<EPI, MF, NF, DEPTH, MH, false><<<tiles * S, 256 * MH, 0, s>>>((const bf16*)X, (const bf16*)W,
                                                             (bf16*)Y, (const bf16*)R, M, N, K, S,
                                                             ws, tk, ra, norm_epi());
}

template <int EPI>
int launch_epi(int variant, const void* X, const void* W, void* Y, const void* R, int M, int N,
               int K, int S, float* ws, int* tk, const RopeArgs& ra, hipStream_t s) {
  // variant = MF-class: 1 (M <= 16), 2 (<= 32), 4 (<= 64), 8 (<= 128)
  switch (variant) {
    case 1: launch_v<EPI, 1, 4, 4>(X, W, Y, R, M, N, K, S, ws, tk, ra, s); return 0;
    case 2: launch_v<EPI, 2, 4, 3>(X, W, Y, R, M, N, K, S, ws, tk, ra, s); return 0;
    case 4: launch_v<EPI, 4, 4, 2>(X, W, Y, R, M, N, K, S, ws, tk, ra, s); return 0;
    case 8: launch_v<EPI, 4, 4, 2, 2>(X, W, Y, R, M, N, K, S, ws, tk, ra, s); return 0;
    default: return 4;
  }
}

int g_stream_force_s = 0;      // tuning: > 0 forces the split count

}  // namespace

// MCP_STREAM_SPLIT_RULE=0: the round-3 split rule and skinny-first test (A/B)
int gemm_stream_rule() {
  static const int r = getenv("MCP_STREAM_SPLIT_RULE") ? atoi(getenv("MCP_STREAM_SPLIT_RULE")) : 1;
  return r;
}

void gemm_stream_force_splits(int S) { g_stream_force_s = S; }

// split count: fill two workgroups per CU with >= 4 k-steps per wave, S <= 8,
// partial tiles within the split-K workspace
int gemm_stream_splits(int M, int N, int K, int epi) {
  const int tiles = N / 64;
  const int nsteps = K / SW_STEP;
  if (g_stream_force_s > 0) return g_stream_force_s;
  // wide projections (gate|up, 448 tiles): measured with cold weights
  // (tools/bench_cold_stream.py) S = 3 at M <= 16, no split above
  if (tiles >= 256) return M <= 16 ? 3 : 1;
  if (gemm_stream_rule() == 0) {                     // round-3 rule (A/B)
    const int target = 2 * gemm256_num_cus();
    int S = 1;
    while (S < 8 && tiles * S * 2 <= target + tiles && nsteps / (2 * S) >= 4 * SW_WAVES) S *= 2;
    return S;
  }
  // about one workgroup per CU (<= 1.5 per CU), >= 4 k-steps per wave:
  // cold-weight sweep (tools/bench_decode_probe.py, profiles/gemm_decode_probe_r4.jsonl):
  // down 4096 x 14336 S = 4 23.6-24.4 us vs S = 8 24.7-25.6; o S = 4 best;
  // qkv S = 4 13.7-14.6 vs S = 2 14.2-15.0, S = 8 16.9-17.4
  const int G = gemm256_num_cus();
  int S = 1;
  while (S < 8 && 2 * tiles * S * 2 <= 3 * G && nsteps / (2 * S) >= 4 * SW_WAVES) S *= 2;
  (void)M;
  (void)epi;
  return S;
}

bool gemm_stream_pick(int M, int N, int K, int epi) {
  // measured on MI355X against the 128^2 split-K path with its reduce
  // kernel (profiles/gemm_stream_sweep.md): the stream kernel wins on the
  // narrow projections (qkv, o, down: N <= 6144) at M <= 32, on o (N K <=
  // 4096^2) up to M = 64; QKV + RoPE (epi 3) also saves the rope_kv launch up
  // to M = 64.  gate|up (N = 28672) keeps the 128^2 path (448 workgroups at
  // S = 2 already stream at ~6 TB/s).
  if (M > 64) return false;
  // gate|up (N >= 16384): cold-weight sweep (tools/bench_cold_stream.py), the
  // stream kernel beats split-K 128^2 at M = 9-32 (48.9-55.3 vs 51.3-59.7 us);
  // M <= 8 / 12 go to the skinny kernel first (gemm.hip skinny_first).
  // MCP_STREAM_WIDE_MAXM: upper M for the wide projections (A/B)
  static const int wide_max = getenv("MCP_STREAM_WIDE_MAXM") ? atoi(getenv("MCP_STREAM_WIDE_MAXM")) : 32;
  if (N >= 16384) return M > 8 && M <= wide_max;
  if (M <= 32 || epi == 3) return true;
  return (long long)N * K <= 4096LL * 4096LL;
}

int gemm_stream_ok(int M, int N, int K, int epi, int D, int Hq, int Hkv) {
  if (M <= 0 || M > GEMM_STREAM_MAX_M || K % SW_STEP || N % 64) return 0;
  if (epi == 3) return D == 128 && N == (Hq + 2 * Hkv) * 128;
  return 1;
}

// epi: 0 plain, 1 + R, 2 SwiGLU (Y [M, N/2]), 3 QKV + RoPE (ra); nonzero if unsupported
int launch_gemm_stream(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                       int epi, const RopeArgs& ra, hipStream_t s) {
  if (!gemm_stream_ok(M, N, K, epi, 128, ra.Hq, ra.Hkv)) return 1;
  int S = gemm_stream_splits(M, N, K, epi);
  float* ws = nullptr;
  int* tk = nullptr;
  const int variant = M <= 16 ? 1 : M <= 32 ? 2 : M <= 64 ? 4 : 8;
  const size_t tile_bytes = (size_t)16 * variant * 64 * 4;
  if (S > 1 && !gemm_splitk_workspace(&ws, &tk, (size_t)(N / 64) * S * tile_bytes, N / 64)) S = 1;
  switch (epi) {
    case 0: return launch_epi<0>(variant, X, W, Y, nullptr, M, N, K, S, ws, tk, ra, s);
    case 1: return launch_epi<1>(variant, X, W, Y, R, M, N, K, S, ws, tk, ra, s);
    case 2: return launch_epi<2>(variant, X, W, Y, nullptr, M, N, K, S, ws, tk, ra, s);
    case 3: return launch_epi<3>(variant, X, W, Y, nullptr, M, N, K, S, ws, tk, ra, s);
    default: return 2;
  }
}
