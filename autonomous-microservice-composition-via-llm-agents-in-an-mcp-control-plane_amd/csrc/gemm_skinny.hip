// K2: skinny GEMM for decode-sized steps (M = tokens in the step <= 128).
//   Y[M,N] = X[M,K] . W[N,K]^T  (+R | SwiGLU), fp32 accumulate, bf16 out.
//
// At small M a projection is a weight stream: 2*M flop per weight byte is far
// below the MI355X ridge point (~400 flop/B), so the kernel's job is to keep
// HBM busy.  The 128^2 / 256^2 tile kernels launch only N/128 workgroups here
// (32 for N = 4096) and leave most of the 256 CUs idle.  Instead:
//
//  * one workgroup = 8 waves per 16 weight rows (32 for SwiGLU: a gate group
//    and its up group), so N = 4096 launches 256 x 8 waves;
//  * the waves split K (128-deep steps, strided) and reduce through LDS;
//  * no LDS staging of W: v_mfma_f32_16x16x32_bf16 takes W straight from
//    registers.  Lane l = (row r = l&15, group g = l>>4) loads
//    W[r][s*128 + 32j + 8g .. +8) with load j = 0..3, so each load instruction
//    reads 64 contiguous bytes of each of 16 rows (the 4 lane groups of a row
//    together), and MFMA j consumes k = 32j .. 32j + 31 of the step; the X
//    fragment uses the same offsets.  (The earlier order, 64 contiguous bytes
//    per LANE over the 4 loads, sent each instruction to 64 scattered 16-B
//    pieces: the activation rows' share of that request traffic cost up to
//    12 us of a 52 us gate|up at M = 8, profiles/gemm_decode_probe_r4.jsonl);
//  * the next step's W is loaded before this step's MFMAs (register double
//    buffer) to keep ~8 KiB per wave in flight;
//  * M > 64 runs ceil(M/64) token groups as extra workgroups placed on the
//    same XCD as their weight rows' first group (shared L2).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int SK_WAVES = 8;
constexpr int SK_STEP = 128;

// NT: non-temporal weight loads (MI355X_MICROARCH.md "nt-weights": a decode
// step streams every weight once, from cold caches)
template <int RB, bool NT>
DEV void load_w(const bf16* const (&wrow)[RB], int k, bf16x8 (&w)[RB][4]) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bf16x8* p = reinterpret_cast<const bf16x8*>(wrow[rb] + k + 32 * j);
      if constexpr (NT) w[rb][j] = __builtin_nontemporal_load(p);
      else w[rb][j] = *p;
    }
}

// WV waves per workgroup split K (wave w takes steps w, w + WV, ...), each
// with a DEPTH-deep register ring of weight steps in flight (DEPTH 1: the
// next step is loaded while this one computes).  The SwiGLU shape (32 rows
// per workgroup, gate|up = 235 MB) streams best with few waves per row group
// and a deep ring was the hypothesis - measured no faster (launch_mb).
// HALF (SwiGLU only): a workgroup owns 8 output features - 8 gate rows and
// their 8 up rows in ONE 16-row MFMA block (lanes r < 8 read gate rows, r >= 8
// up rows; the accumulator's rows 8..15 sit 32 lanes above rows 0..7), so the
// gate|up GEMM launches N / 16 workgroups like the plain one (1,792 for
// Llama-3-8B: 7 per CU) instead of N / 32 (896: 3.5 per CU, the CUs holding 4
// set the time).
template <int EPI, int MB, int WV, int DEPTH, bool NT, bool HALF>
__global__ __launch_bounds__(64 * WV) void gemm_skinny(const bf16* __restrict__ X,
                                                   const bf16* __restrict__ W,
                                                   bf16* __restrict__ Y,
                                                   const bf16* __restrict__ R, int M, int N, int K,
                                                   int nx, int ny, const NormEpi ne, int mload) {
  static_assert(!HALF || EPI == 2, "HALF is a SwiGLU form");
  constexpr int RB = EPI == 2 && !HALF ? 2 : 1;      // 16-row weight blocks per workgroup
  __shared__ f32x4 red[WV][RB][MB][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int lid = xcd_remap(blockIdx.x, nx * ny);
  const int bx = lid / ny, by = lid % ny;
  const int n0 = bx * 16 * RB, m0 = by * 16 * MB;

  const bf16* wrow[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    // HALF: block bx = features 8 bx .. + 8 = pair bx / 2 (32 rows: 16 gate, 16 up), half bx & 1
    const int row = HALF ? 32 * (bx >> 1) + 8 * (bx & 1) + (r & 7) + 16 * (r >> 3) : n0 + rb * 16 + r;
    wrow[rb] = W + (size_t)min(row, N - 1) * K + 8 * g;
  }
  const bf16* xrow[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) xrow[mb] = X + (size_t)min(m0 + mb * 16 + r, mload - 1) * K + 8 * g;

  f32x4 acc[RB][MB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the epilogue's row inputs, loaded before the weight stream (after it they
  // are one more dependent round trip at the end of a ~20-50 us decode kernel):
  // the fused-norm statistic (SwiGLU), the residual piece (EPI 1)
  unsigned long long pre_ss[MB];
  bf16x4 pre_rr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    pre_ss[mb] = 0;
    const int m = min(m0 + mb * 16 + r, M - 1);
    if constexpr (EPI == 1)
      pre_rr[mb] = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + min(n0 + 4 * g, N - 4));
  }
  if (EPI == 2 && ne.ss_in) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) pre_ss[mb] = ne.ss_in[min(m0 + mb * 16 + r, M - 1)];
  }
  auto pre_rs = [&](int mb) -> float {
    return ne.ss_in ? rsqrtf((float)pre_ss[mb] * (1.f / SS_FIX) * ne.inv_h + ne.eps) : 1.f;
  };

  const int nsteps = K / SK_STEP;
  const int count = nsteps > wave ? (nsteps - wave + WV - 1) / WV : 0;
  bf16x8 wr[DEPTH][RB][4];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < count) load_w<RB, NT>(wrow, (wave + d * WV) * SK_STEP, wr[d]);
  for (int i0 = 0; i0 < count; i0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int i = i0 + d;
      if (i < count) {
        const int s = wave + i * WV;
        bf16x8 x[MB][4];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            x[mb][j] = *reinterpret_cast<const bf16x8*>(xrow[mb] + s * SK_STEP + 32 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = mfma16x16x32(wr[d][rb][j], x[mb][j], acc[rb][mb]);
        if (i + DEPTH < count) load_w<RB, NT>(wrow, (s + DEPTH * WV) * SK_STEP, wr[d]);
      }
    }
  }

#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) red[wave][rb][mb][lane] = acc[rb][mb];
  __syncthreads();
  // token group mb of the workgroup is reduced and stored by wave mb % WV
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    if (mb % WV != wave) continue;
    f32x4 tot[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      tot[rb] = red[0][rb][mb][lane];
#pragma unroll
      for (int w = 1; w < WV; ++w) tot[rb] += red[w][rb][mb][lane];
    }
    // C layout: lane holds rows (weight n) 4g..4g+3 of column (token) r
    const int m = m0 + mb * 16 + r;
    if constexpr (HALF) {
      // lanes g < 2: gate features 8 bx + 4 g + q; the up values of the same
      // features sit in lane + 32 (rows 8 + 4 g + q)
      f32x4 up;
#pragma unroll
      for (int q = 0; q < 4; ++q) up[q] = __shfl_xor(tot[0][q], 32, 64);
      if (m >= M || g >= 2) continue;
      const float rs = pre_rs(mb);
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gv = tot[0][q] * rs, uv = up[q] * rs;
        o[q] = (bf16)(gv / (1.f + __expf(-gv)) * uv);
      }
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * (N >> 1) + 8 * bx + 4 * g) = o;
      continue;
    }
    if (m >= M) continue;                            // all four g lanes of token r together
    if constexpr (EPI == 2) {
      const int F = N >> 1, f = (n0 >> 1) + 4 * g;   // f < F: N % 32 == 0 (skinny_ok)
      const float rs = pre_rs(mb);
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gv = tot[0][q] * rs, uv = tot[1][q] * rs;
        o[q] = (bf16)(gv / (1.f + __expf(-gv)) * uv);
      }
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * F + f) = o;
    } else {
      const int n = n0 + 4 * g;                      // n < N: N % 16 == 0 (skinny_ok)
      f32x4 v = tot[0];
      if (EPI == 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += (float)pre_rr[mb][q];
      }
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (bf16)v[q];
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
      if (EPI == 1 && ne.ss_out) {
        // fused RMSNorm statistic: the 16 columns of token r sit in lanes r + 16 g
        float ss = sumsq_bf16x4(o);
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        if (g == 0) ss_atomic_add(ne.ss_out + m, ss);
      }
    }
  }
}

// SwiGLU form: 1 = HALF at M <= 4 (default), 2 = HALF always, 0 = 32-row blocks.
// Cold weights (tools/bench_swiglu_decode.py, profiles/gemm_swiglu_decode_r4.jsonl):
// HALF 40.3-41.1 vs 43.2-43.6 us on 8B gate|up at M = 1-4, equal at 8-16 there,
// but 167 vs 156 us on 70B gate|up at M = 8
int g_skinny_half = -1;

template <int EPI, int MB, int WV, int DEPTH, bool HALF>
void launch_form(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                 hipStream_t s) {
  constexpr int RB = EPI == 2 && !HALF ? 2 : 1;
  const int nx = (N + 16 * RB - 1) / (16 * RB), ny = (M + 16 * MB - 1) / (16 * MB);
  // non-temporal weight loads: measured 12-19 % slower end to end (config 2,
  // profiles/gemm_decode_nt_r4_ab.txt); kept selectable
  static const int nt = getenv("MCP_GEMM_SKINNY_NT") ? atoi(getenv("MCP_GEMM_SKINNY_NT")) : 0;
  // timing probe only (wrong results): every token row loads row 0 of X
  static const int x1 = getenv("MCP_PROBE_SKINNY_X1") ? atoi(getenv("MCP_PROBE_SKINNY_X1")) : 0;
  const int mload = x1 ? 1 : M;
  if (nt)
    gemm_skinny<EPI, MB, WV, DEPTH, true, HALF><<<nx * ny, 64 * WV, 0, s>>>(
        (const bf16*)X, (const bf16*)W, (bf16*)Y, (const bf16*)R, M, N, K, nx, ny, norm_epi(), mload);
  else
    gemm_skinny<EPI, MB, WV, DEPTH, false, HALF><<<nx * ny, 64 * WV, 0, s>>>(
        (const bf16*)X, (const bf16*)W, (bf16*)Y, (const bf16*)R, M, N, K, nx, ny, norm_epi(), mload);
}

template <int EPI, int MB>
void launch_mb(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
               hipStream_t s) {
  // 8 waves x a 1-deep ring: 2 x 2, 4 x 2 and 4 x 4 measured no faster at
  // M = 1-16 on any Llama-3-8B shape, cold weights (profiles/gemm_skinny_forms_r3.jsonl)
  if (g_skinny_half < 0) {
    const char* e = getenv("MCP_GEMM_SKINNY_HALF");
    g_skinny_half = e ? atoi(e) : 1;
  }
  if (EPI == 2 && (g_skinny_half == 2 || (g_skinny_half == 1 && M <= 4))) {
    launch_form<EPI, MB, SK_WAVES, 1, EPI == 2>(X, W, Y, R, M, N, K, s);
    return;
  }
  // MCP_GEMM_SKINNY_FORM (A/B after the round-4 load-order fix, M <= 16):
  // 0 = 8 waves x 1-deep ring, 1 = 8 x 2, 2 = 4 x 2, 3 = 4 x 4, 4 = 8 x 4,
  // 5 = 8 x 4 for EPI 0 / 1 only (form 4 on config 2: 87.7 vs 84.5-85.3 ms)
  // (round 6: at K = 4096 every wave's 4 steps in flight at once, 128 KiB
  // per CU - the o projection of config 2 streams at ~2.5 TB/s with 32 KiB)
  static const int form = getenv("MCP_GEMM_SKINNY_FORM") ? atoi(getenv("MCP_GEMM_SKINNY_FORM")) : 0;
  if constexpr (MB == 1) {
    switch (form) {
      case 1: launch_form<EPI, MB, 8, 2, false>(X, W, Y, R, M, N, K, s); return;
      case 2: launch_form<EPI, MB, 4, 2, false>(X, W, Y, R, M, N, K, s); return;
      case 3: launch_form<EPI, MB, 4, 4, false>(X, W, Y, R, M, N, K, s); return;
      case 4: launch_form<EPI, MB, 8, 4, false>(X, W, Y, R, M, N, K, s); return;
      case 5:                                        // 8 x 4 for the plain / residual GEMMs only
        if constexpr (EPI != 2) {
          launch_form<EPI, MB, 8, 4, false>(X, W, Y, R, M, N, K, s);
          return;
        }
        break;
      default: break;
    }
  }
  launch_form<EPI, MB, SK_WAVES, 1, false>(X, W, Y, R, M, N, K, s);
}

template <int EPI>
void launch_epi(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                hipStream_t s) {
  if (M <= 16) launch_mb<EPI, 1>(X, W, Y, R, M, N, K, s);
  else if (M <= 32) launch_mb<EPI, 2>(X, W, Y, R, M, N, K, s);
  else launch_mb<EPI, 4>(X, W, Y, R, M, N, K, s);
}

}  // namespace

void gemm_skinny_half(int on) { g_skinny_half = on; }

int skinny_ok(int M, int N, int K, int epi) {
  if (M <= 0 || M > SKINNY_MAX_M || K % SK_STEP) return 0;
  if (epi == 2) return N % 32 == 0;
  return N % 16 == 0;
}

// epi: 0 plain, 1 + residual R, 2 SwiGLU (Y is [M, N/2]); returns nonzero if unsupported
int launch_gemm_skinny(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                       int epi, hipStream_t s) {
  if (!skinny_ok(M, N, K, epi)) return 1;
  if (epi == 2) launch_epi<2>(X, W, Y, nullptr, M, N, K, s);
  else if (R) launch_epi<1>(X, W, Y, R, M, N, K, s);
  else launch_epi<0>(X, W, Y, nullptr, M, N, K, s);
  return 0;
}
