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
//    registers.  Lane l = (row r = l&15, group g = l>>4) loads 64 contiguous
//    bytes W[r][s*128 + 32g .. +32) per step; the X fragment uses the SAME
//    k permutation (a dot product is order-free), so MFMA j consumes the 8-wide
//    chunk j of every lane group and four MFMAs cover the 128-k step;
//  * the next step's W is loaded before this step's MFMAs (register double
//    buffer) to keep ~8 KiB per wave in flight;
//  * M > 64 runs ceil(M/64) token groups as extra workgroups placed on the
//    same XCD as their weight rows' first group (shared L2).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int SK_WAVES = 8;
constexpr int SK_STEP = 128;

template <int RB>
DEV void load_w(const bf16* const (&wrow)[RB], int k, bf16x8 (&w)[RB][4]) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int j = 0; j < 4; ++j) w[rb][j] = *reinterpret_cast<const bf16x8*>(wrow[rb] + k + 8 * j);
}

// WV waves per workgroup split K (wave w takes steps w, w + WV, ...), each
// with a DEPTH-deep register ring of weight steps in flight (DEPTH 1: the
// next step is loaded while this one computes).  The SwiGLU shape (32 rows
// per workgroup, gate|up = 235 MB) streams best with few waves per row group
// and a deep ring was the hypothesis - measured no faster (launch_mb).
template <int EPI, int MB, int WV, int DEPTH>
__global__ __launch_bounds__(64 * WV) void gemm_skinny(const bf16* __restrict__ X,
                                                   const bf16* __restrict__ W,
                                                   bf16* __restrict__ Y,
                                                   const bf16* __restrict__ R, int M, int N, int K,
                                                   int nx, int ny, const NormEpi ne) {
  constexpr int RB = EPI == 2 ? 2 : 1;               // 16-row weight blocks per workgroup
  __shared__ f32x4 red[WV][RB][MB][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int lid = xcd_remap(blockIdx.x, nx * ny);
  const int bx = lid / ny, by = lid % ny;
  const int n0 = bx * 16 * RB, m0 = by * 16 * MB;

  const bf16* wrow[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) wrow[rb] = W + (size_t)min(n0 + rb * 16 + r, N - 1) * K + 32 * g;
  const bf16* xrow[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) xrow[mb] = X + (size_t)min(m0 + mb * 16 + r, M - 1) * K + 32 * g;

  f32x4 acc[RB][MB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = K / SK_STEP;
  const int count = nsteps > wave ? (nsteps - wave + WV - 1) / WV : 0;
  bf16x8 wr[DEPTH][RB][4];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < count) load_w<RB>(wrow, (wave + d * WV) * SK_STEP, wr[d]);
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
            x[mb][j] = *reinterpret_cast<const bf16x8*>(xrow[mb] + s * SK_STEP + 8 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = mfma16x16x32(wr[d][rb][j], x[mb][j], acc[rb][mb]);
        if (i + DEPTH < count) load_w<RB>(wrow, (s + DEPTH * WV) * SK_STEP, wr[d]);
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
    if (m >= M) continue;                            // all four g lanes of token r together
    if constexpr (EPI == 2) {
      const int F = N >> 1, f = (n0 >> 1) + 4 * g;   // f < F: N % 32 == 0 (skinny_ok)
      const float rs = norm_row_scale(ne, m);
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
        const bf16x4 rr = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += (float)rr[q];
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

template <int EPI, int MB, int WV, int DEPTH>
void launch_form(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                 hipStream_t s) {
  constexpr int RB = EPI == 2 ? 2 : 1;
  const int nx = (N + 16 * RB - 1) / (16 * RB), ny = (M + 16 * MB - 1) / (16 * MB);
  gemm_skinny<EPI, MB, WV, DEPTH><<<nx * ny, 64 * WV, 0, s>>>(
      (const bf16*)X, (const bf16*)W, (bf16*)Y, (const bf16*)R, M, N, K, nx, ny, norm_epi());
}

template <int EPI, int MB>
void launch_mb(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
               hipStream_t s) {
  // 8 waves x a 1-deep ring: 2 x 2, 4 x 2 and 4 x 4 measured no faster at
  // M = 1-16 on any Llama-3-8B shape, cold weights (profiles/gemm_skinny_forms_r3.jsonl)
  launch_form<EPI, MB, SK_WAVES, 1>(X, W, Y, R, M, N, K, s);
}

template <int EPI>
void launch_epi(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                hipStream_t s) {
  if (M <= 16) launch_mb<EPI, 1>(X, W, Y, R, M, N, K, s);
  else if (M <= 32) launch_mb<EPI, 2>(X, W, Y, R, M, N, K, s);
  else launch_mb<EPI, 4>(X, W, Y, R, M, N, K, s);
}

}  // namespace

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
