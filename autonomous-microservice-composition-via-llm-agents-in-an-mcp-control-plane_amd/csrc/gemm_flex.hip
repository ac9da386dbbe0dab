// K1 at serving-size M (~200-2000 rows): bf16 "TN" GEMM with a tile shape
// picked per (M, N) so that ONE wave of workgroups covers the output.
//
// At these sizes a fixed 128x128 tile leaves the chip part-empty (qkv at
// M = 512: 4 x 48 = 192 tiles for 256 CUs) and split-K pays an fp32 partial
// round trip through HBM plus a reduce launch.  Here the tile is TM x TN with
// TM, TN multiples of 32 (64 ... 256 rows, 32 ... 192 columns) and the
// candidate whose tile count lands at or just under the CU count is chosen
// by the measured plan (tools/tune_gemm_plan.py, code 3 + "flex" index);
// each workgroup walks the whole K, the epilogue (plain / + residual /
// SwiGLU) is applied in registers, no workspace.
//
// Structure = the 128^2 kernel (gemm.hip) generalised: 4 waves in a 2 x 2
// grid, each (TM/2) x (TN/2) = (TM/32) x (TN/32) v_mfma_f32_16x16x32_bf16
// tiles; BK = 64; operands staged global -> LDS by global_load_lds_dwordx4
// (8-row x 128-B pieces, TM/32 + TN/32 per wave), double-buffered, XOR
// swizzle chunk ^= row & 7 on source and read; <= 80 KiB LDS, so two
// workgroups share a CU; XCD-aware grouped tile order.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int FBK = 64;

// SwiGLU epilogue (EPI 2): common.h store_silu (row scales hoisted)
template <int EPI, int MT, int NT>
DEV void flex_store(const f32x4 (&acc)[MT][NT], bf16* __restrict__ Y, const bf16* __restrict__ R,
                    int M, int N, int mb, int nb, int fr, int fq, const NormEpi& ne) {
  if constexpr (EPI == 2) store_silu<MT, NT>(acc, Y, M, N, mb, nb, fr, fq, ne);
  else store_direct<EPI>(acc, Y, R, M, N, mb, nb, fr, fq, ne);
}

template <int EPI, int TM, int TN>     // EPI: 0 plain, 1 + residual, 2 SwiGLU
__global__ __launch_bounds__(256, 2) void gemm_tn_flex(const bf16* __restrict__ X,
                                                       const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y,
                                                       const bf16* __restrict__ R, int M, int N,
                                                       int K, const NormEpi ne) {
  static_assert(TM % 32 == 0 && TN % 32 == 0, "tile dims are multiples of 32");
  static_assert(2 * (TM + TN) * FBK * 2 <= 80 * 1024, "two workgroups per CU");
  constexpr int MT = TM / 32, NT = TN / 32;        // 16-row MFMA tiles per wave
  constexpr int PA = TM / 32, PB = TN / 32;        // 8-row staging pieces per wave
  constexpr int AE = TM * FBK, BE = TN * FBK;      // elements per operand tile
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (AE + BE)];   // [buf][A | B]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nm = (M + TM - 1) / TM, nn = (N + TN - 1) / TN;
  const int nwg = nm * nn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;                         // m-tiles sharing each W panel
  const int per_group = GROUP * nn;
  const int g = wg / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;
  const int m0 = tm * TM, n0 = tn * TN;

  const int lrow = lane >> 3;                      // row inside the 8-row piece
  const int lchunk = (lane & 7) ^ lrow;            // inverse swizzle on the source
  const bf16* srcA[PA];
  const bf16* srcB[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = (wave * PA + i) * 8 + lrow;
    srcA[i] = X + (size_t)min(m0 + row, M - 1) * K + lchunk * 8;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = (wave * PB + i) * 8 + lrow;
    srcB[i] = W + (size_t)min(n0 + row, N - 1) * K + lchunk * 8;
  }
  auto stage = [&](int kt, int buf) {
    bf16* la = smem + buf * (AE + BE);
    bf16* lb = la + AE;
    const int koff = kt * FBK;
#pragma unroll
    for (int i = 0; i < PA; ++i) glds16(srcA[i] + koff, la + (wave * PA + i) * 512);
#pragma unroll
    for (int i = 0; i < PB; ++i) glds16(srcB[i] + koff, lb + (wave * PB + i) * 512);
  };

  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / FBK;
  stage(0, 0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const bf16* la = smem + cur * (AE + BE);
    const bf16* lb = la + AE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int ra = wm * (TM / 2) + t * 16 + fr;
        af[t] = *reinterpret_cast<const bf16x8*>(la + ra * FBK + ((c ^ (ra & 7)) << 3));
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int rb = wn * (TN / 2) + t * 16 + fr;
        bfr[t] = *reinterpret_cast<const bf16x8*>(lb + rb * FBK + ((c ^ (rb & 7)) << 3));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(bfr[nt], af[mt], acc[mt][nt]);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds Y[m][n .. n+3]
  flex_store<EPI>(acc, Y, R, M, N, m0 + wm * (TM / 2), n0 + wn * (TN / 2), fr, fq, ne);
}

// Split-K form of the 2-stage flex tile: gridDim.y = S workgroups per tile
// each walk K / S and write fp32 partials [S][M][N] (lane: Y[m][n .. n+3]);
// gemm.hip's splitk_reduce sums them and applies the epilogue.  Serving-M
// tiles that hold all M rows (W read once) but are too few to fill the chip.
template <int TM, int TN>
__global__ __launch_bounds__(256, 2) void gemm_tn_flex_sk(const bf16* __restrict__ X,
                                                          const bf16* __restrict__ W,
                                                          float* __restrict__ ws, int M, int N,
                                                          int K) {
  static_assert(TM % 32 == 0 && TN % 32 == 0, "tile dims are multiples of 32");
  static_assert(2 * (TM + TN) * FBK * 2 <= 80 * 1024, "two workgroups per CU");
  constexpr int MT = TM / 32, NT = TN / 32;
  constexpr int PA = TM / 32, PB = TN / 32;
  constexpr int AE = TM * FBK, BE = TN * FBK;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (AE + BE)];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nm = (M + TM - 1) / TM, nn = (N + TN - 1) / TN;
  const int wg = xcd_remap(blockIdx.x, nm * nn);
  const int tm = wg % nm, tn = wg / nm;
  const int m0 = tm * TM, n0 = tn * TN;
  const int klen = K / (int)gridDim.y, kbeg = (int)blockIdx.y * klen;
  float* Yp = ws + (size_t)blockIdx.y * M * N;

  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const bf16* srcA[PA];
  const bf16* srcB[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = (wave * PA + i) * 8 + lrow;
    srcA[i] = X + (size_t)min(m0 + row, M - 1) * K + kbeg + lchunk * 8;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = (wave * PB + i) * 8 + lrow;
    srcB[i] = W + (size_t)min(n0 + row, N - 1) * K + kbeg + lchunk * 8;
  }
  auto stage = [&](int kt, int buf) {
    bf16* la = smem + buf * (AE + BE);
    bf16* lb = la + AE;
    const int koff = kt * FBK;
#pragma unroll
    for (int i = 0; i < PA; ++i) glds16(srcA[i] + koff, la + (wave * PA + i) * 512);
#pragma unroll
    for (int i = 0; i < PB; ++i) glds16(srcB[i] + koff, lb + (wave * PB + i) * 512);
  };
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = klen / FBK;
  stage(0, 0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const bf16* la = smem + cur * (AE + BE);
    const bf16* lb = la + AE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int ra = wm * (TM / 2) + t * 16 + fr;
        af[t] = *reinterpret_cast<const bf16x8*>(la + ra * FBK + ((c ^ (ra & 7)) << 3));
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int rb = wn * (TN / 2) + t * 16 + fr;
        bfr[t] = *reinterpret_cast<const bf16x8*>(lb + rb * FBK + ((c ^ (rb & 7)) << 3));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(bfr[nt], af[mt], acc[mt][nt]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = m0 + wm * (TM / 2) + mt * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + wn * (TN / 2) + nt * 16 + fq * 4;
      if (n < N) *reinterpret_cast<f32x4*>(Yp + (size_t)m * N + n) = acc[mt][nt];
    }
  }
}

template <int TM, int TN>
void flex_sk_launch(const void* X, const void* W, float* ws, int M, int N, int K, int S,
                    hipStream_t s) {
  const dim3 grid(((M + TM - 1) / TM) * ((N + TN - 1) / TN), S);
  gemm_tn_flex_sk<TM, TN><<<grid, 256, 0, s>>>((const bf16*)X, (const bf16*)W, ws, M, N, K);
}

// One workgroup per CU, NST LDS stages with NST - 2 k-tiles in flight across
// a raw s_barrier and a counted vmcnt: ONE barrier per k-tile (the 2-stage
// loop above drains vmcnt(0) every k-tile - at one wave of workgroups each
// k-tile then waits the full DMA latency).  Every iteration issues one tile's
// DMAs (past the end: the last tile again, into the slot just freed) so the
// vmcnt counts are static.
template <int EPI, int TM, int TN, int NST>
__global__ __launch_bounds__(256, 1) void gemm_tn_flexp(const bf16* __restrict__ X,
                                                        const bf16* __restrict__ W,
                                                        bf16* __restrict__ Y,
                                                        const bf16* __restrict__ R, int M, int N,
                                                        int K, const NormEpi ne) {
  static_assert(TM % 32 == 0 && TN % 32 == 0, "tile dims are multiples of 32");
  static_assert(NST * (TM + TN) * FBK * 2 <= 160 * 1024, "LDS");
  constexpr int MT = TM / 32, NT = TN / 32;
  constexpr int PA = TM / 32, PB = TN / 32;
  constexpr int AE = TM * FBK, BE = TN * FBK;
  constexpr int VM = (NST - 2) * (PA + PB);          // this wave's DMAs still allowed in flight
  static_assert(VM <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) bf16 smem[NST * (AE + BE)];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nm = (M + TM - 1) / TM, nn = (N + TN - 1) / TN;
  const int nwg = nm * nn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * nn;
  const int g = wg / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;
  const int m0 = tm * TM, n0 = tn * TN;

  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const bf16* srcA[PA];
  const bf16* srcB[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = (wave * PA + i) * 8 + lrow;
    srcA[i] = X + (size_t)min(m0 + row, M - 1) * K + lchunk * 8;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = (wave * PB + i) * 8 + lrow;
    srcB[i] = W + (size_t)min(n0 + row, N - 1) * K + lchunk * 8;
  }
  const int nk = K / FBK;
  auto stage = [&](int kt, int slot) {
    const int koff = min(kt, nk - 1) * FBK;
    bf16* la = smem + slot * (AE + BE);
    bf16* lb = la + AE;
#pragma unroll
    for (int i = 0; i < PA; ++i) glds16(srcA[i] + koff, la + (wave * PA + i) * 512);
#pragma unroll
    for (int i = 0; i < PB; ++i) glds16(srcB[i] + koff, lb + (wave * PB + i) * 512);
  };

  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NST - 1; ++t) stage(t, t);
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");   // this wave's DMAs of tile kt landed
    __builtin_amdgcn_s_barrier();                      // ... every wave's; slot of kt-1 is free
    asm volatile("" ::: "memory");
    stage(kt + NST - 1, (kt + NST - 1) % NST);
    const bf16* la = smem + (kt % NST) * (AE + BE);
    const bf16* lb = la + AE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int ra = wm * (TM / 2) + t * 16 + fr;
        af[t] = *reinterpret_cast<const bf16x8*>(la + ra * FBK + ((c ^ (ra & 7)) << 3));
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int rb = wn * (TN / 2) + t * 16 + fr;
        bfr[t] = *reinterpret_cast<const bf16x8*>(lb + rb * FBK + ((c ^ (rb & 7)) << 3));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(bfr[nt], af[mt], acc[mt][nt]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments read before the slot is reused
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the trailing re-loads land before exit

  flex_store<EPI>(acc, Y, R, M, N, m0 + wm * (TM / 2), n0 + wn * (TN / 2), fr, fq, ne);
}

template <int EPI, int TM, int TN>
void flex_launch_epi(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                     hipStream_t s, int pipe) {
  const dim3 grid(((M + TM - 1) / TM) * ((N + TN - 1) / TN));
  // tiles too tall for two workgroups per CU (TM + TN > 320: the whole-M
  // tiles of wide projections, one W read per column panel) have only the
  // one-workgroup-per-CU form, with as many stages as LDS holds
  constexpr bool two = 2 * (TM + TN) * FBK * 2 <= 80 * 1024;
  constexpr int NST = 4 * (TM + TN) * FBK * 2 <= 160 * 1024 ? 4 : 3;
  if (pipe || !two)
    gemm_tn_flexp<EPI, TM, TN, NST><<<grid, 256, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                                         (const bf16*)R, M, N, K, norm_epi());
  else if constexpr (two)
    gemm_tn_flex<EPI, TM, TN><<<grid, 256, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                                   (const bf16*)R, M, N, K, norm_epi());
}

// epi 2 only for tiles whose per-wave column span holds whole gate | up pairs
template <int TM, int TN>
int flex_launch(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                hipStream_t s, int pipe, int epi) {
  if (epi == 2) {
    if constexpr ((TN / 2) % 32 == 0) {
      flex_launch_epi<2, TM, TN>(X, W, Y, nullptr, M, N, K, s, pipe);
      return 0;
    }
    return 3;
  }
  if (epi == 1) flex_launch_epi<1, TM, TN>(X, W, Y, R, M, N, K, s, pipe);
  else flex_launch_epi<0, TM, TN>(X, W, Y, nullptr, M, N, K, s, pipe);
  return 0;
}

}  // namespace

// candidate tiles (TM rows x TN columns); the index is what the plan records
static const int kFlexTiles[][2] = {{64, 64},   {64, 128},  {64, 160},  {96, 64},
                                    {96, 128},  {128, 96},  {128, 128}, {128, 160},
                                    {128, 192}, {256, 32},  {192, 128}, {160, 128}};
// (round 4: whole-M tiles 256 x 128 / 256 x 64 for the wide gate|up at M <=
// 256, one W read per column panel, were timed by the tuner on every gate|up
// shape and won no bucket - profiles/gemm_tuning.md)

int gemm_flex_count() { return (int)(sizeof(kFlexTiles) / sizeof(kFlexTiles[0])); }

int gemm_flex_tiles(int cand, int M, int N) {
  if (cand < 0 || cand >= gemm_flex_count()) return -1;
  return ((M + kFlexTiles[cand][0] - 1) / kFlexTiles[cand][0]) *
         ((N + kFlexTiles[cand][1] - 1) / kFlexTiles[cand][1]);
}

// 0 ok; 1 unknown candidate; 2 shape (K % 64, N % 4; SwiGLU N % 64);
// 3 the candidate has no SwiGLU form.  cand + 32: the 4-stage
// one-workgroup-per-CU form.  epi: 0 plain, 1 + residual R, 2 SwiGLU (Y [M, N/2])
int launch_gemm_flex_epi(const void* X, const void* W, void* Y, const void* R, int M, int N,
                         int K, int cand, int epi, hipStream_t s) {
  if (K % FBK || N % 4 || M <= 0 || (epi == 2 && N % 64)) return 2;
  const int pipe = cand >= 32;
  cand &= 31;
  switch (cand) {
    case 0: return flex_launch<64, 64>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 1: return flex_launch<64, 128>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 2: return flex_launch<64, 160>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 3: return flex_launch<96, 64>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 4: return flex_launch<96, 128>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 5: return flex_launch<128, 96>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 6: return flex_launch<128, 128>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 7: return flex_launch<128, 160>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 8: return flex_launch<128, 192>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 9: return flex_launch<256, 32>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 10: return flex_launch<192, 128>(X, W, Y, R, M, N, K, s, pipe, epi);
    case 11: return flex_launch<160, 128>(X, W, Y, R, M, N, K, s, pipe, epi);
    default: return 1;
  }
}

int launch_gemm_flex(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                     int cand, hipStream_t s) {
  return launch_gemm_flex_epi(X, W, Y, R, M, N, K, cand, R ? 1 : 0, s);
}

// fp32 split-K partials [S][M][N] of flex tile cand (2-stage form) into ws;
// nonzero if unsupported (K % (64 S), N % 4, the 2-stage form's LDS)
int launch_gemm_flex_partials(const void* X, const void* W, float* ws, int M, int N, int K,
                              int cand, int S, hipStream_t s) {
  if (S < 2 || K % (FBK * S) || N % 4 || M <= 0) return 2;
  switch (cand & 31) {
    case 0: flex_sk_launch<64, 64>(X, W, ws, M, N, K, S, s); return 0;
    case 1: flex_sk_launch<64, 128>(X, W, ws, M, N, K, S, s); return 0;
    case 2: flex_sk_launch<64, 160>(X, W, ws, M, N, K, S, s); return 0;
    case 3: flex_sk_launch<96, 64>(X, W, ws, M, N, K, S, s); return 0;
    case 4: flex_sk_launch<96, 128>(X, W, ws, M, N, K, S, s); return 0;
    case 5: flex_sk_launch<128, 96>(X, W, ws, M, N, K, S, s); return 0;
    case 6: flex_sk_launch<128, 128>(X, W, ws, M, N, K, S, s); return 0;
    case 7: flex_sk_launch<128, 160>(X, W, ws, M, N, K, S, s); return 0;
    case 8: flex_sk_launch<128, 192>(X, W, ws, M, N, K, S, s); return 0;
    case 9: flex_sk_launch<256, 32>(X, W, ws, M, N, K, S, s); return 0;
    case 10: flex_sk_launch<192, 128>(X, W, ws, M, N, K, S, s); return 0;
    case 11: flex_sk_launch<160, 128>(X, W, ws, M, N, K, S, s); return 0;
    case 12: flex_sk_launch<256, 64>(X, W, ws, M, N, K, S, s); return 0;
    case 13: flex_sk_launch<192, 64>(X, W, ws, M, N, K, S, s); return 0;
    default: return 1;
  }
}

// 1 if candidate cand (any form) has a SwiGLU epilogue
int gemm_flex_silu_ok(int cand) {
  cand &= 31;
  return cand >= 0 && cand < gemm_flex_count() && (kFlexTiles[cand][1] / 2) % 32 == 0;
}
