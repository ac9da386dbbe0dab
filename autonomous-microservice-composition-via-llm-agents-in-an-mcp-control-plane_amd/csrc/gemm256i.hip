// K1 (large-M path), interleaved variant: 256x256 tile, 8 waves (2 per SIMD,
// 2(M) x 4(N), 128x64 outputs per wave), ONE barrier per 64-deep K-tile.
//   Y[M,N] = X[M,K] . W[N,K]^T (+ R | SwiGLU)   fp32 accumulate, bf16 out
//
// gemm256.hip's multi-phase kernels pass 8 barriers per K-tile (2 per
// 16-MFMA phase); on MI355X those hand-offs leave the MFMA pipe idle ~40 % of
// the time (profiles/gemm_pmc_v8_vs_hipblaslt.txt: MFMA busy 61 % of cycles vs
// 81 % for hipBLASLt).  Here the fragment reads of the NEXT k-half are issued
// between the MFMAs of the current one (register double-buffered fragments,
// pinned with sched_group_barrier), so LDS latency hides behind MFMA work of
// the same wave and the two waves of a SIMD never have to alternate:
//
//   K-tile t (LDS buffer c = t & 1, tile t+1 already in flight into c ^ 1):
//     MFMA(t, k0) from F0   ||  ds_read F1 <- (t, k1)
//     s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier      (tile t+1 landed for all
//                                                    waves; nobody reads c)
//     LDS-DMA tile t+2 -> c
//     MFMA(t, k1) from F1   ||  ds_read F0 <- (t+1, k0)
//
// RAW: a buffer is read only after the barrier that follows every wave's
// vmcnt(0) for it.  WAR: buffer c is restaged only after the barrier that
// follows every wave's lgkmcnt(0) for its last reads.  Each piece is 256 rows
// x 32 k (64-B rows), chunk swizzle ^= ((row >> 2) & 1) << 1 on the LDS-DMA
// source and on the ds_read address (conflict-free, tools/lds_banks.py), the
// same image as gemm256.hip.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64, KH = 32;
constexpr int PIECE = 256 * KH;                 // bf16 elements per piece (16 KiB)

DEV int swz(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }

DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Frags {
  bf16x8 a[8];
  bf16x8 b[4];
};

// sched_group_barrier masks (LLVM AMDGPU)
constexpr int SG_MFMA = 0x008, SG_VMEM = 0x020, SG_DSR = 0x100;

enum Mode { FULL = 0, NOSTAGE = 1, LAST = 2 };

template <int EPI>
DEV void epilogue(bf16* __restrict__ Y, const bf16* __restrict__ R, int M, int N, int m0, int n0,
                  const f32x4 (&acc)[8][4]) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + wm * 128 + mt * 16 + fr;
    if (m >= M) continue;
    if constexpr (EPI == 2) {
      const int F = N >> 1;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int f = ((n0 + wn * 64) >> 1) + p * 16 + fq * 4;
        if (f >= F) continue;
        const f32x4 gv = acc[mt][2 * p], uv = acc[mt][2 * p + 1];
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)(gv[j] / (1.f + __expf(-gv[j])) * uv[j]);
        *reinterpret_cast<bf16x4*>(Y + (size_t)m * F + f) = o;
      }
      continue;
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = n0 + wn * 64 + nt * 16 + fq * 4;
      if (n >= N) continue;
      f32x4 v = acc[mt][nt];
      if (EPI == 1) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += (float)r[j];
      }
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
    }
  }
}

// Grouped tile order: GROUP M-tiles share each W column panel in L2.
DEV void tile_coords(int t, int nm, int nn, int& m0, int& n0) {
  constexpr int GROUP = 4;
  const int per_group = GROUP * nn;
  const int g = t / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  m0 = (first_m + (t % per_group) % gsz) * BM;
  n0 = ((t % per_group) / gsz) * BN;
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_tn_256i(const bf16* __restrict__ X,
                                                       const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y,
                                                       const bf16* __restrict__ R, int M, int N,
                                                       int K) {
  __shared__ __attribute__((aligned(16))) bf16 smem[8 * PIECE];   // [buf][A.k0 B.k0 A.k1 B.k1]
  const int lane = threadIdx.x & 63;
  // wave index in an SGPR: the LDS-DMA destinations (M0) stay scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  int m0, n0;
  tile_coords(xcd_remap(blockIdx.x, nm * nn), nm, nn, m0, n0);

  // ---- LDS-DMA sources: wave w writes 1 KiB instructions 2w, 2w+1 of every
  //      piece, as buffer_load ... lds through SGPR descriptors (T8): 32-bit
  //      per-lane byte offsets, the K position in soffset -> 4 address VGPRs
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)M * K * 2),
                                                     0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((size_t)N * K * 2),
                                                     0x00020000);
  unsigned voffA[2], voffB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (2 * wave + j) * 16 + (lane >> 2);
    const int ch = swz(row, lane & 3);
    voffA[j] = (unsigned)(((size_t)min(m0 + row, M - 1) * K + ch * 8) * 2);
    voffB[j] = (unsigned)(((size_t)min(n0 + row, N - 1) * K + ch * 8) * 2);
  }
  bf16* const dst0 = smem + (2 * wave) * 512;
  auto gl1 = [&](int t, int buf, int i) {                 // piece i >> 1, instruction i & 1
    const int pc = i >> 1, j = i & 1;
    const int soff = (t * BK + (pc >> 1) * KH) * 2;
    auto* lds_dst = (__attribute__((address_space(3))) void*)(dst0 + (buf * 4 + pc) * PIECE + j * 512);
    if (pc & 1) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, lds_dst, 16, voffB[j], soff, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, lds_dst, 16, voffA[j], soff, 0, 0);
  };
  auto stage = [&](int t, int buf) {            // all 4 pieces of K-tile t -> buffer buf
#pragma unroll
    for (int i = 0; i < 8; ++i) gl1(t, buf, i);
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  // fragment mt / nt sits 16 rows (1 KiB) after fragment 0 and shares its
  // swizzle (bit 2 of the row is fr's), so one byte base per operand and
  // buffer plus immediate ds_read offsets address every fragment
  const int rowA = wm * 128 + fr, rowB = wn * 64 + fr;
  const int baseA = (rowA * KH + swz(rowA, fq) * 8) * 2;
  const int baseB = (rowB * KH + swz(rowB, fq) * 8) * 2 + PIECE * 2;
  const char* const lds = reinterpret_cast<const char*>(smem);

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // buffer 1 lies 64 KiB up, past the 16-bit ds_read offset field: its bases
  // are separate registers (opaque, so they are not re-folded into v_adds)
  int baseA1 = baseA + 65536, baseB1 = baseB + 65536;
  asm volatile("" : "+v"(baseA1), "+v"(baseB1));
  // single instructions of a half K-tile, issued in an explicit order
  auto rd1 = [&](auto buf_c, int kh, Frags& f, int i) {   // i < 4: B[i], else A[i - 4]
    constexpr int BUF = decltype(buf_c)::value;
    const int po = kh * 2 * PIECE * 2;
    if (i < 4) {
      const char* pB = lds + (BUF ? baseB1 : baseB);
      f.b[i] = *reinterpret_cast<const bf16x8*>(pB + po + i * 1024);
    } else {
      const char* pA = lds + (BUF ? baseA1 : baseA);
      f.a[i - 4] = *reinterpret_cast<const bf16x8*>(pA + po + (i - 4) * 1024);
    }
  };
  auto mf1 = [&](const Frags& f, int i) {
    const int mt = i >> 2, nt = i & 3;
    acc[mt][nt] = mfma16x16x32(f.b[nt], f.a[mt], acc[mt][nt]);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };

  Frags F0, F1;
  const int nt_k = K / BK;
  // prologue: tiles 0 (and 1) in flight, tile 0 resident, F0 <- (0, k0)
  stage(0, 0);
  stage(1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 12; ++i) rd1(std::integral_constant<int, 0>{}, 0, F0, i);

  // one K-tile; BUF = t & 1 (static so the compiler's LDS-DMA alias tracking
  // sees that the reads never touch the buffer being restaged)
  auto tile = [&](int t, auto buf_c, auto mode_c) {
    constexpr int BUF = decltype(buf_c)::value;
    constexpr int MODE = decltype(mode_c)::value;
    using BC = std::integral_constant<int, BUF>;
    using BN_ = std::integral_constant<int, BUF ^ 1>;
    // ---- half 0: MFMA from F0; F1 <- (t, k1), one read per two MFMAs
    fence();
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      rd1(BC{}, 1, F1, i);
      mf1(F0, 2 * i);
      mf1(F0, 2 * i + 1);
      fence();
    }
#pragma unroll
    for (int i = 24; i < 32; ++i) mf1(F0, i);
    fence();
    if constexpr (MODE != LAST) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
    fence();
    // ---- half 1: MFMA from F1; F0 <- (t+1, k0) first, then restage this
    //      buffer with K-tile t+2 (one LDS-DMA per MFMA)
    if constexpr (MODE != LAST) {
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        rd1(BN_{}, 0, F0, i);
        mf1(F1, 2 * i);
        mf1(F1, 2 * i + 1);
        fence();
      }
    } else {
#pragma unroll
      for (int i = 0; i < 24; ++i) mf1(F1, i);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (MODE == FULL) gl1(t + 2, BUF, i);
      mf1(F1, 24 + i);
      fence();
    }
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using MF = std::integral_constant<int, FULL>;
  using MN = std::integral_constant<int, NOSTAGE>;
  using ML = std::integral_constant<int, LAST>;

  // nt_k is even (the launcher requires K % 128 == 0): pairs of K-tiles keep
  // the buffer parity static; the last pair stages nothing
  for (int t = 0; t + 2 < nt_k; t += 2) {
    tile(t, B0{}, MF{});
    tile(t + 1, B1{}, MF{});
  }
  tile(nt_k - 2, B0{}, MN{});
  tile(nt_k - 1, B1{}, ML{});
  epilogue<EPI>(Y, R, M, N, m0, n0, acc);
}

}  // namespace

int launch_gemm_tn_256i(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        int epi, hipStream_t s) {
  if (K % (2 * BK)) return 1;                // K-tiles come in pairs
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const dim3 grid(nm * nn);
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  switch (epi) {
    case 0: gemm_tn_256i<0><<<grid, 512, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
    case 1: gemm_tn_256i<1><<<grid, 512, 0, s>>>(x, w, y, r, M, N, K); return 0;
    case 2: gemm_tn_256i<2><<<grid, 512, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
    default: return 2;
  }
}
