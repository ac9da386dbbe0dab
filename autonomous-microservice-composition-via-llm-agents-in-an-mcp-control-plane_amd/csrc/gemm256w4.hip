// K1 (large-M path, v3): 256x256 bf16 TN GEMM, ONE wave per SIMD.
//   Y[M,N] = X[M,K] . W[N,K]^T (+ R)       fp32 accumulate, bf16 out
//
// Measured motivation (profiles/gemm_pmc_*): the 8-wave 256^2 kernel spent 34 %
// of its wave-cycles parked at barriers / waitcnt (SQ_WAIT_ANY, hipBLASLt 6.5 %)
// and issued 1.5x more LDS instructions.  Here 4 waves in a 2x2 grid each own
// a 128x128 sub-tile = 4x4 v_mfma_f32_32x32x16_bf16 tiles (256 fp32
// accumulators per lane, AGPRs), so every fragment read feeds 4 MFMAs of 32
// cycles.
//
// Pipeline: 32-deep k-stages in an S-slot LDS ring (slot = A 256x32 + B 256x32
// = 32 KiB, buffer_load ... lds with 32-bit offsets).  Each stage is two
// 16-deep substeps; fragments are double-buffered per substep (X for sub0,
// Y for sub1: 2 x 8 x b128 = 64 VGPRs), and the reads of the next substep are
// interleaved with the current substep's 16 MFMAs (sched_group_barrier):
//     read sub1(j) -> Y   ||  16 MFMA sub0(j) from X
//     s_waitcnt vmcnt(..) -> stage j+1 landed; s_barrier
//     LDS-DMA stage j+S-1 into the slot of stage j-1
//     read sub0(j+1) -> X ||  16 MFMA sub1(j) from Y
// WAR: the slot refilled at iteration j was last read in iteration j-1's first
// half, whose MFMAs (the consumers) every wave finished before barrier j.
// LDS rows are 64 B; swizzle chunk ^= (row>>2)&3 (conflict-free for 32-row
// fragments, tools/lds_banks.py), applied on the DMA source and the ds_read.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 256, BN = 256, KH = 32;
constexpr int PIECE = 256 * KH;                 // bf16 elements (16 KiB)

DEV int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
// 16-row fragment reads (16x16x32 operands) are conflict-free with this one
DEV int swz16(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }

DEV void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int S, bool RESID>
__global__ __launch_bounds__(256, 1) void gemm_tn_256w4(const bf16* __restrict__ X,
                                                        const bf16* __restrict__ W,
                                                        bf16* __restrict__ Y,
                                                        const bf16* __restrict__ R, int M, int N,
                                                        int K) {
  __shared__ __attribute__((aligned(16))) bf16 smem[S * 2 * PIECE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const int nwg = nm * nn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 4;
  const int per_group = GROUP * nn;
  const int g = wg / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // staging: wave w writes 1 KiB instructions 4w..4w+3 of each 16 KiB piece;
  // rows past M / N fall outside num_records: the range check drops them
  // unsigned 32-bit byte offsets: operands up to 4 GiB (launcher checks)
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0,
                                                     (int)((unsigned)M * (unsigned)K * 2u), 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0,
                                                     (int)((unsigned)N * (unsigned)K * 2u), 0x00020000);
  unsigned voA[4], voB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (4 * wave + i) * 16 + (lane >> 2);
    const int ch = swz(row, lane & 3);
    voA[i] = ((unsigned)(m0 + row) * (unsigned)K + ch * 8) * 2u;
    voB[i] = ((unsigned)(n0 + row) * (unsigned)K + ch * 8) * 2u;
  }
  auto stage = [&](int st) {
    const int soff = st * KH * 2;      // may run past K at the tail (dead slots)
    bf16* slot = smem + (st % S) * 2 * PIECE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(slot + (4 * wave + i) * 512), 16, voA[i],
          soff, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(slot + PIECE + (4 * wave + i) * 512), 16,
          voB[i], soff, 0, 0);
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 31, fh = lane >> 5;
  // fragment element offsets inside a piece: [substep][tile]
  int offA[2][4], offB[2][4];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ra = wm * 128 + t * 32 + fr;
      const int rb = wn * 128 + t * 32 + fr;
      offA[s][t] = ra * KH + swz(ra, 2 * s + fh) * 8;
      offB[s][t] = rb * KH + swz(rb, 2 * s + fh) * 8;
    }

  f32x16 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;

  bf16x8 xa[4], xb[4], ya[4], yb[4];
  auto read = [&](int st, int s, bf16x8 (&af)[4], bf16x8 (&bfr)[4]) {
    const bf16* sA = smem + (st % S) * 2 * PIECE;
    const bf16* sB = sA + PIECE;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bfr[t] = *reinterpret_cast<const bf16x8*>(sB + offB[s][t]);
      af[t] = *reinterpret_cast<const bf16x8*>(sA + offA[s][t]);
    }
  };
  auto mma = [&](const bf16x8 (&af)[4], const bf16x8 (&bfr)[4]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma32(bfr[nt], af[mt], acc[mt][nt]);
  };
  auto interleave_a = [&]() {   // 16 MFMA + 8 ds_read_b128
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
  auto interleave_b = [&]() {   // 16 MFMA + 8 ds_read_b128 + 8 LDS-DMA
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
  };
  const int ns = K / KH;

  // prologue: stages 0..S-2 in flight; stage 0 landed -> substep-0 fragments.
  // Stages >= ns are issued too: they only fill slots that are never read
  // (rows past the matrix end are dropped by the range check), which keeps the
  // loop body one basic block with a constant vmcnt.
#pragma unroll
  for (int st = 0; st < S - 1; ++st) stage(st);
  wait_vm<8 * (S - 2)>();
  bar();
  read(0, 0, xa, xb);

  for (int j = 0; j < ns; ++j) {
    read(j, 1, ya, yb);
    mma(xa, xb);
    interleave_a();
    wait_vm<8 * (S - 3)>();        // stage j+1 landed (this thread)
    bar();                         // ... every thread; stage j-1's slot free
    stage(j + S - 1);
    read(j + 1, 0, xa, xb);        // stale slot at the tail, never used
    mma(ya, yb);
    interleave_b();
  }
  wait_vm<0>();                    // no LDS-DMA may outlive the workgroup

  // epilogue: lane holds Y[m][n .. n+3] for 4 groups of 4 columns per tile
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = m0 + wm * 128 + mt * 32 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * 128 + nt * 32 + 8 * q + 4 * fh;
        if (n >= N) continue;
        f32x4 v = {acc[mt][nt][4 * q], acc[mt][nt][4 * q + 1], acc[mt][nt][4 * q + 2],
                   acc[mt][nt][4 * q + 3]};
        if (RESID) {
          const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
        *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
      }
    }
  }
}

}  // namespace

int launch_gemm_tn_256w4(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                         int stages, hipStream_t s) {
  if (K % 64) return 2;
  if ((size_t)(M + BM) * K * 2 >= (1ull << 32) || (size_t)(N + BN) * K * 2 >= (1ull << 32)) return 3;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const dim3 grid(nm * nn);
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  switch (stages) {
    case 4: if (R) gemm_tn_256w4<4, true><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K);
            else gemm_tn_256w4<4, false><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K); return 0;
    case 5: if (R) gemm_tn_256w4<5, true><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K);
            else gemm_tn_256w4<5, false><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K); return 0;
    default: return 1;
  }
}

// ----------------------------------------------------------------------------
// Same 4-wave pipeline with v_mfma_f32_16x16x32_bf16 (holds a higher clock on
// random data than 32x32x16, MI355X_MICROARCH.md 'DVFS give-back' item 7).
// A k-stage is split by m-halves of the wave's 128 rows: sub0 = rows 0-63 x 128
// cols (32 MFMA), sub1 = rows 64-127 (32 MFMA).  B fragments (8) are read with
// sub0 and double-buffered across stages (loop unrolled by 2; K % 64 == 0).
//   [read A-sub1(j) || MFMA sub0(j)] -> vmcnt, barrier, LDS-DMA j+S-1 ->
//   [read B(j+1), A-sub0(j+1) || MFMA sub1(j)]
namespace {

template <int S, bool RESID>
__global__ __launch_bounds__(256, 1) void gemm_tn_256w4m16(const bf16* __restrict__ X,
                                                           const bf16* __restrict__ W,
                                                           bf16* __restrict__ Y,
                                                           const bf16* __restrict__ R, int M,
                                                           int N, int K) {
  __shared__ __attribute__((aligned(16))) bf16 smem[S * 2 * PIECE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const int nwg = nm * nn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 4;
  const int per_group = GROUP * nn;
  const int g = wg / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0,
                                                     (int)((unsigned)M * (unsigned)K * 2u), 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0,
                                                     (int)((unsigned)N * (unsigned)K * 2u), 0x00020000);
  unsigned voA[4], voB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (4 * wave + i) * 16 + (lane >> 2);
    const int ch = swz16(row, lane & 3);
    voA[i] = ((unsigned)(m0 + row) * (unsigned)K + ch * 8) * 2u;
    voB[i] = ((unsigned)(n0 + row) * (unsigned)K + ch * 8) * 2u;
  }
  auto stage = [&](int st) {
    const int soff = st * KH * 2;
    bf16* slot = smem + (st % S) * 2 * PIECE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(slot + (4 * wave + i) * 512), 16, voA[i],
          soff, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(slot + PIECE + (4 * wave + i) * 512), 16,
          voB[i], soff, 0, 0);
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  int offA[8], offB[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int ra = wm * 128 + t * 16 + fr;
    const int rb = wn * 128 + t * 16 + fr;
    offA[t] = ra * KH + swz16(ra, fq) * 8;
    offB[t] = rb * KH + swz16(rb, fq) * 8;
  }
  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[4], ya[4], b0[8], b1[8];
  auto readA = [&](int st, int half, bf16x8 (&af)[4]) {
    const bf16* sA = smem + (st % S) * 2 * PIECE;
#pragma unroll
    for (int t = 0; t < 4; ++t) af[t] = *reinterpret_cast<const bf16x8*>(sA + offA[4 * half + t]);
  };
  auto readB = [&](int st, bf16x8 (&bfr)[8]) {
    const bf16* sB = smem + (st % S) * 2 * PIECE + PIECE;
#pragma unroll
    for (int t = 0; t < 8; ++t) bfr[t] = *reinterpret_cast<const bf16x8*>(sB + offB[t]);
  };
  auto mma = [&](int half, const bf16x8 (&af)[4], const bf16x8 (&bfr)[8]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
        acc[4 * half + mt][nt] = mfma16x16x32(bfr[nt], af[mt], acc[4 * half + mt][nt]);
  };
  auto il_a = [&]() {           // 32 MFMA + 4 ds_read
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
  auto il_b = [&]() {           // 32 MFMA + 12 ds_read + 8 LDS-DMA
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
  const int ns = K / KH;
#pragma unroll
  for (int st = 0; st < S - 1; ++st) stage(st);
  wait_vm<8 * (S - 2)>();
  bar();
  readB(0, b0);
  readA(0, 0, xa);
  auto iteration = [&](int j, bf16x8 (&cb)[8], bf16x8 (&nb)[8]) {
    readA(j, 1, ya);
    mma(0, xa, cb);
    il_a();
    wait_vm<8 * (S - 3)>();
    bar();
    stage(j + S - 1);
    readB(j + 1, nb);
    readA(j + 1, 0, xa);
    mma(1, ya, cb);
    il_b();
  };
  for (int j = 0; j < ns; j += 2) {
    iteration(j, b0, b1);
    iteration(j + 1, b1, b0);
  }
  wait_vm<0>();

#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + wm * 128 + mt * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int n = n0 + wn * 128 + nt * 16 + fq * 4;
      if (n >= N) continue;
      f32x4 v = acc[mt][nt];
      if (RESID) {
        const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
      }
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
    }
  }
}

}  // namespace

int launch_gemm_tn_256w4m16(const void* X, const void* W, void* Y, const void* R, int M, int N,
                            int K, int stages, hipStream_t s) {
  if (K % 64) return 2;
  if ((size_t)(M + BM) * K * 2 >= (1ull << 32) || (size_t)(N + BN) * K * 2 >= (1ull << 32)) return 3;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const dim3 grid(nm * nn);
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  switch (stages) {
    case 4: if (R) gemm_tn_256w4m16<4, true><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K);
            else gemm_tn_256w4m16<4, false><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K); return 0;
    case 5: if (R) gemm_tn_256w4m16<5, true><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K);
            else gemm_tn_256w4m16<5, false><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K); return 0;
    default: return 1;
  }
}
