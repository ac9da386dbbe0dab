// K1 (large-M path), one wave per SIMD with AGPR accumulators: 256x256 tile,
// 4 waves in a 2x2 grid, 128x128 outputs per wave = 8x8 v_mfma_f32_16x16x32_bf16
// tiles whose 256 fp32 accumulators per lane live in the accumulation register
// file (AGPRs) for the whole K loop.
//   Y[M,N] = X[M,K] . W[N,K]^T (+ R | SwiGLU)   fp32 accumulate, bf16 out
//
// Why: the 8-wave kernels (gemm256.hip / gemm256i.hip) read 12 fragments per
// 32 MFMAs (128x64 per wave); a 128x128 wave tile needs 16 per 64, a third less
// LDS traffic per FLOP - but 256 accumulators only fit one wave per SIMD, and
// hipcc then moves them between AGPRs and VGPRs (profiles/gemm_tuning.md,
// variants 20-23).  Here every MFMA is an inline-asm statement whose
// accumulator is an "+a" operand, so the accumulators are pinned to AGPRs and
// the VGPRs hold only fragments, staging registers and addresses.
//
// Staging is through registers (buffer_load_dwordx4 -> ds_write_b128), not
// LDS-DMA: with one wave per SIMD nothing hides the LDS-DMA issue cost
// (MI355X_MICROARCH.md: ~60 cycles per 1 KiB piece among MFMAs).
//
// Pipeline over 32-deep k-steps; a ring of S slots {A 256x32, B 256x32}
// (32 KiB each); step s computes from fragments F[s&1] read during step s-1:
//   S = 4: barrier after every step;  step s loads step s+3 into registers,
//          writes step s+2 (loaded in step s-1) to slot (s+2)%4, reads the
//          fragments of step s+1 from slot (s+1)%4.
//          WAR: slot (s+2)%4 was last read in step s-3; RAW: step s+1 was
//          written in step s-1, before barrier s-1.
//   S = 5: barrier after odd steps only (160 KiB LDS, half the barriers);
//          step s loads s+4, writes s+3 to slot (s+3)%5, reads s+1.
//          RAW: step s+1 was written in step s-2 and a barrier (end of s-1
//          or s-2, whichever is odd) lies between; WAR: slot (s+3)%5 was
//          last read in step s-3, and one of steps s-3..s-1 ends in a barrier.
// Every wave drains its LDS ops (lgkmcnt(0)) before each barrier.
// LDS rows are 64 B (32 bf16), chunk swizzle ^= ((row >> 2) & 1) << 1 applied
// on the ds_write and ds_read addresses (conflict-free, tools/lds_banks.py).
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 256, BN = 256, KS = 32;
constexpr int PIECE = 256 * KS;                     // bf16 elements per operand piece (16 KiB)
constexpr int SLOT_BYTES = 2 * PIECE * 2;           // A + B = 32 KiB

DEV int swz(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }

DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// acc (AGPR) += B-fragment x A-fragment; opaque to the compiler's scheduler,
// so issue order is program order
DEV void mfma_a(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

struct Frags {
  bf16x8 a[8];
  bf16x8 b[8];
};

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

// SCHED: 0 = one staging / fragment op after every MFMA pair, spread over the
// step; 1 = the same ops bunched into the first 20 pairs.  S: LDS ring slots.
// DMA: stage with buffer_load ... lds straight into the ring (no staging
// registers, no ds_write), loop unrolled by S so every slot index is static.
template <int EPI, int SCHED = 0, int S = 4, bool DMA = false, int DMAPOS = 0>
__global__ __launch_bounds__(256, 1) void gemm_tn_256a(const bf16* __restrict__ X,
                                                       const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y,
                                                       const bf16* __restrict__ R, int M, int N,
                                                       int K) {
  static_assert(S == 4 || S == 5, "ring of 4 or 5 slots");
  static_assert(!DMA || (S == 4 && SCHED == 0), "LDS-DMA staging: 4 slots, spread schedule");
  constexpr int LA = S - 1;          // a step loads step s + LA into registers ...
  constexpr int WA = S - 2;          // ... and writes step s + WA to the LDS ring
  __shared__ __attribute__((aligned(16))) bf16 smem[S * 2 * PIECE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  int m0, n0;
  {
    const int t = xcd_remap(blockIdx.x, nm * nn);
    constexpr int GROUP = 4;
    const int per_group = GROUP * nn;
    const int g = t / per_group;
    const int first_m = g * GROUP;
    const int gsz = min(nm - first_m, GROUP);
    m0 = (first_m + (t % per_group) % gsz) * BM;
    n0 = ((t % per_group) / gsz) * BN;
  }

  // ---- global -> register staging: per operand and k-step, thread t loads the
  //      16-B chunks (row t/4 + 64 i, chunk t%4), i = 0..3
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)M * K * 2),
                                                     0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((size_t)N * K * 2),
                                                     0x00020000);
  const int srow = tid >> 2, sch = tid & 3;
  // rows beyond M / N re-read the last row (their outputs are never stored)
  unsigned goffA[4], goffB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    goffA[i] = (unsigned)(((size_t)min(m0 + srow + 64 * i, M - 1) * K + sch * 8) * 2);
    goffB[i] = (unsigned)(((size_t)min(n0 + srow + 64 * i, N - 1) * K + sch * 8) * 2);
  }
  // LDS byte offset of this thread's chunk i inside a piece: rows srow + 64 i
  // share bit 2 of the row, hence the swizzle; +4 KiB per i
  const int wofs = (srow * KS + swz(srow, sch) * 8) * 2;
  char* const lds = reinterpret_cast<char*>(smem);
  // LDS-DMA: instruction i (0..3) of this wave fills rows (4 wave + i) * 16 +
  // lane / 4 of a piece lane-linearly; the chunk swizzle moves to the source
  unsigned doffA[4], doffB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // DMAPOS 3 (timing-only probe, wrong results): 8 rows x 128 B per instruction
    const int row = DMAPOS == 3 ? (4 * wave + i) * 8 + (lane >> 3) : (4 * wave + i) * 16 + (lane >> 2);
    const int ch = DMAPOS == 3 ? (lane & 7) : swz(row, lane & 3);
    doffA[i] = (unsigned)(((size_t)min(m0 + row, M - 1) * K + ch * 8) * 2);
    doffB[i] = (unsigned)(((size_t)min(n0 + row, N - 1) * K + ch * 8) * 2);
  }
  auto dma1 = [&](int st, int slot, int i) {           // i < 4: A instruction i, else B i-4
    const int soff = min(st, K / KS - 1) * KS * 2;   // soffset is not range-checked
    auto* dst = (__attribute__((address_space(3))) void*)(
        smem + slot * 2 * PIECE + (i < 4 ? 0 : PIECE) + (4 * wave + (i & 3)) * 512);
    if (i < 4) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, doffA[i], soff, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, dst, 16, doffB[i - 4], soff, 0, 0);
  };

  u32x4_t G[2][8];                                   // [set][A0..3 | B0..3], set = step & 1
  auto gload1 = [&](int st, u32x4_t (&g)[8], int i) {      // i < 4: A chunk i, else B chunk i-4
    const int soff = min(st, K / KS - 1) * KS * 2;   // soffset is not range-checked
    if (i < 4)
      g[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rsA, goffA[i], soff, 0));
    else
      g[i] = __builtin_bit_cast(u32x4_t,
                                __builtin_amdgcn_raw_buffer_load_b128(rsB, goffB[i - 4], soff, 0));
  };
  auto lwrite1 = [&](int slot, const u32x4_t (&g)[8], int i) {
    char* base = lds + slot * SLOT_BYTES + wofs + (i < 4 ? 0 : PIECE * 2);
    *reinterpret_cast<u32x4_t*>(base + (i & 3) * 4096) = g[i];
  };
  auto gload = [&](int st, u32x4_t (&g)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) gload1(st, g, i);
  };
  auto lwrite = [&](int slot, const u32x4_t (&g)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) lwrite1(slot, g, i);
  };

  // ---- fragment reads: wave (wm, wn) owns rows wm*128.., cols wn*128..
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int rowA = wm * 128 + fr, rowB = wn * 128 + fr;
  const int rA = (rowA * KS + swz(rowA, fq) * 8) * 2;   // fragment mt: + mt * 1 KiB
  const int rB = (rowB * KS + swz(rowB, fq) * 8) * 2 + PIECE * 2;
  auto fread1 = [&](int slot, Frags& f, int i) {           // i < 8: B[i], else A[i-8]
    if (i < 8)
      f.b[i] = *reinterpret_cast<const bf16x8*>(lds + slot * SLOT_BYTES + rB + i * 1024);
    else
      f.a[i - 8] = *reinterpret_cast<const bf16x8*>(lds + slot * SLOT_BYTES + rA + (i - 8) * 1024);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ns = K / KS;                             // even, >= 4 (launcher)
  Frags F[2];
  if constexpr (DMA) {
    // prologue: steps 0, 1, 2 in flight into slots 0, 1, 2; step 0 landed
#pragma unroll
    for (int st = 0; st < 3; ++st)
#pragma unroll
      for (int i = 0; i < 8; ++i) dma1(st, st, i);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
  // prologue: steps 0 .. WA-1 in the ring, step WA loaded into G[WA & 1]
  gload(0, G[0]);
  gload(1, G[1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lwrite(0, G[0]);
  lwrite(1, G[1]);
  if constexpr (S == 5) {
    gload(2, G[0]);
    gload(3, G[1]);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    lwrite(2, G[0]);
  } else {
    gload(2, G[0]);
  }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 16; ++i) fread1(0, F[0], i);
  __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0): clean waitcnt state at the loop head

  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  // one k-step; P = s & 1 static (the loop is unrolled by two), no branches in
  // the body (a conditional load makes hipcc's waitcnt analysis fall back to
  // draining every outstanding load).  64 MFMAs in pairs with the staging /
  // fragment operations placed between the pairs (one wave per SIMD: nothing
  // else fills the MFMA pipe while a VMEM / LDS instruction issues)
  auto step = [&](int s, auto p_c) {
    constexpr int P = decltype(p_c)::value;         // DMA: s % 4, else s & 1
    constexpr int GL = (LA & 1) ? (P & 1) ^ 1 : (P & 1);   // register set of step s + LA
    Frags& cur = F[P & 1];
    Frags& nxt = F[(P & 1) ^ 1];
    const int rslot = DMA ? (P + 1) % S : (s + 1) % S, wslot = (s + WA) % S;
    fence();
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int i0 = 2 * j, i1 = 2 * j + 1;
      mfma_a(acc[i0 >> 3][i0 & 7], cur.b[i0 & 7], cur.a[i0 >> 3]);
      mfma_a(acc[i1 >> 3][i1 & 7], cur.b[i1 & 7], cur.a[i1 >> 3]);
      if constexpr (DMA) {                      // DMA of step s+3 into the slot of step s-1
        // DMAPOS (tuning): 0 one DMA per 4 pairs, 1 all 8 after pair 0,
        // 2 none (timing-only upper bound: wrong results)
        const int k = j >> 2;
        if ((DMAPOS == 0 || DMAPOS == 3) && (j & 3) == 0) dma1(s + 3, (P + 3) % S, k);
        if (DMAPOS == 1 && j == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) dma1(s + 3, (P + 3) % S, i);
        }
        if ((j & 3) == 1 || (j & 3) == 2)
          fread1(rslot, nxt, 2 * k + (j & 3) - 1);
      } else if constexpr (SCHED == 0) {        // spread over the whole step
        const int k = j >> 2;
        if ((j & 3) == 0)
          gload1(s + LA, G[GL], k);             // G[GL] went to the ring in step s-1
        else if ((j & 3) == 3)
          lwrite1(wslot, G[GL ^ 1], k);         // step s+WA, loaded in step s-1
        else
          fread1(rslot, nxt, 2 * k + (j & 3) - 1);
      } else {                                  // bunched early
        if (j < 8) gload1(s + LA, G[GL], j);
        if (j < 16) fread1(rslot, nxt, j);
        if (j >= 12 && j < 20) lwrite1(wslot, G[GL ^ 1], j - 12);
      }
      fence();
    }
    // keep this step's fragments allocated to the end of the step: hipcc does
    // not know the asm MFMAs read them over several cycles and would otherwise
    // hand their registers to a load issued right after (WAR on an in-flight
    // MFMA source, which inline asm does not pad)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" :: "v"(cur.a[i]), "v"(cur.b[i]));
    if constexpr (DMA) {
      // step s+2's DMA (issued in step s-1) landed; step s+3's 8 stay in flight
      if constexpr (DMAPOS == 2) __builtin_amdgcn_s_waitcnt(0xC07F);
      else __builtin_amdgcn_s_waitcnt(0x0078);      // vmcnt(8) lgkmcnt(0)
      raw_barrier();
    } else if (S == 4 || (P & 1) == 1) {
      // lgkmcnt(0) as a builtin (vmcnt/expcnt left at their maxima), so hipcc
      // knows every LDS op is done and never re-waits for the fragment reads
      __builtin_amdgcn_s_waitcnt(0xC07F);
      raw_barrier();
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // ns is even (K % 64 == 0, launcher).  Every step runs the full body, also
  // the last ones: their loads of steps >= ns read bytes that are never used
  // (in-bounds rows, or zeros past the end of the buffer descriptor) and their
  // writes go to slots that are never read again.  A peeled tail would be
  // separate code in which hipcc re-assigns the accumulators with
  // v_accvgpr_mov's - VALU writes that the inline-asm MFMAs next to them are
  // not padded against.
  // Accumulator zeroing (VALU v_accvgpr_write) -> first MFMA reading them as
  // srcC needs wait states: pin the writes before a nop (asm statements keep
  // their order; the empty "+a" asms depend on the writes).
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4" ::: "memory");
  if constexpr (DMA) {
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    for (int s = 0; s < ns; s += 4) {               // ns % 4 == 0 (launcher)
      step(s, I0{});
      step(s + 1, I1{});
      step(s + 2, I2{});
      step(s + 3, I3{});
    }
  } else {
    for (int s = 0; s < ns; s += 2) {
      step(s, I0{});
      step(s + 1, I1{});
    }
  }
  // MFMA results -> VALU reads: 8-pass XDL needs its wait states (inline asm is not padded)
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

  // ---- epilogue: lane holds Y[m][n .. n+3] of each 16x16 tile
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + wm * 128 + mt * 16 + fr;
    if (m >= M) continue;
    if constexpr (EPI == 2) {
      const int F2 = N >> 1;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int f = ((n0 + wn * 128) >> 1) + p * 16 + fq * 4;
        if (f >= F2) continue;
        const f32x4 gv = acc[mt][2 * p], uv = acc[mt][2 * p + 1];
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)(gv[j] / (1.f + __expf(-gv[j])) * uv[j]);
        *reinterpret_cast<bf16x4*>(Y + (size_t)m * F2 + f) = o;
      }
      continue;
    }
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int n = n0 + wn * 128 + nt * 16 + fq * 4;
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

}  // namespace

int launch_gemm_tn_256a(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        int epi, hipStream_t s) {
  if (K % (2 * KS) || K / KS < 4) return 1;
  if ((size_t)M * K * 2 >= (1ull << 31) || (size_t)N * K * 2 >= (1ull << 31)) return 3;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const dim3 grid(nm * nn);
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  if (epi >= 10) {                                   // structure variants (tuning), plain epilogue
    switch (epi - 10) {
      case 0: gemm_tn_256a<0, 0, 4><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
      case 1: gemm_tn_256a<0, 1, 4><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
      case 2: gemm_tn_256a<0, 0, 5><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
      case 3: gemm_tn_256a<0, 1, 5><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
      case 4:
        if (K % (4 * KS)) return 1;
        gemm_tn_256a<0, 0, 4, true><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K);
        return 0;
      case 5:
        if (K % (4 * KS)) return 1;
        gemm_tn_256a<0, 0, 4, true, 2><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K);
        return 0;
      case 6:
        if (K % (4 * KS)) return 1;
        gemm_tn_256a<0, 0, 4, true, 1><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K);
        return 0;
      case 7:
        if (K % (4 * KS)) return 1;
        gemm_tn_256a<0, 0, 4, true, 3><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K);
        return 0;
      default: return 2;
    }
  }
  switch (epi) {
    case 0: gemm_tn_256a<0><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
    case 1: gemm_tn_256a<1><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K); return 0;
    case 2: gemm_tn_256a<2><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K); return 0;
    default: return 2;
  }
}
