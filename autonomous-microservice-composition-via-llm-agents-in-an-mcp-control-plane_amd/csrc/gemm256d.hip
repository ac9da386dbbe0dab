// K1 (large-M path), production: 256x256 tile, ONE wave per SIMD (4 waves,
// 2x2), 128x128 outputs per wave = 8x8 v_mfma_f32_16x16x32_bf16 tiles whose
// 256 fp32 accumulators live in AGPRs, operands staged by LDS-DMA in
// 128-byte rows.
//   Y[M,N] = X[M,K] . W[N,K]^T (+ R | SwiGLU)   fp32 accumulate, bf16 out
//
// How it got here (profiles/gemm_tuning.md): the 8-wave kernels (gemm256.hip)
// read 12 fragments per 32 MFMAs; a 128x128 wave tile reads 16 per 64.  With
// the MFMAs as inline asm whose accumulators are "+a" operands
// (gemm256a.hip), hipcc keeps the 256 accumulators in AGPRs, so one wave per
// SIMD fits.  Without any staging that loop runs at 1.6-1.8 PF/s; the cost
// left is the LDS-DMA issue (~60 cycles per 1 KiB instruction among MFMAs,
// MI355X_MICROARCH.md), which falls by a third when an instruction covers
// 8 rows x 128 B instead of 16 rows x 64 B (fewer cache lines per request)
// - hence 64-deep k-tiles stored as 128-byte rows here.
//
// Pipeline, per 64-deep k-tile t (LDS slot c = t & 1, 64 KiB = A | B, each
// 256 rows x 128 B; fragments F[0] = k-half 0, F[1] = k-half 1):
//   half 0: 64 MFMAs from F[0]          || ds_read F[1] <- (t, k1) from slot c
//   s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier
//           (tile t+1's DMA, issued in half 1 of tile t-1, landed for every
//            wave; nobody reads slot c any more)
//   half 1: 64 MFMAs from F[1]          || ds_read F[0] <- (t+1, k0) from slot c^1
//                                       || LDS-DMA tile t+2 -> slot c
// One barrier per 128 MFMAs.  RAW: a slot is read only after the barrier that
// follows every wave's vmcnt(0) for its DMA.  WAR: slot c is refilled only
// after the barrier that follows every wave's lgkmcnt(0) for its last reads.
// LDS rows of 128 B, 16-B chunk swizzle ^= row & 7, applied on the DMA source
// address and the ds_read address (conflict-free: tools/lds_banks.py).
// Rows past M re-read row M-1 (clamped per-lane offsets); their outputs are
// never stored.
//
// Tile height BMT = 128, 160, 192, 224 or 256 rows (BMT / 2 rows per wave =
// BMT / 32 MFMA row tiles of 16).  One wave of workgroups is the unit of
// time at one workgroup per CU, so the height that makes ceil(M / BMT) x
// (N / 256) closest to a whole number of waves wins: for N = 4096 (16 column
// tiles) every M in 1792..4096 has a height with 14-16 row tiles (>= 88 % of
// the 256 CUs busy), e.g. M = 2560 = 16 x 160 - where 256-row tiles fill
// 160 of 256 CUs.  The measured plan (ops/gemm_plan_gfx950.json, codes 1-5)
// picks the height per 64-row M bucket; smaller heights read more LDS and
// issue more DMA per MFMA (8 + MTW fragment reads per 8 MTW MFMAs).
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BN = 256, BK = 64;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
constexpr int ROWB = BK * 2;                        // 128-byte LDS rows
constexpr int PIECE_BB = 256 * ROWB;                // the W operand of a slot: 32 KiB

DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// acc (AGPR) += B-fragment x A-fragment; an opaque statement, so hipcc keeps
// the accumulator in AGPRs and issue order is program order
DEV void mfma_a(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

template <int MTW>
struct Frags {
  bf16x8 a[MTW];
  bf16x8 b[8];
};

// grouped tile order: ``group`` M-tiles share each W column panel (a launch
// argument: gemm256d_group picks it per shape)
DEV void tile_coords(int t, int nm, int nn, int bm, int group, int& m0, int& n0) {
  const int per_group = group * nn;
  const int g = t / per_group;
  const int first_m = g * group;
  const int gsz = min(nm - first_m, group);
  m0 = (first_m + (t % per_group) % gsz) * bm;
  n0 = ((t % per_group) / gsz) * BN;
}

// ops n spread over P slots: how many start at slot j, and the first index
constexpr int ops_at(int j, int n, int P) { return ((j + 1) * n) / P - (j * n) / P; }
constexpr int op0_at(int j, int n, int P) { return (j * n) / P; }

// The epilogue goes through LDS (row-contiguous 16-B stores); the direct
// MFMA-layout store measured 10-15 % slower (profiles/gemm_tuning.md).
// PROBE (timing / power ladder only, tools/gemm_power_ladder.py; results are
// not a product): 0 = production; 1 = the MFMA issue alone (fragments read
// once, no DMA, no barriers, no stores); 2 = + the ds_read fragment schedule
// and the barriers (no DMA, no stores); 3 = + the LDS-DMA (the whole
// mainloop, no epilogue stores).  Rung 0 minus rung 3 is the epilogue.
//
// SPLIT = 2 (mid M, one wave of tiles too few for the chip: gate|up at
// M = 129-256 has 112 column tiles for 256 CUs): two workgroups per tile, each
// walks half of K; grid = 2 x tiles, tile = id / 2 after the XCD remap (a
// tile's halves usually share an XCD, which only matters for speed).  The
// hand-off is the sc1 counter form of cdna_hip_programming.md §5 "Projection
// GEMM at M = 256" item 2, made wait-free for the first arriver: each half
// draws a ticket on cnt[tile] when its mainloop is done; ticket 0 stores its
// fp32 accumulators (sc1, write-through) to the tile's slab, drains, bumps
// the counter again and exits; ticket 1 polls (relaxed) until the counter
// reads 3 - it only ever waits on a workgroup that is already running, so no
// residency assumption - re-arms it, adds the slab (sc1 loads, every one) to
// its accumulators and runs the epilogue.  ws: >= tiles x BMT x 256 floats.
//
// PF = 1 (mid-M forms, where each workgroup streams its W panel straight from
// HBM): the 2-slot pipeline waits for tile t+1's DMAs at tile t's half-way
// barrier, so it covers 1-1.5 half-tiles of DMA latency (~0.25-0.75 us), under
// a loaded HBM round trip.  Each wave also pulls its 64 W rows of tile t+4
// into L2 (one 4-byte load per lane = one 128-B line per row, into a sink
// register) at the end of tile t; loads retire in issue order, so the
// half-way wait becomes vmcnt(1) (vmcnt(2) at tile 0) and each L2 fill gets
// three half-tiles before the wait that covers it.
template <int EPI, int BMT, bool WIDE = false, int PROBE = 0, int SPLIT = 1, int PF = 0>
__global__ __launch_bounds__(256, 1) void gemm_tn_256d(const bf16* __restrict__ X,
                                                       const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y,
                                                       const bf16* __restrict__ R, int M, int N,
                                                       int K, int group, const RopeArgs ra,
                                                       const NormEpi ne, f32x4* __restrict__ ws,
                                                       int* __restrict__ cnt) {
  static_assert(SPLIT == 1 || (SPLIT == 2 && PROBE == 0 && WIDE && EPI != 3), "split forms: wide epilogue");
  static_assert(PF == 0 || PROBE == 0, "prefetch: production forms");
  static_assert(BMT % 32 == 0 && BMT >= 128 && BMT <= 256, "tile height");
  constexpr int MTW = BMT / 32;                     // 16-row MFMA tiles per wave (4..8)
  constexpr int WROWS = BMT / 2;                    // rows per wave (64..128)
  constexpr int PIECE_A = BMT * ROWB;               // the X operand of a slot
  constexpr int SLOT_B = PIECE_A + PIECE_BB;
  constexpr int QA = BMT / 32;                      // A DMA instructions per wave (4..8)
  constexpr int NDMA = QA + 8;                      // DMA instructions per wave and k-tile
  constexpr int NRD = 8 + MTW;                      // fragment reads per wave and k-half
  constexpr int NMF = MTW * 8;                      // MFMAs per wave and k-half
  constexpr int NP = NMF / 2;                       // MFMA pairs per k-half
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT_B];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nm = (M + BMT - 1) / BMT, nn = (N + BN - 1) / BN;
  int m0, n0;
  // grid = the first gridDim.x tiles of the grouped order (all of them, or the
  // full waves of a hybrid launch whose tail runs stream-K, gemm256sk.hip);
  // SPLIT 2: two workgroups per tile, K halves
  const int wgl = xcd_remap(blockIdx.x, gridDim.x);
  const int tl = SPLIT == 2 ? wgl >> 1 : wgl;
  const int kslice = SPLIT == 2 ? wgl & 1 : 0;
  tile_coords(tl, nm, nn, BMT, group, m0, n0);

  // ---- LDS-DMA: instruction q of an operand fills rows 8q..8q+7,
  //      lane-linearly (row 8q + lane/8, LDS chunk lane%8, swizzled source
  //      chunk); wave w issues A's q = QA w .. QA w + QA-1 and W's 8w .. 8w+7.
  //      The k position goes in soffset.
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)M * K * 2),
                                                     0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((size_t)N * K * 2),
                                                     0x00020000);
  // The buffer range check covers voffset (+ the instruction offset) but NOT
  // soffset: X rows past M (the last M-tile) go in voffset, so they fall
  // outside the descriptor and read nothing (their outputs are never stored);
  // instruction q reads rows 8 q further, + 16 q K bytes - a wave-uniform
  // addend, one VALU add per DMA instead of QA live offsets.  W rows are
  // always in range (N % 256 == 0, launcher) and step through soffset.
  const int chunk = (lane & 7) ^ (lane >> 3);
  const unsigned offA0 = (unsigned)(((size_t)(m0 + 8 * QA * wave + (lane >> 3)) * K + chunk * 8) * 2);
  const unsigned offB = (unsigned)(((lane >> 3) * K + chunk * 8) * 2);
  const int rowB0 = n0 + 64 * wave;                  // first W row of this wave's instructions
  // k-tile t of the trailing (unconsumed) DMAs is clamped to the last one:
  // soffset is outside the range check, so t >= nt would read past the end of
  // the last row of X / W
  const int nt = K / BK / SPLIT;                     // >= 2, even (launcher)
  const int kb0 = kslice * nt * BK * 2;              // this workgroup's K half (SPLIT 2)
  auto dma1 = [&](int t, int slot, int i) {          // i < QA: A instruction i, else B i-QA
    if (PROBE == 1 || PROBE == 2) {
      if (t > 1) return;                             // probes: the prologue's tiles only
    }
    const bool b = i >= QA;
    const int q = b ? i - QA : i;
    const int kb = kb0 + min(t, nt - 1) * BK * 2;
    auto* dst = (__attribute__((address_space(3))) void*)(
        smem + slot * SLOT_B + (b ? PIECE_A + (8 * wave + q) * 1024 : (QA * wave + q) * 1024));
    if (b)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, dst, 16, offB, (rowB0 + 8 * q) * K * 2 + kb, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, offA0 + q * 16 * K, kb, 0, 0);
  };

  // ---- PF: L2 fill of this wave's 64 W rows of k-tile t (clamped), one line per lane
  [[maybe_unused]] int pf_sink = 0;
  [[maybe_unused]] const bf16* pfw = W + (size_t)(rowB0 + lane) * K + kb0 / 2;
  auto pf1 = [&](int t) {
    if constexpr (PF) {
      const bf16* p = pfw + min(t, nt - 1) * BK;
      asm volatile("global_load_dword %0, %1, off" : "+v"(pf_sink) : "v"(p));
    }
  };

  // ---- fragment reads: wave (wm, wn) owns rows wm*WROWS.., cols wn*128..;
  //      lane (fr, fq) reads row fr of fragment i, k-chunk 4 kh + fq.  Fragment
  //      i sits i * 2 KiB after fragment 0 with the same swizzle (row & 7 = fr & 7).
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  int rbase[2][2][2];                                // [slot][kh][A|B] LDS byte offsets
#pragma unroll
  for (int sl = 0; sl < 2; ++sl)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int ch = ((4 * kh + fq) ^ (fr & 7)) * 16;
      rbase[sl][kh][0] = sl * SLOT_B + (wm * WROWS + fr) * ROWB + ch;
      rbase[sl][kh][1] = sl * SLOT_B + PIECE_A + (wn * 128 + fr) * ROWB + ch;
    }
  bool prologue = true;                              // PROBE 1 reads fragments here only
  auto fread1 = [&](int slot, int kh, Frags<MTW>& f, int i) {   // i < 8: B[i], else A[i-8]
    if constexpr (PROBE == 1) {
      if (!prologue) return;
    }
    if (i < 8)
      f.b[i] = *reinterpret_cast<const bf16x8*>(smem + rbase[slot][kh][1] + i * 2048);
    else
      f.a[i - 8] = *reinterpret_cast<const bf16x8*>(smem + rbase[slot][kh][0] + (i - 8) * 2048);
  };

  f32x4 acc[MTW][8];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // accumulator zeroing (VALU v_accvgpr_write) -> first MFMA reading them as
  // srcC needs wait states: pin the writes before a nop (asm statements keep
  // their order; the empty "+a" statements depend on the writes)
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));

  Frags<MTW> F[2];
  // prologue: tiles 0 and 1 in flight, tile 0 landed, F[0] <- (0, k0)
#pragma unroll
  for (int i = 0; i < NDMA; ++i) dma1(0, 0, i);
#pragma unroll
  for (int i = 0; i < NDMA; ++i) dma1(1, 1, i);
  if constexpr (PF) {
    pf1(2);
    pf1(3);
  }
  // tile 0 landed (own DMAs): the NDMA of tile 1 (+ 2 fills) may still be in flight
  if constexpr (PF) {
    if constexpr (NDMA == 16) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else if constexpr (NDMA == 15) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
    else if constexpr (NDMA == 14) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (NDMA == 13) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  } else if constexpr (NDMA == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (NDMA == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else if constexpr (NDMA == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  else if constexpr (NDMA == 13) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < NRD; ++i) fread1(0, 0, F[0], i);
  if constexpr (PROBE == 1) {                        // both fragment sets hold real data
#pragma unroll
    for (int i = 0; i < NRD; ++i) fread1(0, 1, F[1], i);
    prologue = false;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0): clean waitcnt state at the loop head
  asm volatile("s_nop 4" ::: "memory");

  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  auto keep = [](const Frags<MTW>& f) {              // fragments stay allocated to here: hipcc
#pragma unroll                                       // does not know the asm MFMAs read them
    for (int i = 0; i < MTW; ++i) asm volatile("" :: "v"(f.a[i]));
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" :: "v"(f.b[i]));
  };
  // one 64-deep k-tile; C = t & 1 static (the loop is unrolled by two).  Every
  // tile runs the full body, also the last two: their DMAs (clamped to the last
  // k-tile) and their reads of tile nt are never consumed (a peeled tail would be separate
  // code where hipcc re-assigns the accumulators with v_accvgpr_mov's, VALU
  // writes the unpadded asm MFMAs next to them race with).  The reads and
  // DMAs are spread evenly over the MFMA pairs of each half.
  auto tile = [&](int t, auto c_c) {
    constexpr int C = decltype(c_c)::value;
    fence();
#pragma unroll
    for (int j = 0; j < NP; ++j) {                   // half 0: F[0], reads of (t, k1)
      const int i0 = 2 * j, i1 = 2 * j + 1;
      mfma_a(acc[i0 >> 3][i0 & 7], F[0].b[i0 & 7], F[0].a[i0 >> 3]);
      mfma_a(acc[i1 >> 3][i1 & 7], F[0].b[i1 & 7], F[0].a[i1 >> 3]);
#pragma unroll
      for (int r = 0; r < ops_at(j, NRD, NP); ++r) fread1(C, 1, F[1], op0_at(j, NRD, NP) + r);
      fence();
    }
    keep(F[0]);
    // tile t+1 landed (own DMAs), and this wave's reads of slot C are done
    if constexpr (PROBE != 1) {
      if constexpr (PF) {                            // the youngest fill(s) may stay in flight
        if (C == 0 && t == 0) __builtin_amdgcn_s_waitcnt(0x0072);   // vmcnt(2) lgkmcnt(0)
        else __builtin_amdgcn_s_waitcnt(0x0071);                    // vmcnt(1) lgkmcnt(0)
      } else {
        __builtin_amdgcn_s_waitcnt(0x0070);          // vmcnt(0) lgkmcnt(0)
      }
      raw_barrier();
    }
    fence();
#pragma unroll
    for (int j = 0; j < NP; ++j) {                   // half 1: F[1], reads of (t+1, k0), DMA t+2
      const int i0 = 2 * j, i1 = 2 * j + 1;
      mfma_a(acc[i0 >> 3][i0 & 7], F[1].b[i0 & 7], F[1].a[i0 >> 3]);
      mfma_a(acc[i1 >> 3][i1 & 7], F[1].b[i1 & 7], F[1].a[i1 >> 3]);
#pragma unroll
      for (int r = 0; r < ops_at(j, NRD, NP); ++r) fread1(C ^ 1, 0, F[0], op0_at(j, NRD, NP) + r);
#pragma unroll
      for (int d = 0; d < ops_at(j, NDMA, NP); ++d) dma1(t + 2, C, op0_at(j, NDMA, NP) + d);
      fence();
    }
    pf1(t + 4);                                      // after this tile's DMAs (in-order retire)
    keep(F[1]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  for (int t = 0; t < nt; t += 2) {
    tile(t, C0{});
    tile(t + 1, C1{});
  }
  // drain the trailing (unconsumed) DMAs before the workgroup's LDS is released,
  // and pad MFMA results -> VALU reads (inline asm is not padded)
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  if constexpr (PF) asm volatile("" :: "v"(pf_sink));   // the sink register stays reserved to here
  if constexpr (PROBE != 0) {
    // probes store nothing; one accumulator reaches memory under a condition
    // no launch meets, so the MFMA results stay live
    if (M == -7 && lane == 0) {
      f32x4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) t += acc[i][j];
      *reinterpret_cast<f32x4*>(Y) = t;
    }
    return;
  }

  // SPLIT 2: the slab of the other K half, added in the (wide) epilogue
  constexpr int NACC = MTW * 8;                      // f32x4 per lane
  [[maybe_unused]] const SlabIn<std::remove_const_t<decltype(rsA)>> slab{
      __builtin_amdgcn_make_buffer_rsrc((void*)(ws + (size_t)tl * NACC * 256), (short)0, NACC * 256 * 16,
                                        0x00020000),
      (unsigned)tid * 16};
  if constexpr (SPLIT == 2) {
    // ---- K-half hand-off (see the SPLIT note above the kernel)
    int* tick = reinterpret_cast<int*>(smem);        // the one LDS array (no second __shared__)
    __syncthreads();                                 // every wave is done with the slots
    if (tid == 0) *tick = __hip_atomic_fetch_add(cnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int ticket = *tick;
    f32x4* sbase = ws + (size_t)tl * NACC * 256 + tid;
    if (ticket == 0) {
      // straight from the AGPRs (a builtin store makes hipcc copy them all to
      // VGPRs first and spill); sc1 = write-through, no release fence needed
#pragma unroll
      for (int r = 0; r < NACC; ++r)
        asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(sbase + r * 256), "a"(acc[r >> 3][r & 7])
                     : "memory");
      asm volatile("s_nop 1\n\ts_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {
      // the partner drew ticket 0, so it is running and its store + bump come;
      // the bound (~1 s) only keeps a broken invariant from hanging the GPU
      for (int spin = 0; spin < (1 << 24); ++spin) {
        if (__hip_atomic_load(cnt + tl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3) break;
        __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(cnt + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-arm
    }
    __syncthreads();
  }

  if constexpr (WIDE && EPI != 3) {
    // ---- wide direct epilogue (common.h store_wide): straight from the
    //      accumulators, 16-B stores after a permlane16 exchange, no LDS
    const int ldy = EPI == 2 ? N / 2 : N;
    const int col0 = EPI == 2 ? (n0 + wn * 128) / 2 : n0 + wn * 128;
    float rsc[MTW];
    int rrow[MTW];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) rrow[mt] = min(m0 + wm * WROWS + mt * 16 + fr, M - 1);
    if constexpr (EPI == 2) norm_row_scales(ne, rrow, rsc);
    const auto rsY = __builtin_amdgcn_make_buffer_rsrc((void*)Y, (short)0, (int)((size_t)M * ldy * 2),
                                                       0x00020000);
    if constexpr (SPLIT == 2)
      store_wide_slab<EPI, MTW>(acc, rsY, R, M, ldy, m0 + wm * WROWS, col0, fr, fq, rsc, ne, slab);
    else
      store_wide<EPI, MTW>(acc, rsY, R, M, ldy, m0 + wm * WROWS, col0, fr, fq, rsc, ne);
  } else {
    // ---- staged epilogue.  The direct one below stores 8 B per lane in
    //      32-B row pieces (the MFMA layout: lane = 4 columns of one row); at
    //      one workgroup per CU nothing hides those stores and they cost
    //      10-15 % of a K = 4096 projection (no-store probe, gemm_tuning.md).
    //      Here each wave converts its tile to bf16 (bias / SwiGLU applied)
    //      into its own LDS region - rows of OUTW columns, 16-B chunks
    //      swizzled ^= row - and stores it back as 16 B per lane, 256 B per
    //      row: four times fewer, fully coalesced stores.
    constexpr int OUTW = EPI == 2 ? 64 : 128;        // output columns per wave
    constexpr int RB = OUTW * 2;                     // staged row bytes
    constexpr int NCH = RB / 16;                     // 16-B chunks per row
    constexpr int RPS = 1024 / RB;                   // rows per 1 KiB wave access
    static_assert(4 * WROWS * RB <= 2 * SLOT_B, "epilogue staging fits the operand slots");
    __syncthreads();                                 // every wave is done with the slots
    char* stg = smem + wave * (WROWS * RB);
    const int lr = lane / NCH, lc = lane % NCH;
    constexpr int NST = WROWS / RPS;                 // store rows per lane
    const int ldy = EPI == 2 ? N / 2 : N;
    const int col0 = EPI == 2 ? (n0 + wn * 128) / 2 : n0 + wn * 128;
    // EPI 1: this lane's residual rows, all loaded up front (clamped rows, no
    // branch) so their latency hides behind the LDS staging below; loaded
    // behind the per-row "m < M" store guard they serialised on one L2 / HBM
    // round trip per row (cdna_hip_programming.md §5 "Projection GEMM at
    // M = 256" item 4(c): ~10 us per o projection at M = 2560)
    bf16x8 rres[EPI == 1 ? NST : 1];
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        const int m = min(m0 + wm * WROWS + i * RPS + lr, M - 1);
        rres[i] = *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldy + col0 + lc * 8);
      }
    }
    auto put = [&](int row, int col, const bf16x4& v) {
      const int byte = col * 2;
      *reinterpret_cast<bf16x4*>(stg + row * RB + (((byte >> 4) ^ (row & (NCH - 1))) << 4) +
                                 (byte & 15)) = v;
    };
    // EPI 3: this wave's 128 columns are one head (n0 % 256 == 0)
    const int head = (n0 + wn * 128) >> 7;
    const bool rotate = EPI == 3 && head < ra.Hq + ra.Hkv;
    int rpos[MTW];                                   // EPI 3: positions, loaded up front
    if (EPI == 3 && rotate) {
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) rpos[mt] = ra.pos[min(m0 + wm * WROWS + mt * 16 + fr, M - 1)];
    }
    // EPI 2 / 3: fused RMSNorm of the input rows (1 when none), loaded up front
    float rsc[EPI >= 2 ? MTW : 1];
    if constexpr (EPI >= 2) {
      int rrow[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) rrow[mt] = min(m0 + wm * WROWS + mt * 16 + fr, M - 1);
      norm_row_scales(ne, rrow, rsc);
    }
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int row = mt * 16 + fr;
      if (EPI == 3 && rotate) {
        // rotate-half RoPE on the fp32 accumulators: d and d + 64 of the
        // head are acc[mt][nt] and acc[mt][nt + 4] of this lane; (cos, sin)
        // of d = 16 nt + 4 fq + j .. +3 are 32 contiguous bytes: two 16-B loads
        const f32x4* cs = reinterpret_cast<const f32x4*>(ra.cos_sin) + (size_t)rpos[mt] * 32;
        f32x4 c4[4][2];
#pragma unroll
        for (int nt_ = 0; nt_ < 4; ++nt_) {
          c4[nt_][0] = cs[nt_ * 8 + fq * 2];
          c4[nt_][1] = cs[nt_ * 8 + fq * 2 + 1];
        }
#pragma unroll
        for (int nt_ = 0; nt_ < 4; ++nt_) {
          bf16x4 o1, o2;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 cc = c4[nt_][j >> 1];
            const float rc = cc[(j & 1) * 2], rs = cc[(j & 1) * 2 + 1];
            const float x1 = acc[mt][nt_][j] * rsc[mt], x2 = acc[mt][nt_ + 4][j] * rsc[mt];
            o1[j] = (bf16)(x1 * rc - x2 * rs);
            o2[j] = (bf16)(x2 * rc + x1 * rs);
          }
          put(row, nt_ * 16 + fq * 4, o1);
          put(row, (nt_ + 4) * 16 + fq * 4, o2);
        }
        continue;
      }
      if constexpr (EPI == 2) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const f32x4 gv = acc[mt][2 * p] * rsc[mt], uv = acc[mt][2 * p + 1] * rsc[mt];
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = (bf16)(gv[j] / (1.f + __expf(-gv[j])) * uv[j]);
          put(row, p * 16 + fq * 4, o);
        }
      } else {
#pragma unroll
        for (int nt_ = 0; nt_ < 8; ++nt_) {
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = (bf16)(EPI == 3 ? acc[mt][nt_][j] * rsc[mt] : acc[mt][nt_][j]);
          put(row, nt_ * 16 + fq * 4, o);
        }
      }
    }
    // EPI 3, K / V heads: this lane's rows' cache slots, loaded up front (a
    // load per row inside the loop would serialise on its latency)
    int rslot[EPI == 3 ? NST : 1];
    if (EPI == 3 && head >= ra.Hq) {
#pragma unroll
      for (int i = 0; i < NST; ++i)
        rslot[i] = ra.slots[min(m0 + wm * WROWS + i * RPS + lr, M - 1)];
    }
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int row = i * RPS + lr;
      const int m = m0 + wm * WROWS + row;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(stg + row * RB + ((lc ^ (row & (NCH - 1))) << 4));
      if (EPI == 3 && m < M) {                       // q rows / paged K and V rows
        bf16* dst;
        if (head < ra.Hq) {
          dst = reinterpret_cast<bf16*>(ra.q_out) + ((size_t)m * ra.Hq + head) * 128;
        } else {
          const int slot = rslot[EPI == 3 ? i : 0];
          if (slot < 0) continue;
          const bool isk = head < ra.Hq + ra.Hkv;
          const int hk = head - ra.Hq - (isk ? 0 : ra.Hkv);
          dst = reinterpret_cast<bf16*>(isk ? ra.k_cache : ra.v_cache) +
                (((size_t)(slot / ra.BS) * ra.Hkv + hk) * ra.BS + slot % ra.BS) * 128;
        }
        *reinterpret_cast<bf16x8*>(dst + lc * 8) = v;
        continue;
      }
      if constexpr (EPI == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)rres[i][j]);
      }
      if (m < M) *reinterpret_cast<bf16x8*>(Y + (size_t)m * ldy + col0 + lc * 8) = v;
      if (EPI == 1 && ne.ss_out) {
        // fused RMSNorm statistic: the row's 128 columns sit in the NCH = 16
        // lanes lr * 16 + lc; one atomic per row and wave
        float ss = m < M ? sumsq_bf16x8(v) : 0.f;
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        ss += __shfl_xor(ss, 4, 64);
        ss += __shfl_xor(ss, 8, 64);
        if (lc == 0 && m < M) ss_atomic_add(ne.ss_out + m, ss);
      }
    }
  }
}

}  // namespace

// 0 ok; 1 K not a multiple of 128; 2 N not a multiple of 256; 3 an operand
// past the 2 GiB buffer range
int gemm256d_ok(int M, int N, int K) {
  if (K % (2 * BK)) return 1;
  if (N % BN) return 2;
  if ((size_t)M * K * 2 >= (1ull << 31) || (size_t)N * K * 2 >= (1ull << 31)) return 3;
  return 0;
}

// Tile height by waves of tiles on the CUs (one workgroup per CU at every
// height): time ~ ceil(tiles / G) x tile time, a tile of h rows costing h / 256
// of a 256-row one divided by the height's relative MFMA efficiency (more LDS
// reads and DMA per MFMA at smaller heights; profiles/gemm_tuning.md).
// MCP_GEMM_BM=<height> forces one; the measured plan (codes 1-5) wins over
// this model wherever it has the shape.
static int g_cus = 0;
static double height_eff(int bm) {
  switch (bm) {
    case 256: return 1.0;
    case 224: return 0.98;
    case 192: return 0.96;
    case 160: return 0.92;
    default: return 0.87;
  }
}
double gemm256d_waves_bm(int M, int N, int K, int bm) {
  if (!g_cus) {
    int d = 0;
    hipDeviceProp_t prop;
    (void)hipGetDevice(&d);
    g_cus = hipGetDeviceProperties(&prop, d) == hipSuccess && prop.multiProcessorCount > 0
                ? prop.multiProcessorCount : 256;
  }
  const double tiles = (double)((M + bm - 1) / bm) * ((N + BN - 1) / BN);
  return ceil(tiles / g_cus) * bm / 256.0 / height_eff(bm);   // in 256-row tile times
}

// plan code -> tile height (gemm.hip's measured plan; 0 = the 128^2 kernel)
int gemm256d_code_height(int code) {
  switch (code) {
    case 1: return 256;
    case 2: return 192;
    case 3: return 160;
    case 4: return 224;
    case 5: return 128;
    default: return 0;
  }
}

int gemm256d_height(int M, int N, int K) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("MCP_GEMM_BM");
    forced = e ? atoi(e) : 0;
  }
  if (forced >= 128 && forced <= 256 && forced % 32 == 0) return forced;
  const int plan_h = gemm256d_code_height(gemm_plan_lookup(M, N, K));   // measured (gemm.hip)
  if (plan_h) return plan_h;
  int best = 256;
  double bc = gemm256d_waves_bm(M, N, K, 256);
  for (int bm = 224; bm >= 128; bm -= 32) {
    const double c = gemm256d_waves_bm(M, N, K, bm);
    if (c < bc) {
      bc = c;
      best = bm;
    }
  }
  return best;
}

// bm: tile height 128-256 (0: pick by gemm256d_height); ra: EPI 3 only
int launch_gemm_tn_256sk_tail(const void* X, const void* W, void* Y, const void* R, int M, int N,
                              int K, int epi, int tile0, hipStream_t s);

// hybrid data-parallel + stream-K tail: the full waves here, a tail wave at
// most a quarter full spread over every CU (MCP_GEMM_HYBRID=0 disables).
// gate|up (N = 28672, 32 k-units) with cold weights: tails of 16 / 32 tiles
// gain 2-6 %, 64 is even, 96 / 128 lose 2-6 % to the slab hand-offs
// (M = 2368-2560: 473 vs 446 us plain; profiles/gemm_tuning.md)
static int hybrid_tile0(int M, int N, int bm, int epi) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("MCP_GEMM_HYBRID");
    on = e ? atoi(e) : 1;
  }
  if (!on || bm != 256 || epi < 0 || epi > 2) return 0;
  if (!g_cus) gemm256d_waves_bm(M, N, 128, 256);     // initialises g_cus
  const int T = ((M + 255) / 256) * ((N + BN - 1) / BN);
  const int full = (T / g_cus) * g_cus, tail = T - full;
  return (full > 0 && tail > 0 && 4 * tail <= g_cus) ? full : 0;
}

// Tile group (M-tiles per W panel in the grouped order).  4 was fixed from
// warm-weight timings; a serving step streams cold weights, where sharing a
// W panel across more M-tiles in one pass can read it from HBM fewer times.
// gemm_group_force (tools) / MCP_GEMM_GROUP override; the plan's "group"
// entry per M bucket otherwise, default 4.
static int g_group_force = 0;
void gemm_group_force(int g) { g_group_force = g; }
int gemm256d_group(int M, int N, int K) {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("MCP_GEMM_GROUP");
    env = e ? atoi(e) : 0;
  }
  if (g_group_force > 0) return g_group_force;
  if (env > 0) return env;
  const int g = gemm_plan_group(M, N, K);
  return g > 0 ? g : 4;
}

// Wide direct epilogue (store_wide) instead of the LDS-staged one.  Bitwise
// the same outputs; over the headline's GEMM mix (cold weights, one process,
// profiles/gemm_tuning.md round 5) gate|up + SwiGLU +1.6 %, o +0.1 %, down
// -0.8 %: default (-1) = SwiGLU only; MCP_GEMM_WIDE_EPI / gemm_wide_force
// 0 = never, 1 = every plain / residual / SwiGLU epilogue.  The output must
// be < 2 GiB (buffer descriptor).
static int g_wide_force = -1;
void gemm_wide_force(int w) { g_wide_force = w; }
bool gemm_wide_on(int M, int N, int epi) {
  static const int env = getenv("MCP_GEMM_WIDE_EPI") ? atoi(getenv("MCP_GEMM_WIDE_EPI")) : -1;
  const int on = g_wide_force >= 0 ? g_wide_force : env;
  if (epi < 0 || epi > 2 || (size_t)M * (epi == 2 ? N / 2 : N) * 2 >= (1ull << 31)) return false;
  return on < 0 ? epi == 2 : on != 0;
}

template <int BMT>
static int launch_height(const void* X, const void* W, void* Y, const void* R, int M, int N,
                         int K, int epi, dim3 grid, int group, const RopeArgs& ra, hipStream_t s) {
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  if (gemm_wide_on(M, N, epi)) {
    switch (epi) {
      case 0: gemm_tn_256d<0, BMT, true><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
      case 1: gemm_tn_256d<1, BMT, true><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
      case 2: gemm_tn_256d<2, BMT, true><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
      default: return 2;
    }
  }
  switch (epi) {
    case 0: gemm_tn_256d<0, BMT><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
    case 1: gemm_tn_256d<1, BMT><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
    case 2: gemm_tn_256d<2, BMT><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
    case 3: gemm_tn_256d<3, BMT><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), nullptr, nullptr); return 0;
    default: return 2;
  }
}

// Persistent form (gemm256p.hip): -1 = plan / MCP_GEMM_PERSIST, 0 = off,
// 1 = whenever the tiles exceed one wave of workgroups, 2 = always
static int g_persist_force = -1;
void gemm_persist_force(int p) { g_persist_force = p; }
int gemm256d_persist(int M, int N, int K, int tiles) {
  static int env = -2;
  if (env == -2) {
    const char* e = getenv("MCP_GEMM_PERSIST");
    env = e ? atoi(e) : -1;
  }
  int mode = g_persist_force >= 0 ? g_persist_force : env;
  if (mode < 0) mode = gemm_plan_persist(M, N, K) ? 1 : 0;
  if (!g_cus) gemm256d_waves_bm(M, N, K, 256);
  return mode == 2 || (mode == 1 && tiles > g_cus);
}

static int launch_256d_impl(const void* X, const void* W, void* Y, const void* R, int M, int N,
                            int K, int epi, int bm, const RopeArgs& ra, hipStream_t s) {
  if (const int rc = gemm256d_ok(M, N, K)) return rc;
  if (bm == 0) bm = gemm256d_height(M, N, K);
  const int nm = (M + bm - 1) / bm, nn = (N + BN - 1) / BN;
  if (gemm256d_persist(M, N, K, nm * nn))
    return launch_gemm_tn_256p(X, W, Y, R, M, N, K, epi, bm, g_cus, gemm256d_group(M, N, K), ra, s);
  // at most half the CUs' worth of 256-row tiles: the whole product runs
  // stream-K (every tile over >= 2 workgroups, last arriver sums the slabs)
  // instead of leaving half the chip idle (MCP_GEMM_SK_SMALL=0 disables)
  static const int sk_small = getenv("MCP_GEMM_SK_SMALL") ? atoi(getenv("MCP_GEMM_SK_SMALL")) : 1;
  if (sk_small && bm == 256 && epi >= 0 && epi <= 2) {
    if (!g_cus) gemm256d_waves_bm(M, N, K, 256);
    if (2 * nm * nn <= g_cus) return launch_gemm_tn_256sk_tail(X, W, Y, R, M, N, K, epi, 0, s);
  }
  const int group = gemm256d_group(M, N, K);
  // the stream-K tail kernel walks the tiles in the group-4 order
  const int tile0 = group == 4 ? hybrid_tile0(M, N, bm, epi) : 0;
  const dim3 grid(tile0 > 0 ? tile0 : nm * nn);
  if (tile0 > 0) {
    // full waves first (same stream: the tail starts when they are done)
    if (const int rc = launch_height<256>(X, W, Y, R, M, N, K, epi, grid, group, ra, s)) return rc;
    return launch_gemm_tn_256sk_tail(X, W, Y, R, M, N, K, epi, tile0, s);
  }
  switch (bm) {
    case 256: return launch_height<256>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 224: return launch_height<224>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 192: return launch_height<192>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 160: return launch_height<160>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 128: return launch_height<128>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    default: return 4;
  }
}

int launch_gemm_tn_256d_bm(const void* X, const void* W, void* Y, const void* R, int M, int N,
                           int K, int epi, int bm, hipStream_t s) {
  return launch_256d_impl(X, W, Y, R, M, N, K, epi, bm, RopeArgs{}, s);
}

// One QKV + RoPE + K/V-write path by code (the tuner's candidates and the
// "rope" plan):
//   1..5            AGPR kernel, EPI 3, at the height of plan code c
//   200             weight-streaming kernel, EPI 3 (M <= 128)
//   500             the GEMM by the code / flex plan into qkv, then rope_kv
//   1000 + 16 c + S flex tile c x S-way split-K, the reduce applies RoPE
// nonzero: not supported for this shape (nothing launched)
int launch_qkv_rope_algo(const void* X, const void* W, void* qkv, int M, int N, int K, int D,
                         const RopeArgs& ra, int algo, hipStream_t s) {
  if (D != 128 || N != (ra.Hq + 2 * ra.Hkv) * 128) return 1;
  if (algo >= 1000)
    return launch_qkv_rope_flex_split(X, W, M, N, K, D, ra, (algo - 1000) / 16, (algo - 1000) % 16, s);
  if (algo == 500) {
    launch_gemm_tn(X, W, qkv, nullptr, M, N, K, s);
    launch_rope_kv(qkv, ra.pos, ra.slots, ra.cos_sin, ra.q_out, ra.k_cache, ra.v_cache, M, ra.Hq,
                   ra.Hkv, D, ra.BS, s);
    return 0;
  }
  if (algo == 200) return launch_gemm_stream(X, W, nullptr, nullptr, M, N, K, 3, ra, s);
  if (algo >= 1 && algo <= 5) {
    if (gemm256d_ok(M, N, K)) return 4;
    return launch_256d_impl(X, W, nullptr, nullptr, M, N, K, 3, gemm256d_code_height(algo), ra, s);
  }
  return 5;
}

// QKV + RoPE + paged K/V write (EPI 3) on the AGPR kernel when the selector
// picks it for this shape; otherwise the plain GEMM into qkv and rope_kv
void launch_qkv_rope(const void* X, const void* W, void* qkv, int M, int N, int K, int D,
                     const RopeArgs& ra, hipStream_t s) {
  static const int fused = getenv("MCP_QKV_ROPE_FUSED") ? atoi(getenv("MCP_QKV_ROPE_FUSED")) : 1;
  // a measured path for the bucket (timed at its top row; the decode sizes
  // below 33 rows keep the stream kernel)
  const int rp = (fused && M > 32) ? gemm_plan_rope(M, N, K) : -1;
  if (rp >= 0 && launch_qkv_rope_algo(X, W, qkv, M, N, K, D, ra, rp, s) == 0) return;
  if (fused && gemm_stream_enabled() && gemm_stream_pick(M, N, K, 3) &&
      launch_gemm_stream(X, W, nullptr, nullptr, M, N, K, 3, ra, s) == 0)
    return;
  // a measured flex x split-K bucket (timed against the AGPR heights by the
  // tuner): the reduce applies RoPE and writes the cache
  if (fused && launch_qkv_rope_fsplit(X, W, M, N, K, D, ra, s) == 0) return;
  if (fused && D == 128 && N == (ra.Hq + 2 * ra.Hkv) * 128 && M > SKINNY_MAX_M &&
      gemm_select(M, N, K) == 1 && gemm256d_ok(M, N, K) == 0 &&
      launch_256d_impl(X, W, nullptr, nullptr, M, N, K, 3, 0, ra, s) == 0)
    return;
  launch_gemm_tn(X, W, qkv, nullptr, M, N, K, s);
  launch_rope_kv(qkv, ra.pos, ra.slots, ra.cos_sin, ra.q_out, ra.k_cache, ra.v_cache, M, ra.Hq,
                 ra.Hkv, D, ra.BS, s);
}

int launch_gemm_tn_256d(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        int epi, hipStream_t s) {
  return launch_gemm_tn_256d_bm(X, W, Y, R, M, N, K, epi, 0, s);
}

// the power / issue ladder of the production gate|up kernel (SwiGLU, wide
// epilogue, 256-row tiles) and of a plain 256-row one: rung 0 = production,
// 1-3 = the PROBE forms above (tools/gemm_power_ladder.py); nonzero if the
// shape is not a whole-tile one
int launch_gemm_probe(const void* X, const void* W, void* Y, int M, int N, int K, int epi,
                      int probe, hipStream_t s) {
  if (M % 256 || N % BN || K % (2 * BK) || (epi != 0 && epi != 2) || probe < 0 || probe > 3)
    return 1;
  const dim3 grid((M / 256) * (N / BN));
  const int group = gemm256d_group(M, N, K);
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  const RopeArgs ra{};
  const NormEpi ne{};
#define PROBE_LAUNCH(E, P) gemm_tn_256d<E, 256, true, P><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, ne, nullptr, nullptr)
  if (epi == 2) {
    switch (probe) {
      case 0: PROBE_LAUNCH(2, 0); break;
      case 1: PROBE_LAUNCH(2, 1); break;
      case 2: PROBE_LAUNCH(2, 2); break;
      default: PROBE_LAUNCH(2, 3); break;
    }
  } else {
    switch (probe) {
      case 0: PROBE_LAUNCH(0, 0); break;
      case 1: PROBE_LAUNCH(0, 1); break;
      case 2: PROBE_LAUNCH(0, 2); break;
      default: PROBE_LAUNCH(0, 3); break;
    }
  }
#undef PROBE_LAUNCH
  return 0;
}

// ---- SPLIT 2 (K halves, in-launch hand-off): slabs + tile counters, one set
//      per device, allocated at library load (gemm_splitk_init), never inside
//      a hipGraph capture.  Counters start at 0 and every tile's last arriver
//      re-arms its own, so graph replays need no memset node.  One launch at a
//      time (the model's stream), as for the stream-K slabs.
namespace {
constexpr int SPLIT_MAX_TILES = 128;                 // one wave: 2 x 128 workgroups
int g_pf_force = -1;                                 // gemm_pf_force (tests, A/B)
struct Split2State {
  f32x4* ws = nullptr;
  int* cnt = nullptr;
};
Split2State* split2_state() {
  static Split2State devs[64];
  int d = 0;
  (void)hipGetDevice(&d);
  Split2State& st = devs[d & 63];
  if (!st.ws) {
    f32x4* ws = nullptr;
    int* cnt = nullptr;
    if (hipMalloc(&ws, (size_t)SPLIT_MAX_TILES * 256 * 256 * sizeof(float)) != hipSuccess) return nullptr;
    if (hipMalloc(&cnt, SPLIT_MAX_TILES * sizeof(int)) != hipSuccess) {
      (void)hipFree(ws);
      return nullptr;
    }
    (void)hipMemset(cnt, 0, SPLIT_MAX_TILES * sizeof(int));
    (void)hipDeviceSynchronize();
    st.ws = ws;
    st.cnt = cnt;
  }
  return &st;
}

template <int BMT>
int launch_split2_height(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                         int epi, int group, const Split2State& st, hipStream_t s) {
  const int tiles = ((M + BMT - 1) / BMT) * (N / BN);
  if (tiles > SPLIT_MAX_TILES) return 6;
  const dim3 grid(2 * tiles);
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  const RopeArgs ra{};
  // always the wide epilogue (it adds the other half's slab); Y < 2 GiB
  if ((size_t)M * (epi == 2 ? N / 2 : N) * 2 >= (1ull << 31)) return 8;
  // W L2 fills ahead of the DMA (PF): MCP_GEMM_PF=1 / gemm_pf_force
  static const int pf_env = getenv("MCP_GEMM_PF") ? atoi(getenv("MCP_GEMM_PF")) : 0;
  if (g_pf_force >= 0 ? g_pf_force : pf_env) {
    switch (epi) {
      case 0: gemm_tn_256d<0, BMT, true, 0, 2, 1><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), st.ws, st.cnt); return 0;
      case 1: gemm_tn_256d<1, BMT, true, 0, 2, 1><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, group, ra, norm_epi(), st.ws, st.cnt); return 0;
      case 2: gemm_tn_256d<2, BMT, true, 0, 2, 1><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), st.ws, st.cnt); return 0;
      default: return 2;
    }
  }
  switch (epi) {
    case 0: gemm_tn_256d<0, BMT, true, 0, 2><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), st.ws, st.cnt); return 0;
    case 1: gemm_tn_256d<1, BMT, true, 0, 2><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, group, ra, norm_epi(), st.ws, st.cnt); return 0;
    case 2: gemm_tn_256d<2, BMT, true, 0, 2><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi(), st.ws, st.cnt); return 0;
    default: return 2;
  }
}
}  // namespace

int gemm256d_split2_prealloc() { return split2_state() ? 0 : 1; }
void gemm_pf_force(int p) { g_pf_force = p; }

// Y = X W^T (+ R | SwiGLU) with every tile over two workgroups (K halves);
// bm = a tile height 128-256.  Nonzero (nothing launched): 1-3 gemm256d_ok,
// 4 bad height, 5 K not a multiple of 256 (each half an even number of
// 64-deep k-tiles), 6 more than 128 tiles, 7 no workspace, 2 epilogue
int launch_gemm_tn_256d_split2(const void* X, const void* W, void* Y, const void* R, int M, int N,
                               int K, int epi, int bm, hipStream_t s) {
  if (const int rc = gemm256d_ok(M, N, K)) return rc;
  if (K % (4 * BK)) return 5;
  Split2State* st = split2_state();
  if (!st) return 7;
  const int group = gemm256d_group(M, N, K);
  switch (bm) {
    case 256: return launch_split2_height<256>(X, W, Y, R, M, N, K, epi, group, *st, s);
    case 224: return launch_split2_height<224>(X, W, Y, R, M, N, K, epi, group, *st, s);
    case 192: return launch_split2_height<192>(X, W, Y, R, M, N, K, epi, group, *st, s);
    case 160: return launch_split2_height<160>(X, W, Y, R, M, N, K, epi, group, *st, s);
    case 128: return launch_split2_height<128>(X, W, Y, R, M, N, K, epi, group, *st, s);
    default: return 4;
  }
}
