// K1, persistent form of the AGPR kernel (gemm256d.hip): one workgroup per CU
// walks tiles j = blockIdx.x, + G, + 2G, ... (G = gridDim.x = CUs), in the
// same grouped + XCD-remapped order as the one-tile-per-workgroup launch (tile
// j runs on the XCD block j would have run on), with the SAME mainloop -
// 256-column tiles of BMT rows, one wave per SIMD, 256 fp32 accumulators in
// AGPRs, 64-deep k-tiles staged by LDS-DMA in 128-byte rows, one barrier per
// 128 MFMAs.  What the persistence changes:
//
//  * no cold start per tile: the last two k-tiles of tile j DMA tile j+G's
//    k-tiles 0 and 1 (the pipeline's trailing loads, unconsumed in the
//    one-tile form), and the fragment reads of the last half already fetch
//    tile j+G's first fragments - the next tile's mainloop starts on landed
//    operands;
//  * the epilogue's global stores overlap the next tile's mainloop: the
//    staged epilogue runs through a LDS region of its own (the 32 KiB the two
//    operand slots leave of 160 KiB at 256 rows; 8 KiB per wave, so a wave's
//    128-row tile goes out in passes of 32 rows), the output stores are
//    range-checked buffer stores (a fixed count per wave: rows past M are
//    dropped by the buffer descriptor, not branched around), and the first
//    barrier of the next tile waits only for the DMAs older than them
//    (s_waitcnt vmcnt(<that count>)): the stores drain while the next tile's
//    first 64 MFMAs run.
//
// The rest - fragment layouts, swizzles, the fused epilogues (residual, SwiGLU,
// QKV + RoPE + paged K/V write, the RMSNorm statistics) - is gemm256d.hip's.
// Launched only when the tiles exceed one wave of workgroups
// (launch_gemm_tn_256p: MCP_GEMM_PERSIST / the plan's "persist" entry).
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BN = 256, BK = 64;
constexpr int ROWB = BK * 2;                        // 128-byte LDS rows
constexpr int PIECE_BB = 256 * ROWB;                // the W operand of a slot: 32 KiB
constexpr int LDS_BYTES = 160 * 1024;

DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

DEV void mfma_a(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

template <int MTW>
struct Frags {
  bf16x8 a[MTW];
  bf16x8 b[8];
};

DEV void tile_coords(int t, int nm, int nn, int bm, int group, int& m0, int& n0) {
  const int per_group = group * nn;
  const int g = t / per_group;
  const int first_m = g * group;
  const int gsz = min(nm - first_m, group);
  m0 = (first_m + (t % per_group) % gsz) * bm;
  n0 = ((t % per_group) / gsz) * BN;
}

constexpr int ops_at(int j, int n, int P) { return ((j + 1) * n) / P - (j * n) / P; }
constexpr int op0_at(int j, int n, int P) { return (j * n) / P; }

template <int EPI, int BMT, bool WIDE = false>
struct Geo {
  static constexpr int MTW = BMT / 32;              // 16-row MFMA tiles per wave
  static constexpr int WROWS = BMT / 2;             // rows per wave
  static constexpr int PIECE_A = BMT * ROWB;
  static constexpr int SLOT_B = PIECE_A + PIECE_BB;
  static constexpr int QA = BMT / 32;
  static constexpr int NDMA = QA + 8;
  static constexpr int NRD = 8 + MTW;
  static constexpr int NP = MTW * 4;                // MFMA pairs per k-half
  static constexpr int OUTW = EPI == 2 ? 64 : 128;  // output columns per wave
  static constexpr int RB = OUTW * 2;               // staged row bytes
  static constexpr int NCH = RB / 16;
  static constexpr int RPS = 1024 / RB;             // rows per 1 KiB wave access
  static constexpr int STG_W = ((LDS_BYTES - 2 * SLOT_B) / 4) & ~1023;   // staging per wave
  static constexpr int PMT = STG_W / (16 * RB) < MTW ? STG_W / (16 * RB) : MTW;  // m-tiles per pass
  static constexpr int NPASS = (MTW + PMT - 1) / PMT;
  // VMEM instructions every wave's epilogue issues for sure (range-checked
  // buffer stores; EPI 1 also its residual loads): the next tile's first
  // barrier leaves that many younger than the DMAs it waits for in flight
  // (the wide epilogue: MTW x 4 (EPI 2: x 2) stores, EPI 1 as many residual loads)
  static constexpr int NEPI_RAW = EPI == 3 ? 0
                                  : WIDE ? MTW * (EPI == 2 ? 2 : 4) * (EPI == 1 ? 2 : 1)
                                         : (WROWS / RPS) * (EPI == 1 ? 2 : 1);
  static constexpr int NEPI = NEPI_RAW > 63 ? 63 : NEPI_RAW;
};

template <int N>
DEV void waitcnt_vm_lgkm0() {
  // s_waitcnt vmcnt(N) lgkmcnt(0)
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}

// per-tile DMA state: X row offsets (clamped rows) and the first W row
// (vector-typed so it stays in registers: an array member whose address a
// select could take goes to scratch).  At namespace scope: a class local to
// the kernel, used by the kernel's lambdas, leaves hipcc's host pass without
// the kernel's launch stub (undefined symbol at load time).
struct TileDma {
  unsigned offA0;                                   // this lane's X row of A instruction 0
  int rowB0;
};

template <int EPI, int BMT, bool WIDE = false>
__global__ __launch_bounds__(256, 1) void gemm_tn_256p(const bf16* __restrict__ X,
                                                       const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y,
                                                       const bf16* __restrict__ R, int M, int N,
                                                       int K, int group, const RopeArgs ra,
                                                       const NormEpi ne) {
  using G_ = Geo<EPI, BMT, WIDE>;
  constexpr int MTW = G_::MTW, WROWS = G_::WROWS, PIECE_A = G_::PIECE_A, SLOT_B = G_::SLOT_B;
  constexpr int QA = G_::QA, NDMA = G_::NDMA, NRD = G_::NRD, NP = G_::NP;
  constexpr int OUTW = G_::OUTW, RB = G_::RB, NCH = G_::NCH, RPS = G_::RPS;
  constexpr int STG_W = G_::STG_W, PMT = G_::PMT, NPASS = G_::NPASS;
  static_assert(BMT % 32 == 0 && BMT >= 128 && BMT <= 256, "tile height");
  static_assert(PMT >= 1 && 2 * SLOT_B + 4 * STG_W <= LDS_BYTES, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT_B + 4 * STG_W];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nm = (M + BMT - 1) / BMT, nn = (N + BN - 1) / BN;
  const int ntiles = nm * nn;
  const int GR = gridDim.x;                          // workgroups (<= tiles)

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)M * K * 2),
                                                     0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((size_t)N * K * 2),
                                                     0x00020000);
  const int ldy = EPI == 2 ? N / 2 : N;
  const auto rsY = __builtin_amdgcn_make_buffer_rsrc((void*)Y, (short)0,
                                                     (int)((size_t)M * ldy * 2), 0x00020000);
  const int chunk = (lane & 7) ^ (lane >> 3);
  const unsigned offB = (unsigned)(((lane >> 3) * K + chunk * 8) * 2);
  const int nt = K / BK;                             // >= 2, even (launcher)

  // X rows past M fall outside the buffer descriptor (voffset range check):
  // their LDS rows are never stored, so no clamp; instruction q reads the rows
  // 8 q further: + 16 q K bytes, a wave-uniform addend (one VALU add per DMA
  // instead of 8 live offsets, which spilled at 256 rows)
  auto tile_dma = [&](int m0, int n0, TileDma& d) {
    d.offA0 = (unsigned)(((size_t)(m0 + 8 * QA * wave + (lane >> 3)) * K + chunk * 8) * 2);
    d.rowB0 = n0 + 64 * wave;
  };
  TileDma dstate;
  // DMA instruction i of k-tile kt into slot, from the operands ``dst_`` points
  // at: the current tile's, switched to the next tile's before the DMAs of its
  // k-tiles 0 / 1 (one state object: a select between two would take their
  // addresses and send both to scratch)
  auto dma1 = [&](int kt, int slot, int i) __attribute__((always_inline)) {
    const bool b = i >= QA;
    const int q = b ? i - QA : i;
    const int kb = kt * BK * 2;
    auto* dst = (__attribute__((address_space(3))) void*)(
        smem + slot * SLOT_B + (b ? PIECE_A + (8 * wave + q) * 1024 : (QA * wave + q) * 1024));
    if (b)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, dst, 16, offB, (dstate.rowB0 + 8 * q) * K * 2 + kb, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, dstate.offA0 + q * 16 * K, kb, 0, 0);
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  int rbase[2][2][2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int ch = ((4 * kh + fq) ^ (fr & 7)) * 16;
      rbase[sl][kh][0] = sl * SLOT_B + (wm * WROWS + fr) * ROWB + ch;
      rbase[sl][kh][1] = sl * SLOT_B + PIECE_A + (wn * 128 + fr) * ROWB + ch;
    }
  auto fread1 = [&](int slot, int kh, Frags<MTW>& f, int i) __attribute__((always_inline)) {
    if (i < 8)
      f.b[i] = *reinterpret_cast<const bf16x8*>(smem + rbase[slot][kh][1] + i * 2048);
    else
      f.a[i - 8] = *reinterpret_cast<const bf16x8*>(smem + rbase[slot][kh][0] + (i - 8) * 2048);
  };

  f32x4 acc[MTW][8];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  };

  // ---- the first tile: as the one-tile kernel's prologue
  int j = blockIdx.x;
  int m0, n0;
  tile_coords(xcd_remap(j, ntiles), nm, nn, BMT, group, m0, n0);
  tile_dma(m0, n0, dstate);
  int jn = j + GR;
  bool has_next = jn < ntiles;
  int m0n = m0, n0n = n0;
  if (has_next) tile_coords(xcd_remap(jn, ntiles), nm, nn, BMT, group, m0n, n0n);

  zero_acc();
  Frags<MTW> F[2];
#pragma unroll
  for (int i = 0; i < NDMA; ++i) dma1(0, 0, i);
#pragma unroll
  for (int i = 0; i < NDMA; ++i) dma1(1, 1, i);
  if constexpr (NDMA == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (NDMA == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else if constexpr (NDMA == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  else if constexpr (NDMA == 13) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < NRD; ++i) fread1(0, 0, F[0], i);
  __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0)
  asm volatile("s_nop 4" ::: "memory");

  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  auto keep = [](const Frags<MTW>& f) {
#pragma unroll
    for (int i = 0; i < MTW; ++i) asm volatile("" :: "v"(f.a[i]));
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" :: "v"(f.b[i]));
  };
  // after_epi: the first k-tile of a tile that follows an epilogue - its
  // mid barrier leaves the epilogue's NEPI stores in flight
  auto tile = [&](int t, auto c_c, bool after_epi) __attribute__((always_inline)) {
    constexpr int C = decltype(c_c)::value;
    fence();
#pragma unroll
    for (int jj = 0; jj < NP; ++jj) {
      const int i0 = 2 * jj, i1 = 2 * jj + 1;
      mfma_a(acc[i0 >> 3][i0 & 7], F[0].b[i0 & 7], F[0].a[i0 >> 3]);
      mfma_a(acc[i1 >> 3][i1 & 7], F[0].b[i1 & 7], F[0].a[i1 >> 3]);
#pragma unroll
      for (int r = 0; r < ops_at(jj, NRD, NP); ++r) fread1(C, 1, F[1], op0_at(jj, NRD, NP) + r);
      fence();
    }
    keep(F[0]);
    if (after_epi)
      waitcnt_vm_lgkm0<G_::NEPI>();
    else
      __builtin_amdgcn_s_waitcnt(0x0070);            // vmcnt(0) lgkmcnt(0)
    raw_barrier();
    fence();
    // DMA of k-tile t + 2: this tile's, else the next tile's first two, else
    // a clamped reload nobody consumes
    const bool own = t + 2 < nt;
    if (t + 2 == nt && has_next) tile_dma(m0n, n0n, dstate);   // switch to the next tile
    const int kt = own ? t + 2 : (has_next ? t + 2 - nt : nt - 1);
#pragma unroll
    for (int jj = 0; jj < NP; ++jj) {
      const int i0 = 2 * jj, i1 = 2 * jj + 1;
      mfma_a(acc[i0 >> 3][i0 & 7], F[1].b[i0 & 7], F[1].a[i0 >> 3]);
      mfma_a(acc[i1 >> 3][i1 & 7], F[1].b[i1 & 7], F[1].a[i1 >> 3]);
#pragma unroll
      for (int r = 0; r < ops_at(jj, NRD, NP); ++r) fread1(C ^ 1, 0, F[0], op0_at(jj, NRD, NP) + r);
#pragma unroll
      for (int dd = 0; dd < ops_at(jj, NDMA, NP); ++dd) dma1(kt, C, op0_at(jj, NDMA, NP) + dd);
      fence();
    }
    keep(F[1]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;

  char* stg = smem + 2 * SLOT_B + wave * STG_W;
  const int lr = lane / NCH, lc = lane % NCH;
  bool after_epi = false;
  while (true) {
    for (int t = 0; t < nt; t += 2) {
      tile(t, C0{}, after_epi && t == 0);
      tile(t + 1, C1{}, false);
    }
    // MFMA results -> VALU reads (inline asm is not padded)
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

    // ---- epilogue of tile (m0, n0), through this wave's staging region
    const int col0 = EPI == 2 ? (n0 + wn * 128) / 2 : n0 + wn * 128;
    const int head = (n0 + wn * 128) >> 7;
    const bool rotate = EPI == 3 && head < ra.Hq + ra.Hkv;
    constexpr int NST = WROWS / RPS;                 // store rows per lane, whole tile
    bf16x8 rres[EPI == 1 && !WIDE ? NST : 1];
    if constexpr (EPI == 1 && !WIDE) {
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        const int m = min(m0 + wm * WROWS + i * RPS + lr, M - 1);
        rres[i] = *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldy + col0 + lc * 8);
      }
    }
    int rpos[MTW];
    if (EPI == 3 && rotate) {
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) rpos[mt] = ra.pos[min(m0 + wm * WROWS + mt * 16 + fr, M - 1)];
    }
    float rsc[EPI >= 2 ? MTW : 1];
    if constexpr (EPI >= 2) {
      int rrow[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) rrow[mt] = min(m0 + wm * WROWS + mt * 16 + fr, M - 1);
      norm_row_scales(ne, rrow, rsc);
    }
    int rslot[EPI == 3 ? NST : 1];
    if (EPI == 3 && head >= ra.Hq) {
#pragma unroll
      for (int i = 0; i < NST; ++i)
        rslot[i] = ra.slots[min(m0 + wm * WROWS + i * RPS + lr, M - 1)];
    }
    if constexpr (WIDE && EPI != 3) {
      // wide direct epilogue (common.h store_wide): no staging passes, no
      // barrier; the stores drain under the next tile's first k-tiles
      float rsc2[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        if constexpr (EPI == 2) rsc2[mt] = rsc[mt];
        else rsc2[mt] = 1.f;
      }
      store_wide<EPI, MTW>(acc, rsY, R, M, ldy, m0 + wm * WROWS, col0, fr, fq, rsc2, ne);
    } else {
    auto put = [&](int row, int col, const bf16x4& v) __attribute__((always_inline)) {
      const int byte = col * 2;
      *reinterpret_cast<bf16x4*>(stg + row * RB + (((byte >> 4) ^ (row & (NCH - 1))) << 4) +
                                 (byte & 15)) = v;
    };
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      // m-tiles [p PMT, p PMT + PMT) -> staging rows (mt - p PMT) * 16 + fr;
      // the guards below are constants once the loops are unrolled
#pragma unroll
      for (int mq = 0; mq < PMT; ++mq) {
        const int mt = p * PMT + mq;
        if (mt >= MTW) continue;
        const int row = mq * 16 + fr;
        if (EPI == 3 && rotate) {
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
            for (int e = 0; e < 4; ++e) {
              const f32x4 cc = c4[nt_][e >> 1];
              const float rc = cc[(e & 1) * 2], rs = cc[(e & 1) * 2 + 1];
              const float x1 = acc[mt][nt_][e] * rsc[mt], x2 = acc[mt][nt_ + 4][e] * rsc[mt];
              o1[e] = (bf16)(x1 * rc - x2 * rs);
              o2[e] = (bf16)(x2 * rc + x1 * rs);
            }
            put(row, nt_ * 16 + fq * 4, o1);
            put(row, (nt_ + 4) * 16 + fq * 4, o2);
          }
          continue;
        }
        if constexpr (EPI == 2) {
#pragma unroll
          for (int pp = 0; pp < 4; ++pp) {
            const f32x4 gv = acc[mt][2 * pp] * rsc[mt], uv = acc[mt][2 * pp + 1] * rsc[mt];
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (bf16)(gv[e] / (1.f + __expf(-gv[e])) * uv[e]);
            put(row, pp * 16 + fq * 4, o);
          }
        } else {
#pragma unroll
          for (int nt_ = 0; nt_ < 8; ++nt_) {
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (bf16)(EPI == 3 ? acc[mt][nt_][e] * rsc[mt] : acc[mt][nt_][e]);
            put(row, nt_ * 16 + fq * 4, o);
          }
        }
      }
      // staged rows of this pass -> global, 16 B per lane, 256 B per row
#pragma unroll
      for (int ii = 0; ii < PMT * 16 / RPS; ++ii) {
        const int i = p * PMT * 16 / RPS + ii;       // whole-tile store index (rres / rslot)
        if (i >= NST) continue;
        const int srow = ii * RPS + lr;              // staging row
        const int m = m0 + wm * WROWS + i * RPS + lr;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(stg + srow * RB + ((lc ^ (srow & (NCH - 1))) << 4));
        if constexpr (EPI == 3) {
          if (m < M) {
            bf16* dst;
            bool ok = true;
            if (head < ra.Hq) {
              dst = reinterpret_cast<bf16*>(ra.q_out) + ((size_t)m * ra.Hq + head) * 128;
            } else {
              const int slot = rslot[i];
              ok = slot >= 0;
              const bool isk = head < ra.Hq + ra.Hkv;
              const int hk = head - ra.Hq - (isk ? 0 : ra.Hkv);
              const int sl = max(slot, 0);
              dst = reinterpret_cast<bf16*>(isk ? ra.k_cache : ra.v_cache) +
                    (((size_t)(sl / ra.BS) * ra.Hkv + hk) * ra.BS + sl % ra.BS) * 128;
            }
            if (ok) *reinterpret_cast<bf16x8*>(dst + lc * 8) = v;
          }
        } else {
          if constexpr (EPI == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)rres[i][e]);
          }
          // range-checked: rows >= M fall outside the descriptor and are dropped
          const unsigned off = (unsigned)(((size_t)m * ldy + col0 + lc * 8) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsY,
                                                 m < M ? off : 0x80000000u, 0, 0);
          if (EPI == 1 && ne.ss_out) {
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
    }
    if (!has_next) break;
    // ---- next tile: its k-tiles 0 / 1 are in slots 0 / 1 (or in flight), its
    //      first fragments in F[0]
    j = jn;
    m0 = m0n;
    n0 = n0n;                                      // dstate already points at this tile
    jn = j + GR;
    has_next = jn < ntiles;
    if (has_next) tile_coords(xcd_remap(jn, ntiles), nm, nn, BMT, group, m0n, n0n);
    zero_acc();
    asm volatile("s_nop 4" ::: "memory");
    after_epi = true;
  }
  // drain the trailing (unconsumed) DMAs and the stores before the LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// (outside the anonymous namespace, as gemm256d.hip's launch_height: a kernel
// template launched from a launcher template inside it gets no host stub)
template <int BMT>
static int launch_p_height(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                    int epi, int grid, int group, const RopeArgs& ra, hipStream_t s) {
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  if (gemm_wide_on(M, N, epi)) {
    switch (epi) {
      case 0: gemm_tn_256p<0, BMT, true><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi()); return 0;
      case 1: gemm_tn_256p<1, BMT, true><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, group, ra, norm_epi()); return 0;
      case 2: gemm_tn_256p<2, BMT, true><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi()); return 0;
      default: return 2;
    }
  }
  switch (epi) {
    case 0: gemm_tn_256p<0, BMT><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi()); return 0;
    case 1: gemm_tn_256p<1, BMT><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, group, ra, norm_epi()); return 0;
    case 2: gemm_tn_256p<2, BMT><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi()); return 0;
    case 3: gemm_tn_256p<3, BMT><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, group, ra, norm_epi()); return 0;
    default: return 2;
  }
}

// Persistent AGPR GEMM: grid = min(tiles, CUs) workgroups, each walking tiles
// blockIdx.x + k * grid.  Same shape rules as gemm256d_ok (K % 128 == 0,
// N % 256 == 0, operands < 2 GiB); EPI 2 writes [M, N/2].
int launch_gemm_tn_256p(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        int epi, int bm, int cus, int group, const RopeArgs& ra, hipStream_t s) {
  if (K % (2 * BK) || N % BN) return 1;
  const int ldy = epi == 2 ? N / 2 : N;
  if ((size_t)M * K * 2 >= (1ull << 31) || (size_t)N * K * 2 >= (1ull << 31) ||
      (size_t)M * ldy * 2 >= (1ull << 31))
    return 3;
  const int T = ((M + bm - 1) / bm) * (N / BN);
  const int grid = T < cus ? T : cus;
  switch (bm) {
    case 256: return launch_p_height<256>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 224: return launch_p_height<224>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 192: return launch_p_height<192>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 160: return launch_p_height<160>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    case 128: return launch_p_height<128>(X, W, Y, R, M, N, K, epi, grid, group, ra, s);
    default: return 4;
  }
}
