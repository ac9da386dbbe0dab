// Shared device helpers for the gfx950 (CDNA4) kernels of the planner engine.
// Wave size is 64 everywhere (cdna_hip_programming.md §1); bf16 is the native
// __bf16 type so float->bf16 casts lower to v_cvt_pk_bf16_f32 (NaN-safe,
// MI355X_MICROARCH.md "Correctness boundaries").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define WAVE 64
#define DEV __device__ __forceinline__

#define HIP_CHECK_LAUNCH() do { (void)hipGetLastError(); } while (0)

DEV float bf2f(bf16 x) { return (float)x; }
DEV bf16 f2bf(float x) { return (bf16)x; }

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 2^x as the bare v_exp_f32: exp2f adds a denormal-range fixup (compare,
// select, ldexp: ~4 extra VALU ops per call, a third of the softmax VALU of
// the attention loops); results below 2^-126 flush to 0, which a softmax
// weight can take
DEV float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

DEV f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// async global -> LDS copy, 16 B per lane; the LDS destination of one
// wave-instruction is (wave-uniform base) + lane*16 (cdna_hip_programming.md §5 Caveat).
DEV void glds16(const void* gptr, void* lds_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gptr,
      (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// XCD-aware bijective remap of a linear workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks b and b+8 share an XCD, so give each
// XCD a contiguous range of logical tiles.
DEV int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// counter-based RNG (splitmix64 finaliser) for Gumbel-max sampling
DEV uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
DEV float uniform01(uint64_t seed, uint64_t a, uint64_t b) {
  uint64_t h = mix64(seed ^ mix64(a * 0x100000001B3ull + b));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
}

// RMSNorm fused into GEMM epilogues (kernels.h NormEpi, passed to kernels by
// value).  The per-row sums of squares are 64-bit fixed point (2^-20 units):
// integer atomic adds are order-independent, so the fused norm is bitwise
// deterministic whatever order the producing tiles finish in (fp32 atomics
// would not be).  Headroom: one add carries one wave's 128-column partial,
// clamped at 2^56 units (|x| ~ 2.3e4 on every element of the partial), and a
// row takes at most 64 adds (H = 8192), so the sum stays below 2^62 and reads
// back correctly as torch's signed int64; a row of |x| ~ 3e3 at H = 8192 is
// 2^36 units.  Precision: 2^-21 per add, ~1e-6 of a row of |x| ~ 1e-2.
constexpr float SS_FIX = 1048576.f;                   // 2^20
constexpr float SS_ADD_MAX = 72057594037927936.f;     // 2^56: one add of a partial
constexpr float SS_ROW_MAX = 4611686018427387904.f;   // 2^62: a whole row stored at once
DEV unsigned long long ss_fixed(float v, float cap = SS_ADD_MAX) {
  return (unsigned long long)__float2ull_rn(fminf(v * SS_FIX, cap));
}
DEV void ss_atomic_add(unsigned long long* p, float v) {
  __hip_atomic_fetch_add(p, ss_fixed(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// row scale of a consumer epilogue (1 when no norm is fused)
template <class NE>
DEV float norm_row_scale(const NE& ne, int m) {
  if (!ne.ss_in) return 1.f;
  const float ss = (float)ne.ss_in[m] * (1.f / SS_FIX);
  return rsqrtf(ss * ne.inv_h + ne.eps);
}
// the row scales of N rows at once: the wave-uniform "no norm" test is hoisted
// out and every load issued before the first use (norm_row_scale in an
// unrolled loop makes hipcc branch around each load and wait vmcnt(0) per
// row - N dependent round trips, and a drain of every DMA still in flight:
// cdna_hip_programming.md §5 item 4(c), T20)
template <int N, class NE>
DEV void norm_row_scales(const NE& ne, const int (&m)[N], float (&out)[N]) {
  if (!ne.ss_in) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = 1.f;
    return;
  }
  unsigned long long v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = ne.ss_in[m[i]];
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = rsqrtf((float)v[i] * (1.f / SS_FIX) * ne.inv_h + ne.eps);
}
// sum of squares of the bf16-rounded values a residual epilogue stores
DEV float sumsq_bf16x4(const bf16x4& v) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += (float)v[j] * (float)v[j];
  return s;
}
DEV float sumsq_bf16x8(const bf16x8& v) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += (float)v[j] * (float)v[j];
  return s;
}

// Plain / residual epilogue of an MFMA 16x16x32 accumulator grid in the direct
// layout: lane (fr = lane & 15, fq = lane >> 4) holds rows mb + 16 mt + fr,
// columns nb + 16 nt + 4 fq .. +3.  EPI 1 adds R, whose rows are all loaded up
// front (clamped, no branch) so their latency overlaps instead of serialising
// behind the per-row guards (cdna_hip_programming.md §5 "Projection GEMM at
// M = 256" item 4(c)); with ne.ss_out it also adds each stored row's sum of
// squares (the fused RMSNorm statistic: the 4 fq lanes of a row, then one
// atomic per row and wave).  N % 4 == 0.
template <int EPI, int MT, int NT, class NE>
DEV void store_direct(const f32x4 (&acc)[MT][NT], bf16* __restrict__ Y,
                      const bf16* __restrict__ R, int M, int N, int mb, int nb, int fr, int fq,
                      const NE& ne) {
  bf16x4 rres[EPI == 1 ? MT : 1][EPI == 1 ? NT : 1];
  if constexpr (EPI == 1) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int m = min(mb + mt * 16 + fr, M - 1);
        const int n = min(nb + nt * 16 + fq * 4, N - 4);
        rres[mt][nt] = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n);
      }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mb + mt * 16 + fr;
    float ss = 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nb + nt * 16 + fq * 4;
      f32x4 v = acc[mt][nt];
      if constexpr (EPI == 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += (float)rres[mt][nt][j];
      }
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
      if (m < M && n < N) {
        *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
        if (EPI == 1) ss += sumsq_bf16x4(o);
      }
    }
    if (EPI == 1 && ne.ss_out) {
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (fq == 0 && m < M) ss_atomic_add(ne.ss_out + m, ss);
    }
  }
}

// SwiGLU epilogue of a wave's MT x NT 16x16x32 accumulator tiles (W rows
// interleaved [gate 16 | up 16] per 32-row group, so column tiles 2p / 2p + 1
// hold gate / up of the same 4 features in the same lane); Y is [M, N / 2],
// the fused RMSNorm row scale of the input applied first.  The rows' scale
// loads are issued together before any store (norm_row_scales), not behind
// a per-row guard (cdna_hip_programming.md §5 item 4(c)).
template <int MT, int NT, class NE>
DEV void store_silu(const f32x4 (&acc)[MT][NT], bf16* __restrict__ Y, int M, int N, int mb,
                    int nb, int fr, int fq, const NE& ne) {
  static_assert(NT % 2 == 0, "gate / up tile pairs");
  const int F = N >> 1;
  int rows[MT];
  float rs[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) rows[mt] = min(mb + mt * 16 + fr, M - 1);
  norm_row_scales(ne, rows, rs);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mb + mt * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int p = 0; p < NT / 2; ++p) {
      const int f = (nb >> 1) + p * 16 + fq * 4;
      if (f >= F) continue;
      const f32x4 gv = acc[mt][2 * p] * rs[mt], uv = acc[mt][2 * p + 1] * rs[mt];
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)(gv[j] / (1.f + __expf(-gv[j])) * uv[j]);
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * F + f) = o;
    }
  }
}

// Wide direct epilogue of a wave's 16x16x32 accumulator grid, 8 column tiles
// (128 columns) per wave: lane (fr = lane & 15, fq = lane >> 4) holds rows
// mb + 16 mt + fr, columns 16 nt + 4 fq .. +3.  Column-tile pairs (2p, 2p+1)
// are exchanged across lane rows by v_permlane16_swap (odd 16-lane rows of the
// first operand <-> even rows of the second), after which lane fq holds the 8
// consecutive columns 32 p + 16 (fq & 1) + 8 (fq >> 1) .. +7: one 16-B store
// per lane, 64 contiguous bytes per row per instruction, no LDS staging and no
// barrier (cdna_hip_programming.md T21, here for the 16x16 layout).
DEV void swap_col_pairs(u32x2& a, u32x2& b) {
  const auto r0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  a.x = r0[0];
  b.x = r0[1];
  a.y = r1[0];
  b.y = r1[1];
}

// EPI 0 plain, 1 residual (bf16 product + R, as the staged epilogue rounds it;
// with ne.ss_out each stored row's sum of squares), 2 SwiGLU of interleaved
// gate | up 16-column groups (64 output columns per wave; rsc = the fused
// RMSNorm row scales of the wave's MT row tiles).  Y / R rows have ``ldy``
// elements; the wave's first output column is ``col0``.  Stores go through a
// range-checked buffer descriptor (rows >= M dropped, no branch); R rows are
// clamped and all loaded up front.
template <int EPI, int MT, class RS, class NE>
DEV void store_wide(const f32x4 (&acc)[MT][8], RS rsY, const bf16* __restrict__ R, int M, int ldy,
                    int mb, int col0, int fr, int fq, const float* rsc, const NE& ne) {
  constexpr int NPAIR = EPI == 2 ? 2 : 4;
  const int lcol = 16 * (fq & 1) + 8 * (fq >> 1);
  bf16x8 rres[EPI == 1 ? MT * NPAIR : 1];
  if constexpr (EPI == 1) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        const int m = min(mb + mt * 16 + fr, M - 1);
        rres[mt * NPAIR + p] = *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldy + col0 + 32 * p + lcol);
      }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mb + mt * 16 + fr;
    float ss = 0.f;
#pragma unroll
    for (int p = 0; p < NPAIR; ++p) {
      bf16x4 oa, ob;
      if constexpr (EPI == 2) {
        const float s = rsc[mt];
        const f32x4 ga = acc[mt][4 * p] * s, ua = acc[mt][4 * p + 1] * s;
        const f32x4 gb = acc[mt][4 * p + 2] * s, ub = acc[mt][4 * p + 3] * s;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          oa[e] = (bf16)(ga[e] / (1.f + __expf(-ga[e])) * ua[e]);
          ob[e] = (bf16)(gb[e] / (1.f + __expf(-gb[e])) * ub[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          oa[e] = (bf16)acc[mt][2 * p][e];
          ob[e] = (bf16)acc[mt][2 * p + 1][e];
        }
      }
      u32x2 a = __builtin_bit_cast(u32x2, oa), b = __builtin_bit_cast(u32x2, ob);
      swap_col_pairs(a, b);
      bf16x8 v = __builtin_bit_cast(bf16x8, u32x4{a.x, a.y, b.x, b.y});
      if constexpr (EPI == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)rres[mt * NPAIR + p][e]);
        if (ne.ss_out) ss += m < M ? sumsq_bf16x8(v) : 0.f;
      }
      const unsigned off = (unsigned)(((size_t)m * ldy + col0 + 32 * p + lcol) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsY,
                                             m < M ? off : 0x80000000u, 0, 0);
    }
    if (EPI == 1 && ne.ss_out) {
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (fq == 0 && m < M) ss_atomic_add(ne.ss_out + m, ss);
    }
  }
}

// store_wide plus ``sl`` (gemm256d.hip SPLIT 2): the other K half's fp32 partials, added to
// the accumulators here, one row tile at a time, two row tiles of loads in
// flight (a separate add pass over all MT x 8 accumulators makes hipcc copy
// them out of the AGPRs at once and spill): f32x4 r = (mt, nt) of this lane
// sits at byte r * 4096 + lane_off of the slab, read with sc1 loads.
template <class RS>
struct SlabIn {
  static constexpr bool on = true;
  RS rs;
  unsigned lane_off;
};
template <int EPI, int MT, class RS, class NE, class SL>
DEV void store_wide_slab(const f32x4 (&acc)[MT][8], RS rsY, const bf16* __restrict__ R, int M, int ldy,
                         int mb, int col0, int fr, int fq, const float* rsc, const NE& ne,
                         const SL& sl) {
  constexpr int NPAIR = EPI == 2 ? 2 : 4;
  f32x4 pre[2][SL::on ? 8 : 1];
  auto slab_load = [&](int mt, int b) {
    if constexpr (SL::on) {
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
        pre[b][nt] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(sl.rs, sl.lane_off, (mt * 8 + nt) * 4096, 16));
    }
  };
  if constexpr (SL::on) {
    slab_load(0, 0);
    if (MT > 1) slab_load(1, 1);
  }
  const int lcol = 16 * (fq & 1) + 8 * (fq >> 1);
  bf16x8 rres[EPI == 1 ? MT * NPAIR : 1];
  if constexpr (EPI == 1) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        const int m = min(mb + mt * 16 + fr, M - 1);
        rres[mt * NPAIR + p] = *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldy + col0 + 32 * p + lcol);
      }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mb + mt * 16 + fr;
    float ss = 0.f;
    f32x4 sum[SL::on ? 8 : 1];
    if constexpr (SL::on) {
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) sum[nt] = acc[mt][nt] + pre[mt & 1][nt];
      if (mt + 2 < MT) slab_load(mt + 2, mt & 1);
    }
    auto av = [&](int nt) -> f32x4 {
      if constexpr (SL::on) return sum[nt];
      else return acc[mt][nt];
    };
#pragma unroll
    for (int p = 0; p < NPAIR; ++p) {
      bf16x4 oa, ob;
      if constexpr (EPI == 2) {
        const float s = rsc[mt];
        const f32x4 ga = av(4 * p) * s, ua = av(4 * p + 1) * s;
        const f32x4 gb = av(4 * p + 2) * s, ub = av(4 * p + 3) * s;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          oa[e] = (bf16)(ga[e] / (1.f + __expf(-ga[e])) * ua[e]);
          ob[e] = (bf16)(gb[e] / (1.f + __expf(-gb[e])) * ub[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          oa[e] = (bf16)av(2 * p)[e];
          ob[e] = (bf16)av(2 * p + 1)[e];
        }
      }
      u32x2 a = __builtin_bit_cast(u32x2, oa), b = __builtin_bit_cast(u32x2, ob);
      swap_col_pairs(a, b);
      bf16x8 v = __builtin_bit_cast(bf16x8, u32x4{a.x, a.y, b.x, b.y});
      if constexpr (EPI == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)rres[mt * NPAIR + p][e]);
        if (ne.ss_out) ss += m < M ? sumsq_bf16x8(v) : 0.f;
      }
      const unsigned off = (unsigned)(((size_t)m * ldy + col0 + 32 * p + lcol) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsY,
                                             m < M ? off : 0x80000000u, 0, 0);
    }
    if (EPI == 1 && ne.ss_out) {
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (fq == 0 && m < M) ss_atomic_add(ne.ss_out + m, ss);
    }
  }
}
