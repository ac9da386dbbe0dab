// K1 stream-K form of the one-wave-per-SIMD AGPR GEMM (gemm256d.hip) for wave
// quantisation.  At a decode step of the headline bench (M ~ 2600 tokens) the
// N = 4096 projections have 11 x 16 = 176 256x256 tiles for 256 CUs: one
// workgroup per tile leaves 31 % of the chip idle for the whole GEMM (the
// down projection: 112 k-units of 128 per tile).  Here a persistent grid of
// one workgroup per CU splits the T x U (tile, 128-deep k-unit) iterations
// evenly; workgroup w runs its range [w*T*U/G, (w+1)*T*U/G) as segments.
//   * every segment stores its fp32 accumulators (register order, 256
//     KiB) to its slab - slot 0 for the first segment of the range, 1 for the
//     last - with sc1 (write-through) stores, publishes them (drain, then a
//     relaxed agent-scope ticket on the tile's counter,
//     cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2, the sc1
//     form) and, if its ticket is the tile's last, sums the tile's slabs (sc1
//     loads) in segment order and runs the epilogue (re-arming the counter).
// No workgroup ever waits for another, so residency does not matter.
// The mainloop is gemm256d.hip's (see there for the pipeline, the LDS image
// and the inline-asm rules); it is repeated here rather than shared so the
// two kernels' register allocations cannot perturb each other.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int ROWB = BK * 2;
constexpr int PIECE_B = 256 * ROWB;
constexpr int SLOT_B = 2 * PIECE_B;
constexpr int SLAB_F4 = 64 * 256;                   // float4 per partial slab (256 KiB)

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

DEV void mfma_a(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

struct Frags {
  bf16x8 a[8];
  bf16x8 b[8];
};

DEV void tile_coords(int t, int nm, int nn, int& m0, int& n0) {
  constexpr int GROUP = 4;
  const int per_group = GROUP * nn;
  const int g = t / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  m0 = (first_m + (t % per_group) % gsz) * BM;
  n0 = ((t % per_group) / gsz) * BN;
}

// The epilogue inputs of one accumulator row mt, loaded before the slab sums
// that precede its stores (clamped rows, no branch: loads issued behind a
// per-row guard serialise, cdna_hip_programming.md §5 item 4(c)): the fused
// RMSNorm scale (EPI 2) or the residual row piece (EPI 1)
struct RowIn {
  float rs;
  bf16x4 rr[8];
};
template <int EPI>
DEV void load_row_in(RowIn& in, const bf16* __restrict__ R, int M, int N, int m0, int n0, int wm,
                     int wn, int fr, int fq, int mt, const NormEpi& ne) {
  const int m = min(m0 + wm * 128 + mt * 16 + fr, M - 1);
  if constexpr (EPI == 2) {
    int rows[1] = {m};
    float rs[1];
    norm_row_scales(ne, rows, rs);
    in.rs = rs[0];
  }
  if constexpr (EPI == 1) {                          // N % 256 == 0
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
      in.rr[nt] = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + n0 + wn * 128 + nt * 16 + fq * 4);
  }
}

// the epilogue for one accumulator row mt from per-element values v(nt)
template <int EPI, class V>
DEV void store_row(bf16* __restrict__ Y, int M, int N, int m0, int n0, int wm, int wn, int fr,
                   int fq, int mt, const NormEpi& ne, const RowIn& in, V&& v) {
  const int m = m0 + wm * 128 + mt * 16 + fr;
  if (m >= M) return;                                // the 4 fq lanes of the row together
  if constexpr (EPI == 2) {
    const int F2 = N >> 1;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int f = ((n0 + wn * 128) >> 1) + p * 16 + fq * 4;
      if (f >= F2) continue;
      const f32x4 gv = v(2 * p) * in.rs, uv = v(2 * p + 1) * in.rs;
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)(gv[j] / (1.f + __expf(-gv[j])) * uv[j]);
      *reinterpret_cast<bf16x4*>(Y + (size_t)m * F2 + f) = o;
    }
    return;
  }
  float ss = 0.f;
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    const int n = n0 + wn * 128 + nt * 16 + fq * 4;
    f32x4 x = v(nt);
    if (EPI == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] += (float)in.rr[nt][j];
    }
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)x[j];
    *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
    if (EPI == 1) ss += sumsq_bf16x4(o);
  }
  if (EPI == 1 && ne.ss_out) {                       // fused RMSNorm statistic of the row
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (fq == 0) ss_atomic_add(ne.ss_out + m, ss);
  }
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_tn_256sk(const bf16* __restrict__ X,
                                                        const bf16* __restrict__ W,
                                                        bf16* __restrict__ Y,
                                                        const bf16* __restrict__ R, int M, int N,
                                                        int K, f32x4* __restrict__ ws,
                                                        int* __restrict__ cnt, int tile0,
                                                        const NormEpi ne) {
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT_B];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  // tiles [tile0, nm nn) in the data-parallel kernel's grouped order: the
  // hybrid launch gives the full waves to gemm256d.hip and only the tail here
  const int T = nm * nn - tile0, U = K / (2 * BK);
  const int G = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, G);           // range neighbours share an XCD
  const long long I = (long long)T * U;
  auto range_start = [&](int w) { return (int)((long long)w * I / G); };
  auto owner_of = [&](int i) {                       // the workgroup whose range holds iteration i
    int w = (int)((long long)i * G / I);
    while (w + 1 < G && range_start(w + 1) <= i) ++w;
    while (w > 0 && range_start(w) > i) --w;
    return w;
  };

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)M * K * 2),
                                                     0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((size_t)N * K * 2),
                                                     0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)ws, (short)0, 0x7FFFFFFF, 0x00020000);
  const int chunk = (lane & 7) ^ (lane >> 3);
  const unsigned offB = (unsigned)(((lane >> 3) * K + chunk * 8) * 2);
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  int rbase[2][2][2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int ch = ((4 * kh + fq) ^ (fr & 7)) * 16;
      rbase[sl][kh][0] = sl * SLOT_B + (wm * 128 + fr) * ROWB + ch;
      rbase[sl][kh][1] = sl * SLOT_B + PIECE_B + (wn * 128 + fr) * ROWB + ch;
    }
  auto fread1 = [&](int slot, int kh, Frags& f, int i) {
    if (i < 8)
      f.b[i] = *reinterpret_cast<const bf16x8*>(smem + rbase[slot][kh][1] + i * 2048);
    else
      f.a[i - 8] = *reinterpret_cast<const bf16x8*>(smem + rbase[slot][kh][0] + (i - 8) * 2048);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  auto keep = [](const Frags& f) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" :: "v"(f.a[i]), "v"(f.b[i]));
  };

  const int it_begin = range_start(wg), it_end = range_start(wg + 1);
  int it = it_begin;
  while (it < it_end) {
    const int tile = it / U, u0 = it % U, u1 = min(U, u0 + (it_end - it));
    int m0, n0;
    tile_coords(tile0 + tile, nm, nn, m0, n0);
    unsigned offA[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      offA[q] = (unsigned)(((size_t)min(m0 + 64 * wave + 8 * q + (lane >> 3), M - 1) * K + chunk * 8) * 2);
    const int rowB0 = n0 + 64 * wave;
    const int kt0 = 2 * u0, nkt = 2 * (u1 - u0);
    auto dma1 = [&](int t, int slot, int i) {        // k clamped: soffset is not range-checked
      const bool b = i >= 8;
      const int q = i & 7;
      const int kb = (kt0 + min(t, nkt - 1)) * BK * 2;
      auto* dst = (__attribute__((address_space(3))) void*)(
          smem + slot * SLOT_B + (b ? PIECE_B : 0) + (8 * wave + q) * 1024);
      if (b)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, dst, 16, offB, (rowB0 + 8 * q) * K * 2 + kb, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, offA[q], kb, 0, 0);
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));

    Frags F[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) dma1(0, 0, i);
#pragma unroll
    for (int i = 0; i < 16; ++i) dma1(1, 1, i);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    raw_barrier();
#pragma unroll
    for (int i = 0; i < 16; ++i) fread1(0, 0, F[0], i);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_nop 4" ::: "memory");
    auto ktile = [&](int t, auto c_c) {
      constexpr int C = decltype(c_c)::value;
      fence();
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int i0 = 2 * j, i1 = 2 * j + 1;
        mfma_a(acc[i0 >> 3][i0 & 7], F[0].b[i0 & 7], F[0].a[i0 >> 3]);
        mfma_a(acc[i1 >> 3][i1 & 7], F[0].b[i1 & 7], F[0].a[i1 >> 3]);
        if ((j & 1) == 0) fread1(C, 1, F[1], j >> 1);
        fence();
      }
      keep(F[0]);
      __builtin_amdgcn_s_waitcnt(0x0070);            // vmcnt(0) lgkmcnt(0)
      raw_barrier();
      fence();
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int i0 = 2 * j, i1 = 2 * j + 1;
        mfma_a(acc[i0 >> 3][i0 & 7], F[1].b[i0 & 7], F[1].a[i0 >> 3]);
        mfma_a(acc[i1 >> 3][i1 & 7], F[1].b[i1 & 7], F[1].a[i1 >> 3]);
        if ((j & 1) == 0) fread1(C ^ 1, 0, F[0], j >> 1);
        else dma1(t + 2, C, j >> 1);
        fence();
      }
      keep(F[1]);
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    for (int t = 0; t < nkt; t += 2) {
      ktile(t, C0{});
      ktile(t + 1, C1{});
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    {
      // ---- every segment goes through its slab, also a whole tile (rare in
      //      the stream-K regime; a second, direct epilogue of the AGPR
      //      accumulators makes hipcc spill them): slot 0 = the first
      //      segment of the range, 1 = the last
      const int slab = wg * 2 + (it == it_begin ? 0 : 1);
#pragma unroll
      for (int r = 0; r < 64; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[r >> 3][r & 7]), rsW,
                                               tid * 16, (slab * SLAB_F4 + r * 256) * 16, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* last = reinterpret_cast<int*>(smem);       // LDS is free here (all DMAs drained)
      if (tid == 0) {
        const int w_first = owner_of(tile * U), w_last = owner_of(tile * U + U - 1);
        // slabs are stored and loaded sc1 (write-through / past the XCD L2),
        // so no release / acquire fence - an agent-scope fence writes back or
        // invalidates the whole XCD L2 (cdna_hip_programming.md §5, item 2)
        const int prev = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int is_last = prev == w_last - w_first;
        if (is_last) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last = is_last;
      }
      __syncthreads();
      const int is_last = *last;
      __syncthreads();                               // the flag word is LDS the next segment refills
      if (is_last) {
        // ---- sum the tile's slabs in segment order (w_first's last segment,
        //      then every later workgroup's first), two accumulator rows per batch
        const int w_first = owner_of(tile * U), w_last = owner_of(tile * U + U - 1);
        for (int rb = 0; rb < 4; ++rb) {
          RowIn in[2];
#pragma unroll
          for (int h = 0; h < 2; ++h)
            load_row_in<EPI>(in[h], R, M, N, m0, n0, wm, wn, fr, fq, 2 * rb + h, ne);
          f32x4 P[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) P[i] = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int w = w_first; w <= w_last; ++w) {
            const int sl = w * 2 + (range_start(w) < tile * U ? 1 : 0);
            f32x4 q[16];
#pragma unroll
            for (int i = 0; i < 16; ++i)
              q[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                  rsW, tid * 16, (sl * SLAB_F4 + (rb * 16 + i) * 256) * 16, 16));
#pragma unroll
            for (int i = 0; i < 16; ++i) P[i] += q[i];
          }
#pragma unroll
          for (int h = 0; h < 2; ++h)
            store_row<EPI>(Y, M, N, m0, n0, wm, wn, fr, fq, 2 * rb + h, ne, in[h],
                           [&](int nt) { return P[h * 8 + nt]; });
        }
      }
    }
    it += u1 - u0;
    if (it < it_end) __syncthreads();                // the next segment's prologue refills the LDS
  }
}

struct SkState {
  int G = 0;
  f32x4* ws = nullptr;
  int* cnt = nullptr;
  int cnt_n = 0;
};

// per-device persistent grid size, slabs (two per workgroup) and tile
// counters; allocated on first use (stream-K runs only for large eager steps,
// never inside a graph capture)
SkState* sk_state(int tiles) {
  static SkState devs[64];
  int d = 0;
  (void)hipGetDevice(&d);
  SkState& st = devs[d & 63];
  if (st.G == 0) {
    hipDeviceProp_t prop;
    const int G = hipGetDeviceProperties(&prop, d) == hipSuccess && prop.multiProcessorCount > 0
                      ? prop.multiProcessorCount : 256;
    if (hipMalloc(&st.ws, (size_t)G * 2 * SLAB_F4 * sizeof(f32x4)) != hipSuccess) return nullptr;
    st.G = G;
  }
  if (tiles > st.cnt_n) {
    if (st.cnt) (void)hipFree(st.cnt);
    const int n = tiles < 4096 ? 4096 : tiles;
    if (hipMalloc(&st.cnt, sizeof(int) * n) != hipSuccess) {
      st.cnt = nullptr;
      st.cnt_n = 0;
      return nullptr;
    }
    (void)hipMemset(st.cnt, 0, sizeof(int) * n);
    (void)hipDeviceSynchronize();
    st.cnt_n = n;
  }
  return &st;
}

int streamk_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("MCP_GEMM_STREAMK");
    // default OFF: measured slower than the data-parallel kernel on every
    // Llama shape (profiles/gemm_tuning.md: workgroups at different k offsets
    // stop sharing A / W panels in L2, the per-unit mainloop turns HBM-bound)
    mode = e ? atoi(e) : 0;                          // 0 off, 1 always, 2 auto
  }
  return mode;
}

// stream-K pays when the data-parallel grid's last wave is mostly empty:
// data-parallel ~ ceil(T / G) tile times, stream-K ~ T / G plus the slab
// hand-offs (about one 128-deep k-unit of store + the last arriver's sums)
double sk_cost(int T, int U, int G) { return (double)T / G + 3.0 / U; }

}  // namespace

int gemm256d_ok(int M, int N, int K);

// tile-time cost of the 256 path for this shape (gemm.hip's selection)
double gemm256sk_waves(int M, int N, int K) {
  const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN), U = K / (2 * BK);
  const int G = 256;
  const double dp = ceil((double)T / G);
  if (streamk_mode() == 0 || gemm256d_ok(M, N, K) != 0) return dp;
  return streamk_mode() == 1 ? sk_cost(T, U, G) : fmin(dp, sk_cost(T, U, G));
}

// returns 0 when it launched; nonzero = caller falls back (data-parallel)
int launch_gemm_tn_256sk(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                         int epi, int force, hipStream_t s) {
  if (gemm256d_ok(M, N, K) != 0) return 1;
  const int mode = force ? 1 : streamk_mode();
  if (mode == 0) return 2;
  const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN), U = K / (2 * BK);
  SkState* st = sk_state(T);
  if (!st) return 3;
  if (mode == 2 && !(sk_cost(T, U, st->G) < 0.92 * ceil((double)T / st->G))) return 4;
  // never more workgroups than (tile, k-unit) iterations: an empty range
  // would still be counted between a tile's first and last owner
  const dim3 grid((unsigned)std::min<long long>(st->G, (long long)T * U));
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  switch (epi) {
    case 0: gemm_tn_256sk<0><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, st->ws, st->cnt, 0, norm_epi()); return 0;
    case 1: gemm_tn_256sk<1><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, st->ws, st->cnt, 0, norm_epi()); return 0;
    case 2: gemm_tn_256sk<2><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, st->ws, st->cnt, 0, norm_epi()); return 0;
    default: return 5;
  }
}

// Hybrid tail: tiles [tile0, T) of the data-parallel order, stream-K over one
// persistent wave (gemm256d.hip launches the full waves [0, tile0) first).
// The tail wave of a data-parallel grid that is at most half full costs a
// whole tile time; spread over every CU it costs tail / G of one plus the
// slab hand-offs, while the full waves keep their L2 panel sharing.
int launch_gemm_tn_256sk_tail(const void* X, const void* W, void* Y, const void* R, int M, int N,
                              int K, int epi, int tile0, hipStream_t s) {
  if (gemm256d_ok(M, N, K) != 0) return 1;
  const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN) - tile0, U = K / (2 * BK);
  if (T <= 0 || tile0 < 0) return 2;
  SkState* st = sk_state(T);
  if (!st) return 3;
  // at most MCP_GEMM_TAIL_SPLIT (4) workgroups per tail tile: the last arriver
  // sums every slab of its tile, so wider splits lose to the fix-up
  static const int smax = getenv("MCP_GEMM_TAIL_SPLIT") ? atoi(getenv("MCP_GEMM_TAIL_SPLIT")) : 4;
  const dim3 grid((unsigned)std::min<long long>(std::min<long long>(st->G, (long long)T * smax),
                                                (long long)T * U));
  auto x = (const bf16*)X;
  auto w = (const bf16*)W;
  auto y = (bf16*)Y;
  auto r = (const bf16*)R;
  switch (epi) {
    case 0: gemm_tn_256sk<0><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, st->ws, st->cnt, tile0, norm_epi()); return 0;
    case 1: gemm_tn_256sk<1><<<grid, 256, 0, s>>>(x, w, y, r, M, N, K, st->ws, st->cnt, tile0, norm_epi()); return 0;
    case 2: gemm_tn_256sk<2><<<grid, 256, 0, s>>>(x, w, y, nullptr, M, N, K, st->ws, st->cnt, tile0, norm_epi()); return 0;
    default: return 5;
  }
}

// workspace / counters allocated before any graph capture (library load)
int gemm256sk_prealloc() { return sk_state(4096) ? 0 : 1; }
