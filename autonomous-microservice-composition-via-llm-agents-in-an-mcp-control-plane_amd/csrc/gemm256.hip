// K1 (large-M path): 256x256-tile bf16 TN GEMM with a 4-phase-per-K-tile
// pipeline whose LDS-DMA prefetch stays in flight across barriers.
//   Y[M,N] = X[M,K] . W[N,K]^T (+ R)        fp32 accumulate, bf16 out
//
// Why (cdna_hip_programming.md §5 "The step-3 structure's ~900 TF ceiling"):
// a 128^2 tile with one vmcnt(0)+__syncthreads per K-step stalls on every
// prefetch.  Here one workgroup (8 waves, 2(M) x 4(N), 128x64 outputs per wave)
// owns a 256x256 tile; each 64-deep K-tile is split into four 16 KiB pieces
// {A.k0, B.k0, A.k1, B.k1} (k0/k1 = the two 32-deep halves) held in an 8-slot
// LDS ring (two K-tiles, 128 KiB, one __shared__ array).  Phase p of K-tile t:
//
//   ds_read fragments (A: 4 x b128, B: 4 x b128 on even phases)
//   issue piece p of K-tile t+1 (2 x global_load_lds_dwordx4 per thread)
//   16 x v_mfma_f32_16x16x32_bf16 (m-half p&1, k-half p>>1), s_setprio 1
//   [p = 1, 3: s_waitcnt vmcnt(4) -> the pieces the next phase reads landed]
//   s_barrier
//
// so every load has >= 2 phases of MFMA work to land, and vmcnt never drains
// to 0 inside the main loop (T3+T4).  The waits are hand-counted: each thread
// issues exactly 2 LDS-DMA ops per phase and no other VMEM op in the loop.
// WAR safety: piece p of tile t+1 overwrites the slot of piece p of tile t-1,
// whose last read precedes the barrier that ends tile t-1.
// LDS rows are 64 B (32 bf16); swizzle chunk ^= ((row>>2)&1)<<1 on the glds
// SOURCE and the ds_read address (conflict-free, tools/lds_banks.py).
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64, KH = 32;
constexpr int PIECE = 256 * KH;                 // bf16 elements per piece (16 KiB)

DEV int swz(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }

DEV void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Structural variants (A/B-tested in one process, tools/bench_gemm.py):
//   BAR4  : barrier after every phase (else only where a new piece is consumed
//           next, i.e. after phases 1 and 3 -- WAR/RAW need nothing more)
//   PREA  : even phases also read the odd phase's A fragments, so odd phases
//           issue no LDS reads and their MFMAs start immediately
//   PRIO  : s_setprio 1 around the MFMA cluster
//   GFIRST: issue the next K-tile's LDS-DMA piece before this phase's ds_reads
//   PP    : ping-pong (cdna_hip_programming.md §5 8-phase template): two
//           barriers per phase {reads + LDS-DMA issue | barrier | MFMA |
//           barrier} and the two M-half wave groups offset by one barrier, so
//           on every SIMD one wave runs its MFMA cluster while the other
//           issues its LDS reads and loads.
template <bool BAR4, bool PREA, bool PRIO, bool GFIRST, bool PP = false>
struct V256 {
  static constexpr bool bar4 = BAR4, prea = PREA, prio = PRIO, gfirst = GFIRST, pp = PP;
};

DEV void sched_barrier_full() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// production default: ping-pong without s_setprio (variant 25), +5-12 % over the
// best non-staggered variant 8 on the Llama-3-8B projection shapes
// (profiles/gemm_tuning.md, profiles/gemm_variants_m4096.jsonl)
using V256Default = V256<false, false, false, true, true>;

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

// K-tiles [kt0, kt1) of the 256x256 tile at (m0, n0) accumulated into acc.
// Starts with a barrier (the LDS ring may still be read by a previous tile).
template <class VAR>
DEV void mainloop(const bf16* __restrict__ X, const bf16* __restrict__ W, int M, int N, int K,
                  int m0, int n0, int kt0, int kt1, bf16* smem, f32x4 (&acc)[2][4][4]) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // ---- staging: wave w writes 1 KiB instructions 2w, 2w+1 of every piece
  //      (rows (2w+j)*16 + lane/4, 16-B chunk lane%4 of the 64-B row)
  const bf16* srcA[2];
  const bf16* srcB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (2 * wave + j) * 16 + (lane >> 2);
    const int ch = swz(row, lane & 3);
    srcA[j] = X + (size_t)min(m0 + row, M - 1) * K + ch * 8;
    srcB[j] = W + (size_t)min(n0 + row, N - 1) * K + ch * 8;
  }
  // t counts K-tiles from kt0 (slot parity t & 1 is then static after the
  // compiler's unrolling, which keeps its LDS-DMA alias tracking from adding a
  // vmcnt(0) before every ds_read)
  const bf16* const kbaseA[2] = {srcA[0] + (size_t)kt0 * BK, srcA[1] + (size_t)kt0 * BK};
  const bf16* const kbaseB[2] = {srcB[0] + (size_t)kt0 * BK, srcB[1] + (size_t)kt0 * BK};
  auto stage = [&](int t, int i) {          // piece i of K-tile kt0 + t
    const int koff = t * BK + (i >> 1) * KH;
    bf16* slot = smem + ((t & 1) * 4 + i) * PIECE;
    const bf16* const* src = (i & 1) ? kbaseB : kbaseA;
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(src[j] + koff, slot + (2 * wave + j) * 512);
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[a][b][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment offsets inside a piece (elements)
  int offA[2][4], offB[4];
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int row = wm * 128 + mh * 64 + mt * 16 + fr;
      offA[mh][mt] = row * KH + swz(row, fq) * 8;
    }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int row = wn * 64 + nt * 16 + fr;
    offB[nt] = row * KH + swz(row, fq) * 8;
  }

  barrier();
  // prologue: K-tile kt0 fully resident
#pragma unroll
  for (int i = 0; i < 4; ++i) stage(0, i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();

  bf16x8 bfr[4];
  bf16x8 afr[2][4];
  auto phase = [&](int t, int p, bool prefetch, bool last) {
    const int kh = p >> 1, mh = p & 1;
    const bf16* sA = smem + ((t & 1) * 4 + 2 * kh) * PIECE;
    const bf16* sB = sA + PIECE;
    if (VAR::gfirst && prefetch) stage(t + 1, p);
    if (mh == 0) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bfr[nt] = *reinterpret_cast<const bf16x8*>(sB + offB[nt]);
    }
    if (!VAR::prea || mh == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        afr[mh][mt] = *reinterpret_cast<const bf16x8*>(sA + offA[mh][mt]);
    }
    if (VAR::prea && mh == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) afr[1][mt] = *reinterpret_cast<const bf16x8*>(sA + offA[1][mt]);
    }
    if (!VAR::gfirst && prefetch) stage(t + 1, p);
    if constexpr (VAR::pp) {
      // RAW: pieces read first in phase 0 / 2 of a K-tile retire here in
      // phases 3 / 1, before the barrier both wave groups pass before reading
      if (p == 1) {
        if (last) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else if (p == 3 && !last) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      sched_barrier_full();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (VAR::prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mh][mt][nt] = mfma16x16x32(bfr[nt], afr[mh][mt], acc[mh][mt][nt]);
      if (VAR::prio) __builtin_amdgcn_s_setprio(0);
      sched_barrier_full();
      return;
    }
    if (VAR::prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mh][mt][nt] = mfma16x16x32(bfr[nt], afr[mh][mt], acc[mh][mt][nt]);
    if (VAR::prio) __builtin_amdgcn_s_setprio(0);
    if (p == 1) {
      if (last) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else if (p == 3 && !last) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    if (VAR::bar4 || p == 1 || p == 3) barrier();
  };

  if (VAR::pp && wm == 1) sched_barrier_full();    // stagger the two wave groups
  const int nt = kt1 - kt0;
  for (int t = 0; t + 1 < nt; ++t) {
    phase(t, 0, true, false);
    phase(t, 1, true, false);
    phase(t, 2, true, false);
    phase(t, 3, true, false);
  }
  {
    const int t = nt - 1;
    phase(t, 0, false, true);
    phase(t, 1, false, true);
    phase(t, 2, false, true);
    phase(t, 3, false, true);
  }
  if (VAR::pp && wm == 0) sched_barrier_full();
}

// lane holds Y[m][n .. n+3] of each 16x16 fragment
template <int EPI>
DEV void epilogue(bf16* __restrict__ Y, const bf16* __restrict__ R, int M, int N, int m0, int n0,
                  const f32x4 (&acc)[2][4][4]) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wm * 128 + mh * 64 + mt * 16 + fr;
      if (m >= M) continue;
      if constexpr (EPI == 2) {
        const int F = N >> 1;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int f = ((n0 + wn * 64) >> 1) + p * 16 + fq * 4;
          if (f >= F) continue;
          const f32x4 gv = acc[mh][mt][2 * p], uv = acc[mh][mt][2 * p + 1];
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
        f32x4 v = acc[mh][mt][nt];
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

template <int EPI, class VAR = V256Default>   // EPI: 0 plain, 1 +residual, 2 SwiGLU
__global__ __launch_bounds__(512, 1) void gemm_tn_256(const bf16* __restrict__ X,
                                                      const bf16* __restrict__ W,
                                                      bf16* __restrict__ Y,
                                                      const bf16* __restrict__ R, int M, int N,
                                                      int K) {
  __shared__ __attribute__((aligned(16))) bf16 smem[8 * PIECE];
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  int m0, n0;
  tile_coords(xcd_remap(blockIdx.x, nm * nn), nm, nn, m0, n0);
  f32x4 acc[2][4][4];
  mainloop<VAR>(X, W, M, N, K, m0, n0, 0, K / BK, smem, acc);
  epilogue<EPI>(Y, R, M, N, m0, n0, acc);
}

// ---------------------------------------------------------------------------
// Split-K for wave quantisation: 336 tiles on 256 CUs run as 2 waves at 66 %
// occupancy.  Splitting every tile's K range into s parts gives tiles*s
// workgroups of 1/s tile each; s is chosen to minimise ceil(tiles*s/G)/s
// (3 for 336 tiles: 1.33 tile-times instead of 2).  Each workgroup runs ONE
// mainloop (a loop around it makes the compiler's LDS-DMA alias tracking put
// a vmcnt(0) before every ds_read), stores its fp32 partial (register order,
// coalesced float4) to its workspace slot, releases it (agent-scope fence:
// the 8 XCD L2s are not coherent) and bumps the tile's arrival counter; the
// last of the s contributors to arrive sums the partials in split order
// (deterministic), applies the epilogue and re-arms the counter.
template <int EPI, class VAR = V256Default>
__global__ __launch_bounds__(512, 1) void gemm_tn_256_splitk(const bf16* __restrict__ X,
                                                             const bf16* __restrict__ W,
                                                             bf16* __restrict__ Y,
                                                             const bf16* __restrict__ R, int M,
                                                             int N, int K, int splits,
                                                             float* __restrict__ ws,
                                                             int* __restrict__ cnt) {
  // ONE __shared__ array: a second LDS object (even the 4-byte last-arriver
  // flag) makes hipcc put vmcnt(0) before every ds_read of the K-loop
  // (cdna_hip_programming.md §5 "Three .s-level traps" (a))
  __shared__ __attribute__((aligned(16))) bf16 smem[8 * PIECE];
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  // splits of one tile are consecutive logical ids -> same XCD (shared L2 for the fixup)
  const int lid = xcd_remap(blockIdx.x, nm * nn * splits);
  const int t = lid / splits, sp = lid % splits;
  const int nk = K / BK;
  const int k0 = (int)((long long)sp * nk / splits), k1 = (int)((long long)(sp + 1) * nk / splits);
  int m0, n0;
  tile_coords(t, nm, nn, m0, n0);
  f32x4 acc[2][4][4];
  mainloop<VAR>(X, W, M, N, K, m0, n0, k0, k1, smem, acc);
  f32x4* wsv = reinterpret_cast<f32x4*>(ws) + (size_t)t * splits * 32 * 512;
#pragma unroll
  for (int q = 0; q < 32; ++q) wsv[((size_t)sp * 32 + q) * 512 + threadIdx.x] = (&acc[0][0][0])[q];
  // publish (guide §5 "Projection GEMM at M = 256" item 2): drain, one agent
  // release by lane 0, ticket; the last arriver acquires once and reduces
  int* flag = reinterpret_cast<int*>(smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == splits - 1;
    if (prev == splits - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cnt[t] = 0;                               // re-arm for the next launch
    }
  }
  __syncthreads();
  if (!*flag) return;
#pragma unroll
  for (int q = 0; q < 32; ++q) (&acc[0][0][0])[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < splits; ++c) {
#pragma unroll
    for (int q = 0; q < 32; ++q)
      (&acc[0][0][0])[q] += wsv[((size_t)c * 32 + q) * 512 + threadIdx.x];
  }
  epilogue<EPI>(Y, R, M, N, m0, n0, acc);
}

template <class VAR>
void launch_var(const void* X, const void* W, void* Y, int M, int N, int K, hipStream_t s) {
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  gemm_tn_256<0, VAR><<<dim3(nm * nn), 512, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                                    nullptr, M, N, K);
}

}  // namespace

int launch_gemm_tn_256_mode(const void* X, const void* W, void* Y, int M, int N, int K, int mode,
                            int pingpong, hipStream_t s);
int launch_gemm_tn_256d(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        int epi, hipStream_t s);
int gemm256d_ok(int M, int N, int K);
int launch_gemm_tn_256sk(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                         int epi, int force, hipStream_t s);
double gemm256sk_waves(int M, int N, int K);
int launch_gemm_tn_256d_bm(const void* X, const void* W, void* Y, const void* R, int M, int N,
                           int K, int epi, int bm, hipStream_t s);
int gemm256d_height(int M, int N, int K);
double gemm256d_waves_bm(int M, int N, int K, int bm);

// tuning / test entry for the kernels the production selector can reach
// (profiles/gemm_tuning.md keeps the measurements of the retired variants):
//   8  ping-pong-free base body        25 ping-pong (production fallback body)
//   30 data-parallel  31 forced 3-way split-K (base body)  32 auto  33 split-K + ping-pong
//   49 AGPR 256-row tiles  50 AGPR stream-K  51 AGPR 192-row tiles  52 AGPR, height by model
int launch_gemm_tn_256_variant(const void* X, const void* W, void* Y, int M, int N, int K, int v,
                               hipStream_t s) {
  switch (v) {
    case 8: launch_var<V256<false, false, false, true>>(X, W, Y, M, N, K, s); return 0;
    case 25: launch_var<V256Default>(X, W, Y, M, N, K, s); return 0;
    case 30: return launch_gemm_tn_256_mode(X, W, Y, M, N, K, 1, 1, s);
    case 31: return launch_gemm_tn_256_mode(X, W, Y, M, N, K, 2, 0, s);
    case 32: return launch_gemm_tn_256_mode(X, W, Y, M, N, K, 0, 1, s);
    case 33: return launch_gemm_tn_256_mode(X, W, Y, M, N, K, 2, 1, s);
    case 49: return launch_gemm_tn_256d_bm(X, W, Y, nullptr, M, N, K, 0, 256, s);
    case 50: return launch_gemm_tn_256sk(X, W, Y, nullptr, M, N, K, 0, 1, s);
    case 51: return launch_gemm_tn_256d_bm(X, W, Y, nullptr, M, N, K, 0, 192, s);
    case 52: return launch_gemm_tn_256d(X, W, Y, nullptr, M, N, K, 0, s);
    case 53: return launch_gemm_tn_256d_bm(X, W, Y, nullptr, M, N, K, 0, 160, s);
    case 54: return launch_gemm_tn_256d_bm(X, W, Y, nullptr, M, N, K, 0, 224, s);
    case 55: return launch_gemm_tn_256d_bm(X, W, Y, nullptr, M, N, K, 0, 128, s);
    default: return 1;
  }
}

namespace {

struct SkDevice {
  int G = 0;
  float* ws = nullptr;
  int* cnt = nullptr;
  size_t ws_tiles = 0;     // partial-tile slots in ws
  int cnt_tiles = 0;
};

constexpr int SPLIT_MAX = 8;
constexpr size_t TILE_PARTIAL_BYTES = 32 * 512 * sizeof(f32x4);   // 256 KiB fp32

// CU count and split-K workspace of the current device (allocated on first
// use / growth, outside any graph capture)
SkDevice& sk_device() {
  static SkDevice devs[64];
  int d = 0;
  (void)hipGetDevice(&d);
  SkDevice& sd = devs[d & 63];
  if (sd.G == 0) {
    hipDeviceProp_t prop;
    sd.G = hipGetDeviceProperties(&prop, d) == hipSuccess && prop.multiProcessorCount > 0
               ? prop.multiProcessorCount : 256;
  }
  return sd;
}

bool sk_reserve(SkDevice& sd, int tiles, int splits) {
  const size_t need = (size_t)tiles * splits;
  if (need > sd.ws_tiles) {
    if (sd.ws) (void)hipFree(sd.ws);
    if (hipMalloc(&sd.ws, need * TILE_PARTIAL_BYTES) != hipSuccess) {
      sd.ws = nullptr;
      sd.ws_tiles = 0;
      return false;
    }
    sd.ws_tiles = need;
  }
  if (tiles > sd.cnt_tiles) {
    if (sd.cnt) (void)hipFree(sd.cnt);
    const int n = tiles * 2;
    if (hipMalloc(&sd.cnt, sizeof(int) * n) != hipSuccess) {
      sd.cnt = nullptr;
      sd.cnt_tiles = 0;
      return false;
    }
    (void)hipMemset(sd.cnt, 0, sizeof(int) * n);
    (void)hipDeviceSynchronize();
    sd.cnt_tiles = n;
  }
  return true;
}

// waves per split factor, with a 3 % per-extra-split charge for the partial
// traffic and the shorter pipelines
double split_cost(int tiles, int G, int s) {
  return ceil((double)tiles * s / G) / s * (1.0 + 0.03 * (s - 1));
}

// Auto split-K is OFF by default: with 256 KiB fp32 slabs per split and tile
// the publish + last-arriver reduction costs more than the quantisation it
// removes on every Llama-3 shape measured (profiles/gemm_tuning.md); forced
// splits stay available (gemm_variant 31/33) and MCP_GEMM_SPLITK=1 enables auto.
static bool splitk_auto() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("MCP_GEMM_SPLITK");
    on = e && e[0] == '1';
  }
  return on == 1;
}

static bool use_256d() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("MCP_GEMM256");
    on = !(e && e[0] == 'p' && e[1] == 'p');
  }
  return on == 1;
}

int choose_splits(int M, int N, int K, int G) {
  if (!splitk_auto()) return 1;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nk = K / BK;
  int best = 1;
  double bc = split_cost(tiles, G, 1);
  for (int s = 2; s <= SPLIT_MAX && nk / s >= 4; ++s) {
    const double c = split_cost(tiles, G, s);
    if (c < bc - 1e-9) {
      bc = c;
      best = s;
    }
  }
  return best;
}

template <int EPI, class VAR = V256Default>
void launch_256(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                int splits, hipStream_t s) {
  // splits: 0 auto, 1 data-parallel, >1 forced split-K
  // production: the one-wave-per-SIMD AGPR kernel (gemm256d.hip) wherever its
  // shape rules hold (K % 128, N % 256); MCP_GEMM256=pp keeps the ping-pong kernel
  if (splits <= 1 && use_256d() && gemm256d_ok(M, N, K) == 0) {
    // stream-K (gemm256sk.hip) where the data-parallel grid's last wave is mostly empty
    if (splits <= 0 && launch_gemm_tn_256sk(X, W, Y, R, M, N, K, EPI, 0, s) == 0) return;
    if (launch_gemm_tn_256d(X, W, Y, R, M, N, K, EPI, s) == 0) return;
  }
  SkDevice& sd = sk_device();
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (splits <= 0) splits = choose_splits(M, N, K, sd.G);
  splits = min(splits, max(1, K / BK));
  if (splits > 1 && sk_reserve(sd, tiles, splits)) {
    gemm_tn_256_splitk<EPI, VAR><<<tiles * splits, 512, 0, s>>>(
        (const bf16*)X, (const bf16*)W, (bf16*)Y, (const bf16*)R, M, N, K, splits, sd.ws, sd.cnt);
    return;
  }
  gemm_tn_256<EPI, VAR><<<dim3(tiles), 512, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                                    (const bf16*)R, M, N, K);
}

}  // namespace

// effective waves of the 256^2 kernel (stream-K / split-K trim the quantisation of the last wave)
double gemm256_waves(int M, int N, int K) {
  if (use_256d() && gemm256d_ok(M, N, K) == 0)       // tile height chosen per shape (256 / 192)
    return fmin(gemm256d_waves_bm(M, N, K, gemm256d_height(M, N, K)), gemm256sk_waves(M, N, K));
  SkDevice& sd = sk_device();
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  return split_cost(tiles, sd.G, choose_splits(M, N, K, sd.G));
}

int gemm256_num_cus() { return sk_device().G; }

// sustained rate of the 256^2 path for this shape, PF/s (tools/bench_gemm.py):
// the AGPR kernel where it applies, else the ping-pong kernel
double gemm256_rate(int M, int N, int K) {
  return use_256d() && gemm256d_ok(M, N, K) == 0 ? 1.40 : 1.22;
}

void launch_gemm_tn_256(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                        hipStream_t s) {
  if (R) launch_256<1>(X, W, Y, R, M, N, K, 0, s);
  else launch_256<0>(X, W, Y, nullptr, M, N, K, 0, s);
}

void launch_gemm_tn_256_silu(const void* X, const void* W, void* Y, int M, int N, int K,
                             hipStream_t s) {
  launch_256<2>(X, W, Y, nullptr, M, N, K, 0, s);
}

int launch_gemm_tn_256_mode(const void* X, const void* W, void* Y, int M, int N, int K, int mode,
                            int pingpong, hipStream_t s) {
  // mode: 0 auto split, 1 data-parallel, 2 forced 3-way split
  const int splits = mode == 0 ? 0 : mode == 1 ? 1 : 3;
  if (pingpong) launch_256<0, V256Default>(X, W, Y, nullptr, M, N, K, splits, s);
  else launch_256<0, V256<false, false, false, true>>(X, W, Y, nullptr, M, N, K, splits, s);
  return 0;
}
