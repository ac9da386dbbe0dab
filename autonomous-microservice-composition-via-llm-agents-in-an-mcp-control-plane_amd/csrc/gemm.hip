// K1/K2: bf16 "TN" GEMM on MFMA for every Llama projection.
//   Y[M,N] = X[M,K] · W[N,K]^T   epilogues: plain, + R[M,N] (residual add),
//   or SwiGLU: W rows interleaved [gate 16 | up 16] per 32-row group, so each
//   lane's adjacent 16-column tiles hold gate and up of the same 4 features and
//   Y[M, N/2] = silu(gate) * up is written directly (no [M, N] intermediate).
// X = activations (row-major, K contiguous), W = nn.Linear weight (out x in,
// K contiguous), fp32 accumulation, bf16 out.
//
// Structure (cdna_hip_programming.md §5, "Minimum 2-phase" T3+T4 recipe):
//  * 128x128 block tile, BK = 64, 256 threads = 4 waves in a 2x2 grid, each wave
//    64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles.
//  * global -> LDS with global_load_lds_dwordx4 (one 1 KiB wave-instruction = 8
//    rows x 128 B), double-buffered: tile k+1 is in flight while tile k is read.
//  * LDS image is lane-linear; the XOR swizzle chunk ^= row&7 is applied on the
//    SOURCE address and on the ds_read_b128 address (rule 21) -> conflict-free
//    (tools/lds_banks.py).
//  * operands swapped in the MFMA (W as A, X as B) so each lane ends with 4
//    consecutive output columns of one row -> 8-byte bf16 stores.
//  * XCD-aware bijective block remap + grouped tile order for L2 reuse (T1).
#include <vector>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_ELEMS = 128 * BK;          // one operand tile, bf16 elements (16 KiB)

// SPLIT: split-K partial - blockIdx.y = split s of gridDim.y, K range
// [s K/S, (s+1) K/S), fp32 partial tile to Y + s M N (EPI 0, OutT float);
// splitk_reduce sums the partials and applies the epilogue.
template <int EPI, typename OutT = bf16, bool SPLIT = false>     // EPI: 0 plain, 1 +residual, 2 SwiGLU
__global__ __launch_bounds__(256, 2) void gemm_tn_128(const bf16* __restrict__ X,
                                                      const bf16* __restrict__ W,
                                                      OutT* __restrict__ Y,
                                                      const bf16* __restrict__ R, int M, int N,
                                                      int K, const NormEpi ne) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE_ELEMS];   // [buf][A|B][128][64]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const int nwg = nm * nn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  // grouped ordering: GROUP m-tiles share each W panel
  constexpr int GROUP = 8;
  const int per_group = GROUP * nn;
  const int g = wg / per_group;
  const int first_m = g * GROUP;
  const int gsz = min(nm - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int klen = SPLIT ? K / (int)gridDim.y : K;
  const int kbeg = SPLIT ? (int)blockIdx.y * klen : 0;
  if constexpr (SPLIT) Y += (size_t)blockIdx.y * M * N;

  // ---- staging addresses: wave w stages pieces 4w..4w+3 of each operand
  const int lrow = lane >> 3;                  // row inside the 8-row piece
  const int lchunk = (lane & 7) ^ lrow;        // inverse swizzle on the source
  const bf16* srcA[4];
  const bf16* srcB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 8 + lrow;
    const int ra = min(m0 + row, M - 1);
    const int rb = min(n0 + row, N - 1);
    srcA[i] = X + (size_t)ra * K + kbeg + lchunk * 8;
    srcB[i] = W + (size_t)rb * K + kbeg + lchunk * 8;
  }
  auto stage = [&](int kt, int buf) {
    bf16* la = smem + (buf * 2 + 0) * TILE_ELEMS;
    bf16* lb = smem + (buf * 2 + 1) * TILE_ELEMS;
    const int koff = kt * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(srcA[i] + koff, la + (wave * 4 + i) * 512);
      glds16(srcB[i] + koff, lb + (wave * 4 + i) * 512);
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = klen / BK;
  stage(0, 0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const bf16* la = smem + (cur * 2 + 0) * TILE_ELEMS;
    const bf16* lb = smem + (cur * 2 + 1) * TILE_ELEMS;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int ra = wm * 64 + t * 16 + fr;
        const int rb = wn * 64 + t * 16 + fr;
        af[t] = *reinterpret_cast<const bf16x8*>(la + ra * BK + ((c ^ (ra & 7)) << 3));
        bfr[t] = *reinterpret_cast<const bf16x8*>(lb + rb * BK + ((c ^ (rb & 7)) << 3));
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16x16x32(bfr[nt], af[mt], acc[mt][nt]);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds Y[m][n..n+3]
  if constexpr (sizeof(OutT) == 2 && EPI != 2) {
    store_direct<EPI>(acc, (bf16*)Y, R, M, N, m0 + wm * 64, n0 + wn * 64, fr, fq, ne);
    return;
  }
  if constexpr (EPI == 2) {                          // row scales hoisted (common.h)
    store_silu<4, 4>(acc, (bf16*)Y, M, N, m0 + wm * 64, n0 + wn * 64, fr, fq, ne);
    return;
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = m0 + wm * 64 + mt * 16 + fr;
    if (m >= M) continue;
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
      if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<f32x4*>(Y + (size_t)m * N + n) = v;
      } else {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
        *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
      }
    }
  }
}

// Sum of the S fp32 split-K partials [S][M][N] + the epilogue; one thread per
// 4 outputs (EPI 2: gate column 32 j + i pairs with up column 32 j + 16 + i,
// the interleaved SwiGLU layout, output f = 16 j + i).
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ ws, int S,
                                                     bf16* __restrict__ Y,
                                                     const bf16* __restrict__ R, int M, int N,
                                                     const NormEpi ne) {
  const int NO = EPI == 2 ? N / 2 : N;               // output columns
  const size_t total = (size_t)M * NO / 4;
  const size_t i4 = (size_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = i4 < total;
  const size_t iv = valid ? i4 : total - 1;
  const int m = (int)(iv / (NO / 4));
  const int c = (int)(iv % (NO / 4)) * 4;            // first output column
  const size_t MN = (size_t)M * N;
  bf16x4 o;
  if constexpr (EPI == 2) {
    const int cg = 32 * (c / 16) + c % 16;           // gate column (up = +16)
    const float* p = ws + (size_t)m * N + cg;
    f32x4 g = *reinterpret_cast<const f32x4*>(p), u = *reinterpret_cast<const f32x4*>(p + 16);
    for (int s = 1; s < S; ++s) {
      g += *reinterpret_cast<const f32x4*>(p + s * MN);
      u += *reinterpret_cast<const f32x4*>(p + s * MN + 16);
    }
    const float rs = norm_row_scale(ne, m);          // fused RMSNorm of the input row
    g *= rs;
    u *= rs;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)(g[j] / (1.f + __expf(-g[j])) * u[j]);
  } else {
    const float* p = ws + (size_t)m * N + c;
    f32x4 v = *reinterpret_cast<const f32x4*>(p);
    for (int s = 1; s < S; ++s) v += *reinterpret_cast<const f32x4*>(p + s * MN);
    if (EPI == 1) {
      const bf16x4 r = *reinterpret_cast<const bf16x4*>(R + (size_t)m * N + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += (float)r[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
  }
  if (valid) *reinterpret_cast<bf16x4*>(Y + (size_t)m * NO + c) = o;
  if (EPI == 1 && ne.ss_out) {
    // fused RMSNorm statistic: one atomic per wave when the wave's 64 threads
    // cover one row (NO / 4 a multiple of 64), else one per thread
    float ss = valid ? sumsq_bf16x4(o) : 0.f;
    const size_t w0 = i4 & ~(size_t)63;
    const bool one_row = (NO / 4) % 64 == 0 && w0 < total;
    if (one_row) {
      ss = wave_sum(ss);
      if ((threadIdx.x & 63) == 0) ss_atomic_add(ne.ss_out + m, ss);
    } else if (valid) {
      ss_atomic_add(ne.ss_out + m, ss);
    }
  }
}

}  // namespace

int gemm_tn_check(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 1;
  if (K % 64) return 2;
  if (N % 4) return 3;
  return 0;
}

// Tile selection by a wave-quantisation time model calibrated on MI355X
// (tools/bench_gemm.py): the 256x256 kernels sustain ~1.40 PF/s (AGPR kernel,
// gemm256d.hip, 256- or 192-row tiles) / ~1.22 PF/s (ping-pong) with one
// workgroup per CU (256 concurrent tiles), the 128x128 kernel ~0.9 PF/s with
// two per CU (512).  Predicted time = full waves of tiles x
// per-wave time; pick the smaller.
double gemm256_waves(int M, int N, int K);
double gemm256_rate(int M, int N, int K);
int gemm256_num_cus();

// ---- measured tile plans (tools/tune_gemm_plan.py -> profiles/gemm_plan_*.json,
// loaded by ops.lib()): per (N, K) weight shape one code per 64-row M bucket
// (bucket b = rows (64 b, 64 b + 64]; every tile height divides 64, so all M
// of a bucket have the tile counts of its top row, the row that was timed):
// 0 = 128^2 kernel, 1..5 = AGPR kernel (gemm256d.hip) with 256-, 192-, 160-,
// 224- or 128-row tiles (gemm256d_code_height).
// Written once at load, before any launch; read-only afterwards.
namespace {
struct GemmPlan {
  int N, K;
  std::vector<signed char> code;
  std::vector<signed char> split;    // measured split-K of the 128^2 path (0: the rule)
  std::vector<signed char> flex;     // measured flex tile (gemm_flex.hip) or -1
  std::vector<signed char> group;    // measured tile group of the AGPR kernel (0: default)
  std::vector<signed char> persist;  // 1: the persistent AGPR kernel (gemm256p.hip) measured faster
  std::vector<short> fsplit;         // measured flex tile x split-K (16 cand + S) or -1
  std::vector<short> silu;           // gate|up: measured SwiGLU path (launch_gemm_silu_algo) or -1
  std::vector<short> rope;           // qkv: measured QKV + RoPE path (launch_qkv_rope_algo) or -1
};
std::vector<GemmPlan> g_plans;
}  // namespace

void gemm_plan_set(int N, int K, const int* codes, int n) {
  std::vector<signed char> c(codes, codes + n);
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.code = std::move(c);
      return;
    }
  g_plans.push_back({N, K, std::move(c), {}, {}, {}, {}});
}

void gemm_plan_set_splits(int N, int K, const int* splits, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.split.assign(splits, splits + n);
      return;
    }
  g_plans.push_back({N, K, {}, std::vector<signed char>(splits, splits + n), {}, {}, {}});
}

void gemm_plan_set_flex(int N, int K, const int* flex, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.flex.assign(flex, flex + n);
      return;
    }
  g_plans.push_back({N, K, {}, {}, std::vector<signed char>(flex, flex + n), {}, {}});
}

void gemm_plan_set_group(int N, int K, const int* group, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.group.assign(group, group + n);
      return;
    }
  g_plans.push_back({N, K, {}, {}, {}, std::vector<signed char>(group, group + n), {}});
}

void gemm_plan_set_persist(int N, int K, const int* persist, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.persist.assign(persist, persist + n);
      return;
    }
  g_plans.push_back({N, K, {}, {}, {}, {}, std::vector<signed char>(persist, persist + n)});
}

int gemm_plan_persist(int M, int N, int K) {
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.persist.size() ? p.persist[b] : 0;
    }
  return 0;
}

// measured tile group of the AGPR kernel for this M bucket (0 = none recorded)
int gemm_plan_group(int M, int N, int K) {
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.group.size() ? p.group[b] : 0;
    }
  return 0;
}

// measured flex tile candidate for this M bucket (-1 = none: the code path)
int gemm_plan_flex(int M, int N, int K) {
  static const int on = getenv("MCP_GEMM_FLEX") ? atoi(getenv("MCP_GEMM_FLEX")) : 1;
  if (!on) return -1;
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.flex.size() ? p.flex[b] : -1;
    }
  return -1;
}

// measured split count for the 128^2 path at this M bucket (0 = none recorded)
int gemm_plan_split(int M, int N, int K) {
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.split.size() ? p.split[b] : 0;
    }
  return 0;
}

void gemm_plan_set_fsplit(int N, int K, const int* fs, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.fsplit.assign(fs, fs + n);
      return;
    }
  GemmPlan q{N, K, {}, {}, {}, {}, {}, {}, {}, {}};
  q.fsplit.assign(fs, fs + n);
  g_plans.push_back(std::move(q));
}

// measured flex tile with split-K for this M bucket: 16 cand + S, -1 = none
// (MCP_GEMM_FSPLIT=0 disables)
int gemm_plan_fsplit(int M, int N, int K) {
  static const int on = getenv("MCP_GEMM_FSPLIT") ? atoi(getenv("MCP_GEMM_FSPLIT")) : 1;
  if (!on) return -1;
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.fsplit.size() ? p.fsplit[b] : -1;
    }
  return -1;
}

void gemm_plan_set_silu(int N, int K, const int* codes, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.silu.assign(codes, codes + n);
      return;
    }
  GemmPlan q{N, K, {}, {}, {}, {}, {}, {}, {}, {}};
  q.silu.assign(codes, codes + n);
  g_plans.push_back(std::move(q));
}

// gate|up with the SwiGLU epilogue: the path measured fastest WITH that
// epilogue for this M bucket (tools/tune_gemm_plan.py --silu), -1 = none (the
// rule).  The code plan above is timed with the plain epilogue, and its AGPR
// heights were never reached below M = 256 (gemm_select).  MCP_GEMM_SILU_PLAN=0
// disables.
int gemm_plan_silu(int M, int N, int K) {
  static const int on = getenv("MCP_GEMM_SILU_PLAN") ? atoi(getenv("MCP_GEMM_SILU_PLAN")) : 1;
  if (!on) return -1;
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.silu.size() ? p.silu[b] : -1;
    }
  return -1;
}

void gemm_plan_set_rope(int N, int K, const int* codes, int n) {
  for (auto& p : g_plans)
    if (p.N == N && p.K == K) {
      p.rope.assign(codes, codes + n);
      return;
    }
  GemmPlan q{N, K, {}, {}, {}, {}, {}, {}, {}, {}};
  q.rope.assign(codes, codes + n);
  g_plans.push_back(std::move(q));
}

// QKV + RoPE + K/V write: the path measured fastest with that epilogue for
// this M bucket (tools/tune_gemm_plan.py MCP_TUNE_ROPE=1), -1 = none (the
// rule).  MCP_GEMM_ROPE_PLAN=0 disables.
int gemm_plan_rope(int M, int N, int K) {
  static const int on = getenv("MCP_GEMM_ROPE_PLAN") ? atoi(getenv("MCP_GEMM_ROPE_PLAN")) : 1;
  if (!on) return -1;
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.rope.size() ? p.rope[b] : -1;
    }
  return -1;
}

void gemm_plan_clear() { g_plans.clear(); }

// -1 = no measured plan for this shape
int gemm_plan_lookup(int M, int N, int K) {
  for (const auto& p : g_plans)
    if (p.N == N && p.K == K) {
      const size_t b = (size_t)((M + 63) / 64) - 1;
      return b < p.code.size() ? p.code[b] : -1;
    }
  return -1;
}

int gemm_select(int M, int N, int K) {
  if (M < 256 || N < 256 || K < 128) return 0;
  // a fused RMSNorm needs an epilogue that implements it: the 256^2
  // ping-pong fallback (shapes the AGPR kernel rejects) does not
  const NormEpi& ne = norm_epi();
  if ((ne.ss_in || ne.ss_out) && gemm256d_ok(M, N, K) != 0) return 0;
  const int plan = gemm_plan_lookup(M, N, K);
  if (plan >= 0 && (plan == 0 || gemm256d_ok(M, N, K) == 0)) return plan == 0 ? 0 : 1;
  const double G = (double)gemm256_num_cus();
  const double t128 = (double)(((M + 127) / 128) * ((N + 127) / 128));
  // 256^2 waves (stream-K hybrid where it pays) vs 128^2 waves at 2 blocks/CU
  const double cost256 = gemm256_waves(M, N, K) * G * 4.0 / gemm256_rate(M, N, K);   // 128^2 units / PF
  // 128^2 kernel: ~0.9 PF/s at the decode-step shapes (M ~ 2600, measured
  // 0.68-1.07; profiles/gemm_tuning.md)
  const double cost128 = ceil(t128 / (2.0 * G)) * 2.0 * G / 0.90;
  return cost256 < cost128 ? 1 : 0;
}

// ---- split-K for the 128^2 kernel at small M: N = 4096 at M = 256 is 64
// tiles for 256 CUs (two per CU fit), so one projection ran at a quarter of
// the chip.  S splits of K (each >= 8 k-tiles) fill it; the fp32 partials go
// to a workspace allocated once when the library loads (never inside a graph
// capture), and a reduce kernel applies the epilogue.
namespace {
float* g_splitk_ws = nullptr;
size_t g_splitk_ws_bytes = 0;
int* g_splitk_tickets = nullptr;       // per-tile arrival tickets (gemm_stream.hip)
constexpr size_t MAX_SPLIT_TILES = 1 << 16;
int g_split_force = -1;                // gemm_splitk_force (tests, tuning)
}  // namespace

void gemm_splitk_force(int S) { g_split_force = S; }

bool gemm_splitk_workspace(float** ws, int** tickets, size_t bytes, size_t tiles) {
  if (!g_splitk_ws || !g_splitk_tickets || bytes > g_splitk_ws_bytes || tiles > MAX_SPLIT_TILES)
    return false;
  *ws = g_splitk_ws;
  *tickets = g_splitk_tickets;
  return true;
}

int gemm_stream_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("MCP_GEMM_STREAM");
    on = e ? atoi(e) : 1;
  }
  return on;
}

int gemm256sk_prealloc();
int gemm256d_split2_prealloc();

int gemm_splitk_init(size_t bytes) {
  // the stream-K tail's slabs / counters too (gemm256sk.hip): both are
  // allocated here, at library load, never inside a hipGraph capture
  if (gemm256sk_prealloc() != 0 || gemm256d_split2_prealloc() != 0) return 2;
  if (!g_splitk_tickets) {
    if (hipMalloc(&g_splitk_tickets, MAX_SPLIT_TILES * sizeof(int)) != hipSuccess) {
      g_splitk_tickets = nullptr;
      return 1;
    }
    if (hipMemset(g_splitk_tickets, 0, MAX_SPLIT_TILES * sizeof(int)) != hipSuccess) return 1;
    (void)hipDeviceSynchronize();
  }
  if (g_splitk_ws_bytes >= bytes) return 0;
  if (g_splitk_ws) (void)hipFree(g_splitk_ws);
  g_splitk_ws = nullptr;
  g_splitk_ws_bytes = 0;
  if (hipMalloc(&g_splitk_ws, bytes) != hipSuccess) {
    g_splitk_ws = nullptr;
    return 1;
  }
  g_splitk_ws_bytes = bytes;
  return 0;
}

// splits for the 128^2 path (1 = none): the fewest that give >= 2 workgroups
// per CU, K / S a multiple of 64 with >= 8 k-tiles, partials within the
// workspace.  MCP_GEMM_SPLITK128=0 disables, =S > 1 forces S where K allows.
int gemm128_splits(int M, int N, int K) {
  static int enabled = -1;
  if (enabled < 0) {
    const char* e = getenv("MCP_GEMM_SPLITK128");
    enabled = e ? atoi(e) : 1;
  }
  if (!enabled || !g_splitk_ws) return 1;
  if (g_split_force >= 0) {
    const int S = g_split_force, nkt = K / BK;
    return (S > 1 && nkt % S == 0 && nkt / S >= 4 &&
            (size_t)S * M * N * sizeof(float) <= g_splitk_ws_bytes) ? S : 1;
  }
  const int G = gemm256_num_cus();
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (enabled > 1) {                                 // MCP_GEMM_SPLITK128=S forces S (tuning)
    const int S = enabled, nkt = K / BK;
    return (nkt % S == 0 && (size_t)S * M * N * sizeof(float) <= g_splitk_ws_bytes) ? S : 1;
  }
  const int nkt = K / BK;
  // a measured split (tools/tune_gemm_plan.py) for this (N, K, M bucket) wins
  // over the rule below where it is admissible
  const int ps = gemm_plan_split(M, N, K);
  if (ps == 1) return 1;
  if (ps > 1 && nkt % ps == 0 && nkt / ps >= 4 && (size_t)ps * M * N * sizeof(float) <= g_splitk_ws_bytes)
    return ps;
  if (tiles > G) return 1;
  // fewest splits that give every CU a workgroup while each keeps <= 32
  // k-tiles: fewer fp32 partials to write and reduce.  Measured at M = 64-256
  // on the 8B shapes (profiles/gemm_small_m_splitk_sweep.jsonl): gate|up 2 vs
  // 4 splits -18..-20 %, qkv / o at M = 192-256 4 vs 8 -5..-16 %, down
  // (K = 14336) keeps 8.  Applied in the measured range M <= 256 only.
  for (int S = 2; S <= 16 && M <= 256; S *= 2) {
    if (nkt % S || nkt / S < 8 || nkt / S > 32) continue;
    if ((size_t)S * M * N * sizeof(float) > g_splitk_ws_bytes) break;
    if (tiles * S >= G) return S;
  }
  for (int S = 2; S <= 16; ++S) {
    if (nkt % S || nkt / S < 8) continue;
    if ((size_t)S * M * N * sizeof(float) > g_splitk_ws_bytes) break;
    if (tiles * S >= 2 * G || S == 16) return S;
  }
  // largest admissible S below the target
  int best = 1;
  for (int S = 2; S <= 16; ++S)
    if (nkt % S == 0 && nkt / S >= 8 && (size_t)S * M * N * sizeof(float) <= g_splitk_ws_bytes)
      best = S;
  return best;
}

// EPI 0/1/2 through S split-K partials + the reduce; false if not split
static bool launch_gemm_128_split(const void* X, const void* W, void* Y, const void* R, int M,
                                  int N, int K, int epi, hipStream_t s) {
  const int S = gemm128_splits(M, N, K);
  if (S <= 1) return false;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  gemm_tn_128<0, float, true><<<dim3(nm * nn, S), 256, 0, s>>>(
      (const bf16*)X, (const bf16*)W, g_splitk_ws, nullptr, M, N, K, NormEpi{});
  const size_t n4 = (size_t)M * (epi == 2 ? N / 2 : N) / 4;
  const dim3 rg((unsigned)((n4 + 255) / 256));
  switch (epi) {
    case 0: splitk_reduce<0><<<rg, 256, 0, s>>>(g_splitk_ws, S, (bf16*)Y, nullptr, M, N, norm_epi()); break;
    case 1: splitk_reduce<1><<<rg, 256, 0, s>>>(g_splitk_ws, S, (bf16*)Y, (const bf16*)R, M, N, norm_epi()); break;
    default: splitk_reduce<2><<<rg, 256, 0, s>>>(g_splitk_ws, S, (bf16*)Y, nullptr, M, N, norm_epi()); break;
  }
  return true;
}

// QKV split-K reduce with the RoPE / paged K-V write fused in (the rope_kv
// kernel's work, elementwise.hip, on the fp32 sums instead of a bf16 qkv
// round trip): one thread per (token, head, 8-wide chunk of the first half)
// of the S partials [S][M][(Hq + 2 Hkv) D]; V heads are copied to the cache
template <int D>
__global__ __launch_bounds__(256) void splitk_reduce_rope(const float* __restrict__ ws, int S, int M,
                                                          const RopeArgs ra, const NormEpi ne) {
  constexpr int CH = D / 16;
  const int heads = ra.Hq + 2 * ra.Hkv;
  const int N = heads * D;
  const size_t total = (size_t)M * heads * CH;
  const size_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % CH);
  const int h = (int)((i / CH) % heads);
  const int t = (int)(i / ((size_t)CH * heads));
  const int d0 = c * 8;
  const size_t MN = (size_t)M * N;
  const float* p = ws + (size_t)t * N + (size_t)h * D + d0;
  f32x4 lo0 = *reinterpret_cast<const f32x4*>(p), lo1 = *reinterpret_cast<const f32x4*>(p + 4);
  f32x4 hi0 = *reinterpret_cast<const f32x4*>(p + D / 2), hi1 = *reinterpret_cast<const f32x4*>(p + D / 2 + 4);
  for (int sp = 1; sp < S; ++sp) {
    const float* q = p + sp * MN;
    lo0 += *reinterpret_cast<const f32x4*>(q);
    lo1 += *reinterpret_cast<const f32x4*>(q + 4);
    hi0 += *reinterpret_cast<const f32x4*>(q + D / 2);
    hi1 += *reinterpret_cast<const f32x4*>(q + D / 2 + 4);
  }
  const float rs = norm_row_scale(ne, t);
  float lo[8], hi[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lo[j] = lo0[j] * rs;
    lo[4 + j] = lo1[j] * rs;
    hi[j] = hi0[j] * rs;
    hi[4 + j] = hi1[j] * rs;
  }
  bf16x8 olo, ohi;
  bf16* dst;
  if (h >= ra.Hq + ra.Hkv) {                           // V: copy into the cache
    const int slot = ra.slots[t];
    if (slot < 0) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      olo[j] = (bf16)lo[j];
      ohi[j] = (bf16)hi[j];
    }
    dst = reinterpret_cast<bf16*>(ra.v_cache) +
          (((size_t)(slot / ra.BS) * ra.Hkv + (h - ra.Hq - ra.Hkv)) * ra.BS + slot % ra.BS) * D;
  } else {
    const float2* cs = reinterpret_cast<const float2*>(ra.cos_sin) + (size_t)ra.pos[t] * (D / 2) + d0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 r = cs[j];
      olo[j] = (bf16)(lo[j] * r.x - hi[j] * r.y);
      ohi[j] = (bf16)(hi[j] * r.x + lo[j] * r.y);
    }
    if (h < ra.Hq) {
      dst = reinterpret_cast<bf16*>(ra.q_out) + ((size_t)t * ra.Hq + h) * D;
    } else {
      const int slot = ra.slots[t];
      if (slot < 0) return;
      dst = reinterpret_cast<bf16*>(ra.k_cache) +
            (((size_t)(slot / ra.BS) * ra.Hkv + (h - ra.Hq)) * ra.BS + slot % ra.BS) * D;
    }
  }
  *reinterpret_cast<bf16x8*>(dst + d0) = olo;
  *reinterpret_cast<bf16x8*>(dst + d0 + D / 2) = ohi;
}

// QKV + RoPE + K/V write through the plan's flex x split-K entry for this
// bucket, the reduce doing the rope_kv work; nonzero: not taken
// flex tile cand x S-way split-K, the reduce applying RoPE + the K/V write
int launch_qkv_rope_flex_split(const void* X, const void* W, int M, int N, int K, int D,
                               const RopeArgs& ra, int cand, int S, hipStream_t s) {
  if (D != 128 || N != (ra.Hq + 2 * ra.Hkv) * D) return 1;
  if (!g_splitk_ws || (size_t)S * M * N * sizeof(float) > g_splitk_ws_bytes) return 4;
  if (launch_gemm_flex_partials(X, W, g_splitk_ws, M, N, K, cand, S, s)) return 2;
  const size_t total = (size_t)M * (ra.Hq + 2 * ra.Hkv) * (D / 16);
  splitk_reduce_rope<128><<<(unsigned)((total + 255) / 256), 256, 0, s>>>(g_splitk_ws, S, M, ra,
                                                                            norm_epi());
  return 0;
}

int launch_qkv_rope_fsplit(const void* X, const void* W, int M, int N, int K, int D,
                           const RopeArgs& ra, hipStream_t s) {
  static const int on = getenv("MCP_QKV_ROPE_FSPLIT") ? atoi(getenv("MCP_QKV_ROPE_FSPLIT")) : 1;
  if (!on) return 1;
  const int fs = gemm_plan_fsplit(M, N, K);
  if (fs < 0) return 1;
  return launch_qkv_rope_flex_split(X, W, M, N, K, D, ra, fs / 16, fs % 16, s);
}

// flex tile cand, S-way split-K through the fp32 workspace + the reduce
// (epilogue 0/1/2); nonzero if unsupported or the workspace is too small
int launch_gemm_flex_split(const void* X, const void* W, void* Y, const void* R, int M, int N,
                           int K, int cand, int S, int epi, hipStream_t s) {
  if (!g_splitk_ws || (size_t)S * M * N * sizeof(float) > g_splitk_ws_bytes) return 4;
  if (epi == 2 && N % 64) return 2;
  const int rc = launch_gemm_flex_partials(X, W, g_splitk_ws, M, N, K, cand, S, s);
  if (rc) return rc;
  const size_t n4 = (size_t)M * (epi == 2 ? N / 2 : N) / 4;
  const dim3 rg((unsigned)((n4 + 255) / 256));
  switch (epi) {
    case 0: splitk_reduce<0><<<rg, 256, 0, s>>>(g_splitk_ws, S, (bf16*)Y, nullptr, M, N, norm_epi()); break;
    case 1: splitk_reduce<1><<<rg, 256, 0, s>>>(g_splitk_ws, S, (bf16*)Y, (const bf16*)R, M, N, norm_epi()); break;
    default: splitk_reduce<2><<<rg, 256, 0, s>>>(g_splitk_ws, S, (bf16*)Y, nullptr, M, N, norm_epi()); break;
  }
  return 0;
}

static void launch_gemm_tn_128(const void* X, const void* W, void* Y, const void* R, int M, int N,
                               int K, hipStream_t s) {
  if (launch_gemm_128_split(X, W, Y, R, M, N, K, R ? 1 : 0, s)) return;
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  const dim3 grid(nm * nn);
  if (R)
    gemm_tn_128<1><<<grid, 256, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                        (const bf16*)R, M, N, K, norm_epi());
  else
    gemm_tn_128<0><<<grid, 256, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y, nullptr, M, N,
                                        K, norm_epi());
}

// fp32-output variant (retrieval scores: bf16 would tie near-equal cosines)
void launch_gemm_tn_f32out(const void* X, const void* W, float* Y, int M, int N, int K,
                           hipStream_t s) {
  const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
  gemm_tn_128<0, float><<<dim3(nm * nn), 256, 0, s>>>((const bf16*)X, (const bf16*)W, Y,
                                                      nullptr, M, N, K, NormEpi{});
}

// A few rows (single-intent decode): the skinny kernel streams the weights at
// the HBM roof with COLD weights (the serving case, tools/bench_cold_small_m.py:
// gate|up 38.8-44.5 us at M = 1-8 = 6 TB/s, vs 54 us through split-K 128^2 or
// the stream kernel; o / down / qkv 2-4 % faster at M <= 4)
static bool skinny_first(int M, int N, int K) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("MCP_GEMM_SKINNY_FIRST");
    on = e ? atoi(e) : 1;
  }
  // wide (gate|up) projections: skinny up to MCP_GEMM_SKINNY_WIDE_MAXM rows
  static const int wide = getenv("MCP_GEMM_SKINNY_WIDE_MAXM") ? atoi(getenv("MCP_GEMM_SKINNY_WIDE_MAXM")) : 8;
  // o-proj sized (N, K <= 4096): skinny up to 16 rows (8.0-10.0 vs 7.8-10.5 us)
  // tall-K projections (down: K >= 2 N) go to the split-K stream kernel even at
  // M <= 4: N / 16 workgroups each walking all of K lose to it (4096 x 14336,
  // M = 1-4: 28.1-29.2 vs 23.6-23.8 us cold, profiles/gemm_decode_probe_r4.jsonl)
  const bool tall = gemm_stream_rule() != 0 && K >= 2 * N;
  return on && ((M <= 4 && !tall) || (N >= 16384 && M <= wide) || (N <= 4096 && K <= 4096 && M <= 16));
}

void launch_gemm_tn(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                    hipStream_t s) {
  if (skinny_first(M, N, K) && launch_gemm_skinny(X, W, Y, R, M, N, K, R ? 1 : 0, s) == 0) return;
  if (gemm_stream_enabled() && gemm_stream_pick(M, N, K, R ? 1 : 0) &&
      launch_gemm_stream(X, W, Y, R, M, N, K, R ? 1 : 0, RopeArgs{}, s) == 0)
    return;
  // M <= 128: split-K over the 128^2 kernel beats the weight-streaming skinny
  // kernel wherever it applies (tools/bench_small_m.py: 1.5-4x at N, K >= 4096)
  if (M <= SKINNY_MAX_M && gemm128_splits(M, N, K) <= 1 &&
      launch_gemm_skinny(X, W, Y, R, M, N, K, R ? 1 : 0, s) == 0)
    return;
  // serving-size M: a flex tile with split-K through the fp32 workspace,
  // measured faster than every other path for this bucket (plan "fsplit": the
  // narrow projections at M = 65-512, e.g. down 4096 x 14336 at M = 320-384
  // 59-64 vs 72-76 us, profiles/gemm_flex_split_r4.jsonl)
  const int fs = gemm_plan_fsplit(M, N, K);
  if (fs >= 0 && launch_gemm_flex_split(X, W, Y, R, M, N, K, fs / 16, fs % 16, R ? 1 : 0, s) == 0)
    return;
  // serving-size M: a tile shape that fills one wave of workgroups, measured
  // faster than the 128^2 split-K / AGPR paths for this bucket (plan "flex")
  const int fx = gemm_plan_flex(M, N, K);
  if (fx >= 0 && launch_gemm_flex(X, W, Y, R, M, N, K, fx, s) == 0) return;
  if (gemm_select(M, N, K) == 1)
    launch_gemm_tn_256(X, W, Y, R, M, N, K, s);
  else
    launch_gemm_tn_128(X, W, Y, R, M, N, K, s);
}

void launch_gemm_tn_algo(const void* X, const void* W, void* Y, const void* R, int M, int N, int K,
                         int algo, hipStream_t s) {
  // tuning: 1000 + 16 cand + S = flex tile cand with S-way split-K
  if (algo >= 1000 && launch_gemm_flex_split(X, W, Y, R, M, N, K, (algo - 1000) / 16,
                                             (algo - 1000) % 16, R ? 1 : 0, s) == 0)
    return;
  if (algo >= 16 && algo < 1000 && launch_gemm_flex(X, W, Y, R, M, N, K, algo - 16, s) == 0) return;   // tuning
  // 9..13: the AGPR kernel at the tile height of plan code algo - 8 (tuning)
  if (algo >= 9 && algo <= 13 &&
      launch_gemm_tn_256d_bm(X, W, Y, R, M, N, K, R ? 1 : 0, gemm256d_code_height(algo - 8), s) == 0)
    return;
  if (algo < 0) launch_gemm_tn(X, W, Y, R, M, N, K, s);
  else if (algo == 3 && launch_gemm_stream(X, W, Y, R, M, N, K, R ? 1 : 0, RopeArgs{}, s) == 0) return;
  else if (algo == 2 && launch_gemm_skinny(X, W, Y, R, M, N, K, R ? 1 : 0, s) == 0) return;
  else if (algo == 1) launch_gemm_tn_256(X, W, Y, R, M, N, K, s);
  else launch_gemm_tn_128(X, W, Y, R, M, N, K, s);
}

// SwiGLU-fused projection: W rows interleaved [gate 16 | up 16]; Y is [M, N/2]
void launch_gemm_tn_256_silu(const void* X, const void* W, void* Y, int M, int N, int K,
                             hipStream_t s);

// One SwiGLU path by code (the tuner's candidates and the "silu" plan):
//   1..5          AGPR kernel at the height of plan code c (gemm256d_code_height)
//   100 + S       128^2 kernel, S-way split-K through the reduce (S = 1: none)
//   200           weight-streaming kernel (M <= 128)
//   300 + f       flex tile candidate f (+32: 4-stage) with the SwiGLU epilogue
//   400 + c       AGPR kernel at the height of code c, K halves over two
//                 workgroups per tile (SPLIT 2, in-launch hand-off); 400 =
//                 the smallest height >= M (M <= 224, else nonzero)
//   1000 + 16 c + S  flex tile c with S-way split-K, the reduce applies SwiGLU
// nonzero: not supported for this shape (nothing launched)
int launch_gemm_silu_algo(const void* X, const void* W, void* Y, int M, int N, int K, int algo,
                          hipStream_t s) {
  if (N % 64) return 1;
  if (algo >= 1000)
    return launch_gemm_flex_split(X, W, Y, nullptr, M, N, K, (algo - 1000) / 16, (algo - 1000) % 16, 2, s);
  if (algo >= 401 && algo <= 405)                    // AGPR kernel, K halves over two workgroups
    return launch_gemm_tn_256d_split2(X, W, Y, nullptr, M, N, K, 2, gemm256d_code_height(algo - 400), s);
  if (algo == 400) {
    // K halves at the smallest tile height that holds all M rows, up to 224
    // (gate|up at M = 129-224: one wave of 2 x 112 workgroups, W streamed
    // once; profiles/gate_up_midm_r6.md).  Past 224 rows nonzero: the
    // caller's rule path runs.  MCP_GEMM_SPLIT2=0 turns it off (A/B).
    static const int on = getenv("MCP_GEMM_SPLIT2") ? atoi(getenv("MCP_GEMM_SPLIT2")) : 1;
    if (!on || M > 224) return 6;
    const int bm = M <= 128 ? 128 : M <= 160 ? 160 : M <= 192 ? 192 : 224;
    return launch_gemm_tn_256d_split2(X, W, Y, nullptr, M, N, K, 2, bm, s);
  }
  if (algo >= 300) {
    if (!gemm_flex_silu_ok(algo - 300)) return 2;
    return launch_gemm_flex_epi(X, W, Y, nullptr, M, N, K, algo - 300, 2, s);
  }
  if (algo == 200) return launch_gemm_stream(X, W, Y, nullptr, M, N, K, 2, RopeArgs{}, s);
  if (algo >= 100) {
    const int S = algo - 100;
    if (S > 1) {
      const int nkt = K / BK;
      if (!g_splitk_ws || nkt % S || nkt / S < 4 || (size_t)S * M * N * sizeof(float) > g_splitk_ws_bytes)
        return 3;
      const int saved = g_split_force;
      g_split_force = S;
      const bool split = launch_gemm_128_split(X, W, Y, nullptr, M, N, K, 2, s);
      g_split_force = saved;
      if (!split) return 3;
      return 0;
    }
    const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
    gemm_tn_128<2><<<dim3(nm * nn), 256, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                                 nullptr, M, N, K, norm_epi());
    return 0;
  }
  if (algo >= 1 && algo <= 5) {
    if (gemm256d_ok(M, N, K)) return 4;
    return launch_gemm_tn_256d_bm(X, W, Y, nullptr, M, N, K, 2, gemm256d_code_height(algo), s);
  }
  return 5;
}

int launch_gemm_silu(const void* X, const void* W, void* Y, int M, int N, int K, hipStream_t s) {
  if (N % 64) return 1;
  if (skinny_first(M, N, K) && launch_gemm_skinny(X, W, Y, nullptr, M, N, K, 2, s) == 0) return 0;
  // a measured SwiGLU path for the bucket (timed at its top row: below 33
  // rows the stream / skinny rules, measured per M, keep the decode sizes)
  const int sp = M > 32 ? gemm_plan_silu(M, N, K) : -1;
  if (sp >= 0 && launch_gemm_silu_algo(X, W, Y, M, N, K, sp, s) == 0) return 0;
  if (gemm_stream_enabled() && gemm_stream_pick(M, N, K, 2) &&
      launch_gemm_stream(X, W, Y, nullptr, M, N, K, 2, RopeArgs{}, s) == 0)
    return 0;
  if (M <= SKINNY_MAX_M && gemm128_splits(M, N, K) <= 1 &&
      launch_gemm_skinny(X, W, Y, nullptr, M, N, K, 2, s) == 0)
    return 0;
  // serving-size M: a measured flex tile with split-K (plan "fsplit"; the
  // reduce applies the SwiGLU) or with the SwiGLU epilogue (plan "flex")
  const int fs = gemm_plan_fsplit(M, N, K);
  if (fs >= 0 && launch_gemm_flex_split(X, W, Y, nullptr, M, N, K, fs / 16, fs % 16, 2, s) == 0)
    return 0;
  const int fx = gemm_plan_flex(M, N, K);
  if (fx >= 0 && gemm_flex_silu_ok(fx) &&
      launch_gemm_flex_epi(X, W, Y, nullptr, M, N, K, fx, 2, s) == 0)
    return 0;
  if (gemm_select(M, N, K) == 1) {
    launch_gemm_tn_256_silu(X, W, Y, M, N, K, s);
  } else if (!launch_gemm_128_split(X, W, Y, nullptr, M, N, K, 2, s)) {
    const int nm = (M + BM - 1) / BM, nn = (N + BN - 1) / BN;
    gemm_tn_128<2><<<dim3(nm * nn), 256, 0, s>>>((const bf16*)X, (const bf16*)W, (bf16*)Y,
                                                 nullptr, M, N, K, norm_epi());
  }
  return 0;
}
