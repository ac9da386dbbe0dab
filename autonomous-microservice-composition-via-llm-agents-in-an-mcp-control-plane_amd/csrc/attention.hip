// K5/K6: unified paged, causal, GQA attention for ragged batches (prefill,
// extend/jump-forward chunks and single-token decode in ONE kernel family).
//
// Layouts
//   q       [T, Hq, D]            rotated queries (rope_kv output)
//   k/v     [num_blocks, Hkv, 64, D]  paged cache, block = one 64-key tile
//   out     [T, Hq, D]
// Work item = (sequence, q-tile of QT tokens) x kv-head.  All G = Hq/Hkv query
// heads that share a kv head are processed together, so each K/V tile is read
// once per group (GQA), and the 16 MFMA rows of a wave are (16/G tokens) x G heads.
//
// Math per wave (D = 128, v_mfma_f32_16x16x32_bf16):
//   S^T[key][qrow] = K . Q^T  (K from LDS as the A operand, Q in registers as B)
//   -> every lane owns one query row (lane&15): the online-softmax rescale of O
//      is a per-lane scalar, row max/sum need two xor-shuffles (16, 32);
//   O^T[d][qrow] += V^T . P^T with P^T taken straight from the S^T accumulators
//      (key order permuted identically in both operands,
//      cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's
//      operand") and V^T read with ds_read_b64_tr_b16 (T10).
// K/V tiles: global_load_lds_dwordx4 into a double-buffered LDS ring with the
// 256-B-row XOR swizzle chunk ^= row&15 on source and read (tools/lds_banks.py).
//
// Split-KV (K6, KSPLIT): a decode step of few sequences with long contexts has
// few work items (one 1-wave item per sequence and kv head: batch 1 on 8B is 8
// workgroups on 256 CUs).  Such steps split each item's key range over
// gridDim.z workgroups; each writes its normalised fp32 partial O and its
// log2-sum-exp (split 0 folds in the cascade prefix partial), and
// attn_split_combine merges the splits with LSE weights.
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int D = 128;
constexpr int KT = 64;                        // keys per tile == cache block size
constexpr int TILE = KT * D;                  // bf16 elements per K or V tile (16 KiB)
typedef __attribute__((ext_vector_type(4))) short s16x4;

DEV bf16x4 tr_read(const bf16* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// Block-table entries of a key walk, 64 tiles per VGPR (lane i: tile base + i),
// read back with v_readlane.  Reading bt[kt + 1] inside the loop put a global
// load and its vmcnt(0) in front of every tile's DMA: two dependent memory
// round trips per key tile (table entry, then K / V) instead of one.  One
// load per 64 tiles, issued before the first DMA.
struct BtLanes {
  const int* bt;
  int end, base, v;
  DEV BtLanes(const int* bt_, int kt0, int end_) : bt(bt_), end(end_), base(kt0) { fill(); }
  DEV void fill() {
    const int i = base + (int)(threadIdx.x & 63);
    v = i < end ? bt[i] : 0;
  }
  DEV int operator()(int kt) {         // kt uniform, non-decreasing, < end
    if (kt - base >= 64) {
      base = kt;
      fill();
    }
    return __builtin_amdgcn_readlane(v, kt - base);
  }
};

struct AttnArgs {
  const bf16* q;
  const bf16* kc;
  const bf16* vc;
  bf16* out;
  const int* q_start;
  const int* q_len;
  const int* ctx_len;
  const int* block_table;
  int max_blocks;
  const int* work_seq;
  const int* work_q0;
  int Hq, Hkv;
  float scale_log2;
  // cascade (shared-prefix) attention
  const int* kv_begin;     // MODE 0: per-sequence first key (multiple of 64) or null
  const bf16* pre_o;       // MODE 0: normalised prefix partial O [T, Hq, D] to merge
  const float* pre_lse;    // MODE 0: its log2-sum-exp [T, Hq]
  float* lse_out;          // MODE 1: log2-sum-exp of the prefix partial
  // split-KV (KSPLIT): partials [nsplit][rows][D] fp32 and [nsplit][rows] LSE
  float* split_o;
  float* split_lse;
  int rows;                // T * Hq
  const int* pre_bt;       // MODE 1: block table of the shared prefix
  int pre_keys;            // MODE 1: prefix keys (multiple of 64)
  int pre_tokens;          // MODE 1: query tokens [0, pre_tokens) of the flat batch
  // MODE 1 inside a captured hipGraph: device [pre_tokens, pre_keys] read by
  // the kernel (the grid covers the bucket's token capacity; items past
  // pre_tokens exit, pre_tokens = 0 = no cascade this step)
  const int* pre_dims;
  // MODE 0, concurrent cascade: rows whose sequence starts past the prefix
  // (kv_begin > 0) write their own normalised O and its LSE here instead of
  // merging the prefix partial (which is computed at the same time on a side
  // stream); attn_cascade_merge combines the two afterwards
  float* own_lse;
  // MODE 1: grid (Hkv, token blocks) instead of (token blocks, Hkv), so that
  // block id % 8 (the XCD) is the kv head when Hkv = 8: each XCD's L2 then
  // holds one head's prefix K/V (352 KiB) instead of all eight
  int head_major;
  // shared-prefix pass: lazy max rescaling (MCP_ATTN_LAZY_RESCALE) - the
  // running max and the O / row-sum rescale are updated only when some row of
  // the wave's tile grows its max by more than LAZY_T (log2 units); otherwise
  // the scores are exponentiated against the stale max (p <= 2^LAZY_T)
  int lazy;
  // MIXED split launch (split-KV steps): blocks [0, nwork4) run the 4-wave
  // list (work_seq / work_q0), blocks [nwork4, ...) the 1-wave list
  // (work_seq1 / work_q01) as 4-wave blocks whose waves 1-3 hold no rows;
  // split_cnt (per block x kv head arrival tickets, zero between launches):
  // the last split to arrive merges every split's partial (no combine kernel)
  const int* work_seq1;
  const int* work_q01;
  int nwork4;
  int* split_cnt;
};

// Fused split-KV combine (MIXED launches).  Every split writes its
// normalised fp32 partial O and its log2-sum-exp write-through (sc1 buffer
// stores), drains them, and lane 0 takes the (block, kv head) ticket; the
// split whose ticket is the last merges all partials with LSE weights (sc1
// loads: the hand-off of MI355X_MICROARCH.md "Valid forms", row 1 - the same
// protocol as gemm_stream.hip's split-K) and writes the bf16 rows.  Split 0
// folds in the cascade prefix partial exactly as the unfused KSPLIT path.
// Every wave reaches both barriers (rows without a query are predicated off,
// never returned early).
template <int NW, int G>
DEV void split_fused_epilogue(const AttnArgs& a, f32x4 (&o)[8], float m_run, float l_tot,
                              bool qvalid, size_t row, int s, int fq, bf16* smem) {
  const int nz = gridDim.z, z = blockIdx.z;
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  float lse = l_tot > 0.f ? m_run + __log2f(l_tot) : -INFINITY;
  const bool merge_pre = a.pre_o != nullptr && a.kv_begin != nullptr && a.kv_begin[s] > 0;
  float wa = 0.f, wb = 1.f;
  // the prefix partial's LSE and 8 row pieces, loaded together before any
  // store (a load per dt behind a runtime test waits vmcnt(0) after each)
  bf16x4 pa[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) pa[dt] = bf16x4{};
  if (z == 0 && merge_pre && qvalid) {
    const bf16* pp = a.pre_o + row * D + 4 * fq;
    const float lse_a = a.pre_lse[row];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) pa[dt] = *reinterpret_cast<const bf16x4*>(pp + dt * 16);
    const float mx = fmaxf(lse_a, lse);
    const float ea = fexp2(lse_a - mx), eb = lse == -INFINITY ? 0.f : fexp2(lse - mx);
    wa = ea / (ea + eb);
    wb = eb / (ea + eb);
    lse = mx + __log2f(ea + eb);
  }
  const auto rso = __builtin_amdgcn_make_buffer_rsrc(a.split_o, (short)0, 0x7FFFFFFF, 0x00020000);
  const auto rsl = __builtin_amdgcn_make_buffer_rsrc(a.split_lse, (short)0, 0x7FFFFFFF, 0x00020000);
  if (qvalid) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      f32x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = o[dt][r] * inv * wb + (float)pa[dt][r] * wa;
      o[dt] = w;                                      // this split's partial, kept for the merge
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, w), rso,
          (unsigned)((((size_t)z * a.rows + row) * D + 4 * fq + 16 * dt) * 4), 0, 16);
    }
    if (fq == 0)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, lse), rsl,
                                            (unsigned)(((size_t)z * a.rows + row) * 4), 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                   // every wave's partial is out
  int* flag = reinterpret_cast<int*>(smem);          // the K/V ring is free after the loop
  if (threadIdx.x == 0) {
    int* cnt = a.split_cnt + (size_t)blockIdx.x * gridDim.y + blockIdx.y;
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nz - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag || !qvalid) return;
  // ---- last arriver: LSE-weighted sum over the splits, this lane's row.
  //      Every split (its own too) is read back from the workspace, in split
  //      order - deterministic whichever split arrives last - with the loads
  //      of 8 (LSE) / 4 (O) splits in flight instead of one L2 round trip each
  float mx = -INFINITY;
#pragma unroll 8
  for (int j = 0; j < nz; ++j)
    mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                       rsl, (unsigned)(((size_t)j * a.rows + row) * 4), 0, 16)));
  const float mu = mx == -INFINITY ? 0.f : mx;
  float den = 0.f;
  f32x4 acc[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int j = 0; j < nz; ++j) {
    const float lj = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
        rsl, (unsigned)(((size_t)j * a.rows + row) * 4), 0, 16));
    f32x4 pj[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      pj[dt] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
          rso, (unsigned)((((size_t)j * a.rows + row) * D + 4 * fq + 16 * dt) * 4), 0, 16));
    const float wj = lj == -INFINITY ? 0.f : fexp2(lj - mu);   // 0 for empty splits
    den += wj;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) acc[dt] += pj[dt] * wj;
  }
  const float dinv = den > 0.f ? 1.f / den : 0.f;
  if (a.own_lse != nullptr && fq == 0 && a.kv_begin != nullptr && a.kv_begin[s] > 0)
    a.own_lse[row] = den > 0.f ? mu + __log2f(den) : -INFINITY;
  bf16* op = a.out + row * D + 4 * fq;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    bf16x4 w;
#pragma unroll
    for (int r = 0; r < 4; ++r) w[r] = (bf16)(acc[dt][r] * dinv);
    *reinterpret_cast<bf16x4*>(op + dt * 16) = w;
  }
}

// MODE 0: per (sequence, q-tile) work item, causal over keys
//         [kv_begin[s], ctx_len[s]); merges the prefix partial when present.
// MODE 1: shared-prefix pass: the flat query tokens [0, pre_tokens) of every
//         sequence that shares one registry prefix, 16-token tiles that mix
//         sequences (they attend to the same K/V), no mask (every query sits
//         after the prefix).  Writes normalised O and its LSE.
template <int NW, int G, int MODE, int NBUF_ = 0, bool KSPLIT = false, int WPE = 1,
          bool MIXED = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void attn_kernel(const AttnArgs a) {
  static_assert(!MIXED || (NW == 4 && MODE == 0 && KSPLIT), "mixed lists: 4-wave split items");
  constexpr int TPW = 16 / G;                 // tokens per wave
  constexpr int QT = NW * TPW;                // tokens per work item
  constexpr int PIECES = 2 * TILE * 2 / 1024; // 1 KiB pieces of the K and V tiles (32)
  static_assert(PIECES % NW == 0, "pieces split evenly");
  // 1-wave (decode) items are latency-bound: one 32 KiB K|V buffer instead of
  // two lets 5 instead of 2 of them share a CU (LDS 160 KiB)
  constexpr int NBUF = NBUF_ > 0 ? NBUF_ : (NW == 1 ? 1 : 2);
  __shared__ __attribute__((aligned(16))) bf16 smem[NBUF * 2 * TILE];   // [buf][K|V][64][128]

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool hm = MODE == 1 && a.head_major;
  const int kvh = hm ? blockIdx.x : blockIdx.y;
  const int qblk = hm ? blockIdx.y : blockIdx.x;
  const int fr = lane & 15, fq = lane >> 4;
  const int head = kvh * G + fr % G;
  const int Hq = a.Hq, Hkv = a.Hkv;

  int s = 0, qs, ql, cl, tok, qpos, kt0, ntiles;
  int kv_stop = 1 << 30;                                  // MODE 0: the item's last key + 1
  bool qvalid;
  const int* bt;
  if (MODE == 1) {
    const int pre_tokens = a.pre_dims ? a.pre_dims[0] : a.pre_tokens;
    const int pre_keys = a.pre_dims ? a.pre_dims[1] : a.pre_keys;
    if (qblk * QT >= pre_tokens) return;                 // whole block idle (before any barrier)
    tok = qblk * QT + wave * TPW + fr / G;                // flat token index
    qvalid = tok < pre_tokens;
    qs = 0;
    ql = pre_tokens;
    cl = pre_keys;
    qpos = 1 << 30;                                       // no causal limit inside the prefix
    kt0 = 0;
    ntiles = pre_keys / KT;
    bt = a.pre_bt;
    if constexpr (KSPLIT) {                               // this split's share of the prefix tiles
      const int span = ntiles, z = blockIdx.z, nz = gridDim.z;
      kt0 = span * z / nz;
      ntiles = span * (z + 1) / nz;
    }
  } else {
    int q0, item_waves = NW;
    if constexpr (MIXED) {
      const int b = blockIdx.x;
      const bool wide = b < a.nwork4;
      s = wide ? a.work_seq[b] : a.work_seq1[b - a.nwork4];
      q0 = wide ? a.work_q0[b] : a.work_q01[b - a.nwork4];
      item_waves = wide ? NW : 1;
    } else {
      s = a.work_seq[blockIdx.x];
      q0 = a.work_q0[blockIdx.x];
    }
    qs = a.q_start[s];
    ql = a.q_len[s];
    cl = a.ctx_len[s];
    bt = a.block_table + (size_t)s * a.max_blocks;
    tok = q0 + wave * TPW + fr / G;                       // index inside the query span
    qvalid = tok < ql && wave < item_waves;
    qpos = cl - ql + tok;
    const int last_tok = min(q0 + item_waves * TPW, ql) - 1;
    const int kv_end = cl - ql + last_tok + 1;
    kv_stop = kv_end;
    ntiles = (kv_end + KT - 1) / KT;
    kt0 = a.kv_begin ? a.kv_begin[s] / KT : 0;
    if constexpr (KSPLIT) {                               // this split's share of the tiles
      const int span = max(ntiles - kt0, 0), z = blockIdx.z, nz = gridDim.z;
      const int b0 = kt0 + span * z / nz, b1 = kt0 + span * (z + 1) / nz;
      kt0 = b0;
      ntiles = b1;
    }
  }

  // Q fragments (B operand): lane holds Q[row fr][d = 32ks + 8fq + j]
  bf16x8 qf[4];
  {
    const bf16* qp = a.q + ((size_t)(qs + (qvalid ? tok : 0)) * Hq + head) * D + 8 * fq;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 32 * ks);
      if (!qvalid) qf[ks] = bf16x8{};
    }
  }

  // staging: piece p covers rows 4p..4p+3 of the K (p<16) or V (p>=16) tile.
  // A sequence's last tile is read only up to its last key: pieces wholly
  // past it are not fetched (HBM bytes the per-request pass - bandwidth
  // bound - would otherwise spend on rows every query masks); their V rows
  // are zeroed in LDS instead (P is 0 there, and 0 x stale LDS could be NaN),
  // their K rows stay stale (those scores are masked before the softmax)
  const int srow = lane >> 4;
  BtLanes bt_at(bt, kt0, ntiles);
  auto stage = [&](int kt, int buf) {
    const size_t blk = (size_t)bt_at(kt);
    const bf16* kb = a.kc + (blk * Hkv + kvh) * (size_t)TILE;
    const bf16* vb = a.vc + (blk * Hkv + kvh) * (size_t)TILE;
    bf16* base = smem + buf * 2 * TILE;
    const int rows_valid = kv_stop - kt * KT;              // >= 1 for a staged tile
    if (rows_valid >= KT) {
      // a full tile (every tile but a sequence's last): the straight DMA run
      // - per-piece tests here cost a one-wave item walking ~11 tiles 43 %
      // (one sequence, 700 keys: 27.0 vs 18.8 us, profiles/decode_unsplit_kernels_r6.md)
#pragma unroll
      for (int i = 0; i < PIECES / NW; ++i) {
        const int p = wave * (PIECES / NW) + i;
        const int tile = p >> 4, pr = p & 15;
        const int row = pr * 4 + srow;
        const int chunk = (lane & 15) ^ (row & 15);
        glds16((tile ? vb : kb) + row * D + chunk * 8, base + tile * TILE + pr * 512);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < PIECES / NW; ++i) {
      const int p = wave * (PIECES / NW) + i;
      const int tile = p >> 4, pr = p & 15;
      if (pr * 4 >= rows_valid) {                          // wave-uniform
        if (tile) *reinterpret_cast<u32x4*>(base + TILE + pr * 512 + lane * 8) = u32x4{0, 0, 0, 0};
        continue;
      }
      const int row = pr * 4 + srow;
      const int chunk = (lane & 15) ^ (row & 15);
      const bf16* src = (tile ? vb : kb) + row * D + chunk * 8;
      glds16(src, base + tile * TILE + pr * 512);
    }
  };

  f32x4 o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_part = 0.f;

  if (NBUF == 2 && kt0 < ntiles) stage(kt0, 0);
  if (NBUF == 2) __syncthreads();
  for (int kt = kt0; kt < ntiles; ++kt) {
    const int cur = NBUF == 2 ? (kt - kt0) & 1 : 0;
    if (NBUF == 1) {
      stage(kt, 0);
      __syncthreads();             // its fence drains the LDS-DMA (vmcnt(0))
    } else if (kt + 1 < ntiles) {
      stage(kt + 1, cur ^ 1);
    }
    const bf16* Kl = smem + cur * 2 * TILE;
    const bf16* Vl = Kl + TILE;

    // ---- S^T = K Q^T : 4 key sub-tiles x 4 d-steps
    f32x4 sacc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sacc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = nt * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int c = ks * 4 + fq;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kl + row * D + ((c ^ (row & 15)) << 3));
        sacc[nt] = mfma16x16x32(kf, qf[ks], sacc[nt]);
      }
    }
    // ---- mask + online softmax (this lane: query row fr, keys 16nt + 4fq + r)
    float tmax = -INFINITY;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * KT + nt * 16 + fq * 4 + r;
        // unscaled (max commutes with the positive scale; one fma per score below)
        const float v = (key <= qpos && key < cl) ? sacc[nt][r] : -INFINITY;
        sacc[nt][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax * a.scale_log2);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = fexp2(m_run - m_use);
    m_run = m_new;
    float psum = 0.f;
    bf16x8 pf[2];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fexp2(fmaf(sacc[nt][r], a.scale_log2, -m_use));
        psum += p;
        pf[nt >> 1][(nt & 1) * 4 + r] = (bf16)p;
      }
    l_part = l_part * alpha + psum;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;

    // ---- O^T += V^T P^T  (V^T via transposed LDS reads, permuted key order)
    const int tq = (lane & 15) >> 2, tp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int col = dt * 16 + tp * 4;
      const int chunk = col >> 3, half = (col & 7);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int key0 = k2 * 32 + fq * 4 + tq;
        const int key1 = key0 + 16;
        const bf16x4 v0 = tr_read(Vl + key0 * D + ((chunk ^ (key0 & 15)) << 3) + half);
        const bf16x4 v1 = tr_read(Vl + key1 * D + ((chunk ^ (key1 & 15)) << 3) + half);
        const bf16x8 vf = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        o[dt] = mfma16x16x32(vf, pf[k2], o[dt]);
      }
    }
    __syncthreads();
  }

  // ---- normalise and store: lane holds O[row fr][d = 16dt + 4fq + r]
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if constexpr (MIXED) {
    split_fused_epilogue<NW, G>(a, o, m_run, l_tot, qvalid, (size_t)(qs + (qvalid ? tok : 0)) * Hq + head,
                                s, fq, smem);
    return;
  }
  if (!qvalid) return;
  const size_t row = (size_t)(qs + tok) * Hq + head;
  float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if constexpr (KSPLIT) {
    // normalised partial + its LSE; split 0 also carries the cascade prefix.
    // The prefix partial's LSE and its 8 row pieces are loaded together, in
    // one branch, before any store: a load per dt behind the `pp` test made
    // hipcc wait vmcnt(0) after each (8 dependent round trips per item)
    float lse = l_tot > 0.f ? m_run + __log2f(l_tot) : -INFINITY;
    float wa = 0.f, wb = 1.f;
    const bool merge = blockIdx.z == 0 && a.pre_o != nullptr && a.kv_begin != nullptr &&
                       a.kv_begin[s] > 0;
    bf16x4 pa[8];
    if (merge) {
      const bf16* pp = a.pre_o + row * D + 4 * fq;
      const float lse_a = a.pre_lse[row];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) pa[dt] = *reinterpret_cast<const bf16x4*>(pp + dt * 16);
      const float mx = fmaxf(lse_a, lse);
      const float ea = fexp2(lse_a - mx), eb = lse == -INFINITY ? 0.f : fexp2(lse - mx);
      wa = ea / (ea + eb);
      wb = eb / (ea + eb);
      lse = mx + __log2f(ea + eb);
    } else {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) pa[dt] = bf16x4{};
    }
    float* po32 = a.split_o + ((size_t)blockIdx.z * a.rows + row) * D + 4 * fq;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      f32x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = o[dt][r] * inv * wb + (float)pa[dt][r] * wa;
      *reinterpret_cast<f32x4*>(po32 + dt * 16) = w;
    }
    if (fq == 0) a.split_lse[(size_t)blockIdx.z * a.rows + row] = lse;
    return;
  }
  float wa = 0.f, wb = 1.f;
  bool merge = false;
  bf16x4 pa[8];
  if (MODE == 0 && a.own_lse != nullptr && a.kv_begin != nullptr && a.kv_begin[s] > 0) {
    if (fq == 0) a.own_lse[row] = l_tot > 0.f ? m_run + __log2f(l_tot) : -INFINITY;
  } else if (MODE == 0 && a.kv_begin != nullptr && a.kv_begin[s] > 0) {
    // merge with the shared-prefix partial: weights from the two log2-sum-exps.
    // Its LSE and all 8 row pieces are loaded together before any store (a
    // load per dt behind a runtime test waited vmcnt(0) after each one)
    merge = true;
    const bf16* po = a.pre_o + row * D + 4 * fq;
    const float lse_a = a.pre_lse[row];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) pa[dt] = *reinterpret_cast<const bf16x4*>(po + dt * 16);
    const float lse_b = m_run + __log2f(l_tot);
    const float mx = fmaxf(lse_a, lse_b);
    wa = fexp2(lse_a - mx);
    wb = fexp2(lse_b - mx);
    const float den = 1.f / (wa + wb);
    wa *= den;
    wb *= den;
  }
  if (MODE == 1 && fq == 0) a.lse_out[row] = m_run + __log2f(l_tot);
  bf16* op = a.out + row * D + 4 * fq;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    bf16x4 w;
    if (merge) {
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[dt][r] * inv * wb + (float)pa[dt][r] * wa);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[dt][r] * inv);
    }
    *reinterpret_cast<bf16x4*>(op + dt * 16) = w;
  }
}

// Shared-prefix pass with RT row tiles per wave.  The one-tile form
// (attn_kernel MODE 1) reads the whole 32 KiB K|V tile from LDS per 16 query
// rows: 1 KiB of LDS reads per 16x16x32 MFMA, so the four SIMDs of a CU ask
// for ~4x the LDS port at MFMA peak and the pass ran at ~0.5 PF/s.  Here each
// K fragment (S^T = K Q^T) and each transposed V fragment (O^T += V^T P^T)
// read from LDS feeds RT MFMAs, one per row tile, which cuts the LDS bytes
// per FLOP by RT.  Every query of the pass sits after the prefix, so there is
// no mask (pre_keys is a multiple of 64).  Same row layout, online softmax,
// swizzled double-buffered LDS-DMA ring and outputs (normalised O + LSE) as
// MODE 1; the key-split form for few tokens stays on attn_kernel.
//
// PP (ping-pong, 8 waves): waves 0-3 and 4-7 - one of each per SIMD - run the
// tile loop half a phase apart.  Group A does QK^T, softmax, PV of tile kt
// between two barriers; group B does softmax + PV of tile kt - 1, then QK^T of
// tile kt.  So while one wave of a SIMD issues MFMAs the other issues the
// softmax VALU, instead of both waiting on the same unit (in lock step, the
// two waves' MFMA, VALU and LDS-read phases each took ~1/3 of a tile step and
// did not overlap; profiles/attention_tuning.md).  B reads the V tile of the
// previous step while the next tile is staged, so the ring has 3 buffers
// (96 KiB); every wave passes the same barriers.
constexpr float LAZY_T = 8.f;                // lazy rescale: p <= 2^8 against a stale max

// SW: the K|V image's 16-B chunk swizzle.  false: chunk ^ (row & 15) (the
// image of attn_kernel); true: chunk ^ ((row & 7) << 1), which keeps the K
// row reads (ds_read_b128) conflict-free and makes the transposed V reads
// (ds_read_b64_tr_b16: a 32-lane half reads 8 consecutive keys) conflict-free
// too - 2-way on the first image (tools/lds_banks.py; round-5 PMC: LDS
// bank-conflict cycles 2.9 M against 2.6 M active on this pass)
template <int NW, int G, int RT, bool PP = false, bool SW = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(RT >= 4 ? 1 : 2)))
void attn_prefix_kernel(const AttnArgs a) {
  static_assert(!PP || NW == 8, "ping-pong: two groups of 4 waves");
  constexpr int TPT = 16 / G;                 // tokens per 16-row tile
  constexpr int QT = NW * RT * TPT;           // tokens per block
  constexpr int PIECES = 2 * TILE * 2 / 1024; // 1 KiB pieces of the K and V tiles (32)
  constexpr int NB = PP ? 3 : 2;              // K|V ring depth
  static_assert(PIECES % NW == 0, "pieces split evenly");
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * 2 * TILE];   // [buf][K|V][64][128]

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kvh = a.head_major ? blockIdx.x : blockIdx.y;
  const int qblk = a.head_major ? blockIdx.y : blockIdx.x;
  const int fr = lane & 15, fq = lane >> 4;
  const int head = kvh * G + fr % G;
  const int Hq = a.Hq, Hkv = a.Hkv;
  const int pre_tokens = a.pre_dims ? a.pre_dims[0] : a.pre_tokens;
  const int pre_keys = a.pre_dims ? a.pre_dims[1] : a.pre_keys;
  if (qblk * QT >= pre_tokens) return;        // whole block idle (before any barrier)
  const int ntiles = pre_keys / KT;

  int tok[RT];
  bf16x8 qf[RT][4];                           // B operands: Q[row fr][d = 32ks + 8fq + j]
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    tok[r] = qblk * QT + (wave * RT + r) * TPT + fr / G;
    const bool v = tok[r] < pre_tokens;
    const bf16* qp = a.q + ((size_t)(v ? tok[r] : 0) * Hq + head) * D + 8 * fq;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[r][ks] = *reinterpret_cast<const bf16x8*>(qp + 32 * ks);
      if (!v) qf[r][ks] = bf16x8{};
    }
  }

  const int srow = lane >> 4;
  BtLanes bt_at(a.pre_bt, 0, ntiles);
  // Piece pr of a K or V tile is rows 4 pr + srow, the lane's 16-B chunk at
  // chunk ^ (row & 15).  The 8-wave lock-step form DMAs from 64-bit addresses
  // (global_load_lds); the 4-wave and ping-pong forms through per-tile buffer
  // resources with 4 per-lane offsets (the chunk depends on pr & 3 only, the
  // row step goes in soffset): one 64-bit address per piece kept
  // 2 x PIECES / NW VGPRs live across the loop and the 4-wave form spilled,
  // while the buffer form measured ~3 % slower on the 8-wave one (r5c7)
  constexpr bool BUF_DMA = NW == 4 || PP;
  auto pswz = [](int row) { return SW ? ((row & 7) << 1) : (row & 15); };
  unsigned voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) voff[i] = (unsigned)((srow * D + (((lane & 15) ^ pswz(4 * i + srow)) << 3)) * 2);
  auto stage = [&](int kt, int buf) {
    const size_t blk = (size_t)bt_at(kt);
    const size_t off = (blk * Hkv + kvh) * (size_t)TILE;
    bf16* base = smem + buf * 2 * TILE;
    if constexpr (BUF_DMA) {
      const auto rk = __builtin_amdgcn_make_buffer_rsrc((void*)(a.kc + off), (short)0, TILE * 2, 0x00020000);
      const auto rv = __builtin_amdgcn_make_buffer_rsrc((void*)(a.vc + off), (short)0, TILE * 2, 0x00020000);
#pragma unroll
      for (int i = 0; i < PIECES / NW; ++i) {
        const int p = wave * (PIECES / NW) + i;
        const int tile = p >> 4, pr = p & 15;
        auto* dst = (__attribute__((address_space(3))) void*)(base + tile * TILE + pr * 512);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(tile ? rv : rk, dst, 16, voff[pr & 3], pr * 4 * D * 2, 0, 0);
      }
    } else {
      const bf16* kb = a.kc + off;
      const bf16* vb = a.vc + off;
#pragma unroll
      for (int i = 0; i < PIECES / NW; ++i) {
        const int p = wave * (PIECES / NW) + i;
        const int tile = p >> 4, pr = p & 15;
        const int row = pr * 4 + srow;
        const int chunk = (lane & 15) ^ pswz(row);
        glds16((tile ? vb : kb) + row * D + chunk * 8, base + tile * TILE + pr * 512);
      }
    }
  };

  f32x4 o[RT][8];
  float m_run[RT], l_part[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[r][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run[r] = -INFINITY;
    l_part[r] = 0.f;
  }

  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const float c = a.scale_log2;
  // ---- S^T = K Q^T: each K fragment feeds the RT row tiles
  auto qk = [&](const bf16* Kl, f32x4 (&sacc)[RT][4]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int r = 0; r < RT; ++r) sacc[r][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = nt * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int cc = ks * 4 + fq;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kl + row * D + ((cc ^ pswz(row)) << 3));
#pragma unroll
        for (int r = 0; r < RT; ++r) sacc[r][nt] = mfma16x16x32(kf, qf[r][ks], sacc[r][nt]);
      }
    }
  };
  // ---- online softmax per row tile (lane: query row fr, keys 16nt + 4fq + r).
  //      The scores stay unscaled: the max commutes with the positive scale,
  //      and exp2(s c - m) is one fma + exp per score
  auto softmax = [&](f32x4 (&sacc)[RT][4], bf16x8 (&pf)[RT][2]) {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      float tmax = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) tmax = fmaxf(tmax, sacc[r][nt][e]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float m_new = fmaxf(m_run[r], tmax * c);
      // lazy: keep the stale max unless some row of this wave's tile grew it
      // by more than LAZY_T (wave-uniform test, so the rescale is skipped
      // for the whole wave - the softmax chain loses the exp and the 32 + 1
      // multiplies of the O / sum rescale on most tiles)
      const bool rescale = !a.lazy || __builtin_amdgcn_ballot_w64(m_new > m_run[r] + LAZY_T) != 0;
      float psum = 0.f;
      if (rescale) {
        const float alpha = fexp2(m_run[r] - m_new);
        m_run[r] = m_new;
        l_part[r] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[r][dt] *= alpha;
      }
      const float mu = m_run[r];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = fexp2(fmaf(sacc[r][nt][e], c, -mu));
          psum += p;
          pf[r][nt >> 1][(nt & 1) * 4 + e] = (bf16)p;
        }
      l_part[r] += psum;
    }
  };
  // ---- O^T += V^T P^T: each transposed V fragment feeds the RT row tiles
  auto pv = [&](const bf16* Vl, bf16x8 (&pf)[RT][2]) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int col = dt * 16 + tp * 4;
      const int chunk = col >> 3, half = (col & 7);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int key0 = k2 * 32 + fq * 4 + tq;
        const int key1 = key0 + 16;
        const bf16x4 v0 = tr_read(Vl + key0 * D + ((chunk ^ pswz(key0)) << 3) + half);
        const bf16x4 v1 = tr_read(Vl + key1 * D + ((chunk ^ pswz(key1)) << 3) + half);
        const bf16x8 vf = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int r = 0; r < RT; ++r) o[r][dt] = mfma16x16x32(vf, pf[r][k2], o[r][dt]);
      }
    }
  };

  f32x4 sacc[RT][4];
  bf16x8 pf[RT][2];
  if (ntiles > 0) stage(0, 0);
  __syncthreads();
  if constexpr (!PP) {
    for (int kt = 0; kt < ntiles; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < ntiles) stage(kt + 1, cur ^ 1);
      const bf16* Kl = smem + cur * 2 * TILE;
      qk(Kl, sacc);
      softmax(sacc, pf);
      pv(Kl + TILE, pf);
      __syncthreads();             // its fence also drains the next tile's LDS-DMA
    }
  } else {
    const bool lag = wave >= NW / 2;          // group B: half a phase behind
    int cur = 0, prev = 2;                    // ring slots of tiles kt and kt - 1
    for (int kt = 0; kt < ntiles; ++kt) {
      const int nxt = cur == 2 ? 0 : cur + 1;
      if (kt + 1 < ntiles) stage(kt + 1, nxt);   // slot of tile kt - 2: read by nobody now
      const bf16* Kl = smem + cur * 2 * TILE;
      if (!lag) {
        qk(Kl, sacc);
        softmax(sacc, pf);
        pv(Kl + TILE, pf);
      } else {
        if (kt > 0) {
          softmax(sacc, pf);                  // tile kt - 1's scores, from the last step
          pv(smem + prev * 2 * TILE + TILE, pf);
        }
        qk(Kl, sacc);
      }
      __syncthreads();             // tile kt + 1 landed; slot prev free for the next stage
      prev = cur;
      cur = nxt;
    }
    if (lag && ntiles > 0) {       // group B's last tile (nothing is staged any more)
      softmax(sacc, pf);
      pv(smem + prev * 2 * TILE + TILE, pf);
    }
  }

  // ---- normalise and store: lane holds O[row fr][d = 16dt + 4fq + e]
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    float l_tot = l_part[r] + __shfl_xor(l_part[r], 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (tok[r] >= pre_tokens) continue;
    const size_t row = (size_t)tok[r] * Hq + head;
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (fq == 0) a.lse_out[row] = m_run[r] + __log2f(l_tot);
    bf16* op = a.out + row * D + 4 * fq;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (bf16)(o[r][dt][e] * inv);
      *reinterpret_cast<bf16x4*>(op + dt * 16) = w;
    }
  }
}

// Merge of the split-KV partials of 1-wave items: one workgroup per (item,
// kv head) = 16 rows (TPW tokens x G heads).  Wave w takes splits w, w + 4,
// ...; lane = (row l & 15, 32-wide d slice).  Each wave keeps its own running
// max / weighted sum (loads of 4 splits in flight), then the 4 waves' partial
// results are merged through LDS.
template <int G, int NWI = 1>
__global__ __launch_bounds__(256) void attn_split_combine(const AttnArgs a, int nsplit) {
  // NWI = waves of the split items: a 4-wave item's 4 row groups of 16 are
  // merged by 4 consecutive workgroups
  constexpr int CW = 4;
  constexpr int TPW = 16 / G;
  __shared__ float red_m[CW][64], red_d[CW][64];
  __shared__ float red_o[CW][32][65];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, dq = lane >> 4;
  const int item = blockIdx.x / NWI, sub = blockIdx.x % NWI;
  const int s = a.work_seq[item];
  const int tok = a.work_q0[item] + sub * TPW + fr / G;
  const bool valid = tok < a.q_len[s];
  const int head = blockIdx.y * G + fr % G;
  const size_t row = (size_t)(a.q_start[s] + (valid ? tok : 0)) * a.Hq + head;
  float m = -INFINITY;
#pragma unroll 4
  for (int z = wave; z < nsplit; z += CW) m = fmaxf(m, a.split_lse[(size_t)z * a.rows + row]);
  float acc[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) acc[j] = 0.f;
  float den = 0.f;
  const float mu = m == -INFINITY ? 0.f : m;
#pragma unroll 4
  for (int z = wave; z < nsplit; z += CW) {
    const float w = fexp2(a.split_lse[(size_t)z * a.rows + row] - mu);   // 0 for empty splits
    den += w;
    const f32x4* p = reinterpret_cast<const f32x4*>(a.split_o + ((size_t)z * a.rows + row) * D + 32 * dq);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 v = p[j];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[4 * j + r] += w * v[r];
    }
  }
  red_m[wave][lane] = m;
  red_d[wave][lane] = den;
#pragma unroll
  for (int j = 0; j < 32; ++j) red_o[wave][j][lane] = acc[j];
  __syncthreads();
  if (wave != 0 || !valid) return;
  float mt = -INFINITY;
#pragma unroll
  for (int w = 0; w < CW; ++w) mt = fmaxf(mt, red_m[w][lane]);
  const float mtu = mt == -INFINITY ? 0.f : mt;
  float sc[CW], dt = 0.f;
#pragma unroll
  for (int w = 0; w < CW; ++w) {
    const float mw = red_m[w][lane];
    sc[w] = mw == -INFINITY ? 0.f : fexp2(mw - mtu);
    dt += sc[w] * red_d[w][lane];
  }
  const float inv = dt > 0.f ? 1.f / dt : 0.f;
  if (a.own_lse != nullptr && dq == 0 && a.kv_begin != nullptr && a.kv_begin[s] > 0)
    a.own_lse[row] = dt > 0.f ? mtu + __log2f(dt) : -INFINITY;
  bf16* op = a.out + row * D + 32 * dq;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bf16x8 o;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < CW; ++w) v += sc[w] * red_o[w][8 * j + r][lane];
      o[r] = (bf16)(v * inv);
    }
    *reinterpret_cast<bf16x8*>(op + 8 * j) = o;
  }
}

// Merge of the key-split prefix pass: rows [0, pre_tokens) x Hq, one thread
// per (row, 8 dims); writes the normalised bf16 prefix partial and its LSE
// exactly as the unsplit pass does (the per-sequence pass merges it next).
__global__ __launch_bounds__(256) void attn_prefix_combine(const AttnArgs a, int nsplit) {
  const int pre_tokens = a.pre_dims ? a.pre_dims[0] : a.pre_tokens;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long row = i / (D / 8);
  const int d0 = (int)(i % (D / 8)) * 8;
  if (row >= (long long)pre_tokens * a.Hq) return;
  float m = -INFINITY;
  for (int z = 0; z < nsplit; ++z) m = fmaxf(m, a.split_lse[(size_t)z * a.rows + row]);
  const float mu = m == -INFINITY ? 0.f : m;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float den = 0.f;
  for (int z = 0; z < nsplit; ++z) {
    const float w = fexp2(a.split_lse[(size_t)z * a.rows + row] - mu);   // 0 for empty splits
    den += w;
    const f32x4* p = reinterpret_cast<const f32x4*>(a.split_o + ((size_t)z * a.rows + row) * D + d0);
    const f32x4 v0 = p[0], v1 = p[1];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc[r] += w * v0[r];
      acc[4 + r] += w * v1[r];
    }
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  bf16x8 o;
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = (bf16)(acc[r] * inv);
  *reinterpret_cast<bf16x8*>(a.out + row * D + d0) = o;
  if (d0 == 0) a.lse_out[row] = den > 0.f ? mu + __log2f(den) : -INFINITY;
}

// Concurrent cascade: out[row] (the sequence's own-key partial, normalised,
// LSE own_lse) merged with the shared-prefix partial (pre_o, pre_lse) for the
// rows [0, pre_tokens) x Hq; one thread per (row, 8 dims).
__global__ __launch_bounds__(256) void attn_cascade_merge(const AttnArgs a) {
  const int pre_tokens = a.pre_dims ? a.pre_dims[0] : a.pre_tokens;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long row = i / (D / 8);
  const int d0 = (int)(i % (D / 8)) * 8;
  if (row >= (long long)pre_tokens * a.Hq) return;
  const float la = a.pre_lse[row], lb = a.own_lse[row];
  const float mx = fmaxf(la, lb);
  const float mu = mx == -INFINITY ? 0.f : mx;
  float wa = la == -INFINITY ? 0.f : fexp2(la - mu), wb = lb == -INFINITY ? 0.f : fexp2(lb - mu);
  const float den = wa + wb;
  wa = den > 0.f ? wa / den : 0.f;
  wb = den > 0.f ? wb / den : 0.f;
  const bf16x8 pa = *reinterpret_cast<const bf16x8*>(a.pre_o + row * D + d0);
  bf16x8* op = reinterpret_cast<bf16x8*>(a.out + row * D + d0);
  const bf16x8 pb = *op;
  bf16x8 o;
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = (bf16)((float)pa[r] * wa + (float)pb[r] * wb);
  *op = o;
}

template <int G>
void attn_dispatch(int nw, const AttnArgs& a, int nwork, hipStream_t s, int nsplit = 1) {
  // split items double-buffer their K/V tiles (one tile in flight while the
  // previous is consumed): 10-25 % faster than the single-buffer decode form
  // at 8k-128k (profiles/attention_splitkv.md)
  static const int split_bufs = getenv("MCP_ATTN_SPLIT_BUFS") ? atoi(getenv("MCP_ATTN_SPLIT_BUFS")) : 2;
  if (nw == 1 && nsplit > 1) {
    if (split_bufs == 2)
      attn_kernel<1, G, 0, 2, true><<<dim3(nwork, a.Hkv, nsplit), 64, 0, s>>>(a);
    else
      attn_kernel<1, G, 0, 0, true><<<dim3(nwork, a.Hkv, nsplit), 64, 0, s>>>(a);
    attn_split_combine<G><<<dim3(nwork, a.Hkv), 256, 0, s>>>(a, nsplit);
    return;
  }
  if (nw == 4 && nsplit > 1) {
    // 4-wave items (jump-forward spans) of a few long-context sequences
    attn_kernel<4, G, 0, 2, true><<<dim3(nwork, a.Hkv, nsplit), 256, 0, s>>>(a);
    attn_split_combine<G, 4><<<dim3(nwork * 4, a.Hkv), 256, 0, s>>>(a, nsplit);
    return;
  }
  const dim3 grid(nwork, a.Hkv);
  static const int nw1_bufs = getenv("MCP_ATTN_NW1_BUFS") ? atoi(getenv("MCP_ATTN_NW1_BUFS")) : 1;
  // 4-wave items single-buffered at <= 168 VGPRs (150 + 0 AGPRs, 3 waves per
  // SIMD): 3 blocks per CU (96 KiB LDS) instead of 2 double-buffered ones
  // (178 registers): per-request pass 3-6 % faster at 10-32 tokens per request,
  // equal at 6-8 (profiles/attention_tuning.md); MCP_ATTN_NW4_FORM=0 = old form
  static const int nw4_form = getenv("MCP_ATTN_NW4_FORM") ? atoi(getenv("MCP_ATTN_NW4_FORM")) : 1;
  if (nw == 1 && nw1_bufs == 2)
    attn_kernel<1, G, 0, 2><<<grid, 64, 0, s>>>(a);
  else if (nw == 1)
    attn_kernel<1, G, 0><<<grid, 64, 0, s>>>(a);
  else if (nw4_form == 1)
    attn_kernel<4, G, 0, 1, false, 3><<<grid, 256, 0, s>>>(a);
  else
    attn_kernel<4, G, 0><<<grid, 256, 0, s>>>(a);
}

// per-device arrival tickets of the fused split-KV launch (zeroed once here,
// at library load - never inside a graph capture; each last arriver re-arms
// its own ticket)
constexpr int SPLIT_CNT_MAX = 1 << 16;
int* g_split_cnt[64] = {};

int* split_counters() {
  int d = 0;
  (void)hipGetDevice(&d);
  return g_split_cnt[d & 63];
}

// waves per block of the shared-prefix pass: MCP_ATTN_PREFIX_NW = 4 / 8
// forces one; by default 4-wave blocks (half the tokens per block) when the
// 8-wave grid would not give every CU a block.  tools/bench_attention.py,
// 704-key prefix, 16 new tokens per request (prefix pass us, 8 / 4 waves):
// 8 requests 31.0 / 23.5, 36 32.6 / 25.3, 64 34.4 / 27.1, 128 39.0 / 41.6,
// 256 78.1 / 76.3; 8 tokens each: 36 31.6 / 24.0, 128 33.9 / 27.1
// (profiles/attention_tuning.md, round 3)
int prefix_nw(int tokens, int tok_per_block8, int hkv) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("MCP_ATTN_PREFIX_NW");
    forced = e ? atoi(e) : 0;
    if (forced != 4 && forced != 8) forced = 0;
  }
  if (forced) return forced;
  const long long blocks8 = (long long)((tokens + tok_per_block8 - 1) / tok_per_block8) * hkv;
  return blocks8 < gemm256_num_cus() ? 4 : 8;
}

// MCP_ATTN_PREFIX_PP=1: the ping-pong form of the 8-wave prefix pass (read
// per launch: the GPU tests compare the forms in one process)
static bool prefix_pp() {
  const char* e = getenv("MCP_ATTN_PREFIX_PP");
  return e && e[0] == '1';
}
// MCP_ATTN_PREFIX_SWZ=1: the conflict-free K|V image (attn_prefix_kernel SW)
// for the lock-step forms (read per launch: the tests compare both images)
static bool prefix_swz() {
  const char* e = getenv("MCP_ATTN_PREFIX_SWZ");
  return e && e[0] == '1';
}

// Shared-prefix pass: 8 waves per block (32 tokens x G heads) -> half the K/V
// tile staging per query of the 4-wave item and 4 waves per SIMD at 2 blocks/CU
template <int G>
void attn_prefix_dispatch(const AttnArgs& a, hipStream_t s, int nsplit = 1) {
  if (nsplit > 1) {
    // key-split prefix pass (few query tokens: the unsplit grid is a few
    // dozen workgroups each walking every prefix tile), then the merge
    constexpr int QT = 8 * (16 / G);
    const int nblk = (a.pre_tokens + QT - 1) / QT;
    const dim3 grid = a.head_major ? dim3(a.Hkv, nblk, nsplit) : dim3(nblk, a.Hkv, nsplit);
    attn_kernel<8, G, 1, 0, true><<<grid, 512, 0, s>>>(a);
    const long long n = (long long)a.pre_tokens * a.Hq * (D / 8);
    attn_prefix_combine<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a, nsplit);
    return;
  }
  // MCP_ATTN_PREFIX_RT: row tiles per wave of the prefix pass (2 = default,
  // 1 = the attn_kernel MODE 1 forms below, A/B)
  // (read per launch: the GPU tests compare the forms in one process)
  const char* rt_env = getenv("MCP_ATTN_PREFIX_RT");
  const int rt = rt_env ? atoi(rt_env) : 2;
  if (rt == 2 || rt == 4) {
    auto grid_for = [&](int qt) {
      const int nblk = (a.pre_tokens + qt - 1) / qt;
      return a.head_major ? dim3(a.Hkv, nblk) : dim3(nblk, a.Hkv);
    };
    if (rt == 4)
      attn_prefix_kernel<4, G, 4><<<grid_for(4 * 4 * (16 / G)), 256, 0, s>>>(a);
    else if (prefix_nw(a.pre_tokens, 8 * 2 * (16 / G), a.Hkv) == 4 && prefix_swz())
      attn_prefix_kernel<4, G, 2, false, true><<<grid_for(4 * 2 * (16 / G)), 256, 0, s>>>(a);
    else if (prefix_nw(a.pre_tokens, 8 * 2 * (16 / G), a.Hkv) == 4)
      attn_prefix_kernel<4, G, 2><<<grid_for(4 * 2 * (16 / G)), 256, 0, s>>>(a);
    else if (prefix_pp())
      attn_prefix_kernel<8, G, 2, true><<<grid_for(8 * 2 * (16 / G)), 512, 0, s>>>(a);
    else if (prefix_swz())
      attn_prefix_kernel<8, G, 2, false, true><<<grid_for(8 * 2 * (16 / G)), 512, 0, s>>>(a);
    else
      attn_prefix_kernel<8, G, 2><<<grid_for(8 * 2 * (16 / G)), 512, 0, s>>>(a);
    return;
  }
  if (prefix_nw(a.pre_tokens, 8 * (16 / G), a.Hkv) == 4) {
    constexpr int QT = 4 * (16 / G);
    const int nblk = (a.pre_tokens + QT - 1) / QT;
    const dim3 grid = a.head_major ? dim3(a.Hkv, nblk) : dim3(nblk, a.Hkv);
    attn_kernel<4, G, 1><<<grid, 256, 0, s>>>(a);
  } else {
    constexpr int QT = 8 * (16 / G);
    const int nblk = (a.pre_tokens + QT - 1) / QT;
    const dim3 grid = a.head_major ? dim3(a.Hkv, nblk) : dim3(nblk, a.Hkv);
    attn_kernel<8, G, 1><<<grid, 512, 0, s>>>(a);
  }
}

}  // namespace

int attn_tokens_per_item(int nw, int group) { return nw * (16 / group); }

// shared-prefix pass lazy rescaling: -1 = MCP_ATTN_LAZY_RESCALE (default 1:
// tools/bench_attention.py 16, same box alternated, prefix pass 77.7 / 78.3
// -> 75.3 / 75.7 us, headline within noise; profiles/attention_prefix_r6.md)
static int g_lazy_rescale = -1;
void attn_lazy_rescale(int on) { g_lazy_rescale = on; }

int* attn_split_counters() { return split_counters(); }

int attn_split_init() {
  int d = 0;
  (void)hipGetDevice(&d);
  if (g_split_cnt[d & 63]) return 0;
  int* p = nullptr;
  if (hipMalloc(&p, SPLIT_CNT_MAX * sizeof(int)) != hipSuccess) return 1;
  if (hipMemset(p, 0, SPLIT_CNT_MAX * sizeof(int)) != hipSuccess) return 1;
  (void)hipDeviceSynchronize();
  g_split_cnt[d & 63] = p;
  return 0;
}

#define ATTN_SWITCH_G(G_, CALL)                     \
  switch (G_) {                                     \
    case 1: { constexpr int GG = 1; CALL; } break;  \
    case 2: { constexpr int GG = 2; CALL; } break;  \
    case 4: { constexpr int GG = 4; CALL; } break;  \
    case 8: { constexpr int GG = 8; CALL; } break;  \
    case 16: { constexpr int GG = 16; CALL; } break; \
    default: return 3;                              \
  }

int launch_paged_attention(const void* q, const void* k_cache, const void* v_cache, void* out,
                           const int* q_start, const int* q_len, const int* ctx_len,
                           const int* block_table, int max_blocks, const int* work_seq,
                           const int* work_q0, int nwork, int nw, int Hq, int Hkv, int head_dim,
                           float scale, const int* kv_begin, const void* pre_o,
                           const float* pre_lse, hipStream_t s, int nsplit, float* split_o,
                           float* split_lse, int rows, float* own_lse) {
  if (head_dim != D) return 1;
  if (nw != 1 && nw != 4) return 2;
  if (nwork <= 0) return 0;
  if (nsplit > 1 && (!split_o || !split_lse)) return 4;
  AttnArgs a{};
  a.q = (const bf16*)q;
  a.kc = (const bf16*)k_cache;
  a.vc = (const bf16*)v_cache;
  a.out = (bf16*)out;
  a.q_start = q_start;
  a.q_len = q_len;
  a.ctx_len = ctx_len;
  a.block_table = block_table;
  a.max_blocks = max_blocks;
  a.work_seq = work_seq;
  a.work_q0 = work_q0;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.kv_begin = kv_begin;
  a.pre_o = (const bf16*)pre_o;
  a.pre_lse = pre_lse;
  a.split_o = split_o;
  a.split_lse = split_lse;
  a.rows = rows;
  a.own_lse = own_lse;
  ATTN_SWITCH_G(Hq / Hkv, attn_dispatch<GG>(nw, a, nwork, s, nsplit))
  return 0;
}

// Split-KV step in ONE launch: both work lists (4-wave items, then 1-wave
// items run as 4-wave blocks) x Hkv x nsplit, the combine fused in (last
// arriver per item and kv head).  Returns nonzero (caller falls back to the
// per-list launches + attn_split_combine) when the tickets or the 2 GiB
// buffer range of the partials do not cover the launch.
int launch_paged_attention_mixed(const void* q, const void* k_cache, const void* v_cache,
                                 void* out, const int* q_start, const int* q_len,
                                 const int* ctx_len, const int* block_table, int max_blocks,
                                 const int* work_seq4, const int* work_q04, int nwork4,
                                 const int* work_seq1, const int* work_q01, int nwork1, int Hq,
                                 int Hkv, int head_dim, float scale, const int* kv_begin,
                                 const void* pre_o, const float* pre_lse, hipStream_t s,
                                 int nsplit, float* split_o, float* split_lse, int rows,
                                 float* own_lse) {
  if (head_dim != D) return 1;
  if (nsplit < 2 || !split_o || !split_lse) return 4;
  const int nitems = nwork4 + nwork1;
  if (nitems <= 0) return 0;
  int* cnt = split_counters();
  if (!cnt || (long long)nitems * Hkv > SPLIT_CNT_MAX) return 5;
  if ((long long)nsplit * rows * D * 4 >= (1ll << 31)) return 6;
  AttnArgs a{};
  a.q = (const bf16*)q;
  a.kc = (const bf16*)k_cache;
  a.vc = (const bf16*)v_cache;
  a.out = (bf16*)out;
  a.q_start = q_start;
  a.q_len = q_len;
  a.ctx_len = ctx_len;
  a.block_table = block_table;
  a.max_blocks = max_blocks;
  a.work_seq = work_seq4;
  a.work_q0 = work_q04;
  a.work_seq1 = work_seq1;
  a.work_q01 = work_q01;
  a.nwork4 = nwork4;
  a.split_cnt = cnt;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.kv_begin = kv_begin;
  a.pre_o = (const bf16*)pre_o;
  a.pre_lse = pre_lse;
  a.split_o = split_o;
  a.split_lse = split_lse;
  a.rows = rows;
  a.own_lse = own_lse;
  const dim3 grid(nitems, Hkv, nsplit);
  ATTN_SWITCH_G(Hq / Hkv, (attn_kernel<4, GG, 0, 2, true, 1, true><<<grid, 256, 0, s>>>(a)))
  return 0;
}

int launch_prefix_attention(const void* q, const void* k_cache, const void* v_cache, void* out,
                            float* lse_out, const int* pre_bt, int pre_keys, int pre_tokens,
                            int Hq, int Hkv, int head_dim, float scale, hipStream_t s,
                            const int* pre_dims, int nsplit, float* split_o, float* split_lse) {
  // pre_dims != null: pre_tokens is the grid's token capacity, the actual
  // [pre_tokens, pre_keys] are read on the device (hipGraph replay)
  if (head_dim != D) return 1;
  if (!pre_dims && pre_keys % KT) return 2;
  if (pre_tokens <= 0 || (!pre_dims && pre_keys <= 0)) return 0;
  AttnArgs a{};
  a.q = (const bf16*)q;
  a.kc = (const bf16*)k_cache;
  a.vc = (const bf16*)v_cache;
  a.out = (bf16*)out;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.lse_out = lse_out;
  a.pre_bt = pre_bt;
  a.pre_keys = pre_keys;
  a.pre_tokens = pre_tokens;
  a.pre_dims = pre_dims;
  if (nsplit > 1 && (!split_o || !split_lse)) return 4;
  a.split_o = split_o;
  a.split_lse = split_lse;
  a.rows = pre_tokens * Hq;
  // MCP_ATTN_PREFIX_HEAD_MAJOR=0: token-major grid (A/B)
  static const int head_major = getenv("MCP_ATTN_PREFIX_HEAD_MAJOR") ? atoi(getenv("MCP_ATTN_PREFIX_HEAD_MAJOR")) : 1;
  a.head_major = head_major;
  if (g_lazy_rescale < 0)
    g_lazy_rescale = getenv("MCP_ATTN_LAZY_RESCALE") ? atoi(getenv("MCP_ATTN_LAZY_RESCALE")) : 1;
  a.lazy = g_lazy_rescale;
  ATTN_SWITCH_G(Hq / Hkv, attn_prefix_dispatch<GG>(a, s, nsplit))
  return 0;
}

// concurrent cascade: merge the own-key partial in out with the prefix partial
int launch_cascade_merge(void* out, const float* own_lse, const void* pre_o, const float* pre_lse,
                         int pre_tokens, const int* pre_dims, int Hq, int head_dim, hipStream_t s) {
  if (head_dim != D) return 1;
  if (pre_tokens <= 0) return 0;
  AttnArgs a{};
  a.out = (bf16*)out;
  a.own_lse = (float*)own_lse;
  a.pre_o = (const bf16*)pre_o;
  a.pre_lse = pre_lse;
  a.pre_tokens = pre_tokens;
  a.pre_dims = pre_dims;
  a.Hq = Hq;
  const long long n = (long long)pre_tokens * Hq * (D / 8);
  attn_cascade_merge<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a);
  return 0;
}
