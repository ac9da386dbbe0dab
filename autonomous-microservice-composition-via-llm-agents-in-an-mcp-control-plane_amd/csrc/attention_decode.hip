// K6 (v2): split-KV attention for decode-sized steps - few sequences, a few
// new query tokens each (single intent, low-QPS serving: config 2 / 5).
//
// Measured first (tools/bench_attention_decode.py, hipGraph-replayed,
// profiles/attention_decode_r3_baseline.jsonl): the work-list kernel
// (attention.hip, MIXED split launch) takes ~10-12 us warm and 19.4 us in the
// config-2 trace for one sequence over 700-1100 keys (4.5 MB of K/V: the HBM
// time is < 1 us; an empty kernel in a graph costs 2.2 us).  The time is a
// chain of dependent memory round trips - work item -> sequence sizes ->
// block table -> K/V DMA -> next tile's DMA -> partial / ticket / merge -
// each an HBM miss during serving (the weights streamed since the last step
// evicted everything).  Here:
//
//  * the key tiles of a block are fixed by its grid position alone: block z
//    covers absolute tiles [z C, z C + C), C = 4 x tpw, wave w the tiles
//    z C + w + 4 j.  So the block-table entry of a wave's first tile is read
//    in the same round trip as the sequence's sizes, and its K / V loads and
//    the Q loads go out together in the next;
//  * the 4 waves of a block work on 4 different tiles at once: K straight
//    into registers as the MFMA A operand (16 x 16 B per lane), V by LDS-DMA
//    into the wave's own 16 KiB buffer (no barrier between a wave's DMA and
//    its transposed reads; 64 KiB per block, two blocks per CU);
//  * one 16-row tile (16 / G tokens x G heads) per block: a 4-wave work item
//    (16 x 4 / G tokens) runs as 4 blocks, so no wave carries several row
//    tiles through the softmax chain;
//  * the 4 waves' (max, sum, O) merge through LDS (the V buffers hold the
//    fp32 O afterwards), then - only when the item spans more than one block
//    - the blocks merge by the last-arriver protocol of attention.hip (sc1
//    partials + agent-scope ticket, block order, so the result does not
//    depend on which block arrives last); the cascade prefix partial, if any,
//    is folded in once by whoever writes the rows.
// Same math as attention.hip's attn_kernel (S^T = K Q^T, online softmax per
// lane, O^T += V^T P^T with V^T from ds_read_b64_tr_b16 and P^T straight from
// the S^T accumulators).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int D = 128;
constexpr int KT = 64;                     // keys per tile == cache block
constexpr int TILE = KT * D;               // bf16 elements of a K or V tile (16 KiB)
constexpr int NWV = 4;                     // waves per block
typedef __attribute__((ext_vector_type(4))) short s16x4;

DEV bf16x4 tr_read(const bf16* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

struct DecArgs {
  const bf16* q;
  const bf16* kc;
  const bf16* vc;
  bf16* out;
  const int* q_start;
  const int* q_len;
  const int* ctx_len;
  const int* block_table;
  int max_blocks;
  const int* work_seq4;    // 4-wave items: blocks [0, 4 nwork4), 4 row tiles each
  const int* work_q04;
  int nwork4;
  const int* work_seq1;    // 1-wave items: blocks [4 nwork4, ...)
  const int* work_q01;
  int Hq, Hkv;
  float scale_log2;
  const int* kv_begin;     // cascade: first own key per sequence (multiple of 64) or null
  const bf16* pre_o;       // cascade: normalised prefix partial [T, Hq, D]
  const float* pre_lse;    // cascade: its log2-sum-exp [T, Hq]
  float* split_o;          // [nz][rows][D] fp32 partials of multi-block items
  float* split_lse;        // [nz][rows]
  int rows;                // T * Hq
  int* split_cnt;          // per (block row, kv head) arrival tickets, zero between launches
  int tpw;                 // tiles per wave
  int rel;                 // 1: block z covers the own tiles [kt0 + z C, ...), kt0 = kv_begin / 64
  int sc1_out;             // 1: out rows stored write-through (sc1) - the fused o-projection's hand-off
};

// one 16-B piece of an output row: plain, or write-through (sc1: leaves the
// XCD's L2 at once, MI355X_MICROARCH.md "Valid forms" producer condition (2))
template <bool SC1>
DEV void store_out(const DecArgs& a, size_t elem, const bf16x8& v) {
  if (SC1 && a.sc1_out) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, (unsigned)(elem * 2), 0, 16);
  } else {
    *reinterpret_cast<bf16x8*>(a.out + elem) = v;
  }
}

// One block of the decode attention: work item b, kv head kvh, key block z
// (the grid position of attn_decode_kernel; attn_oproj_kernel maps a flat id).
// Returns (block-uniform) 1 when this block wrote its item's output rows (the
// item's only block), 2 when it did as the last arriving block of a split
// item, 0 when it wrote none.
// SC1: the fused form's write-through outputs are compiled in (attn_oproj_kernel
// only; the plain kernel keeps round 5's direct stores and codegen)
template <int G, bool SC1 = false>
DEV int attn_decode_body(const DecArgs& a, const int b, const int kvh, const int z) {
  constexpr int TPR = 16 / G;                        // tokens per 16-row tile
  __shared__ __attribute__((aligned(16))) bf16 smem[NWV * TILE];   // per wave: V tile, then O
  __shared__ float s_ml[NWV][2][16];                 // per wave: row max, row sum
  __shared__ int s_last;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const bool wide = b < 4 * a.nwork4;
  const int s = wide ? a.work_seq4[b >> 2] : a.work_seq1[b - 4 * a.nwork4];
  const int q0 = wide ? a.work_q04[b >> 2] + (b & 3) * TPR : a.work_q01[b - 4 * a.nwork4];
  const int C = NWV * a.tpw;
  const int* bt = a.block_table + (size_t)s * a.max_blocks;
  bf16* vl = smem + wave * TILE;                     // this wave's V buffer

  // K of cache block blk -> registers: A fragment (nt, ks) = K[key 16 nt + fr]
  // [d 32 ks + 8 fq ..]; V -> LDS by 16 DMA pieces of 4 rows, row 4 pr + srow's
  // 16-B chunk c at chunk c ^ (row & 15) - which depends on pr & 3 only: 4
  // per-lane offsets, the row step in soffset
  const int srow = lane >> 4;
  unsigned voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) voff[i] = (unsigned)((srow * D + (((lane & 15) ^ (4 * i + srow)) << 3)) * 2);
  const unsigned koff = (unsigned)((fr * D + 8 * fq) * 2);
  bf16x8 kf[4][4];
  auto load_tile = [&](int blk) {
    blk = __builtin_amdgcn_readfirstlane(blk);
    if (blk < 0) blk = 0;                            // never for a used tile (padding guard)
    const size_t base = ((size_t)blk * a.Hkv + kvh) * (size_t)TILE;
    const auto rk = __builtin_amdgcn_make_buffer_rsrc((void*)(a.kc + base), (short)0, TILE * 2, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc((void*)(a.vc + base), (short)0, TILE * 2, 0x00020000);
#pragma unroll
    for (int pr = 0; pr < 16; ++pr) {
      auto* dst = (__attribute__((address_space(3))) void*)(vl + pr * 512);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, dst, 16, voff[pr & 3], pr * 4 * D * 2, 0, 0);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        kf[nt][ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rk, koff, (nt * 16 * D + 32 * ks) * 2, 0));
  };

  // the first tile's block id needs only the grid position: read in the same
  // round trip as the sequence's sizes; its K / V and the Q loads go next.
  // rel: the tiles count from the sequence's first own key tile (one more
  // round trip, for kv_begin), so a step of many sequences behind a cascade
  // prefix launches ceil(own tiles / C) blocks per item instead of
  // ceil(table width / C), most of which would find nothing to do
  const int kvb = a.kv_begin ? a.kv_begin[s] : 0;
  const int zbase = (a.rel ? kvb / KT : 0) + z * C;  // this block's first tile
  const int kt_first = zbase + wave;
  const int blk0 = kt_first < a.max_blocks ? bt[kt_first] : -1;
  const int qs = a.q_start[s], ql = a.q_len[s], cl = a.ctx_len[s];
  const int last_tok = min(q0 + TPR, ql) - 1;
  const int kv_end = cl - ql + last_tok + 1;
  const int kt0 = kvb / KT, kt1 = (kv_end + KT - 1) / KT;
  const int z_first = a.rel ? 0 : kt0 / C;
  const int z_last = a.rel ? (kt1 - 1 - kt0) / C : (kt1 - 1) / C;
  // padding items / row tiles past the span, blocks wholly outside the own keys
  if (q0 >= ql || kt1 <= kt0 || z < z_first || z > z_last) return 0;
  const int nact = z_last - z_first + 1;
  if (kt_first >= kt0 && kt_first < kt1) load_tile(blk0);

  // Q fragment (B operand): lane holds Q[row fr][d = 32 ks + 8 fq + j]
  const int tok = q0 + fr / G;
  const bool qvalid = tok < ql;
  const int qpos = qvalid ? cl - ql + tok : -1;      // -1: no key passes the mask
  bf16x8 qf[4];
  {
    const bf16* qp = a.q + ((size_t)(qs + (qvalid ? tok : 0)) * a.Hq + kvh * G + fr % G) * D + 8 * fq;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 32 * ks) : bf16x8{};
  }

  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_part = 0.f;

  for (int j = 0; j < a.tpw; ++j) {
    const int kt = zbase + wave + NWV * j;
    const bool use = kt >= kt0 && kt < kt1;
    if (j > 0 && use) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the last V
      load_tile(bt[kt]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // own K / V landed (own buffer only)
    if (!use) continue;

    // ---- S^T = K Q^T
    f32x4 sacc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sacc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) sacc[nt] = mfma16x16x32(kf[nt][ks], qf[ks], sacc[nt]);
    }
    // ---- mask + online softmax (lane: query row fr, keys 16 nt + 4 fq + r)
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
    // ---- O^T += V^T P^T (V^T via transposed LDS reads, permuted key order)
    const int tq = (lane & 15) >> 2, tp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int col = dt * 16 + tp * 4;
      const int chunk = col >> 3, half = (col & 7);
      f32x4 acc = o[dt] * alpha;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int key0 = k2 * 32 + fq * 4 + tq;
        const int key1 = key0 + 16;
        const bf16x4 v0 = tr_read(vl + key0 * D + ((chunk ^ (key0 & 15)) << 3) + half);
        const bf16x4 v1 = tr_read(vl + key1 * D + ((chunk ^ (key1 & 15)) << 3) + half);
        const bf16x8 vf = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        acc = mfma16x16x32(vf, pf[k2], acc);
      }
      o[dt] = acc;
    }
  }

  // ---- the 4 waves' partials -> LDS: (max, sum) per row and the unnormalised
  //      fp32 O (8 KiB) in the wave's own V buffer, rows of 128 floats with
  //      the 16-B chunk c at c ^ (row & 15) (conflict-free MFMA-layout writes)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  {
    float* ow = reinterpret_cast<float*>(vl);
    float lt = l_part + __shfl_xor(l_part, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (fq == 0) {
      s_ml[wave][0][fr] = m_run;
      s_ml[wave][1][fr] = lt;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      *reinterpret_cast<f32x4*>(ow + fr * D + (((4 * dt + fq) ^ fr) << 2)) = o[dt];
  }
  __syncthreads();

  // ---- merge: thread = (row r = tid / 16, 8 dims c8 = tid % 16)
  const int r = threadIdx.x >> 4, c8 = threadIdx.x & 15;
  const int rtok = q0 + r / G;
  const bool rvalid = rtok < ql;
  const size_t grow = (size_t)(qs + (rvalid ? rtok : 0)) * a.Hq + kvh * G + r % G;
  const bool merge_pre = a.pre_o != nullptr && a.kv_begin != nullptr && kvb > 0;
  const auto rso = __builtin_amdgcn_make_buffer_rsrc(a.split_o, (short)0, 0x7FFFFFFF, 0x00020000);
  const auto rsl = __builtin_amdgcn_make_buffer_rsrc(a.split_lse, (short)0, 0x7FFFFFFF, 0x00020000);
  if (rvalid) {
    float mw[NWV], mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      mw[w] = s_ml[w][0][r];
      mx = fmaxf(mx, mw[w]);
    }
    const float mu = mx == -INFINITY ? 0.f : mx;
    float den = 0.f;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float e = mw[w] == -INFINITY ? 0.f : fexp2(mw[w] - mu);
      den += e * s_ml[w][1][r];
      const float* src = reinterpret_cast<const float*>(smem + w * TILE) + r * D;
      acc0 += e * *reinterpret_cast<const f32x4*>(src + (((2 * c8) ^ r) << 2));
      acc1 += e * *reinterpret_cast<const f32x4*>(src + (((2 * c8 + 1) ^ r) << 2));
    }
    const float inv = den > 0.f ? 1.f / den : 0.f;
    acc0 *= inv;
    acc1 *= inv;
    const float lse = den > 0.f ? mu + __log2f(den) : -INFINITY;
    if (nact == 1) {
      // the item's only block: fold the prefix partial in and write the row
      if (merge_pre) {
        const float lp = a.pre_lse[grow];
        const float m2 = fmaxf(lp, lse);
        const float wa = fexp2(lp - m2), wb = lse == -INFINITY ? 0.f : fexp2(lse - m2);
        const float dn = 1.f / (wa + wb);
        const bf16x8 pa = *reinterpret_cast<const bf16x8*>(a.pre_o + grow * D + 8 * c8);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc0[i] = (acc0[i] * wb + (float)pa[i] * wa) * dn;
          acc1[i] = (acc1[i] * wb + (float)pa[4 + i] * wa) * dn;
        }
      }
      bf16x8 ov;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ov[i] = (bf16)acc0[i];
        ov[4 + i] = (bf16)acc1[i];
      }
      store_out<SC1>(a, grow * D + 8 * c8, ov);
    } else {
      // one of several blocks: its normalised partial, write-through
      const int zr = z - z_first;
      const unsigned off = (unsigned)((((size_t)zr * a.rows + grow) * D + 8 * c8) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc0), rso, off, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc1), rso, off + 16, 0, 16);
      if (c8 == 0)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, lse), rsl,
                                              (unsigned)(((size_t)zr * a.rows + grow) * 4), 0, 16);
    }
  }
  if (nact == 1) return 1;

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                   // every partial of this block is out
  if (threadIdx.x == 0) {
    int* cnt = a.split_cnt + (size_t)b * a.Hkv + kvh;
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nact - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return 0;
  if (!rvalid) return 2;
  // ---- last arriver: every block's partial in block order (deterministic)
  float mx = -INFINITY;
#pragma unroll 8
  for (int jz = 0; jz < nact; ++jz)
    mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                       rsl, (unsigned)(((size_t)jz * a.rows + grow) * 4), 0, 16)));
  float lp = -INFINITY;
  bf16x8 pa{};
  if (merge_pre) {
    lp = a.pre_lse[grow];
    pa = *reinterpret_cast<const bf16x8*>(a.pre_o + grow * D + 8 * c8);
    mx = fmaxf(mx, lp);
  }
  const float mu = mx == -INFINITY ? 0.f : mx;
  float den = 0.f;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int jz = 0; jz < nact; ++jz) {
    const float lj = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
        rsl, (unsigned)(((size_t)jz * a.rows + grow) * 4), 0, 16));
    const unsigned off = (unsigned)((((size_t)jz * a.rows + grow) * D + 8 * c8) * 4);
    const f32x4 p0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rso, off, 0, 16));
    const f32x4 p1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rso, off + 16, 0, 16));
    const float wj = lj == -INFINITY ? 0.f : fexp2(lj - mu);
    den += wj;
    acc0 += p0 * wj;
    acc1 += p1 * wj;
  }
  if (merge_pre) {
    const float wp = fexp2(lp - mu);
    den += wp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc0[i] += (float)pa[i] * wp;
      acc1[i] += (float)pa[4 + i] * wp;
    }
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  bf16x8 ov;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ov[i] = (bf16)(acc0[i] * inv);
    ov[4 + i] = (bf16)(acc1[i] * inv);
  }
  store_out<SC1>(a, grow * D + 8 * c8, ov);
  return 2;
}

template <int G>
__global__ __launch_bounds__(256, 2) void attn_decode_kernel(const DecArgs a) {
  attn_decode_body<G>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---------------------------------------------------------------------------
// Decode attention with the o-projection in the same launch (config 2 / low-QPS
// decode steps, TP = 1).  A decode layer is a chain of short kernels, each
// paying a launch boundary and a weight-stream ramp; the attention in the
// middle is a chain of dependent memory round trips (~14 us over a few MB of
// K / V) during which HBM idles, and the o-projection after it streams 33.5 MB
// of weights (Llama-3-8B) in ~10-13 us, mostly ramp and tail (5.6 us at
// 6 TB/s).  Here the grid is [attention blocks | o-projection blocks]:
//
//  * the o-projection blocks (16 weight rows x all of K each, 4 waves split K)
//    load their whole weight slice into registers at once, while the
//    attention blocks run - the stream overlaps the attention's latency chain;
//  * each attention block, when done (every path, early exits included),
//    drains its stores and publishes with the canonical hand-off
//    (MI355X_MICROARCH.md "Valid forms": stores -> s_waitcnt vmcnt(0) ->
//    barrier -> lane-0 agent release -> s_waitcnt -> relaxed agent counter add);
//  * an o-projection block polls the counter (relaxed agent loads, s_sleep,
//    bounded: a timeout sets the error word and proceeds), takes ONE agent
//    acquire, loads the attention rows (two halves of its K range), and
//    finishes with the residual GEMM epilogue of gemm_skinny (EPI 1: + x in
//    place, the rows' fused-norm statistic);
//  * the last o-projection block past its poll resets both counters (every
//    attention block has counted by then), so hipGraph replays start at 0.
//
// Attention blocks come first in block order: dispatch is in order per XCD
// (observed), so a waiting o-projection block never holds a slot an attention
// block still needs; the grid also fits in two blocks per CU at config 2.
struct OprojArgs {
  const bf16* W;                     // [N, K] o-projection weight
  const bf16* X;                     // [M, K] attention output (= DecArgs.out)
  bf16* Y;                           // [M, N]: residual in, x + X W^T out (in place)
  unsigned long long* ss_out;        // fused-norm statistic of the rows written, or null
  int* sync;                         // [0] attention blocks done, [1] o blocks past the poll
  int* err;                          // nonzero: a poll timed out
  int M, N, K;
  int n_attn, nitems;                // attention blocks, attention grid x extent
  int pace;                          // weight-load pacing (MCP_AOP_PACE): s_sleep(32) x pace between
                                     // k-steps; < 0: load the weights only after the wait
};

constexpr int OP_STEP = 128;

template <int G, int KS>              // k-steps of 128 per wave: K = 4 x 128 x KS
DEV void oproj_block(const DecArgs& a, const OprojArgs& o, const int j) {
  constexpr int TPR = 16 / G;
  __shared__ f32x4 ored[NWV][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = j * 16;
  const int kb = wave * KS * OP_STEP;
  // the weight slice (16 rows x K / 4 per wave) into registers, all in
  // flight while the attention runs (paced: the attention's own round trips
  // queue behind this stream in HBM)
  const bf16* wrow = o.W + (size_t)(n0 + r) * o.K + kb + 8 * g;
  bf16x8 w[KS][4];
  auto load_w = [&]() {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int q = 0; q < 4; ++q) w[s][q] = *reinterpret_cast<const bf16x8*>(wrow + s * OP_STEP + 32 * q);
      for (int p = 0; p < o.pace; ++p) __builtin_amdgcn_s_sleep(32);
    }
  };
  if (o.pace >= 0) load_w();
  const int m = min(r, o.M - 1);
  const bf16x4 rr = *reinterpret_cast<const bf16x4*>(o.Y + (size_t)m * o.N + n0 + 4 * g);
  if (wave == 0) {
    // the writers to wait for: one per (item with rows, kv head) - the item's
    // only block or its last arriving one (attn_decode_body returns nonzero);
    // an item has rows iff q0 < q_len of its sequence (no cascade here, so
    // every such item has keys).  Counted on the device: a hipGraph replay's
    // items are padded, and their real count is only known here
    int cnt = 0;
    for (int b = lane; b < o.nitems; b += 64) {
      const bool wide = b < 4 * a.nwork4;
      const int s = wide ? a.work_seq4[b >> 2] : a.work_seq1[b - 4 * a.nwork4];
      const int q0 = wide ? a.work_q04[b >> 2] + (b & 3) * TPR : a.work_q01[b - 4 * a.nwork4];
      cnt += q0 < a.q_len[s];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane == 0) {
      const int expect = cnt * a.Hkv;
      int spins = 0;
      while (__hip_atomic_load(o.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < expect) {
        __builtin_amdgcn_s_sleep(4);
        if (++spins > (1 << 23)) {                   // ~seconds: never in a healthy launch
          __hip_atomic_store(o.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (o.pace < 0) load_w();
  if (threadIdx.x == 0) {
    const int n_o = o.N / 16;
    const int old = __hip_atomic_fetch_add(o.sync + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == n_o - 1) {                            // every block is past its wait
      __hip_atomic_store(o.sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o.sync + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // the attention rows, in two halves of this wave's K range
  const bf16* xrow = o.X + (size_t)m * o.K + kb + 8 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int H = KS / 2;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    bf16x8 x[H][4];
#pragma unroll
    for (int s = 0; s < H; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        x[s][q] = *reinterpret_cast<const bf16x8*>(xrow + (half * H + s) * OP_STEP + 32 * q);
#pragma unroll
    for (int s = 0; s < H; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = mfma16x16x32(w[half * H + s][q], x[s][q], acc);
  }
  ored[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  f32x4 v = ored[0][lane] + ored[1][lane] + ored[2][lane] + ored[3][lane];
  // C layout: lane holds weight rows n0 + 4 g .. + 3 of token r
  if (r >= o.M) return;                              // all four g lanes of token r together
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] += (float)rr[q];
  bf16x4 out;
#pragma unroll
  for (int q = 0; q < 4; ++q) out[q] = (bf16)v[q];
  *reinterpret_cast<bf16x4*>(o.Y + (size_t)r * o.N + n0 + 4 * g) = out;
  if (o.ss_out) {
    float ss = sumsq_bf16x4(out);
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (g == 0) ss_atomic_add(o.ss_out + r, ss);
  }
}

template <int G, int KS>
__global__ __launch_bounds__(256, 2) void attn_oproj_kernel(const DecArgs a, const OprojArgs o) {
  const int f = blockIdx.x;
  if (f >= o.n_attn) {
    oproj_block<G, KS>(a, o, f - o.n_attn);
    return;
  }
  const int rest = f / o.nitems;
  const int wrote = attn_decode_body<G, true>(a, f - rest * o.nitems, rest % a.Hkv, rest / a.Hkv);
  // hand-off of this block's rows (block-uniform: only writers signal, so the
  // padded items of a graph replay cost no atomics): sc1 stores drained by
  // every wave, a barrier, one relaxed agent-scope add; the reader's acquire
  // completes it (MI355X_MICROARCH.md "Valid forms", producer (2) + (3))
  if (wrote) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(o.sync, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

int* attn_split_counters();   // attention.hip
// the fused kernel's sync words live past the tickets the decode kernel uses
constexpr int AOP_RESERVED = 64;
constexpr int SPLIT_TICKETS = (1 << 16) - AOP_RESERVED;

// tiles per wave for a block-table width: <= 64 blocks per (item, kv head)
int attn_decode_tpw(int max_blocks) {
  const int per_pass = NWV * 64;
  const int tpw = max_blocks <= per_pass ? 1 : (max_blocks + per_pass - 1) / per_pass;
  // MCP_ATTN_DECODE_TPW: at least this many tiles per wave (fewer blocks to
  // merge, more tiles walked per wave; A/B)
  static const int force = getenv("MCP_ATTN_DECODE_TPW") ? atoi(getenv("MCP_ATTN_DECODE_TPW")) : 0;
  return force > tpw ? force : tpw;
}
int attn_decode_blocks(int max_blocks) {
  const int C = NWV * attn_decode_tpw(max_blocks);
  return (max_blocks + C - 1) / C;
}
// own-span (rel) mode: the same rule over the longest own key span
int attn_decode_rel_blocks(int own_tiles) { return attn_decode_blocks(own_tiles > 0 ? own_tiles : 1); }

static int launch_attn_decode_impl(const void* q, const void* k_cache, const void* v_cache,
                                   void* out, const int* q_start, const int* q_len,
                                   const int* ctx_len, const int* block_table, int max_blocks,
                                   const int* work_seq4, const int* work_q04, int nwork4,
                                   const int* work_seq1, const int* work_q01, int nwork1, int Hq,
                                   int Hkv, int head_dim, float scale, const int* kv_begin,
                                   const void* pre_o, const float* pre_lse, float* split_o,
                                   float* split_lse, int rows, int nz, hipStream_t s,
                                   int own_tiles, const OprojArgs* oproj);

// nonzero: not launched (the caller uses the work-list split path)

int launch_attn_decode(const void* q, const void* k_cache, const void* v_cache, void* out,
                       const int* q_start, const int* q_len, const int* ctx_len,
                       const int* block_table, int max_blocks, const int* work_seq4,
                       const int* work_q04, int nwork4, const int* work_seq1, const int* work_q01,
                       int nwork1, int Hq, int Hkv, int head_dim, float scale, const int* kv_begin,
                       const void* pre_o, const float* pre_lse, float* split_o, float* split_lse,
                       int rows, int nz, hipStream_t s, int own_tiles) {
  return launch_attn_decode_impl(q, k_cache, v_cache, out, q_start, q_len, ctx_len, block_table,
                            max_blocks, work_seq4, work_q04, nwork4, work_seq1, work_q01, nwork1,
                            Hq, Hkv, head_dim, scale, kv_begin, pre_o, pre_lse, split_o, split_lse,
                            rows, nz, s, own_tiles, nullptr);
}

// decode attention + o-projection in one launch (attn_oproj_kernel); nonzero:
// not launched (7: shape outside the fused form) - the caller runs both apart
int launch_attn_decode_oproj(const void* q, const void* k_cache, const void* v_cache, void* out,
                             const int* q_start, const int* q_len, const int* ctx_len,
                             const int* block_table, int max_blocks, const int* work_seq4,
                             const int* work_q04, int nwork4, const int* work_seq1,
                             const int* work_q01, int nwork1, int Hq, int Hkv, int head_dim,
                             float scale, float* split_o, float* split_lse, int rows, int nz,
                             const void* Wo, void* x, int M, int N, int K,
                             unsigned long long* ss_out, hipStream_t s) {
  OprojArgs o{};
  o.W = (const bf16*)Wo;
  o.Y = (bf16*)x;
  o.ss_out = ss_out;
  o.M = M;
  o.N = N;
  o.K = K;
  return launch_attn_decode_impl(q, k_cache, v_cache, out, q_start, q_len, ctx_len, block_table,
                            max_blocks, work_seq4, work_q04, nwork4, work_seq1, work_q01, nwork1,
                            Hq, Hkv, head_dim, scale, nullptr, nullptr, nullptr, split_o, split_lse,
                            rows, nz, s, 0, &o);
}

// the fused kernel's error word (nonzero: an o-projection block's wait timed out)
int attn_oproj_error() {
  int* cnt = attn_split_counters();
  if (!cnt) return 0;
  int v = 0;
  if (hipMemcpy(&v, cnt + SPLIT_TICKETS + 2, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

static int launch_attn_decode_impl(const void* q, const void* k_cache, const void* v_cache, void* out,
                       const int* q_start, const int* q_len, const int* ctx_len,
                       const int* block_table, int max_blocks, const int* work_seq4,
                       const int* work_q04, int nwork4, const int* work_seq1, const int* work_q01,
                       int nwork1, int Hq, int Hkv, int head_dim, float scale, const int* kv_begin,
                       const void* pre_o, const float* pre_lse, float* split_o, float* split_lse,
                       int rows, int nz, hipStream_t s, int own_tiles, const OprojArgs* oproj) {
  if (head_dim != D) return 1;
  const int nitems = 4 * nwork4 + nwork1;            // 4-wave items: one block per row tile
  if (nitems <= 0) return oproj ? 7 : 0;
  if (max_blocks <= 0) return 2;
  // own_tiles > 0: own-span mode, the longest own key span in tiles
  const int span = own_tiles > 0 ? own_tiles : max_blocks;
  const int tpw = attn_decode_tpw(span);
  if (nz != attn_decode_blocks(span)) return 3;
  int* cnt = attn_split_counters();
  if (!cnt || (long long)nitems * Hkv > SPLIT_TICKETS) return 5;
  if (nz > 1 && (!split_o || !split_lse || (long long)nz * rows * D * 4 >= (1ll << 31))) return 6;
  DecArgs a{};
  a.q = (const bf16*)q;
  a.kc = (const bf16*)k_cache;
  a.vc = (const bf16*)v_cache;
  a.out = (bf16*)out;
  a.q_start = q_start;
  a.q_len = q_len;
  a.ctx_len = ctx_len;
  a.block_table = block_table;
  a.max_blocks = max_blocks;
  a.work_seq4 = work_seq4;
  a.work_q04 = work_q04;
  a.nwork4 = nwork4;
  a.work_seq1 = work_seq1;
  a.work_q01 = work_q01;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.kv_begin = kv_begin;
  a.pre_o = (const bf16*)pre_o;
  a.pre_lse = pre_lse;
  a.split_o = split_o;
  a.split_lse = split_lse;
  a.rows = rows;
  a.split_cnt = cnt;
  a.tpw = tpw;
  a.rel = own_tiles > 0;
  if (oproj) {
    // fused o-projection (attn_oproj_kernel): K = Hq D = 4 x 128 x KS, KS = 8
    // (Llama-3-8B / 3.2-3B padded heads), one 16-token row tile
    if (own_tiles > 0 || oproj->K != Hq * D || oproj->K != 4 * OP_STEP * 8 || oproj->N % 16 ||
        oproj->M < 1 || oproj->M > 16 || oproj->M * Hq != rows)
      return 7;
    OprojArgs o = *oproj;
    static const int pace = getenv("MCP_AOP_PACE") ? atoi(getenv("MCP_AOP_PACE")) : 0;
    o.pace = pace;
    a.sc1_out = 1;
    o.X = a.out;
    o.sync = cnt + SPLIT_TICKETS;
    o.err = cnt + SPLIT_TICKETS + 2;
    o.nitems = nitems;
    o.n_attn = nitems * Hkv * nz;
    const int grid1 = o.n_attn + o.N / 16;
    switch (Hq / Hkv) {
      case 1: attn_oproj_kernel<1, 8><<<grid1, 256, 0, s>>>(a, o); break;
      case 2: attn_oproj_kernel<2, 8><<<grid1, 256, 0, s>>>(a, o); break;
      case 4: attn_oproj_kernel<4, 8><<<grid1, 256, 0, s>>>(a, o); break;
      case 8: attn_oproj_kernel<8, 8><<<grid1, 256, 0, s>>>(a, o); break;
      default: return 4;
    }
    return 0;
  }
  const dim3 grid(nitems, Hkv, nz);
  switch (Hq / Hkv) {
    case 1: attn_decode_kernel<1><<<grid, 256, 0, s>>>(a); break;
    case 2: attn_decode_kernel<2><<<grid, 256, 0, s>>>(a); break;
    case 4: attn_decode_kernel<4><<<grid, 256, 0, s>>>(a); break;
    case 8: attn_decode_kernel<8><<<grid, 256, 0, s>>>(a); break;
    case 16: attn_decode_kernel<16><<<grid, 256, 0, s>>>(a); break;
    default: return 4;
  }
  return 0;
}
