// Memory-bound kernels of the Llama-3 forward (SURVEY §2.6 K3, K4+K10, K7, K8).
// All loads/stores are 16 B per lane (bf16x8), cdna_hip_programming.md Guideline 13.
#include "common.h"
#include "kernels.h"

// ---------------------------------------------------------------- K3 RMSNorm
// One 256-thread block per row.  VMAX bf16x8 vectors per thread are kept in
// registers between the reduction and the scaled write (single HBM pass).
template <int VMAX, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16* __restrict__ x,
                                                      bf16* __restrict__ residual,
                                                      const bf16* __restrict__ w,
                                                      bf16* __restrict__ out, int H, float eps) {
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * H);
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + (size_t)row * H);
  float v[VMAX][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VMAX; ++i) {
    const int idx = threadIdx.x + i * 256;
    if (idx < nvec) {
      bf16x8 a = xr[idx];
      if (ADD) {
        bf16x8 r = rr[idx];
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f = (float)a[j] + (float)r[j];
          s[j] = (bf16)f;
          v[i][j] = (float)s[j];   // normalise the rounded residual, as a bf16 model would
        }
        rr[idx] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (float)a[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(tot / (float)H + eps);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  bf16x8* orow = reinterpret_cast<bf16x8*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < VMAX; ++i) {
    const int idx = threadIdx.x + i * 256;
    if (idx < nvec) {
      bf16x8 ww = wv[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)(v[i][j] * inv * (float)ww[j]);
      orow[idx] = o;
    }
  }
}

template <bool ADD>
static void rmsnorm_dispatch(const bf16* x, bf16* residual, const bf16* w, bf16* out, int T,
                             int H, float eps, hipStream_t s) {
  const int nvec = H / 8;
  const int vmax = (nvec + 255) / 256;
  if (T <= 0) return;
  if (vmax <= 1)
    rmsnorm_kernel<1, ADD><<<T, 256, 0, s>>>(x, residual, w, out, H, eps);
  else if (vmax <= 2)
    rmsnorm_kernel<2, ADD><<<T, 256, 0, s>>>(x, residual, w, out, H, eps);
  else if (vmax <= 4)
    rmsnorm_kernel<4, ADD><<<T, 256, 0, s>>>(x, residual, w, out, H, eps);
  else
    rmsnorm_kernel<8, ADD><<<T, 256, 0, s>>>(x, residual, w, out, H, eps);
}

void launch_rmsnorm(const void* x, const void* w, void* out, int T, int H, float eps,
                    hipStream_t s) {
  rmsnorm_dispatch<false>((const bf16*)x, nullptr, (const bf16*)w, (bf16*)out, T, H, eps, s);
}

void launch_add_rmsnorm(const void* x, void* residual, const void* w, void* out, int T, int H,
                        float eps, hipStream_t s) {
  rmsnorm_dispatch<true>((const bf16*)x, (bf16*)residual, (const bf16*)w, (bf16*)out, T, H, eps,
                         s);
}

// ---------------------------------------------------------------- K7 SiLU*mul
// x: [T, 2F] (gate | up), y: [T, F]
__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16* __restrict__ x,
                                                       bf16* __restrict__ y, int T, int F) {
  const int fv = F >> 3;
  const size_t total = (size_t)T * fv;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t t = i / fv, c = i % fv;
    const bf16x8 g = reinterpret_cast<const bf16x8*>(x + t * 2 * F)[c];
    const bf16x8 u = reinterpret_cast<const bf16x8*>(x + t * 2 * F + F)[c];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = (float)g[j];
      o[j] = (bf16)(gf / (1.f + __expf(-gf)) * (float)u[j]);
    }
    reinterpret_cast<bf16x8*>(y + t * F)[c] = o;
  }
}

void launch_silu_mul(const void* x, void* y, int T, int F, hipStream_t s) {
  const size_t total = (size_t)T * (F / 8);
  if (!total) return;
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  silu_mul_kernel<<<grid, 256, 0, s>>>((const bf16*)x, (bf16*)y, T, F);
}

// ------------------------------------------- fused-RMSNorm launch context
NormEpi& norm_epi() {
  static NormEpi ne;
  return ne;
}

// per-row sum of squares (the fused norm's statistic of a row nobody's GEMM
// epilogue wrote: the embedding output of layer 0); one wave per row
__global__ __launch_bounds__(256) void row_sumsq_kernel(const bf16* __restrict__ x,
                                                        unsigned long long* __restrict__ ss, int T,
                                                        int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const int lane = threadIdx.x & 63;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * H);
  float acc = 0.f;
  for (int c = lane; c < (H >> 3); c += 64) acc += sumsq_bf16x8(xr[c]);
  acc = wave_sum(acc);
  if (lane == 0) ss[row] = ss_fixed(acc, SS_ROW_MAX);
}

void launch_row_sumsq(const void* x, unsigned long long* ss, int T, int H, hipStream_t s) {
  if (T > 0) row_sumsq_kernel<<<(T + 3) / 4, 256, 0, s>>>((const bf16*)x, ss, T, H);
}

// ---------------------------------------------------------------- K8 embedding
__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ ids,
                                                        const bf16* __restrict__ table,
                                                        bf16* __restrict__ out, int H) {
  const int t = blockIdx.x;
  const int id = ids[t];
  const bf16x8* src = reinterpret_cast<const bf16x8*>(table + (size_t)id * H);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out + (size_t)t * H);
  for (int c = threadIdx.x; c < (H >> 3); c += 256) dst[c] = src[c];
}

void launch_embedding(const int* ids, const void* table, void* out, int T, int H, hipStream_t s) {
  if (T > 0) embedding_kernel<<<T, 256, 0, s>>>(ids, (const bf16*)table, (bf16*)out, H);
}

// ------------------------------------------------------- K4+K10 RoPE + KV write
// qkv: [T, (Hq + 2*Hkv) * D] straight from the QKV projection.
// q_out: [T, Hq, D] rotated queries.  k/v caches: [num_blocks, Hkv, BS, D].
// cos_sin: [max_pos, D/2] float2 (cos, sin), rotate-half (Llama) convention.
// One thread per (token, head, 8-wide dim chunk of the first half).
template <int D>
__global__ __launch_bounds__(256) void rope_kv_kernel(
    const bf16* __restrict__ qkv, const int* __restrict__ pos, const int* __restrict__ slots,
    const float2* __restrict__ cos_sin, bf16* __restrict__ q_out, bf16* __restrict__ k_cache,
    bf16* __restrict__ v_cache, int T, int Hq, int Hkv, int BS, const NormEpi ne) {
  constexpr int CH = D / 16;                 // 8-wide chunks in the first half
  const int heads = Hq + 2 * Hkv;
  const size_t total = (size_t)T * heads * CH;
  const size_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % CH);
  const int h = (int)((i / CH) % heads);
  const int t = (int)(i / ((size_t)CH * heads));
  const bf16* src = qkv + (size_t)t * heads * D + (size_t)h * D;
  const int d0 = c * 8;
  const bf16x8 lo = *reinterpret_cast<const bf16x8*>(src + d0);
  const bf16x8 hi = *reinterpret_cast<const bf16x8*>(src + d0 + D / 2);
  const float rs = norm_row_scale(ne, t);    // fused RMSNorm of the projected row (1 if none)
  if (h >= Hq + Hkv) {                       // V: copy into the cache
    const int slot = slots[t];
    if (slot < 0) return;
    const int hv = h - Hq - Hkv;
    bf16* dst = v_cache + (((size_t)(slot / BS) * Hkv + hv) * BS + (slot % BS)) * D;
    bf16x8 vlo = lo, vhi = hi;
    if (ne.ss_in) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        vlo[j] = (bf16)((float)lo[j] * rs);
        vhi[j] = (bf16)((float)hi[j] * rs);
      }
    }
    *reinterpret_cast<bf16x8*>(dst + d0) = vlo;
    *reinterpret_cast<bf16x8*>(dst + d0 + D / 2) = vhi;
    return;
  }
  const float2* cs = cos_sin + (size_t)pos[t] * (D / 2) + d0;
  bf16x8 olo, ohi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 r = cs[j];
    const float a = (float)lo[j] * rs, b = (float)hi[j] * rs;
    olo[j] = (bf16)(a * r.x - b * r.y);
    ohi[j] = (bf16)(b * r.x + a * r.y);
  }
  bf16* dst;
  if (h < Hq) {
    dst = q_out + ((size_t)t * Hq + h) * D;
  } else {
    const int slot = slots[t];
    if (slot < 0) return;
    const int hk = h - Hq;
    dst = k_cache + (((size_t)(slot / BS) * Hkv + hk) * BS + (slot % BS)) * D;
  }
  *reinterpret_cast<bf16x8*>(dst + d0) = olo;
  *reinterpret_cast<bf16x8*>(dst + d0 + D / 2) = ohi;
}

void launch_rope_kv(const void* qkv, const int* pos, const int* slots, const void* cos_sin,
                    void* q_out, void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D,
                    int BS, hipStream_t s) {
  if (T <= 0) return;
  const size_t total = (size_t)T * (Hq + 2 * Hkv) * (D / 16);
  const int grid = (int)((total + 255) / 256);
  if (D == 128)
    rope_kv_kernel<128><<<grid, 256, 0, s>>>((const bf16*)qkv, pos, slots, (const float2*)cos_sin,
                                             (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, T, Hq,
                                             Hkv, BS, norm_epi());
  else if (D == 64)
    rope_kv_kernel<64><<<grid, 256, 0, s>>>((const bf16*)qkv, pos, slots, (const float2*)cos_sin,
                                            (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, T, Hq,
                                            Hkv, BS, norm_epi());
}

// ------------------------------------------------------------ residual add
__global__ __launch_bounds__(256) void add_kernel(bf16* __restrict__ y, const bf16* __restrict__ x,
                                                  size_t nvec) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
    bf16x8 a = reinterpret_cast<bf16x8*>(y)[i];
    const bf16x8 b = reinterpret_cast<const bf16x8*>(x)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (bf16)((float)a[j] + (float)b[j]);
    reinterpret_cast<bf16x8*>(y)[i] = a;
  }
}

void launch_add_inplace(void* y, const void* x, size_t n, hipStream_t s) {
  const size_t nvec = n / 8;
  if (!nvec) return;
  int grid = (int)((nvec + 255) / 256);
  if (grid > 4096) grid = 4096;
  add_kernel<<<grid, 256, 0, s>>>((bf16*)y, (const bf16*)x, nvec);
}

// ------------------------------------------------------- KV block copy (CoW)
// data: [L, 2, num_blocks, block_elems]; copies block src[i] -> dst[i] for every
// layer and K/V (prefix-cache tail blocks).  16 B per lane; pairs with a
// negative block id are skipped.
__global__ __launch_bounds__(256) void copy_blocks_kernel(bf16* __restrict__ data,
                                                          const int* __restrict__ src,
                                                          const int* __restrict__ dst, int npairs,
                                                          int nb, int block_vecs) {
  const int pair = blockIdx.x % npairs;
  const int lk = blockIdx.x / npairs;           // layer * 2 + kv
  // a negative pair is padding (the fixed-capacity copy list of a captured
  // hipGraph step): the whole workgroup skips it
  if (src[pair] < 0 || dst[pair] < 0) return;
  bf16x8* base = reinterpret_cast<bf16x8*>(data) + (size_t)lk * nb * block_vecs;
  const bf16x8* s = base + (size_t)src[pair] * block_vecs;
  bf16x8* d = base + (size_t)dst[pair] * block_vecs;
  for (int i = threadIdx.x; i < block_vecs; i += 256) d[i] = s[i];
}

void launch_copy_blocks(void* data, const int* src, const int* dst, int npairs, int layers2,
                        int nb, int block_elems, hipStream_t s) {
  if (npairs <= 0) return;
  copy_blocks_kernel<<<npairs * layers2, 256, 0, s>>>((bf16*)data, src, dst, npairs, nb,
                                                      block_elems / 8);
}

