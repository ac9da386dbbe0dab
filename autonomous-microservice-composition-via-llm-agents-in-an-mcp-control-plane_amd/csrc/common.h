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
