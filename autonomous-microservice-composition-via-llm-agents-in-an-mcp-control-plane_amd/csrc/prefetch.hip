// Weight prefetch into the Infinity Cache (MALL, 256 MiB die-level) for
// decode-sized steps.
//
// A single-intent decode step is a chain of weight streams with latency-bound
// work between them: the decode attention of a layer takes ~14 us with the
// HBM nearly idle (a few MB of K/V), then the o-projection streams its 33.5 MB
// of weights from HBM.  Reads with the default cache policy allocate in the
// MALL (MI355X_MICROARCH.md "nt-weights": a back-to-back replay of a launch
// reads its weights faster than its cold run), so a kernel running beside the
// attention on a second stream that reads the next weights once leaves them
// where the GEMM finds them at MALL instead of HBM bandwidth.
//
// The kernel only loads: every lane keeps 8 x 16 B in flight per pass over a
// grid-strided range and folds what it read into one register, written out
// only under a flag the host never sets (so the loads stay live).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int PF_THREADS = 256;
constexpr int PF_UNROLL = 8;

__global__ __launch_bounds__(PF_THREADS) void prefetch_kernel(const uint4* __restrict__ p, size_t n16,
                                                              int* __restrict__ sink, int never) {
  const size_t stride = (size_t)gridDim.x * PF_THREADS;
  size_t i = (size_t)blockIdx.x * PF_THREADS + threadIdx.x;
  unsigned acc = 0;
  for (; i + (PF_UNROLL - 1) * stride < n16; i += PF_UNROLL * stride) {
    uint4 v[PF_UNROLL];
#pragma unroll
    for (int u = 0; u < PF_UNROLL; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < PF_UNROLL; ++u) acc ^= v[u].x ^ v[u].w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (never) sink[threadIdx.x] = (int)acc;
}

}  // namespace

// Read [p, p + bytes) once (16-B granules; a ragged tail is skipped) with
// `wgs` workgroups; nonzero if nothing to do.
int launch_prefetch(const void* p, size_t bytes, int wgs, int* sink, hipStream_t s) {
  const size_t n16 = bytes / 16;
  if (n16 == 0 || wgs <= 0 || !sink) return 1;
  prefetch_kernel<<<wgs, PF_THREADS, 0, s>>>(reinterpret_cast<const uint4*>(p), n16, sink, 0);
  return 0;
}
