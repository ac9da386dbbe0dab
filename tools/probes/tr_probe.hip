// Probe: what does each lane receive from ds_read_b64_tr_b16 ?
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(4))) short s4;
__global__ void k(int* out, int mode) {
  __shared__ __attribute__((aligned(16))) short lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (short)i;
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  int addr;
  if (mode == 0) addr = (4 * g + q) * 64 + 4 * p;     // guide's description
  else addr = l * 4;                                    // lane-linear
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + addr));
  for (int j = 0; j < 4; ++j) out[(mode * 64 + l) * 4 + j] = v[j];
}
int main() {
  int* d; hipMalloc(&d, 2 * 64 * 4 * sizeof(int));
  k<<<1, 64>>>(d, 0); k<<<1, 64>>>(d, 1);
  int h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int m = 0; m < 2; ++m) { printf("mode %d\n", m);
    for (int l = 0; l < 64; ++l) printf("lane %2d: %5d %5d %5d %5d\n", l, h[(m*64+l)*4], h[(m*64+l)*4+1], h[(m*64+l)*4+2], h[(m*64+l)*4+3]); }
  return 0;
}
