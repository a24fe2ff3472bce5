// Probe the lane semantics of ds_read_b64_tr_b16 on gfx950 (printed table, no assumptions).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[8 * 32];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = (short)((i / 32) * 100 + (i % 32));
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
  const int row = (g & 1) * 4 + q, col = (g >> 1) * 16 + 4 * p;   // documented addressing
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + row * 32 + col));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  return 0;
}
