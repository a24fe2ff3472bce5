// Tape-store rate probe (gfx950): the lstm_fwd4 tape pattern with 8-byte lane stores (two per
// 16x16 row block) vs the same bytes as one 16-byte lane store, persistent grid of 256 x 512
// threads, waves 0-6 storing, one barrier per step.  Prints ms and TB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

template <int MODE>  // 0: 2 x 8 B per slot (fwd4 today), 1: 1 x 16 B per slot, 2: no stores
__global__ void __launch_bounds__(512) k(short* tape, int nrb, int Tn) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g4 = lane >> 4, c = 16 * wave + (lane & 15);
  const int wt32 = wave >> 1;
  const int lo8 = (32 * (g4 & 1) + (c & 31)) * 8 + 4 * (g4 >> 1);       // elements
  const int lo16 = (32 * (g4 & 1) + (c & 31)) * 16 + 8 * (g4 >> 1);     // elements
  for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
    for (int t = 0; t < Tn; ++t) {
      if (wave < 7 && c < 100) {
        short* base = tape + (((size_t)rb * Tn + t) * 4 + wt32) * 5 * 1024;
        for (int s = 0; s < 5; ++s) {
          if (MODE == 0) {
            *(v2i*)(base + s * 1024 + lo8) = v2i{t, s};
            *(v2i*)(base + s * 1024 + 512 + lo8) = v2i{t, s};
          } else if (MODE == 1) {
            *(v4i*)(base + s * 1024 + lo16) = v4i{t, s, t, s};
          }
        }
      }
      __syncthreads();
    }
  }
}

template <int MODE>
static float run(short* d, int nrb, int Tn) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(512), 0, 0, d, nrb, Tn);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(512), 0, 0, d, nrb, Tn);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int nrb = 8192, Tn = 24;  // B = 262144
  const size_t elems = (size_t)nrb * Tn * 4 * 5 * 1024;
  short* d;
  if (hipMalloc(&d, elems * 2) != hipSuccess) { printf("alloc failed\n"); return 1; }
  const double gb = elems * 2 * (100.0 / 128.0) / 1e9;  // bytes actually written (units < 100)
  float m0 = run<0>(d, nrb, Tn), m1 = run<1>(d, nrb, Tn), m2 = run<2>(d, nrb, Tn);
  printf("{\"probe\": \"tape_store\", \"GB\": %.2f, \"ms_8B\": %.3f, \"TBps_8B\": %.2f, \"ms_16B\": %.3f, \"TBps_16B\": %.2f, \"ms_barrier_only\": %.3f}\n",
         gb, m0, gb / m0, m1, gb / m1, m2);
  hipFree(d);
  return 0;
}
