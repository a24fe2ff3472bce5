// MFMA issue rate of dependent accumulation chains (gfx950).
//
// Question: does a dependent MFMA (SrcC = the previous MFMA's destination) issue back to back at
// the pipe's throughput, or does it wait for the previous result?  The compiler's scheduler
// groups the fp32 LSTM kernels' MFMAs chain by chain (16 dependent 16x16x4 f32 MFMAs, then the
// next chain), so this decides whether those kernels run at throughput or at latency.
//
// One wave per SIMD (4 waves per workgroup, one workgroup per CU); each wave runs 64 MFMAs per
// iteration as NC interleaved chains (NC = 1, 2, 4), timed with s_memtime (100 MHz constant clock)
// and converted to cycles per MFMA with the shader clock given on the command line (MHz).
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_chain_probe.hip -o scripts/probes/mfma_chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int NC, bool BF16>
__global__ void __launch_bounds__(256) chain(float* out, long long* ticks, int iters) {
  f32x4 acc[4];
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float a = 1e-3f * (threadIdx.x & 7), b = 1e-3f;
  bf16x8 ab;
  for (int i = 0; i < 8; ++i) ab[i] = 0x3a83;  // ~1e-3
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 64 / NC; ++k) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if constexpr (BF16) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, acc[c], 0, 0, 0);
        else acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int c = 0; c < NC; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int NC, bool BF16>
static void run(float* out, long long* ticks, int cus, int iters, double mhz) {
  hipLaunchKernelGGL((chain<NC, BF16>), dim3(cus), dim3(256), 0, 0, out, ticks, iters);
  (void)hipDeviceSynchronize();
  long long* h = (long long*)malloc(cus * sizeof(long long));
  (void)hipMemcpy(h, ticks, cus * sizeof(long long), hipMemcpyDeviceToHost);
  double mx = 0;
  for (int i = 0; i < cus; ++i) mx = h[i] > mx ? h[i] : mx;
  free(h);
  const double ns = mx * 10.0;  // s_memtime: 100 MHz
  const double cyc = ns * mhz / 1000.0 / (64.0 * iters);
  printf("{\"mfma\": \"%s\", \"chains\": %d, \"cycles_per_mfma\": %.2f}\n", BF16 ? "16x16x32_bf16" : "16x16x4_f32", NC, cyc);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double mhz = argc > 1 ? atof(argv[1]) : 2400.0;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  int cus = 256;
  float* out;
  long long* ticks;
  if (hipMalloc(&out, cus * 256 * sizeof(float)) != hipSuccess) return 1;
  if (hipMalloc(&ticks, cus * sizeof(long long)) != hipSuccess) return 1;
  run<1, false>(out, ticks, cus, iters, mhz);
  run<2, false>(out, ticks, cus, iters, mhz);
  run<4, false>(out, ticks, cus, iters, mhz);
  run<1, true>(out, ticks, cus, iters, mhz);
  run<2, true>(out, ticks, cus, iters, mhz);
  run<4, true>(out, ticks, cus, iters, mhz);
  (void)hipFree(out);
  (void)hipFree(ticks);
  return 0;
}
