// MFMA result -> VALU read timing probe (gfx950).
//
// Question: how many wait states must separate a v_mfma_f32_16x16x16_bf16 / 16x16x32_bf16 from a
// VALU instruction that reads its result?  The compiler places such reads 8 wait states after the
// 16x16x16 (K = 16 tail) MFMA in the LSTM kernels; kernel variants showed run-to-run different
// values in exactly one VGPR pair of an accumulator tile.
//
// Each lane runs, inside ONE asm block with fixed physical registers (so no compiler pass can add
// or move wait states): 4 independent MFMAs (pipe pressure), a dependent chain of 4 MFMAs into
// v[40:43] (each adds K to every element), N wait states of s_nop, then v_mov of v40..v43.
// A stale read is a value != 4 K.  Output per N: stale lanes per accumulator register, summed
// over all waves and repetitions.
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_raw_probe.hip -o scripts/probes/mfma_raw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// the MFMA sequence for one opcode and A/B register width
#define SEQ(OPC, AR, BR)                                                   \
  OPC " v[44:47], " AR ", " BR ", v[44:47]\n" OPC " v[48:51], " AR ", " BR ", v[48:51]\n" \
  OPC " v[52:55], " AR ", " BR ", v[52:55]\n" OPC " v[56:59], " AR ", " BR ", v[56:59]\n" \
  OPC " v[40:43], " AR ", " BR ", v[40:43]\n" OPC " v[40:43], " AR ", " BR ", v[40:43]\n" \
  OPC " v[40:43], " AR ", " BR ", v[40:43]\n" OPC " v[40:43], " AR ", " BR ", v[40:43]\n"

#define CLOBBERS "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", \
  "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", \
  "v70", "v71", "v72", "v73"

template <int K32, int N>
__global__ void probe(float* out, int reps) {
  float bad[4] = {0.f, 0.f, 0.f, 0.f};
  const float want = K32 ? 128.f : 64.f;
  for (int r = 0; r < reps; ++r) {
    float o0, o1, o2, o3;
    // init: A = B = bf16 1.0 (0x3F80 in both halves), accumulators zero
#define INIT                                                                                          \
  "v_mov_b32 v60, 0x3f803f80\nv_mov_b32 v61, 0x3f803f80\nv_mov_b32 v62, 0x3f803f80\n"                 \
  "v_mov_b32 v63, 0x3f803f80\nv_mov_b32 v64, 0x3f803f80\nv_mov_b32 v65, 0x3f803f80\n"                 \
  "v_mov_b32 v66, 0x3f803f80\nv_mov_b32 v67, 0x3f803f80\n"                                             \
  "v_mov_b32 v40, 0\nv_mov_b32 v41, 0\nv_mov_b32 v42, 0\nv_mov_b32 v43, 0\n"                          \
  "v_mov_b32 v44, 0\nv_mov_b32 v45, 0\nv_mov_b32 v46, 0\nv_mov_b32 v47, 0\n"                          \
  "v_mov_b32 v48, 0\nv_mov_b32 v49, 0\nv_mov_b32 v50, 0\nv_mov_b32 v51, 0\n"                          \
  "v_mov_b32 v52, 0\nv_mov_b32 v53, 0\nv_mov_b32 v54, 0\nv_mov_b32 v55, 0\n"                          \
  "v_mov_b32 v56, 0\nv_mov_b32 v57, 0\nv_mov_b32 v58, 0\nv_mov_b32 v59, 0\ns_nop 15\n"
#define TAIL                                                                                          \
  "v_mov_b32 v70, v40\nv_mov_b32 v71, v41\nv_mov_b32 v72, v42\nv_mov_b32 v73, v43\ns_nop 15\ns_nop 15\n" \
  "v_mov_b32 %0, v70\nv_mov_b32 %1, v71\nv_mov_b32 %2, v72\nv_mov_b32 %3, v73\n"
    if constexpr (K32) {
      asm volatile(INIT SEQ("v_mfma_f32_16x16x32_bf16", "v[60:63]", "v[64:67]") "s_nop %4\n" TAIL
                   : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)
                   : "i"(N)
                   : CLOBBERS);
    } else {
      asm volatile(INIT SEQ("v_mfma_f32_16x16x16_bf16", "v[60:61]", "v[64:65]") "s_nop %4\n" TAIL
                   : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)
                   : "i"(N)
                   : CLOBBERS);
    }
    bad[0] += o0 != want;
    bad[1] += o1 != want;
    bad[2] += o2 != want;
    bad[3] += o3 != want;
  }
  for (int i = 0; i < 4; ++i) atomicAdd(out + i, bad[i]);
}

template <int K32, int N>
static void run(float* d, int blocks, int reps) {
  (void)hipMemset(d, 0, 4 * sizeof(float));
  hipLaunchKernelGGL((probe<K32, N>), dim3(blocks), dim3(256), 0, 0, d, reps);
  float h[4];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // s_nop N = N + 1 wait states; the TAIL's first v_mov reads v40 right after it
  printf("{\"mfma\": \"%s\", \"wait_states\": %d, \"stale\": [%.0f, %.0f, %.0f, %.0f], \"reads\": %.0f}\n",
         K32 ? "16x16x32_bf16" : "16x16x16_bf16", N + 1, h[0], h[1], h[2], h[3], (double)blocks * 256 * reps);
  fflush(stdout);
}

template <int K32>
static void sweep(float* d, int blocks, int reps) {
  run<K32, 0>(d, blocks, reps);
  run<K32, 1>(d, blocks, reps);
  run<K32, 2>(d, blocks, reps);
  run<K32, 3>(d, blocks, reps);
  run<K32, 4>(d, blocks, reps);
  run<K32, 5>(d, blocks, reps);
  run<K32, 6>(d, blocks, reps);
  run<K32, 7>(d, blocks, reps);
  run<K32, 8>(d, blocks, reps);
  run<K32, 9>(d, blocks, reps);
  run<K32, 10>(d, blocks, reps);
  run<K32, 11>(d, blocks, reps);
  run<K32, 12>(d, blocks, reps);
  run<K32, 15>(d, blocks, reps);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048, reps = argc > 2 ? atoi(argv[2]) : 64;
  float* d;
  if (hipMalloc(&d, 4 * sizeof(float)) != hipSuccess) return 1;
  sweep<0>(d, blocks, reps);
  sweep<1>(d, blocks, reps);
  (void)hipFree(d);
  return 0;
}
