// MFMA source-operand overwrite (WAR) timing probe (gfx950).
//
// Question: how many wait states must separate an MFMA from a VALU instruction that OVERWRITES one
// of its source registers (SrcC held in other registers than the destination, or A)?  The compiler
// lets a v_mov / v_add write an in-flight MFMA's SrcC registers 3 wait states after it in the LSTM
// tangent reverse (scripts/isa_mfma_hazards.py war_census).  The MFMA below computes
// dst = A B + C with C = 1000 in registers other than dst; N wait states later the C registers (mode
// C) or the A registers (mode A) are zeroed.  A clean result is 1000 + K in every register; a result
// of K (C read after the overwrite) or 1000 (A read after it) is counted per register.
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_war_probe.hip -o scripts/probes/mfma_war_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// the MFMA sequence for one opcode and A/B register width
#define SEQ(OPC, AR, BR)                                                   \
  OPC " v[48:51], " AR ", " BR ", v[48:51]\n" OPC " v[52:55], " AR ", " BR ", v[52:55]\n" \
  OPC " v[56:59], " AR ", " BR ", v[56:59]\n" OPC " v[40:43], " AR ", " BR ", v[44:47]\n"

#define CLOBBERS "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", \
  "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", \
  "v70", "v71", "v72", "v73"

template <int K32, int MODE, int N>
__global__ void probe(float* out, int reps) {
  float bad[4] = {0.f, 0.f, 0.f, 0.f};
  const float want = 1000.f + (K32 ? 32.f : 16.f);
  for (int r = 0; r < reps; ++r) {
    float o0, o1, o2, o3;
    // init: A = B = bf16 1.0 (0x3F80 in both halves), accumulators zero
#define INIT                                                                                          \
  "v_mov_b32 v60, 0x3f803f80\nv_mov_b32 v61, 0x3f803f80\nv_mov_b32 v62, 0x3f803f80\n"                 \
  "v_mov_b32 v63, 0x3f803f80\nv_mov_b32 v64, 0x3f803f80\nv_mov_b32 v65, 0x3f803f80\n"                 \
  "v_mov_b32 v66, 0x3f803f80\nv_mov_b32 v67, 0x3f803f80\n"                                             \
  "v_mov_b32 v40, 0\nv_mov_b32 v41, 0\nv_mov_b32 v42, 0\nv_mov_b32 v43, 0\n"                          \
  "v_mov_b32 v44, 0x447a0000\nv_mov_b32 v45, 0x447a0000\nv_mov_b32 v46, 0x447a0000\nv_mov_b32 v47, 0x447a0000\n"                          \
  "v_mov_b32 v48, 0\nv_mov_b32 v49, 0\nv_mov_b32 v50, 0\nv_mov_b32 v51, 0\n"                          \
  "v_mov_b32 v52, 0\nv_mov_b32 v53, 0\nv_mov_b32 v54, 0\nv_mov_b32 v55, 0\n"                          \
  "v_mov_b32 v56, 0\nv_mov_b32 v57, 0\nv_mov_b32 v58, 0\nv_mov_b32 v59, 0\ns_nop 15\n"
#define OVW_C "v_mov_b32 v44, 0\nv_mov_b32 v45, 0\nv_mov_b32 v46, 0\nv_mov_b32 v47, 0\n"
#define OVW_A "v_mov_b32 v60, 0\nv_mov_b32 v61, 0\nv_mov_b32 v62, 0\nv_mov_b32 v63, 0\n"
#define TAIL                                                                                          \
  "s_nop 15\ns_nop 15\nv_mov_b32 v70, v40\nv_mov_b32 v71, v41\nv_mov_b32 v72, v42\nv_mov_b32 v73, v43\ns_nop 15\ns_nop 15\n" \
  "v_mov_b32 %0, v70\nv_mov_b32 %1, v71\nv_mov_b32 %2, v72\nv_mov_b32 %3, v73\n"
#define P(OPC, AR, BR, OVW)                                                                            \
  asm volatile(INIT SEQ(OPC, AR, BR) "s_nop %4\n" OVW TAIL                                                 \
               : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)                                                      \
               : "i"(N)                                                                                        \
               : CLOBBERS)
    if constexpr (K32 && MODE == 0) P("v_mfma_f32_16x16x32_bf16", "v[60:63]", "v[64:67]", OVW_C);
    else if constexpr (K32) P("v_mfma_f32_16x16x32_bf16", "v[60:63]", "v[64:67]", OVW_A);
    else if constexpr (MODE == 0) P("v_mfma_f32_16x16x16_bf16", "v[60:61]", "v[64:65]", OVW_C);
    else P("v_mfma_f32_16x16x16_bf16", "v[60:61]", "v[64:65]", OVW_A);
#undef P
    bad[0] += o0 != want;
    bad[1] += o1 != want;
    bad[2] += o2 != want;
    bad[3] += o3 != want;
  }
  for (int i = 0; i < 4; ++i) atomicAdd(out + i, bad[i]);
}

template <int K32, int MODE, int N>
static void run(float* d, int blocks, int reps) {
  (void)hipMemset(d, 0, 4 * sizeof(float));
  hipLaunchKernelGGL((probe<K32, MODE, N>), dim3(blocks), dim3(256), 0, 0, d, reps);
  float h[4];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // s_nop N = N + 1 wait states; the TAIL's first v_mov reads v40 right after it
  printf("{\"mfma\": \"%s\", \"overwritten\": \"%s\", \"wait_states\": %d, \"bad\": [%.0f, %.0f, %.0f, %.0f], \"reads\": %.0f}\n",
         K32 ? "16x16x32_bf16" : "16x16x16_bf16", MODE ? "A" : "SrcC", N + 1, h[0], h[1], h[2], h[3],
         (double)blocks * 256 * reps);
  fflush(stdout);
}

template <int K32, int MODE>
static void sweep(float* d, int blocks, int reps) {
  run<K32, MODE, 0>(d, blocks, reps);
  run<K32, MODE, 1>(d, blocks, reps);
  run<K32, MODE, 2>(d, blocks, reps);
  run<K32, MODE, 3>(d, blocks, reps);
  run<K32, MODE, 4>(d, blocks, reps);
  run<K32, MODE, 5>(d, blocks, reps);
  run<K32, MODE, 6>(d, blocks, reps);
  run<K32, MODE, 7>(d, blocks, reps);
  run<K32, MODE, 8>(d, blocks, reps);
  run<K32, MODE, 9>(d, blocks, reps);
  run<K32, MODE, 10>(d, blocks, reps);
  run<K32, MODE, 11>(d, blocks, reps);
  run<K32, MODE, 12>(d, blocks, reps);
  run<K32, MODE, 15>(d, blocks, reps);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048, reps = argc > 2 ? atoi(argv[2]) : 64;
  float* d;
  if (hipMalloc(&d, 4 * sizeof(float)) != hipSuccess) return 1;
  sweep<0, 0>(d, blocks, reps);
  sweep<1, 0>(d, blocks, reps);
  sweep<0, 1>(d, blocks, reps);
  sweep<1, 1>(d, blocks, reps);
  (void)hipFree(d);
  return 0;
}
