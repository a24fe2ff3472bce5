// MFMA -> MFMA SrcC forwarding across DIFFERENT opcodes (gfx950).
//
// Question: the compiler chains a 16-wide tail step (v_mfma_f32_16x16x16_bf16) onto a
// v_mfma_f32_16x16x32_bf16 accumulator with as few as 1 wait state between them
// (scripts/isa_mfma_srcc.py over the shipped kernels), as if the pipe forwarded the accumulator between
// the two opcodes.  Does it?  The bf16 tangent reverse (act = sigmoid) loses rows 4 g + {0, 1} of one
// accumulator tile run to run (profiles/r03_race) right where such a pair sits.
//
// One asm block per lane and rep, fixed registers: 4 independent MFMAs keep the pipe busy, then the
// WRITER (ones x ones into v[40:43], from 0) and, N wait states later, the READER with SrcC = v[40:43]
// (dst v[44:47]); all operands are ones, so the reader's result is K_writer + K_reader exactly.  A read
// of the stale accumulator gives K_reader.  Pairs: 0 = 16x16x32 -> 16x16x16 (bf16), 1 = 16x16x16 ->
// 16x16x32, 2 = 16x16x32 -> 16x16x32 (control, same opcode), 3 = 16x16x32 bf16 -> 16x16x4 f32,
// 4 = 16x16x4 f32 -> 16x16x32 bf16, 5 = 16x16x16 -> 16x16x16 (same opcode, the short one).  Output per (pair, N): stale lanes per result register.
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_srcc_probe.hip -o scripts/probes/mfma_srcc_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define INIT                                                                                          \
  "v_mov_b32 v60, 0x3f803f80\nv_mov_b32 v61, 0x3f803f80\nv_mov_b32 v62, 0x3f803f80\n"                 \
  "v_mov_b32 v63, 0x3f803f80\nv_mov_b32 v64, 0x3f803f80\nv_mov_b32 v65, 0x3f803f80\n"                 \
  "v_mov_b32 v66, 0x3f803f80\nv_mov_b32 v67, 0x3f803f80\nv_mov_b32 v68, 1.0\nv_mov_b32 v69, 1.0\n"    \
  "v_mov_b32 v40, 0\nv_mov_b32 v41, 0\nv_mov_b32 v42, 0\nv_mov_b32 v43, 0\n"                          \
  "v_mov_b32 v44, 0\nv_mov_b32 v45, 0\nv_mov_b32 v46, 0\nv_mov_b32 v47, 0\n"                          \
  "v_mov_b32 v48, 0\nv_mov_b32 v49, 0\nv_mov_b32 v50, 0\nv_mov_b32 v51, 0\n"                          \
  "v_mov_b32 v52, 0\nv_mov_b32 v53, 0\nv_mov_b32 v54, 0\nv_mov_b32 v55, 0\n"                          \
  "v_mov_b32 v56, 0\nv_mov_b32 v57, 0\nv_mov_b32 v58, 0\nv_mov_b32 v59, 0\ns_nop 15\n"                 \
  "v_mfma_f32_16x16x32_bf16 v[48:51], v[60:63], v[64:67], v[48:51]\n"                                 \
  "v_mfma_f32_16x16x32_bf16 v[52:55], v[60:63], v[64:67], v[52:55]\n"                                 \
  "v_mfma_f32_16x16x32_bf16 v[56:59], v[60:63], v[64:67], v[56:59]\n"                                 \
  "v_mfma_f32_16x16x32_bf16 v[48:51], v[60:63], v[64:67], v[48:51]\n"
#define M32 "v_mfma_f32_16x16x32_bf16 "
#define M16 "v_mfma_f32_16x16x16_bf16 "
#define MF4 "v_mfma_f32_16x16x4_f32 "
#define W32 M32 "v[40:43], v[60:63], v[64:67], v[40:43]\n"
#define W16 M16 "v[40:43], v[60:61], v[64:65], v[40:43]\n"
#define WF4 MF4 "v[40:43], v68, v69, v[40:43]\n"
#define R32 M32 "v[44:47], v[60:63], v[64:67], v[40:43]\n"
#define R16 M16 "v[44:47], v[60:61], v[64:65], v[40:43]\n"
#define RF4 MF4 "v[44:47], v68, v69, v[40:43]\n"
#define TAIL                                                                                          \
  "s_nop 15\ns_nop 15\nv_mov_b32 %0, v44\nv_mov_b32 %1, v45\nv_mov_b32 %2, v46\nv_mov_b32 %3, v47\n"
#define CLOBBERS "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", \
  "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", \
  "v68", "v69"
#define BODY(W, R) asm volatile(INIT W "s_nop %4\n" R TAIL : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3) : "i"(N) : CLOBBERS)

template <int P, int N>
__global__ void probe(float* out, int reps) {
  float bad[4] = {0.f, 0.f, 0.f, 0.f};
  // K of writer + reader: 32 + 16, 16 + 32, 32 + 32, 32 + 4, 4 + 32
  const float want = P == 0 ? 48.f : P == 1 ? 48.f : P == 2 ? 64.f : P == 3 ? 36.f : P == 4 ? 36.f : 32.f;
  for (int r = 0; r < reps; ++r) {
    float o0, o1, o2, o3;
    if constexpr (P == 0) BODY(W32, R16);
    else if constexpr (P == 1) BODY(W16, R32);
    else if constexpr (P == 2) BODY(W32, R32);
    else if constexpr (P == 3) BODY(W32, RF4);
    else if constexpr (P == 4) BODY(WF4, R32);
    else BODY(W16, R16);
    bad[0] += o0 != want;
    bad[1] += o1 != want;
    bad[2] += o2 != want;
    bad[3] += o3 != want;
  }
  for (int i = 0; i < 4; ++i) atomicAdd(out + i, bad[i]);
}

static const char* PN[6] = {"16x16x32_bf16 -> 16x16x16_bf16", "16x16x16_bf16 -> 16x16x32_bf16",
                            "16x16x32_bf16 -> 16x16x32_bf16", "16x16x32_bf16 -> 16x16x4_f32",
                            "16x16x4_f32 -> 16x16x32_bf16", "16x16x16_bf16 -> 16x16x16_bf16"};

template <int P, int N>
static void run(float* d, int blocks, int reps) {
  (void)hipMemset(d, 0, 4 * sizeof(float));
  hipLaunchKernelGGL((probe<P, N>), dim3(blocks), dim3(256), 0, 0, d, reps);
  float h[4];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("{\"pair\": \"%s\", \"wait_states\": %d, \"stale\": [%.0f, %.0f, %.0f, %.0f], \"reads\": %.0f}\n", PN[P], N + 1,
         h[0], h[1], h[2], h[3], (double)blocks * 256 * reps);
  fflush(stdout);
}

template <int P>
static void sweep(float* d, int blocks, int reps) {
  run<P, 0>(d, blocks, reps);
  run<P, 1>(d, blocks, reps);
  run<P, 2>(d, blocks, reps);
  run<P, 3>(d, blocks, reps);
  run<P, 4>(d, blocks, reps);
  run<P, 5>(d, blocks, reps);
  run<P, 6>(d, blocks, reps);
  run<P, 7>(d, blocks, reps);
  run<P, 8>(d, blocks, reps);
  run<P, 10>(d, blocks, reps);
  run<P, 12>(d, blocks, reps);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048, reps = argc > 2 ? atoi(argv[2]) : 64;
  float* d;
  if (hipMalloc(&d, 4 * sizeof(float)) != hipSuccess) return 1;
  sweep<0>(d, blocks, reps);
  sweep<1>(d, blocks, reps);
  sweep<2>(d, blocks, reps);
  sweep<3>(d, blocks, reps);
  sweep<4>(d, blocks, reps);
  sweep<5>(d, blocks, reps);
  (void)hipFree(d);
  return 0;
}
