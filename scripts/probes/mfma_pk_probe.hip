// MFMA result -> PACKED fp32 VALU read timing probe (gfx950).
//
// Question: does a packed fp32 VALU instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32, which read a
// VGPR PAIR) need more wait states after the MFMA that writes the pair than a plain VALU read
// (mfma_raw_probe.hip: v_mov needs 5 after 16x16x16_bf16, 7 after 16x16x32_bf16)?  The nondeterministic
// bf16 kernel variants (profiles/r02_det) lose exactly one VGPR pair of an accumulator tile, and the
// compiler feeds MFMA results to v_pk_add_f32 8 wait states after the MFMA (scripts/isa_mfma_hazard.py).
//
// Same frame as mfma_raw_probe.hip (one asm block, fixed registers: 4 independent MFMAs, a dependent
// chain of 4 into v[40:43], N wait states of s_nop), then the consumer C reads v[40:41] and v[42:43]:
// C = 0 v_mov (control), 1 v_pk_add_f32 (+ 0), 2 v_pk_mul_f32 (x 1), 3 v_pk_fma_f32 (x 1 + 0).
// A stale read is a value != 4 K.  Output per (opcode, consumer, N): stale lanes per register.
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_pk_probe.hip -o scripts/probes/mfma_pk_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define SEQ(OPC, AR, BR)                                                   \
  OPC " v[44:47], " AR ", " BR ", v[44:47]\n" OPC " v[48:51], " AR ", " BR ", v[48:51]\n" \
  OPC " v[52:55], " AR ", " BR ", v[52:55]\n" OPC " v[56:59], " AR ", " BR ", v[56:59]\n" \
  OPC " v[40:43], " AR ", " BR ", v[40:43]\n" OPC " v[40:43], " AR ", " BR ", v[40:43]\n" \
  OPC " v[40:43], " AR ", " BR ", v[40:43]\n" OPC " v[40:43], " AR ", " BR ", v[40:43]\n"

#define CLOBBERS "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", \
  "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", \
  "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77"

#define INIT                                                                                          \
  "v_mov_b32 v60, 0x3f803f80\nv_mov_b32 v61, 0x3f803f80\nv_mov_b32 v62, 0x3f803f80\n"                 \
  "v_mov_b32 v63, 0x3f803f80\nv_mov_b32 v64, 0x3f803f80\nv_mov_b32 v65, 0x3f803f80\n"                 \
  "v_mov_b32 v66, 0x3f803f80\nv_mov_b32 v67, 0x3f803f80\n"                                             \
  "v_mov_b32 v40, 0\nv_mov_b32 v41, 0\nv_mov_b32 v42, 0\nv_mov_b32 v43, 0\n"                          \
  "v_mov_b32 v44, 0\nv_mov_b32 v45, 0\nv_mov_b32 v46, 0\nv_mov_b32 v47, 0\n"                          \
  "v_mov_b32 v48, 0\nv_mov_b32 v49, 0\nv_mov_b32 v50, 0\nv_mov_b32 v51, 0\n"                          \
  "v_mov_b32 v52, 0\nv_mov_b32 v53, 0\nv_mov_b32 v54, 0\nv_mov_b32 v55, 0\n"                          \
  "v_mov_b32 v56, 0\nv_mov_b32 v57, 0\nv_mov_b32 v58, 0\nv_mov_b32 v59, 0\n"                          \
  "v_mov_b32 v74, 0\nv_mov_b32 v75, 0\nv_mov_b32 v76, 1.0\nv_mov_b32 v77, 1.0\ns_nop 15\n"
#define OUT                                                                                           \
  "s_nop 15\ns_nop 15\nv_mov_b32 %0, v70\nv_mov_b32 %1, v71\nv_mov_b32 %2, v72\nv_mov_b32 %3, v73\n"

#define C_MOV "v_mov_b32 v70, v40\nv_mov_b32 v71, v41\nv_mov_b32 v72, v42\nv_mov_b32 v73, v43\n"
#define C_ADD "v_pk_add_f32 v[70:71], v[40:41], v[74:75]\nv_pk_add_f32 v[72:73], v[42:43], v[74:75]\n"
#define C_MUL "v_pk_mul_f32 v[70:71], v[40:41], v[76:77]\nv_pk_mul_f32 v[72:73], v[42:43], v[76:77]\n"
#define C_FMA "v_pk_fma_f32 v[70:71], v[40:41], v[76:77], v[74:75]\nv_pk_fma_f32 v[72:73], v[42:43], v[76:77], v[74:75]\n"

#define BODY(SEQS, CONS)                                                                   \
  asm volatile(INIT SEQS "s_nop %4\n" CONS OUT : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3) : "i"(N) : CLOBBERS)

template <int K32, int C, int N>
__global__ void probe(float* out, int reps) {
  float bad[4] = {0.f, 0.f, 0.f, 0.f};
  const float want = K32 ? 128.f : 64.f;
  for (int r = 0; r < reps; ++r) {
    float o0, o1, o2, o3;
    if constexpr (K32) {
#define S32 SEQ("v_mfma_f32_16x16x32_bf16", "v[60:63]", "v[64:67]")
      if constexpr (C == 0) BODY(S32, C_MOV);
      else if constexpr (C == 1) BODY(S32, C_ADD);
      else if constexpr (C == 2) BODY(S32, C_MUL);
      else BODY(S32, C_FMA);
    } else {
#define S16 SEQ("v_mfma_f32_16x16x16_bf16", "v[60:61]", "v[64:65]")
      if constexpr (C == 0) BODY(S16, C_MOV);
      else if constexpr (C == 1) BODY(S16, C_ADD);
      else if constexpr (C == 2) BODY(S16, C_MUL);
      else BODY(S16, C_FMA);
    }
    bad[0] += o0 != want;
    bad[1] += o1 != want;
    bad[2] += o2 != want;
    bad[3] += o3 != want;
  }
  for (int i = 0; i < 4; ++i) atomicAdd(out + i, bad[i]);
}

static const char* CN[4] = {"v_mov", "v_pk_add_f32", "v_pk_mul_f32", "v_pk_fma_f32"};

template <int K32, int C, int N>
static void run(float* d, int blocks, int reps) {
  (void)hipMemset(d, 0, 4 * sizeof(float));
  hipLaunchKernelGGL((probe<K32, C, N>), dim3(blocks), dim3(256), 0, 0, d, reps);
  float h[4];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("{\"mfma\": \"%s\", \"consumer\": \"%s\", \"wait_states\": %d, \"stale\": [%.0f, %.0f, %.0f, %.0f], \"reads\": %.0f}\n",
         K32 ? "16x16x32_bf16" : "16x16x16_bf16", CN[C], N + 1, h[0], h[1], h[2], h[3], (double)blocks * 256 * reps);
  fflush(stdout);
}

template <int K32, int C>
static void sweep(float* d, int blocks, int reps) {
  run<K32, C, 2>(d, blocks, reps);
  run<K32, C, 3>(d, blocks, reps);
  run<K32, C, 4>(d, blocks, reps);
  run<K32, C, 5>(d, blocks, reps);
  run<K32, C, 6>(d, blocks, reps);
  run<K32, C, 7>(d, blocks, reps);
  run<K32, C, 8>(d, blocks, reps);
  run<K32, C, 9>(d, blocks, reps);
  run<K32, C, 10>(d, blocks, reps);
  run<K32, C, 11>(d, blocks, reps);
  run<K32, C, 13>(d, blocks, reps);
  run<K32, C, 15>(d, blocks, reps);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048, reps = argc > 2 ? atoi(argv[2]) : 64;
  float* d;
  if (hipMalloc(&d, 4 * sizeof(float)) != hipSuccess) return 1;
  sweep<0, 0>(d, blocks, reps);
  sweep<0, 1>(d, blocks, reps);
  sweep<0, 2>(d, blocks, reps);
  sweep<0, 3>(d, blocks, reps);
  sweep<1, 0>(d, blocks, reps);
  sweep<1, 1>(d, blocks, reps);
  sweep<1, 2>(d, blocks, reps);
  sweep<1, 3>(d, blocks, reps);
  (void)hipFree(d);
  return 0;
}
