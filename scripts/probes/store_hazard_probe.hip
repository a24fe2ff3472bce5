// Buffer-store data hazard probe (gfx950): is a store's data (or address) VGPR read late enough that an
// overwrite by the NEXT VALU instruction lands in memory?
//
// r02 found it for 16-byte stores with a register soffset (LLVM's model: the >8-byte store data hazard
// exists only when soffset is NOT a register, so the compiler added no wait state; rows 14 / 15 of the fp32
// BPTT's dZ tile were corrupt, profiles/r02_hazard).  The bf16 kernel variants that lose one accumulator
// register pair (profiles/r02_det) store their dX through 2-byte buffer stores with a register soffset
// followed by VALU writes of the same registers -- assumed safe by the ISA rule (<= 8 bytes), never
// measured.  Each mode: one asm block per lane and rep, fixed registers:
//   v_mov v40..43 <- data; buffer_store_<kind> v40[..], v44, s[desc], <soff> offen; v_mov v40..43 <- 0xdeadbeef
// then every stored slot is checked.  Mode 8 overwrites the voffset register v44 instead of the data;
// modes 9 / 10: a non-temporal 16- / 8-byte store followed at once by an LDS READ into its data registers
// (the data wave's LDS -> HBM tile copy pattern; the LDS holds 0xdeadbeef).
//
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/store_hazard_probe.hip -o scripts/probes/store_hazard_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __amdgpu_buffer_rsrc_t rsrc_t;

#define PRE "v_mov_b32 v40, %0\nv_mov_b32 v41, %0\nv_mov_b32 v42, %0\nv_mov_b32 v43, %0\nv_mov_b32 v44, %1\ns_nop 4\n"
#define POST "v_mov_b32 v40, 0xdeadbeef\nv_mov_b32 v41, 0xdeadbeef\nv_mov_b32 v42, 0xdeadbeef\nv_mov_b32 v43, 0xdeadbeef\n"
#define POSTA "v_mov_b32 v44, 0x7fff0000\n"
#define CLOB "v40", "v41", "v42", "v43", "v44", "memory"

// MODE: 0 short / 1 short_d16_hi / 2 dword / 3 dwordx2 / 4 dwordx4, soffset = SGPR (the uniform offset)
//       5 dwordx4 / 6 short / 7 dwordx2, soffset = 0 (inline constant)
//       8 short, SGPR soffset, the VOFFSET register overwritten next
template <int MODE>
__global__ void store_k(unsigned* out, int reps) {
  __shared__ unsigned lds[256 * 4];  // 0xdeadbeef everywhere: what a late data read of modes 9 / 10 would store
  for (int i = threadIdx.x; i < 256 * 4; i += blockDim.x) lds[i] = 0xdeadbeefu;
  __syncthreads();
  const unsigned lds_a = (unsigned)(size_t)(lds + 4 * threadIdx.x);
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7ffffff0, 0x00020000);
  for (int r = 0; r < reps; ++r) {
    const unsigned val = 0x40000000u + (unsigned)(r * nth + tid);  // (never 0xdeadbeef)
    const int slot = r * nth + tid;                                // one 16-byte slot per (lane, rep)
    const int soff = __builtin_amdgcn_readfirstlane((r & 7) * 16 * nth);
    const int voff = (slot - (r & 7) * nth) * 16;                  // voff + soff = 16 * slot
    if constexpr (MODE == 0)
      asm volatile(PRE "buffer_store_short v40, v44, %2, %3 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 1)
      asm volatile(PRE "buffer_store_short_d16_hi v40, v44, %2, %3 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 2)
      asm volatile(PRE "buffer_store_dword v40, v44, %2, %3 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 3)
      asm volatile(PRE "buffer_store_dwordx2 v[40:41], v44, %2, %3 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 4)
      asm volatile(PRE "buffer_store_dwordx4 v[40:43], v44, %2, %3 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 5)
      asm volatile(PRE "v_add_u32 v44, %3, v44\nbuffer_store_dwordx4 v[40:43], v44, %2, 0 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 6)
      asm volatile(PRE "v_add_u32 v44, %3, v44\nbuffer_store_short v40, v44, %2, 0 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 7)
      asm volatile(PRE "v_add_u32 v44, %3, v44\nbuffer_store_dwordx2 v[40:41], v44, %2, 0 offen\n" POST ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 8)
      asm volatile(PRE "buffer_store_short v40, v44, %2, %3 offen\n" POSTA ::"v"(val), "v"(voff), "s"(rs), "s"(soff) : CLOB);
    else if constexpr (MODE == 9)  // 16-byte store, then an LDS read into the data registers (no wait)
      asm volatile(PRE "v_add_u32 v44, %3, v44\nbuffer_store_dwordx4 v[40:43], v44, %2, 0 offen nt\nds_read_b128 v[40:43], %4\ns_waitcnt lgkmcnt(0)\n"
                   ::"v"(val), "v"(voff), "s"(rs), "s"(soff), "v"(lds_a) : CLOB);
    else  // 8-byte store, then an LDS read into the data registers
      asm volatile(PRE "v_add_u32 v44, %3, v44\nbuffer_store_dwordx2 v[40:41], v44, %2, 0 offen nt\nds_read_b64 v[40:41], %4\ns_waitcnt lgkmcnt(0)\n"
                   ::"v"(val), "v"(voff), "s"(rs), "s"(soff), "v"(lds_a) : CLOB);
  }
}

// count slots whose stored words differ from the expected value (the bytes a mode writes)
__global__ void check_k(const unsigned* out, int n, int mode, unsigned long long* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned want = 0x40000000u + (unsigned)i;
  const unsigned* s = out + 4 * (size_t)i;
  bool ok;
  switch (mode) {
    case 0: case 6: case 8: ok = (s[0] & 0xffffu) == (want & 0xffffu); break;
    case 1: ok = (s[0] & 0xffffu) == (want >> 16); break;
    case 2: ok = s[0] == want; break;
    case 3: case 7: case 10: ok = s[0] == want && s[1] == want; break;
    default: ok = s[0] == want && s[1] == want && s[2] == want && s[3] == want; break;
  }
  if (!ok) atomicAdd(bad, 1ull);
}

template <int MODE>
static void run(unsigned* d, unsigned long long* bad, int blocks, int reps) {
  const int n = blocks * 256 * reps;
  (void)hipMemset(d, 0, (size_t)n * 16);
  (void)hipMemset(bad, 0, sizeof(*bad));
  hipLaunchKernelGGL(store_k<MODE>, dim3(blocks), dim3(256), 0, 0, d, reps);
  hipLaunchKernelGGL(check_k, dim3((n + 255) / 256), dim3(256), 0, 0, d, n, MODE, bad);
  unsigned long long h = 0;
  (void)hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost);
  static const char* names[] = {"short sgpr-soff", "short_d16_hi sgpr-soff", "dword sgpr-soff", "dwordx2 sgpr-soff",
                                "dwordx4 sgpr-soff", "dwordx4 soff0", "short soff0", "dwordx2 soff0",
                                "short sgpr-soff, voffset overwritten", "dwordx4 nt soff0, then ds_read_b128 into the data",
                                "dwordx2 nt soff0, then ds_read_b64 into the data"};
  printf("{\"mode\": %d, \"store\": \"%s\", \"bad\": %llu, \"stores\": %d}\n", MODE, names[MODE], h, n);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 32;
  unsigned* d;
  unsigned long long* bad;
  if (hipMalloc(&d, (size_t)blocks * 256 * reps * 16) != hipSuccess || hipMalloc(&bad, 8) != hipSuccess) return 1;
  const bool lds_only = argc > 3 && atoi(argv[3]) == 1;
  for (int it = 0; it < 3; ++it) {
    if (lds_only) {
      run<9>(d, bad, blocks, reps);
      run<10>(d, bad, blocks, reps);
      continue;
    }
    run<0>(d, bad, blocks, reps);
    run<1>(d, bad, blocks, reps);
    run<2>(d, bad, blocks, reps);
    run<3>(d, bad, blocks, reps);
    run<4>(d, bad, blocks, reps);
    run<5>(d, bad, blocks, reps);
    run<6>(d, bad, blocks, reps);
    run<7>(d, bad, blocks, reps);
    run<8>(d, bad, blocks, reps);
    run<9>(d, bad, blocks, reps);
    run<10>(d, bad, blocks, reps);
  }
  (void)hipFree(d);
  (void)hipFree(bad);
  return 0;
}
