// LSTM weight gradient v3 (bf16, gfx950): HBM-streaming split-M reduction with an LDS-DMA ring.
//
//     C[Ktot, N] = sum_m A[m,:]^T D[m,:],   A = [X | H_{t-1} | 1],  Ktot = K + Hd + 1,  N = 4 Hd
//
// (same contract as lstm_wgrad2 in gemm2.hip: C rows 0..K-1 -> gW, K..K+Hd-1 -> gU, K+Hd -> gb).
// The op reads ~1 GB per call at the flagship shape and does ~130 GFLOP: it is an HBM-streaming
// problem, so the design is organised around bytes in flight, not MFMA tiling:
//
//  * one workgroup per CU (8 waves, two per SIMD) owning ALL of C in registers: wave w holds i-group
//    w & 3 (i-blocks w & 3 + 4 k) x j-half w >> 2 (13 / 12 of the 25 j-blocks of 16x16 accumulators,
//    208 registers at K = 100); a split of M rows is walked in 32-row chunks, one MFMA k-step each.
//    Round 4 replaced two 208-column j-tiles on paired workgroups (the second X / H read an L2 hit):
//    LDS-DMA is bound per CU (~24 GB/s), so every X / H byte DMA'd twice cost time even from L2 --
//    full width moves 26 % (K = 100) / 22 % (K = 32) fewer bytes per CU and row (2.90 vs 3.40 ms and
//    2.43 vs 2.89 ms per call at the bench shape, profiles/r04_wgrad3);
//  * every chunk lands in LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction):
//    X rows m0..m0+31, H rows m0-1..m0+30 and the D rows are contiguous HBM ranges, copied raw (no transposes, no register staging) into a 4-deep ring, so three chunks
//    (~80 KB per CU) are in flight while the fourth is consumed.  Waits are counted
//    (s_waitcnt vmcnt(2 chunks)) and the barrier is a raw s_barrier, so the DMA is never drained
//    inside the loop;
//  * MFMA operands come straight from the raw row-major images via ds_read_b64_tr_b16 (the
//    reduction index m must sit inside each lane's fragment), with per-lane addresses: the
//    h_{t-1} shift, the m % T == 0 zero rows, the all-ones bias row and the tail mask are pointer
//    selects onto a 16-byte zero / ones pad in LDS, never data movement;
//  * the loop body is instantiated per wave index (wgrad3_wave<K, HD, W>).
// The fp32 partials go to per-split slabs reduced by lstm_wgrad2_reduce_kernel (deterministic).
#include "common.h"
#include "mfma.h"
#include "kernels.h"

namespace hfrep {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int W3_STAGES = 4;
constexpr int W3_WAVES = 8;

template <int K, int HD>
struct W3 {
  static constexpr int N = 4 * HD;
  static constexpr int JT = N;  // one full-width j-tile: each X / H / D chunk is DMA'd once
  static constexpr int NJB = JT / 16;
  static constexpr int NJT = (N + JT - 1) / JT;
  static constexpr int JBW = (NJB + 1) / 2;            // j-blocks per wave (waves 0-3: first half)
  static constexpr int KTOT = K + HD + 1;
  static constexpr int NIB = (KTOT + 15) / 16;
  static constexpr int IBW = (NIB + 3) / 4;            // i-blocks per wave (block ib = (wave & 3) + 4 k)
  static constexpr int XBYTES = 32 * K * 2;
  static constexpr int HBYTES = (8 + 32 * HD * 2 + 15) / 16 * 16;  // + up to 8 B of alignment slack
  static constexpr int XI = (XBYTES + 1023) / 1024;   // 1 KiB DMA instructions per chunk
  static constexpr int HI = (HBYTES + 1023) / 1024;
  static constexpr int DI = (32 * JT * 2) / 1024;
  static constexpr int NI = XI + HI + DI;
  static constexpr int NPW = (NI + W3_WAVES - 1) / W3_WAVES;  // per wave per chunk (uniform: counted waits)
  static constexpr int STAGE = NI * 1024;
  static constexpr int OFF_H = XI * 1024, OFF_D = (XI + HI) * 1024;
  static constexpr int TRASH = W3_STAGES * STAGE;     // dummy DMA target
  static constexpr int PADS = TRASH + 1024;           // 16 B zeros, then 16 B {1, 0, 0, 0} bf16
  static constexpr int LDS = PADS + 32;
  static_assert(K % 4 == 0 && HD % 4 == 0, "4-column groups must not straddle X/H");
  static_assert((32 * JT * 2) % 1024 == 0, "D image is whole DMA instructions");
  static_assert((W3_STAGES - 2) * NPW <= 63, "vmcnt range");
  static_assert(NJT == 1 && JT % 16 == 0, "one full-width tile of whole 16-column blocks");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// LDS-DMA of 16 bytes per lane from sbase + voff into lds_dst + 16 * lane (M0 = lds_dst)
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ bf16x8 tr2(uint32_t lo, uint32_t hi) {
  const v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)lo);
  const v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(uintptr_t)hi);
  bf16x8 f;
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  return f;
}

}  // namespace

// One wave's whole loop, with the wave index W a compile-time constant: the DMA plan (which image
// each of the wave's NPW instructions fills), the i-blocks / j-blocks it owns and their operand kinds
// fold into straight-line code.  With W a run-time value the loop carried ~150 scalar instructions
// and ~50 branches per 32-row chunk and wave (pointer selects per DMA slot, wave-kind tests;
// profiles/r04_wgrad3/README.md), which -- not the bytes -- set the chunk time.
template <int K, int HD, int W>
__device__ __forceinline__ void wgrad3_wave(const bf16_t* __restrict__ X0, const bf16_t* __restrict__ H0,
                                            const bf16_t* __restrict__ D0, const bf16_t* __restrict__ X1,
                                            const bf16_t* __restrict__ H1, const bf16_t* __restrict__ D1,
                                            float* __restrict__ slab, int M, int Tn, int nseg, int rps,
                                            unsigned char* smem, uint32_t lds0, int lane) {
  using G = W3<K, HD>;
  constexpr int w = W;
  constexpr int ig = w & 3, jh = w >> 2;  // i-group, j-half of this wave
  const int z = blockIdx.x, j0 = 0;  // split z: rows z * rps ..
  const int mb = z * rps, me = min(M, mb + rps);
  const int nchs = me > mb ? (me - mb + 31) / 32 : 0;  // chunks per segment
  const int nch = nchs * nseg;

  // ---- per-lane DMA geometry of this wave's NPW instructions (chunk independent)
  uint32_t voff[G::NPW], vdst[G::NPW];
  int vreg[G::NPW];   // 0 X, 1 H, 2 D, 3 dummy  (wave-uniform)
  bool von[G::NPW];   // lane carries bytes (X/H tails; D columns >= N on the last tile)
#pragma unroll
  for (int k = 0; k < G::NPW; ++k) {
    const int n = w + W3_WAVES * k;
    if (n < G::XI) {
      vreg[k] = 0; voff[k] = n * 1024 + lane * 16; vdst[k] = n * 1024; von[k] = voff[k] < (uint32_t)G::XBYTES;
    } else if (n < G::XI + G::HI) {
      const int nh = n - G::XI;
      vreg[k] = 1; voff[k] = nh * 1024 + lane * 16; vdst[k] = G::OFF_H + nh * 1024; von[k] = voff[k] < (uint32_t)G::HBYTES;
    } else if (n < G::NI) {
      const int nd = n - G::XI - G::HI, piece = nd * 64 + lane;
      const int r = piece / (G::JT / 8), cc = piece - r * (G::JT / 8);
      vreg[k] = 2; voff[k] = (uint32_t)(r * G::N * 2 + cc * 16); vdst[k] = G::OFF_D + nd * 1024;
      von[k] = true;  // (one full-width tile: every D piece is a real column)
    } else {
      vreg[k] = 3; voff[k] = 0; vdst[k] = G::TRASH; von[k] = lane == 0;
    }
  }

  // chunk c -> segment, first row m0 and the row the images start at (m0 clamped so the 32 rows exist)
  auto chunk_rows = [&](int c, int& s, int& m0, int& ml) {
    s = c >= nchs;
    m0 = mb + (c - s * nchs) * 32;
    ml = min(m0, M - 32);
  };
  auto issue = [&](int c, int st) {
    const uint32_t sb = lds0 + st * G::STAGE;
    if (c >= nch) {  // ring tail: keep the per-wave count uniform with 16-byte dummies
#pragma unroll
      for (int k = 0; k < G::NPW; ++k)
        if (lane == 0) glds16s(X0, 0u, lds0 + G::TRASH);
      return;
    }
    int s, m0, ml;
    chunk_rows(c, s, m0, ml);
    const char* xb = reinterpret_cast<const char*>(s ? X1 : X0) + (int64_t)ml * K * 2;
    const int64_t hraw = ((int64_t)ml - 1) * HD * 2;
    const char* hb = reinterpret_cast<const char*>(s ? H1 : H0) + (hraw < 0 ? 0 : (hraw & ~(int64_t)15));
    const char* db = reinterpret_cast<const char*>(s ? D1 : D0) + ((int64_t)ml * G::N + j0) * 2;
#pragma unroll
    for (int k = 0; k < G::NPW; ++k) {
      const void* base = vreg[k] == 0 ? (const void*)xb : vreg[k] == 1 ? (const void*)hb : vreg[k] == 2 ? (const void*)db
                                                                                                          : (const void*)X0;
      if (von[k]) glds16s(base, voff[k], (vreg[k] == 3 ? lds0 : sb) + vdst[k]);
    }
  };

  // ---- per-lane fragment geometry (chunk independent)
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int rlo = 8 * g + q;  // chunk rows of this lane's lo / hi tr-reads (hi = rlo + 4)
  int atype[G::IBW], aoff[G::IBW], astr[G::IBW];  // 0 X, 1 H, 2 bias, 3 zero
#pragma unroll
  for (int k = 0; k < G::IBW; ++k) {
    const int i = (ig + 4 * k) * 16 + 4 * p;
    if (i < K) { atype[k] = 0; aoff[k] = i * 2; astr[k] = K * 2; }
    else if (i < K + HD) { atype[k] = 1; aoff[k] = G::OFF_H + (i - K) * 2; astr[k] = HD * 2; }
    else if (i == K + HD) { atype[k] = 2; aoff[k] = 0; astr[k] = 0; }
    else { atype[k] = 3; aoff[k] = 0; astr[k] = 0; }
  }
  const uint32_t zero_pad = lds0 + G::PADS, ones_pad = lds0 + G::PADS + 16;
  const int jb0 = jh * G::JBW;  // first j-block of this wave
  const uint32_t doff = G::OFF_D + rlo * G::JT * 2 + 8 * p + jb0 * 32;

  f32x4 acc[G::IBW][G::JBW];
#pragma unroll
  for (int k = 0; k < G::IBW; ++k)
#pragma unroll
    for (int jb = 0; jb < G::JBW; ++jb) acc[k][jb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: S-1 chunks in flight
#pragma unroll
  for (int c = 0; c < W3_STAGES - 1; ++c) issue(c, c);

  int st = 0;
  for (int c = 0; c < nch; ++c) {
    wait_vm<(W3_STAGES - 2) * G::NPW>();  // this wave's DMA for chunk c has landed
    raw_barrier();                        // ... everyone's, and stage (c-1) is free
    issue(c + W3_STAGES - 1, st == 0 ? W3_STAGES - 1 : st - 1);
    const uint32_t sb = lds0 + st * G::STAGE;
    int s, m0, ml;
    chunk_rows(c, s, m0, ml);
    // H image origin: byte offset of row ml-1 inside the (16-byte aligned) H image
    const int64_t hraw = ((int64_t)ml - 1) * HD * 2;
    const int horg = (int)(hraw - (hraw < 0 ? 0 : (hraw & ~(int64_t)15)));
    const int mlo = ml + rlo, mhi = mlo + 4;
    const bool xlo = mlo >= m0 && mlo < me, xhi = mhi >= m0 && mhi < me;
    const bool hlo = xlo && (mlo % Tn) != 0, hhi = xhi && (mhi % Tn) != 0;
    bf16x8 af[G::IBW];
#pragma unroll
    for (int k = 0; k < G::IBW; ++k) {
      if (ig + 4 * k < G::NIB) {
        uint32_t alo, ahi;
        if (atype[k] == 0) {
          alo = xlo ? sb + aoff[k] + rlo * astr[k] : zero_pad;
          ahi = xhi ? sb + aoff[k] + (rlo + 4) * astr[k] : zero_pad;
        } else if (atype[k] == 1) {
          alo = hlo ? sb + horg + aoff[k] + rlo * astr[k] : zero_pad;
          ahi = hhi ? sb + horg + aoff[k] + (rlo + 4) * astr[k] : zero_pad;
        } else if (atype[k] == 2) {
          alo = (xlo && s == 0) ? ones_pad : zero_pad;
          ahi = (xhi && s == 0) ? ones_pad : zero_pad;
        } else {
          alo = ahi = zero_pad;
        }
        af[k] = tr2(alo, ahi);
      }
    }
#pragma unroll
    for (int jb = 0; jb < G::JBW; ++jb) {
      if (jb0 + jb < G::NJB) {
        const uint32_t d = sb + doff + jb * 32;
        const bf16x8 bfr = tr2(d, d + 4 * G::JT * 2);
#pragma unroll
        for (int k = 0; k < G::IBW; ++k)
          if (ig + 4 * k < G::NIB) acc[k][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], bfr, acc[k][jb], 0, 0, 0);
      }
    }
    st = st == W3_STAGES - 1 ? 0 : st + 1;
  }
  wait_vm<0>();  // retire the ring-tail dummies before the workgroup exits

  // 16x16 accumulator: col = lane & 15, row = 4 (lane >> 4) + reg
  float* out = slab + (size_t)z * G::KTOT * G::N;
#pragma unroll
  for (int k = 0; k < G::IBW; ++k) {
    if (ig + 4 * k >= G::NIB) continue;
#pragma unroll
    for (int jb = 0; jb < G::JBW; ++jb) {
      const int j = j0 + (jb0 + jb) * 16 + (lane & 15);
      if (jb0 + jb >= G::NJB) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = (ig + 4 * k) * 16 + 4 * (lane >> 4) + r;
        if (i < G::KTOT && j < G::N) out[(size_t)i * G::N + j] = acc[k][jb][r];
      }
    }
  }
}

template <int K, int HD>
__global__ void __launch_bounds__(512, 1)
lstm_wgrad3_kernel(const bf16_t* __restrict__ X0, const bf16_t* __restrict__ H0, const bf16_t* __restrict__ D0,
                   const bf16_t* __restrict__ X1, const bf16_t* __restrict__ H1, const bf16_t* __restrict__ D1,
                   float* __restrict__ slab, int M, int Tn, int nseg, int rps) {
  using G = W3<K, HD>;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 16) reinterpret_cast<uint16_t*>(smem + G::PADS)[tid] = (tid == 8) ? (uint16_t)0x3f80 : (uint16_t)0;
  __syncthreads();  // nothing in flight yet: the only full barrier of the kernel
#define HFREP_W3_WAVE(WV) wgrad3_wave<K, HD, WV>(X0, H0, D0, X1, H1, D1, slab, M, Tn, nseg, rps, smem, lds0, lane)
  switch (w) {
    case 0: HFREP_W3_WAVE(0); break;
    case 1: HFREP_W3_WAVE(1); break;
    case 2: HFREP_W3_WAVE(2); break;
    case 3: HFREP_W3_WAVE(3); break;
    case 4: HFREP_W3_WAVE(4); break;
    case 5: HFREP_W3_WAVE(5); break;
    case 6: HFREP_W3_WAVE(6); break;
    default: HFREP_W3_WAVE(7); break;
  }
#undef HFREP_W3_WAVE
}

template <int K, int HD>
static void run_wgrad3(const void* X0, const void* H0, const void* D0, const void* X1, const void* H1, const void* D1,
                       float* gW, float* gU, float* gb, int M, int Tn, int nsplit, float* ws, hipStream_t s) {
  using G = W3<K, HD>;
  int rps = (M + nsplit - 1) / nsplit;
  rps = (rps + 31) / 32 * 32;
  const int nseg = X1 ? 2 : 1;
  static bool attr = false;
  if (!attr) {
    HFREP_CHECK_HIP(hipFuncSetAttribute((const void*)lstm_wgrad3_kernel<K, HD>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  hipLaunchKernelGGL((lstm_wgrad3_kernel<K, HD>), dim3(nsplit * G::NJT), dim3(512), G::LDS, s, (const bf16_t*)X0,
                     (const bf16_t*)H0, (const bf16_t*)D0, (const bf16_t*)X1, (const bf16_t*)H1, (const bf16_t*)D1, ws,
                     M, Tn, nseg, rps);
  launch_lstm_wgrad2_reduce(ws, gW, gU, gb, nsplit, K, HD, G::N, s);
}

// one workgroup (one split of M) per CU at most; small M (the reference preset: B = 32, T = 48) takes
// fewer splits of >= 1024 rows, since every split writes (and the reduce reads) a whole 201 x 400
// fp32 slab (0.32 MB) however few rows it had
static int wgrad3_splits(int64_t M = -1) {
  const int cus = std::max(8, device_cu_count());
  if (M < 0) return cus;  // (workspace sizing: the maximum)
  const int64_t want = (M + 1023) / 1024;
  return (int)std::max<int64_t>(8, std::min<int64_t>(cus, want));
}

bool lstm_wgrad3_supported(int M, int K, int Hd, int N) {
  if (Hd != 100 || N != 4 * Hd || !(K == 32 || K == 100) || M < 64) return false;
  // whole 16-byte DMA pieces at every tensor end
  return ((int64_t)M * K * 2) % 16 == 0 && ((int64_t)M * Hd * 2) % 16 == 0 && ((int64_t)M * N * 2) % 16 == 0;
}

size_t lstm_wgrad3_workspace_floats(int K, int Hd, int N) { return (size_t)wgrad3_splits() * (K + Hd + 1) * N; }

bool launch_lstm_wgrad3(const void* X0, const void* H0, const void* D0, const void* X1, const void* H1, const void* D1,
                        float* gW, float* gU, float* gb, int M, int K, int Hd, int N, int Tn, float* ws, hipStream_t s) {
  if (M <= 0) return true;
  if (!lstm_wgrad3_supported(M, K, Hd, N)) return false;
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!(al(X0) && al(H0) && al(D0) && al(X1) && al(H1) && al(D1))) return false;
  const int ns = wgrad3_splits(M);
  if (K == 32) run_wgrad3<32, 100>(X0, H0, D0, X1, H1, D1, gW, gU, gb, M, Tn, ns, ws, s);
  else run_wgrad3<100, 100>(X0, H0, D0, X1, H1, D1, gW, gU, gb, M, Tn, ns, ws, s);
  return true;
}

}  // namespace hfrep
