// MFMA GEMMs for the dense parts of the GAN/AE models (gfx950).
//
//  * linear:  C[M,N] = act(A[M,K] . W + bias)   (W fp32 (K,N), or W^T for input gradients)
//    -- Keras Dense on the last axis, the LSTM input projection x.W + b, the Flatten->Dense head
//    and every input-gradient product dZ.W^T.  Bias + activation are fused into the epilogue.
//  * wgrad:   gW[K,N] += X^T D, gb += colsum(D)  -- weight gradients reduce over M = batch*T
//    rows (up to millions), so the M axis is split across workgroups into fp32 slabs that one
//    reduce launch folds into the flat gradient buffer.  The bias gradient rides along as an
//    extra all-ones row of X^T (no separate column-sum kernel), and the LSTM's h_{t-1} operand is
//    produced by index arithmetic (shiftT) instead of materialising a shifted copy of h.
//
// Tiles are staged through LDS k-contiguous ([row][k], padded) so every MFMA fragment is one
// conflict-free ds_read (b128 for bf16, b32 for fp32); the blockIdx -> tile map is XCD-aware so
// the N tiles that re-read one A panel share an XCD's L2.
#include "common.h"
#include "mfma.h"
#include "kernels.h"
#include "mlp.h"

namespace hfrep {

constexpr int LBM = 128, LBN = 64, LBK = 32;

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks sharing bid % 8 (one XCD under round-robin dispatch) get contiguous ids
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <typename T>
__global__ void __launch_bounds__(256)
linear_kernel(const T* __restrict__ A, const float* __restrict__ W, const float* __restrict__ bias, T* __restrict__ C,
              int M, int N, int K, int w_trans, int act) {
  using P = MF<T>;
  constexpr int LK = LBK + P::LDS_PAD;
  __shared__ __attribute__((aligned(16))) T As[LBM * LK];
  __shared__ __attribute__((aligned(16))) T Bs[LBN * LK];
  const int ntn = (N + LBN - 1) / LBN, ntm = (M + LBM - 1) / LBM;
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int tm = tile / ntn, tn = tile % ntn;
  const int m0 = tm * LBM, n0 = tn * LBN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  f32x16 acc0 = zero16(), acc1 = zero16();
  for (int k0 = 0; k0 < K; k0 += LBK) {
    // stage A tile [128][32]: consecutive threads walk k (row-major A)
#pragma unroll 4
    for (int it = 0; it < (LBM * LBK) / 256; ++it) {
      const int e = tid + it * 256, r = e / LBK, kk = e % LBK;
      const int gm = m0 + r, gk = k0 + kk;
      As[r * LK + kk] = (gm < M && gk < K) ? A[(size_t)gm * K + gk] : Cvt<T>::from_f(0.f);
    }
    // stage W tile as Bs[n][k]
    if (!w_trans) {
#pragma unroll 4
      for (int it = 0; it < (LBN * LBK) / 256; ++it) {
        const int e = tid + it * 256, kk = e / LBN, n = e % LBN;
        const int gk = k0 + kk, gn = n0 + n;
        Bs[n * LK + kk] = Cvt<T>::from_f((gk < K && gn < N) ? W[(size_t)gk * N + gn] : 0.f);
      }
    } else {
#pragma unroll 4
      for (int it = 0; it < (LBN * LBK) / 256; ++it) {
        const int e = tid + it * 256, n = e / LBK, kk = e % LBK;
        const int gk = k0 + kk, gn = n0 + n;
        Bs[n * LK + kk] = Cvt<T>::from_f((gk < K && gn < N) ? W[(size_t)gn * K + gk] : 0.f);
      }
    }
    __syncthreads();
    const T* arow = As + (w * 32 + (lane & 31)) * LK;
    const T* b0 = Bs + (lane & 31) * LK;
    const T* b1 = Bs + (32 + (lane & 31)) * LK;
#pragma unroll
    for (int ks = 0; ks < LBK / P::KS; ++ks) {
      const typename P::frag a = P::lda(arow, ks, lane);
      acc0 = P::mma(a, P::lda(b0, ks, lane), acc0);
      acc1 = P::mma(a, P::lda(b1, ks, lane), acc1);
    }
    __syncthreads();
  }
  const int col0 = n0 + (lane & 31), col1 = col0 + 32;
  const float bb0 = (bias && col0 < N) ? bias[col0] : 0.f;
  const float bb1 = (bias && col1 < N) ? bias[col1] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + w * 32 + acc32_row(r, lane);
    if (row < M) {
      if (col0 < N) st_f(C + (size_t)row * N + col0, act_f(act, acc0[r] + bb0));
      if (col1 < N) st_f(C + (size_t)row * N + col1, act_f(act, acc1[r] + bb1));
    }
  }
}

// ---------------------------------------------------------------------------------------------
// weight gradient: slab[z][i][j] = sum_{m in split z} Xe(m, i) D(m, j),  i < K + has_bias
// ---------------------------------------------------------------------------------------------
constexpr int WBI = 64, WBJ = 64, WBM = 32;

template <typename T>
__global__ void __launch_bounds__(256)
wgrad_kernel(const T* __restrict__ X, const T* __restrict__ D, float* __restrict__ slab, int M, int K, int N,
             int has_bias, int shiftT, int rows_per_split) {
  using P = MF<T>;
  constexpr int LK = WBM + P::LDS_PAD;
  __shared__ __attribute__((aligned(16))) T As[WBI * LK];
  __shared__ __attribute__((aligned(16))) T Bs[WBJ * LK];
  const int Kr = K + has_bias;
  const int nti = (Kr + WBI - 1) / WBI, ntj = (N + WBJ - 1) / WBJ;
  const int ti = blockIdx.x / ntj, tj = blockIdx.x % ntj;
  const int i0 = ti * WBI, j0 = tj * WBJ;
  const int z = blockIdx.y;
  const int mb = z * rows_per_split, me = min(M, mb + rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wi = w >> 1, wj = w & 1;
  (void)nti;
  f32x16 acc = zero16();
  for (int m0 = mb; m0 < me; m0 += WBM) {
    // stage Xe^T tile: As[i][mm]; consecutive threads walk i (X row-major over i)
#pragma unroll 4
    for (int it = 0; it < (WBI * WBM) / 256; ++it) {
      const int e = tid + it * 256, mm = e / WBI, ii = e % WBI;
      const int gm = m0 + mm, gi = i0 + ii;
      float v = 0.f;
      if (gm < me) {
        if (gi < K) {
          if (shiftT > 0) {
            v = (gm % shiftT == 0) ? 0.f : ld_f(X + (size_t)(gm - 1) * K + gi);
          } else {
            v = ld_f(X + (size_t)gm * K + gi);
          }
        } else if (gi == K && has_bias) {
          v = 1.f;
        }
      }
      As[ii * LK + mm] = Cvt<T>::from_f(v);
    }
#pragma unroll 4
    for (int it = 0; it < (WBJ * WBM) / 256; ++it) {
      const int e = tid + it * 256, mm = e / WBJ, jj = e % WBJ;
      const int gm = m0 + mm, gj = j0 + jj;
      Bs[jj * LK + mm] = (gm < me && gj < N) ? D[(size_t)gm * N + gj] : Cvt<T>::from_f(0.f);
    }
    __syncthreads();
    const T* arow = As + (wi * 32 + (lane & 31)) * LK;
    const T* brow = Bs + (wj * 32 + (lane & 31)) * LK;
#pragma unroll
    for (int ks = 0; ks < WBM / P::KS; ++ks) acc = P::mma(P::lda(arow, ks, lane), P::lda(brow, ks, lane), acc);
    __syncthreads();
  }
  float* out = slab + (size_t)z * Kr * N;
  const int col = j0 + wj * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = i0 + wi * 32 + acc32_row(r, lane);
    if (row < Kr && col < N) out[(size_t)row * N + col] = acc[r];
  }
}

__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ gW, float* __restrict__ gb, int splits, int K,
                    int N, int has_bias) {
  const int Kr = K + has_bias;
  const int64_t total = (int64_t)Kr * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += slab[(size_t)z * total + e];
    const int i = (int)(e / N), j = (int)(e % N);
    if (i < K) gW[(size_t)i * N + j] += s;
    else gb[j] += s;
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 weight gradient on the bf16 matrix pipe for the narrow layers (K + 1 <= 128, N <= 128: the MLP
// generator's / discriminator's Dense layers, GAN/GAN.py:127-158, GAN/WGAN_GP.py:221-253).
// wgrad_kernel<float> above tiles the output 64 x 64 (each X / D element is read once per opposite
// tile), stages with one scalar load + div / mod per element and runs the exact fp32 MFMA
// (v_mfma_f32_32x32x2_f32: 1/16 of the bf16 rate): 2.8 ms per (6.3 M x 100)^T (6.3 M x 100).  Here one
// workgroup owns the whole output and walks 32-row chunks of its row range once: each chunk of X and D
// is loaded with coalesced dword loads (lanes over features, 8 rows per task), split exactly into three
// bf16 planes (hi / mid / lo: 8 mantissa bits each) and stored TRANSPOSED in LDS ([feature][row], 16-byte
// writes); the 6 plane products with terms >= 2^-24 (hh, hm, mh, hl, lh, mm) run on
// v_mfma_f32_32x32x16_bf16 -- the LSTM fp32 kernels' split (lstm_f32.hip split3), error within 2x the exact
// kernel's vs fp64.  The next chunk's loads are issued before the current chunk's MFMAs.  Row K of the X
// image is the ones row (bias gradient).  Slab rows per workgroup, fixed-order reduce (mlp_slab_sum).
// ---------------------------------------------------------------------------------------------
constexpr int WSR = 32;        // rows per chunk
constexpr int WSQ = WSR + 8;   // image row pitch (bf16): 80 bytes
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& mi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float a = v[j];  // (a scalar copy first: tests/test_isa_hazards.py bit_cast lint)
    const uint32_t u = __builtin_bit_cast(uint32_t, a), h = u & 0xffff0000u;
    const float r1 = a - __builtin_bit_cast(float, h);
    const uint32_t m = __builtin_bit_cast(uint32_t, r1) & 0xffff0000u;
    const float r2 = r1 - __builtin_bit_cast(float, m);
    hi[j] = (short)(h >> 16);
    mi[j] = (short)(m >> 16);
    lo[j] = (short)(__builtin_bit_cast(uint32_t, r2) >> 16);
  }
}

template <int NI, int NJ>
__global__ void __launch_bounds__(256)
wgrad_f32s_kernel(const float* __restrict__ X, const float* __restrict__ D, float* __restrict__ slab, int M, int K,
                  int N, int rows_per_split) {
  constexpr int PX = NI * 32 * WSQ, PD = NJ * 32 * WSQ;  // plane sizes (bf16)
  constexpr int TX = (NI + 1) / 2, TD = (NJ + 1) / 2;    // (feature, 8-row group) tasks per thread
  constexpr int TPW = (NI * NJ + 3) / 4;                 // output tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t img[3 * PX + 3 * PD];
  bf16_t* ix = img;
  bf16_t* id = img + 3 * PX;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, cl = lane & 31;
  const int mb = blockIdx.x * rows_per_split, me = min(M, mb + rows_per_split);
  for (int e = tid; e < (3 * PX + 3 * PD) / 8; e += 256) reinterpret_cast<bf16x8*>(img)[e] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  __syncthreads();
  if (tid < WSR) ix[K * WSQ + tid] = (bf16_t)0x3F80;  // ones row (hi plane): the bias gradient
  f32x16 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = zero16();
  float vx[TX][8], vd[TD][8];
  auto load = [&](int m0) {
#pragma unroll
    for (int q = 0; q < TX; ++q) {
      const int e = tid + 256 * q, i = e % K, rg = e / K;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = m0 + 8 * rg + j;
        vx[q][j] = (rg < 4 && r < me) ? X[(size_t)r * K + i] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < TD; ++q) {
      const int e = tid + 256 * q, j0 = e % N, rg = e / N;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = m0 + 8 * rg + j;
        vd[q][j] = (rg < 4 && r < me) ? D[(size_t)r * N + j0] : 0.f;
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int q = 0; q < TX; ++q) {
      const int e = tid + 256 * q, i = e % K, rg = e / K;
      if (rg < 4) {
        bf16x8 a, b, c;
        split8(vx[q], a, b, c);
        const int o = i * WSQ + 8 * rg;
        *reinterpret_cast<bf16x8*>(ix + o) = a;
        *reinterpret_cast<bf16x8*>(ix + PX + o) = b;
        *reinterpret_cast<bf16x8*>(ix + 2 * PX + o) = c;
      }
    }
#pragma unroll
    for (int q = 0; q < TD; ++q) {
      const int e = tid + 256 * q, j0 = e % N, rg = e / N;
      if (rg < 4) {
        bf16x8 a, b, c;
        split8(vd[q], a, b, c);
        const int o = j0 * WSQ + 8 * rg;
        *reinterpret_cast<bf16x8*>(id + o) = a;
        *reinterpret_cast<bf16x8*>(id + PD + o) = b;
        *reinterpret_cast<bf16x8*>(id + 2 * PD + o) = c;
      }
    }
  };
  load(mb);
  for (int m0 = mb; m0 < me; m0 += WSR) {
    stage();
    __syncthreads();
    load(m0 + WSR);  // the next chunk's loads fly during the MFMAs (past me: zeros, no access)
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = w + 4 * t;
      if (tile < NI * NJ) {
        const int ti = tile / NJ, tj = tile - ti * NJ;
#pragma unroll
        for (int ks = 0; ks < WSR / 16; ++ks) {
          const int ao = (32 * ti + cl) * WSQ + 16 * ks + 8 * h, bo = (32 * tj + cl) * WSQ + 16 * ks + 8 * h;
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ix + ao);
          const bf16x8 am = *reinterpret_cast<const bf16x8*>(ix + PX + ao);
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(ix + 2 * PX + ao);
          const bf16x8 bh = *reinterpret_cast<const bf16x8*>(id + bo);
          const bf16x8 bm = *reinterpret_cast<const bf16x8*>(id + PD + bo);
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(id + 2 * PD + bo);
          acc[t] = MF<bf16_t>::mma(am, bm, acc[t]);
          acc[t] = MF<bf16_t>::mma(al, bh, acc[t]);
          acc[t] = MF<bf16_t>::mma(ah, bl, acc[t]);
          acc[t] = MF<bf16_t>::mma(am, bh, acc[t]);
          acc[t] = MF<bf16_t>::mma(ah, bm, acc[t]);
          acc[t] = MF<bf16_t>::mma(ah, bh, acc[t]);
        }
      }
    }
    // The accumulators are read after the loop, behind the wave-uniform tile branch and the loop exit,
    // where LLVM's hazard recognizer does not count the XDL write -> read wait states
    // (tests/test_isa_hazards.py found 11 of 12): 16 explicit ones after each chunk's MFMAs (16 cycles
    // against ~1.5k of MFMA per chunk), which no MFMA may pass
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  }
  const int Kr = K + 1;
  float* out = slab + (size_t)blockIdx.x * Kr * N;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = w + 4 * t;
    if (tile < NI * NJ) {
      const int ti = tile / NJ, tj = tile - ti * NJ, col = 32 * tj + cl;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * ti + acc32_row(r, lane);
        if (row < Kr && col < N) out[(size_t)row * N + col] = acc[t][r];
      }
    }
  }
}

bool fp32_exact_mode() {
  static const bool v = [] {
    const char* e = getenv("HFREP_FP32_EXACT");
    return e && atoi(e) == 1;
  }();
  return v;
}
static bool wgrad_f32s_ok(int K, int N) {
  return !fp32_exact_mode() && K >= 1 && K + 1 <= 128 && N >= 1 && N <= 128;
}
static int wgrad_f32s_splits(int M) {
  const int want = (M + 1023) / 1024;  // >= 32 chunks per workgroup
  return std::max(1, std::min(want, device_cu_count() * 2));
}

static int wgrad_splits(int M, int K, int N) {
  const int Kr = K + 1;
  const int tiles = ((Kr + WBI - 1) / WBI) * ((N + WBJ - 1) / WBJ);
  int splits = (M + 2047) / 2048;                    // >= 2048 rows per split
  const int cap = max(1, 2048 / max(tiles, 1));     // <= ~2048 workgroups total
  splits = max(1, min(splits, cap));
  return splits;
}

size_t wgrad_workspace_floats(int M, int K, int N) {
  const int splits = std::max(wgrad_splits(M, K, N), wgrad_f32s_ok(K, N) ? wgrad_f32s_splits(M) : 1);
  return (size_t)splits * (size_t)(K + 1) * (size_t)N;
}

void launch_linear(int dt, const void* A, const float* W, const float* bias, void* C, int M, int N, int K,
                   int w_trans, int act, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const int nwg = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(linear_kernel<bf16_t>, dim3(nwg), dim3(256), 0, s, (const bf16_t*)A, W, bias, (bf16_t*)C, M,
                       N, K, w_trans, act);
  else
    hipLaunchKernelGGL(linear_kernel<float>, dim3(nwg), dim3(256), 0, s, (const float*)A, W, bias, (float*)C, M, N,
                       K, w_trans, act);
}

// narrow weight gradient (bf16, K % 4 == 0, K + 1 <= 128, N <= 32, no time shift: the generator's
// output Dense(F)): one 32-wide column block, 4 waves x 32 rows of C = [X | 1]^T D.  The generic
// kernel above stages both operands with one 2-byte load + div/mod per element and a 64-wide N
// tile (half of it padding for N = 32): 425 us per (393k x 100)^T (393k x 32) call.  Here rows
// are staged with 8-byte buffer loads (rows past the split read zeros) and transposed into LDS.
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256)
narrow_wgrad_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ D, float* __restrict__ slab, int M,
                    int K, int N, int has_bias, int rows_per_split) {
  using P = MF<bf16_t>;
  constexpr int LK = 32 + 8;
  __shared__ __attribute__((aligned(16))) bf16_t As[128 * LK];  // [i][m]: X^T chunk, row K = ones (bias)
  __shared__ __attribute__((aligned(16))) bf16_t Bs[32 * LK];   // [j][m]: D^T chunk
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int z = blockIdx.x;
  const int mb = z * rows_per_split, me = min(M, mb + rows_per_split);
  for (int i = tid; i < 128 * LK; i += 256) As[i] = 0;
  for (int i = tid; i < 32 * LK; i += 256) Bs[i] = 0;
  const int K4 = K / 4, N4 = (N + 3) / 4;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X + (size_t)mb * K), 0,
                                                                      (me - mb) * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(D + (size_t)mb * N), 0,
                                                                      (me - mb) * N * 2, 0x00020000);
  f32x16 acc = zero16();
  __syncthreads();
  for (int m0 = 0; m0 < me - mb; m0 += 32) {
    for (int e = tid; e < 32 * K4; e += 256) {
      const int r = e / K4, c = e - r * K4;
      const v2i v = __builtin_amdgcn_raw_buffer_load_b64(rx, ((m0 + r) * K + 4 * c) * 2, 0, 0);  // OOB rows -> 0
      const uint32_t lo = (uint32_t)v[0], hi = (uint32_t)v[1];
      As[(4 * c + 0) * LK + r] = (bf16_t)(lo & 0xffffu);
      As[(4 * c + 1) * LK + r] = (bf16_t)(lo >> 16);
      As[(4 * c + 2) * LK + r] = (bf16_t)(hi & 0xffffu);
      As[(4 * c + 3) * LK + r] = (bf16_t)(hi >> 16);
    }
    if (has_bias && tid < 32) As[K * LK + tid] = (m0 + tid < me - mb) ? (bf16_t)0x3f80 : (bf16_t)0;  // 1.0
    for (int e = tid; e < 32 * N4; e += 256) {
      const int r = e / N4, c = e - r * N4;
      const bool ok = 4 * c + 3 < N;  // (N % 4 != 0: the last group element-wise)
      if (ok) {
        const v2i v = __builtin_amdgcn_raw_buffer_load_b64(rd, ((m0 + r) * N + 4 * c) * 2, 0, 0);
        const uint32_t lo = (uint32_t)v[0], hi = (uint32_t)v[1];
        Bs[(4 * c + 0) * LK + r] = (bf16_t)(lo & 0xffffu);
        Bs[(4 * c + 1) * LK + r] = (bf16_t)(lo >> 16);
        Bs[(4 * c + 2) * LK + r] = (bf16_t)(hi & 0xffffu);
        Bs[(4 * c + 3) * LK + r] = (bf16_t)(hi >> 16);
      } else {
        for (int q = 0; q < 4 && 4 * c + q < N; ++q)
          Bs[(4 * c + q) * LK + r] = (bf16_t)__builtin_amdgcn_raw_buffer_load_b16(rd, ((m0 + r) * N + 4 * c + q) * 2, 0, 0);
      }
    }
    __syncthreads();
    const bf16_t* arow = As + (w * 32 + (lane & 31)) * LK;
    const bf16_t* brow = Bs + (lane & 31) * LK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) acc = P::mma(P::lda(arow, ks, lane), P::lda(brow, ks, lane), acc);
    __syncthreads();
  }
  const int Kr = K + has_bias;
  float* out = slab + (size_t)z * Kr * N;
  const int col = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = w * 32 + acc32_row(r, lane);
    if (row < Kr && col < N) out[(size_t)row * N + col] = acc[r];
  }
}

void launch_wgrad(int dt, const void* X, const void* D, float* gW, float* gb, int M, int K, int N, int shiftT,
                  float* ws, hipStream_t s) {
  if (M <= 0) return;
  if (dt == DT_BF16 && shiftT == 0 && K % 4 == 0 && K + 1 <= 128 && N <= 32) {
    const int splits = wgrad_splits(M, K, N);
    const int rps = ((M + splits - 1) / splits + 31) / 32 * 32;
    const int z = (M + rps - 1) / rps;
    hipLaunchKernelGGL(narrow_wgrad_kernel, dim3(z), dim3(256), 0, s, (const bf16_t*)X, (const bf16_t*)D, ws, M, K, N,
                       gb != nullptr ? 1 : 0, rps);
    const int blocks = (int)std::min<int64_t>(((int64_t)(K + 1) * N + 255) / 256, 1024);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, ws, gW, gb, z, K, N, gb != nullptr ? 1 : 0);
    return;
  }
  if (dt == DT_F32 && shiftT == 0 && wgrad_f32s_ok(K, N)) {
    const int P = wgrad_f32s_splits(M);
    const int rps = ((M + P - 1) / P + WSR - 1) / WSR * WSR;
    const int z = (M + rps - 1) / rps;
    const int ni = (K + 1 + 31) / 32, nj = (N + 31) / 32;
    auto go = [&](auto k) {
      hipLaunchKernelGGL(k, dim3(z), dim3(256), 0, s, (const float*)X, (const float*)D, ws, M, K, N, rps);
    };
    switch (ni * 4 + nj) {
      case 1 * 4 + 1: go(wgrad_f32s_kernel<1, 1>); break;
      case 1 * 4 + 2: go(wgrad_f32s_kernel<1, 2>); break;
      case 1 * 4 + 3: go(wgrad_f32s_kernel<1, 3>); break;
      case 1 * 4 + 4: go(wgrad_f32s_kernel<1, 4>); break;
      case 2 * 4 + 1: go(wgrad_f32s_kernel<2, 1>); break;
      case 2 * 4 + 2: go(wgrad_f32s_kernel<2, 2>); break;
      case 2 * 4 + 3: go(wgrad_f32s_kernel<2, 3>); break;
      case 2 * 4 + 4: go(wgrad_f32s_kernel<2, 4>); break;
      case 3 * 4 + 1: go(wgrad_f32s_kernel<3, 1>); break;
      case 3 * 4 + 2: go(wgrad_f32s_kernel<3, 2>); break;
      case 3 * 4 + 3: go(wgrad_f32s_kernel<3, 3>); break;
      case 3 * 4 + 4: go(wgrad_f32s_kernel<3, 4>); break;
      case 4 * 4 + 1: go(wgrad_f32s_kernel<4, 1>); break;
      case 4 * 4 + 2: go(wgrad_f32s_kernel<4, 2>); break;
      case 4 * 4 + 3: go(wgrad_f32s_kernel<4, 3>); break;
      default: go(wgrad_f32s_kernel<4, 4>); break;
    }
    const int64_t stride = (int64_t)(K + 1) * N;
    launch_mlp_slab_sum_cols(ws, z, stride, 0, K * N, gW, s);
    if (gb) launch_mlp_slab_sum_cols(ws, z, stride, K * N, N, gb, s);
    return;
  }
  const int has_bias = gb != nullptr;
  const int Kr = K + has_bias;
  const int splits = wgrad_splits(M, K, N);
  int rps = (M + splits - 1) / splits;
  rps = (rps + WBM - 1) / WBM * WBM;
  const int tiles = ((Kr + WBI - 1) / WBI) * ((N + WBJ - 1) / WBJ);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(wgrad_kernel<bf16_t>, dim3(tiles, splits), dim3(256), 0, s, (const bf16_t*)X,
                       (const bf16_t*)D, ws, M, K, N, has_bias, shiftT, rps);
  else
    hipLaunchKernelGGL(wgrad_kernel<float>, dim3(tiles, splits), dim3(256), 0, s, (const float*)X, (const float*)D,
                       ws, M, K, N, has_bias, shiftT, rps);
  const int64_t total = (int64_t)Kr * N;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, ws, gW, gb, splits, K, N, has_bias);
}

}  // namespace hfrep
