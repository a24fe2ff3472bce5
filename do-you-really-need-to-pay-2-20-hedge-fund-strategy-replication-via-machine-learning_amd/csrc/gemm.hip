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

static int wgrad_splits(int M, int K, int N) {
  const int Kr = K + 1;
  const int tiles = ((Kr + WBI - 1) / WBI) * ((N + WBJ - 1) / WBJ);
  int splits = (M + 2047) / 2048;                    // >= 2048 rows per split
  const int cap = max(1, 2048 / max(tiles, 1));     // <= ~2048 workgroups total
  splits = max(1, min(splits, cap));
  return splits;
}

size_t wgrad_workspace_floats(int M, int K, int N) {
  return (size_t)wgrad_splits(M, K, N) * (size_t)(K + 1) * (size_t)N;
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
