// Skinny GEMMs (bf16 or fp32 activations, N <= 4 output columns, K % 8 == 0): the critic head
// Flatten(T*H) -> Dense(1) of every WGAN family (reference GAN/MTSS_WGAN_GP.py build_critic).
//
// All three products of a Dense(1) layer are HBM-streaming with O(1) arithmetic per byte, so the
// MFMA tile kernels (gemm.hip / gemm2.hip) - which stage a 128-wide W tile for one useful column
// and launch one workgroup per 128 rows - ran them at 0.2-0.6 TB/s.  Here every op is a flat stream
// of 16-byte accesses with enough rows in flight per wave to cover HBM latency:
//
//   skinny_fwd   y[m,n]   = act(sum_k x[m,k] W[k,n] + b[n])   wave per row group, W in LDS,
//                                                            lanes stride the row, shuffle-reduce
//   skinny_wgrad gW[k,n] += sum_m x[m,k] d[m,n]  (+ gb)      thread per 8-column chunk, split-M
//                                                            slabs + one reduce launch (deterministic)
//   skinny_dgrad dx[m,k]  = sum_n d[m,n] W[k,n]              one 16-byte output chunk per thread
#include "common.h"
#include "kernels.h"
#include "mfma.h"

#include <algorithm>
#include <stdexcept>

namespace hfrep {

namespace {

__device__ __forceinline__ float lo_bf(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi_bf(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ void unpack8(const uint4& v, float (&f)[8]) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) { return pk2bf(a, b); }

// 8 consecutive elements of a row: one 16-byte access in bf16, two in fp32
template <typename T> struct Chunk8;
template <> struct Chunk8<bf16_t> {
  uint4 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { v = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ void get(float (&f)[8]) const { unpack8(v, f); }
  __device__ __forceinline__ static void store(bf16_t* p, const float (&o)[8]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
  }
};
template <> struct Chunk8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void get(float (&f)[8]) const {
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&o)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
};

constexpr int SK_ROWS = 4;  // rows per wave in flight (forward)

}  // namespace

template <int N, typename T>
__global__ void __launch_bounds__(256) skinny_fwd_kernel(const T* __restrict__ x, const float* __restrict__ W,
                                                         const float* __restrict__ b, T* __restrict__ y, int M,
                                                         int K, int act) {
  extern __shared__ float wsh[];  // [K][N]
  for (int i = threadIdx.x; i < K * N; i += 256) wsh[i] = W[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int KC = K / 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t m0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * SK_ROWS; m0 < M; m0 += nw * SK_ROWS) {
    float acc[SK_ROWS][N];
#pragma unroll
    for (int r = 0; r < SK_ROWS; ++r)
#pragma unroll
      for (int n = 0; n < N; ++n) acc[r][n] = 0.f;
    for (int c = lane; c < KC; c += 64) {
      Chunk8<T> v[SK_ROWS];
#pragma unroll
      for (int r = 0; r < SK_ROWS; ++r) {
        if (m0 + r < M) v[r].load(x + (m0 + r) * K + 8 * c);
        else v[r].zero();
      }
      float w[8][N];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int n = 0; n < N; ++n) w[j][n] = wsh[(8 * c + j) * N + n];
#pragma unroll
      for (int r = 0; r < SK_ROWS; ++r) {
        float f[8];
        v[r].get(f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int n = 0; n < N; ++n) acc[r][n] = fmaf(f[j], w[j][n], acc[r][n]);
      }
    }
#pragma unroll
    for (int r = 0; r < SK_ROWS; ++r)
#pragma unroll
      for (int n = 0; n < N; ++n) {
        const float s = wave_sum(acc[r][n]);
        if (lane == 0 && m0 + r < M) y[(m0 + r) * N + n] = Cvt<T>::from_f(act_f(act, s + (b ? b[n] : 0.f)));
      }
  }
}

// Linear Dense(1) head forward on rows whose loss gradient is known before the forward: the
// Wasserstein critic loss (W(real, -1) + W(fake, +1), GAN/MTSS_WGAN_GP.py) gives every row of the
// [real; fake] batch the constant ds = wa (rows < split) or wb.  The head's weight gradient
// gW = sum_r ds_r x_r (and gb = sum_r ds_r) is then a signed column sum of the rows the forward streams
// anyway: each lane keeps the sums of its NC column chunks (c = lane + 64 k) in registers and every wave
// writes one slab row [K column sums | weight sum], reduced by skinny_reduce_kernel in a fixed order.
// One pass over x instead of the forward's and skinny_wgrad's two.
template <typename T, int NC>
__global__ void __launch_bounds__(256) skinny_fwd_cs_kernel(const T* __restrict__ x, const float* __restrict__ W,
                                                            const float* __restrict__ b, T* __restrict__ y, int M, int K,
                                                            int split, float wa, float wb, float* __restrict__ slab) {
  extern __shared__ float wsh[];  // [K]
  for (int i = threadIdx.x; i < K; i += 256) wsh[i] = W[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int KC = K / 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float cs[NC][8];
#pragma unroll
  for (int k = 0; k < NC; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) cs[k][j] = 0.f;
  float ws = 0.f;
  for (int64_t m0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * SK_ROWS; m0 < M; m0 += nw * SK_ROWS) {
    float acc[SK_ROWS], wr[SK_ROWS];
#pragma unroll
    for (int r = 0; r < SK_ROWS; ++r) {
      acc[r] = 0.f;
      wr[r] = m0 + r < M ? (m0 + r < split ? wa : wb) : 0.f;
      ws += wr[r];
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c < KC) {
        Chunk8<T> v[SK_ROWS];
#pragma unroll
        for (int r = 0; r < SK_ROWS; ++r) {
          if (m0 + r < M) v[r].load(x + (m0 + r) * K + 8 * c);
          else v[r].zero();
        }
        float w8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w8[j] = wsh[8 * c + j];
#pragma unroll
        for (int r = 0; r < SK_ROWS; ++r) {
          float f[8];
          v[r].get(f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            acc[r] = fmaf(f[j], w8[j], acc[r]);
            cs[k][j] = fmaf(f[j], wr[r], cs[k][j]);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < SK_ROWS; ++r) {
      const float sv = wave_sum(acc[r]);
      if (lane == 0 && m0 + r < M) y[m0 + r] = Cvt<T>::from_f(sv + (b ? b[0] : 0.f));
    }
  }
  float* out = slab + ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (K + 1);
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + 64 * k;
    if (c < KC) {
#pragma unroll
      for (int j = 0; j < 8; ++j) out[8 * c + j] = cs[k][j];
    }
  }
  if (lane == 0) out[K] = ws;  // (every lane summed the same row weights)
}

template <int N, typename T>
__global__ void __launch_bounds__(1024) skinny_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ d,
                                                            float* __restrict__ slab, int M, int K, int rps) {
  const int c = threadIdx.x, KC = K / 8;
  const int z = blockIdx.x;
  const int mb = z * rps, me = min(M, mb + rps);
  float acc[8][N], bacc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    bacc[n] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j][n] = 0.f;
  }
  const bool own = c < KC;
  int m = mb;
  for (; m + 4 <= me; m += 4) {  // four rows in flight
    Chunk8<T> v[4];
    float dv[4][N];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (own) v[r].load(x + (int64_t)(m + r) * K + 8 * c);
      else v[r].zero();
#pragma unroll
      for (int n = 0; n < N; ++n) dv[r][n] = ld_f(d + (int64_t)(m + r) * N + n);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float f[8];
      v[r].get(f);
#pragma unroll
      for (int n = 0; n < N; ++n) {
        bacc[n] += dv[r][n];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j][n] = fmaf(f[j], dv[r][n], acc[j][n]);
      }
    }
  }
  for (; m < me; ++m) {
    Chunk8<T> v;
    if (own) v.load(x + (int64_t)m * K + 8 * c);
    else v.zero();
    float f[8];
    v.get(f);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float dv = ld_f(d + (int64_t)m * N + n);
      bacc[n] += dv;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j][n] = fmaf(f[j], dv, acc[j][n]);
    }
  }
  float* out = slab + (size_t)z * (K + 1) * N;
  if (own) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int n = 0; n < N; ++n) out[(8 * c + j) * N + n] = acc[j][n];
  }
  if (c == 0) {
#pragma unroll
    for (int n = 0; n < N; ++n) out[K * N + n] = bacc[n];
  }
}

// sum the split slabs: 64 consecutive elements per workgroup, 16 waves split the slabs (fixed
// order: deterministic).  Elements [0, KN) accumulate into gW, [KN, KN + N) into gb (if non-null).
__global__ void __launch_bounds__(1024) skinny_reduce_kernel(const float* __restrict__ slab, float* __restrict__ gW,
                                                             float* __restrict__ gb, int splits, int KN, int N) {
  // 16 waves split the slabs (4 independent partial sums each, so loads overlap), fixed order
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int total = KN + N;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (e < total) {
    int z = wv;
    for (; z + 48 < splits; z += 64) {
      s0 += slab[(size_t)z * total + e];
      s1 += slab[(size_t)(z + 16) * total + e];
      s2 += slab[(size_t)(z + 32) * total + e];
      s3 += slab[(size_t)(z + 48) * total + e];
    }
    for (; z < splits; z += 16) s0 += slab[(size_t)z * total + e];
  }
  part[wv][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wv == 0 && e < total) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += part[w][lane];
    if (e < KN) {
      if (gW) gW[e] += t;
    } else if (gb) {
      gb[e - KN] += t;
    }
  }
}

template <int N, typename T>
__global__ void __launch_bounds__(256) skinny_dgrad_kernel(const T* __restrict__ d, const float* __restrict__ W,
                                                           T* __restrict__ dx, int M, int K) {
  const int KC = K / 8;
  const int64_t total = (int64_t)M * KC;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int64_t m = q / KC;
    const int c = (int)(q - m * KC);
    float dv[N];
#pragma unroll
    for (int n = 0; n < N; ++n) dv[n] = ld_f(d + m * N + n);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < N; ++n) s = fmaf(dv[n], W[(8 * c + j) * N + n], s);
      o[j] = s;
    }
    Chunk8<T>::store(dx + m * K + 8 * c, o);
  }
}

// ------------------------------------------------------------------------------------ narrow Dense
// y = act(x W + b) for 4 < N <= 32, K <= 128, bf16 (the generator's output Dense(F), F = 32..36 ->
// N <= 32 covers F = 32; 33..64 use two column tiles).  The generic tile GEMM staged x through LDS
// for a 128-wide N tile and ran at ~1.1 TB/s (1.55 ms per (6.3M x 100) x (100 x 32) call).  Here a
// wave owns one 32-column tile with W as register fragments (ceil(K/16) x 4 VGPRs) and streams
// 32-row tiles (grid-stride) straight from HBM into MFMA A fragments (one 16-byte buffer load
// per k-step per lane, rows past M read zeros, k >= K columns masked).
template <int KS>
__global__ void __launch_bounds__(256) narrow_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ W,
                                                         const float* __restrict__ bias, bf16_t* __restrict__ y, int M,
                                                         int K, int N, int act) {
  using P = MF<bf16_t>;
  const int lane = threadIdx.x & 63;
  const int col0 = blockIdx.y * 32, col = col0 + (lane & 31);
  const int kh = 8 * (lane >> 5);
  typename P::frag wb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * ks + kh + j;
      const float v = W[(size_t)min(k, K - 1) * N + min(col, N - 1)];
      wb[ks][j] = (short)f2bf((k < K && col < N) ? v : 0.f);
    }
  const float bv = (bias && col < N) ? bias[col] : 0.f;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x), 0, (int)std::min<int64_t>((int64_t)M * K * 2, 0x7fff0000), 0x00020000);
  const int ntiles = (M + 31) / 32;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (int tile = wid; tile < ntiles; tile += nw) {
    const int row = tile * 32 + (lane & 31);
    f32x16 acc = zero16();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = 16 * ks + kh;
      const bool ok = row < M && k0 < K;
      bf16x8 a = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                rx, ok ? (int)(((int64_t)row * K + k0) * 2) : 0x7fff0000, 0, 0));
      if (16 * ks + 16 > K) {  // the k-step that crosses K: zero the columns past it (they belong to the next row)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j >= K) a[j] = 0;
      }
      acc = P::mma(a, wb[ks], acc);
    }
    if (col < N) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = tile * 32 + acc32_row(r, lane);
        if (rr < M) y[(size_t)rr * N + col] = f2bf(act_f(act, acc[r] + bv));
      }
    }
  }
}

// K even: a row's 16-byte A load starts on a dword (an odd K put every other row's load at a 2-byte
// offset, which the buffer load does not honour: wrong values -- the bf16 autoencoder decoder at odd
// latent sizes, profiles/r04_ae/README.md)
bool narrow_supported(int K, int N) { return N > 4 && N <= 64 && K >= 2 && K <= 128 && K % 2 == 0; }

void launch_narrow_fwd(const void* x, const float* W, const float* b, void* y, int M, int K, int N, int act,
                       hipStream_t s) {
  const int ntiles = (M + 31) / 32;
  const int bx = std::max(1, std::min((ntiles + 3) / 4, device_cu_count() * 8));
  const dim3 grid(bx, (N + 31) / 32);
  const int ks = (K + 15) / 16;
  const bf16_t* xp = (const bf16_t*)x;
  bf16_t* yp = (bf16_t*)y;
  switch (ks) {
    case 1: hipLaunchKernelGGL(narrow_fwd_kernel<1>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    case 2: hipLaunchKernelGGL(narrow_fwd_kernel<2>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    case 3: hipLaunchKernelGGL(narrow_fwd_kernel<3>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    case 4: hipLaunchKernelGGL(narrow_fwd_kernel<4>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    case 5: hipLaunchKernelGGL(narrow_fwd_kernel<5>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    case 6: hipLaunchKernelGGL(narrow_fwd_kernel<6>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    case 7: hipLaunchKernelGGL(narrow_fwd_kernel<7>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
    default: hipLaunchKernelGGL(narrow_fwd_kernel<8>, grid, dim3(256), 0, s, xp, W, b, yp, M, K, N, act); break;
  }
}

// ------------------------------------------------------------------------------------ narrow fp32
// y = act(x B + b) in exact fp32 for K <= 128 (K % 4 == 0) and 4 < N <= 112, B given by strides
// (B[k][n] = Bp[k sk + n sn]): the generator's output Dense(F) forward (K = 100, N = F) and its input
// gradient dz W^T (K = F, N = 100), the MLP models' 100-wide Dense layers.  hipBLASLt ran the
// forward at ~1.1 ms per 6.3 M-row call on the B = 262k step (Cijk_..._MT32x256x16,
// profiles/r02_end); its tile shape wastes most of a 256-wide N tile on N = 32.
//
// One wave owns a 16-row chunk and ALL NT 16-column output tiles; B^T fragments of the whole
// reduction live in registers (NT x KS), the A operand comes straight from HBM into registers (k is
// permuted inside each 16-wide k group: k-step 4 q + j of lane group g reads k = 16 q + 4 g + j, so
// a lane's four k-steps are one contiguous dwordx4; the remainder k-steps read k = 16 NQ + 4 r + g;
// the sum over k is order-free and A / B use the same map).  The next chunk's A is loaded before
// the current chunk's MFMAs (grid-stride over chunks, 4 waves per block, several blocks per CU).
template <int NT, int NQ, int RS>
__global__ void __launch_bounds__(256) narrowf_kernel(const float* __restrict__ x, const float* __restrict__ Bp, int sk,
                                                      int sn, const float* __restrict__ bias, float* __restrict__ y,
                                                      int M, int N, int act) {
  constexpr int K = 16 * NQ + 4 * RS, KS = 4 * NQ + RS;
  const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  float bw[NT][KS], bv[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int col = 16 * n + c16;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = s < 4 * NQ ? 16 * (s >> 2) + 4 * g + (s & 3) : 16 * NQ + 4 * (s - 4 * NQ) + g;
      bw[n][s] = col < N ? Bp[(size_t)k * sk + (size_t)col * sn] : 0.f;
    }
    bv[n] = (bias && col < N) ? bias[col] : 0.f;
  }
  const int nch = (M + 15) / 16;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  typedef __amdgpu_buffer_rsrc_t rsrc_t;
  auto rsrc_of = [&](int c) -> rsrc_t {  // rows of chunk c (past M: zero-size descriptor, loads read 0)
    const int r0 = c * 16, nr = c < nch ? min(16, M - r0) : 0;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x) + (nr ? (size_t)r0 * K : 0), 0, nr * K * 4, 0x00020000);
  };
  f32x4 a4[2][NQ > 0 ? NQ : 1];
  float ar[2][RS > 0 ? RS : 1];
  const int vo = (c16 * K + 4 * g) * 4;
  auto load = [&](int set, int c) {
    const rsrc_t r = rsrc_of(c);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      a4[set][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 64 * q, 0, 0));
#pragma unroll
    for (int rr = 0; rr < RS; ++rr)
      ar[set][rr] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (c16 * K + 16 * NQ + 4 * rr + g) * 4, 0, 0));
  };
  auto body = [&](int set, int c) {
    f32x4 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float av = s < 4 * NQ ? a4[set][s < 4 * NQ ? s >> 2 : 0][s & 3] : ar[set][s < 4 * NQ ? 0 : s - 4 * NQ];
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bw[n][s], acc[n], 0, 0, 0);
    }
    const int r0 = c * 16 + 4 * g;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = 16 * n + c16;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (col < N && r0 + i < M) y[(size_t)(r0 + i) * N + col] = act_f(act, acc[n][i] + bv[n]);
    }
  };
  int c = wid;
  if (c < nch) load(0, c);
  for (; c < nch; c += 2 * nw) {
    load(1, c + nw);  // (past the end: zero-size descriptor)
    body(0, c);
    if (c + nw >= nch) break;
    load(0, c + 2 * nw);
    body(1, c + nw);
  }
}

// ------------------------------------------------------------------------------------------
// fp32 GEMM for the shapes narrowf cannot hold in registers: widef_kernel
// ------------------------------------------------------------------------------------------
// y = act(x B + b), x (M, K) fp32 row-major with K % 4 == 0 and K <= 320, any N (column blocks of 112 over
// grid.y).  The conv critic's im2col GEMMs (K = k C = 300 at C = 100) and their input gradients (N = k C)
// went to hipBLASLt (K14): narrowf keeps its B fragments in registers (K / 4 per column tile), which at
// K = 300 would be 525 of them.  Here the workgroup's B block (K x 112, zero-padded) is staged once in
// LDS (<= 145 KiB; row stride 116 floats: the four k-rows of a 16x16x4 B fragment land on distinct bank
// halves) and every wave walks 16-row chunks of x with the exact-fp32 v_mfma_f32_16x16x4_f32: per chunk
// the lane's x values are loaded as float4 (k = 16 q + 4 g + 0..3, the same k permutation on both
// operands as narrowf) one chunk ahead, B fragments are single ds_read_b32 per MFMA.  Exact fp32 (an
// fmaf chain per output), any activation in the epilogue.
constexpr int WF_NT = 7, WF_LDB = 16 * WF_NT + 4, WF_KMAX = 320;
template <int NQ>
__global__ void __launch_bounds__(256) widef_kernel(const float* __restrict__ x, const float* __restrict__ Bp, int sk,
                                                    int sn, const float* __restrict__ bias, float* __restrict__ y,
                                                    int M, int K, int N, int act) {
  extern __shared__ __attribute__((aligned(16))) float bsm[];  // [16 NQ][WF_LDB]
  const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int col0 = blockIdx.y * 16 * WF_NT;
  for (int e = threadIdx.x; e < 16 * NQ * WF_LDB; e += 256) {
    const int k = e / WF_LDB, c = e - k * WF_LDB, col = col0 + c;
    bsm[e] = (k < K && c < 16 * WF_NT && col < N) ? Bp[(size_t)k * sk + (size_t)col * sn] : 0.f;
  }
  float bv[WF_NT];
#pragma unroll
  for (int n = 0; n < WF_NT; ++n) {
    const int col = col0 + 16 * n + c16;
    bv[n] = (bias && col < N) ? bias[col] : 0.f;
  }
  __syncthreads();
  const int nch = (M + 15) / 16;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  typedef __amdgpu_buffer_rsrc_t rsrc_t;
  auto rsrc_of = [&](int c) -> rsrc_t {  // rows of chunk c (past M: zero-size descriptor, loads read 0)
    const int r0 = c * 16, nr = c < nch ? min(16, M - r0) : 0;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x) + (nr ? (size_t)r0 * K : 0), 0, nr * K * 4, 0x00020000);
  };
  f32x4 a4[2][NQ];
  auto load = [&](int set, int c) {
    const rsrc_t r = rsrc_of(c);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int k = 16 * q + 4 * g;  // (K % 4 == 0: a float4 is wholly inside the row or past its end)
      a4[set][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, k < K ? (c16 * K + k) * 4 : 0x7fff0000,
                                                                                   0, 0));
    }
  };
  const float* bl = bsm + (4 * g) * WF_LDB + c16;  // B[k = 16 q + 4 g + j][16 n + c16]
  auto body = [&](int set, int c) {
    f32x4 acc[WF_NT];
#pragma unroll
    for (int n = 0; n < WF_NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float av = a4[set][q][j];
#pragma unroll
        for (int n = 0; n < WF_NT; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bl[(16 * q + j) * WF_LDB + 16 * n], acc[n], 0, 0, 0);
      }
    const int r0 = c * 16 + 4 * g;
#pragma unroll
    for (int n = 0; n < WF_NT; ++n) {
      const int col = col0 + 16 * n + c16;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (col < N && r0 + i < M) y[(size_t)(r0 + i) * N + col] = act_f(act, acc[n][i] + bv[n]);
    }
  };
  int c = wid;
  if (c < nch) load(0, c);
  for (; c < nch; c += 2 * nw) {
    load(1, c + nw);
    body(0, c);
    if (c + nw >= nch) break;
    load(0, c + 2 * nw);
    body(1, c + nw);
  }
}

bool widef_supported(int K, int N) { return K >= 4 && K <= WF_KMAX && K % 4 == 0 && N > 4; }

void launch_widef(const float* x, const float* B, int sk, int sn, const float* b, float* y, int M, int K, int N,
                  int act, hipStream_t s) {
  if (M <= 0) return;
  const int nq = (K + 15) / 16, nch = (M + 15) / 16, ncb = (N + 16 * WF_NT - 1) / (16 * WF_NT);
  const size_t smem = (size_t)16 * nq * WF_LDB * 4;
  const int grid = std::max(1, std::min((nch + 3) / 4, std::max(1, device_cu_count() / ncb)));
  // every NQ instantiation needs its own MaxDynamicSharedMemorySize attribute (NQ >= 9 is > 64 KiB of
  // LDS): a flag per NQ, set at that instantiation's first launch
  static bool attr[21] = {};
  auto go = [&](auto kern, int q) {
    if (!attr[q]) {
      HFREP_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                          160 * 1024));
      attr[q] = true;
    }
    hipLaunchKernelGGL(kern, dim3(grid, ncb), dim3(256), smem, s, x, B, sk, sn, b, y, M, K, N, act);
    HFREP_CHECK_HIP(hipGetLastError());
  };
  switch (nq) {
#define HFREP_WIDEF(Q) case Q: go(widef_kernel<Q>, Q); break;
    HFREP_WIDEF(1) HFREP_WIDEF(2) HFREP_WIDEF(3) HFREP_WIDEF(4) HFREP_WIDEF(5) HFREP_WIDEF(6) HFREP_WIDEF(7)
    HFREP_WIDEF(8) HFREP_WIDEF(9) HFREP_WIDEF(10) HFREP_WIDEF(11) HFREP_WIDEF(12) HFREP_WIDEF(13) HFREP_WIDEF(14)
    HFREP_WIDEF(15) HFREP_WIDEF(16) HFREP_WIDEF(17) HFREP_WIDEF(18) HFREP_WIDEF(19)
    default: go(widef_kernel<20>, 20); break;
#undef HFREP_WIDEF
  }
}

bool narrowf_supported(int K, int N) {
  return N > 4 && N <= 112 && (K == 32 || K == 36 || K == 64 || K == 100 || K == 128);
}

void launch_narrowf(const float* x, const float* B, int sk, int sn, const float* b, float* y, int M, int K, int N,
                    int act, hipStream_t s) {
  if (M <= 0) return;
  const int nch = (M + 15) / 16;
  const int grid = std::max(1, std::min((nch + 3) / 4, device_cu_count() * 4));
  const int nt = (N + 15) / 16;
#define HFREP_NARROWF(NQ, RS)                                                                                        \
  switch (nt) {                                                                                                      \
    case 1: hipLaunchKernelGGL((narrowf_kernel<1, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
    case 2: hipLaunchKernelGGL((narrowf_kernel<2, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
    case 3: hipLaunchKernelGGL((narrowf_kernel<3, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
    case 4: hipLaunchKernelGGL((narrowf_kernel<4, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
    case 5: hipLaunchKernelGGL((narrowf_kernel<5, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
    case 6: hipLaunchKernelGGL((narrowf_kernel<6, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
    default: hipLaunchKernelGGL((narrowf_kernel<7, NQ, RS>), dim3(grid), dim3(256), 0, s, x, B, sk, sn, b, y, M, N, act); break; \
  }
  switch (K) {
    case 32: HFREP_NARROWF(2, 0) break;
    case 36: HFREP_NARROWF(2, 1) break;
    case 64: HFREP_NARROWF(4, 0) break;
    case 100: HFREP_NARROWF(6, 1) break;
    default: HFREP_NARROWF(8, 0) break;
  }
#undef HFREP_NARROWF
}

// ------------------------------------------------------------------------------------ host
bool skinny_supported(int K, int N) {
  return N >= 1 && N <= 4 && K % 8 == 0 && K >= 8 && K / 8 <= 1024 && K * N <= 16384;  // W in <= 64 KB LDS
}

#define HFREP_SKINNY_N(N, KERNEL, T, ...)                                  \
  switch (N) {                                                             \
    case 1: hipLaunchKernelGGL((KERNEL<1, T>), __VA_ARGS__); break;        \
    case 2: hipLaunchKernelGGL((KERNEL<2, T>), __VA_ARGS__); break;        \
    case 3: hipLaunchKernelGGL((KERNEL<3, T>), __VA_ARGS__); break;        \
    default: hipLaunchKernelGGL((KERNEL<4, T>), __VA_ARGS__); break;       \
  }

void launch_skinny_fwd(int dt, const void* x, const float* W, const float* b, void* y, int M, int K, int N, int act,
                       hipStream_t s) {
  if (M <= 0) return;
  const int64_t groups = ((int64_t)M + 4 * SK_ROWS - 1) / (4 * SK_ROWS);
  const int grid = (int)std::min<int64_t>(groups, (int64_t)device_cu_count() * 8);
  if (dt == DT_BF16)
    HFREP_SKINNY_N(N, skinny_fwd_kernel, bf16_t, dim3(grid), dim3(256), (size_t)K * N * sizeof(float), s, (const bf16_t*)x,
                   W, b, (bf16_t*)y, M, K, act)
  else
    HFREP_SKINNY_N(N, skinny_fwd_kernel, float, dim3(grid), dim3(256), (size_t)K * N * sizeof(float), s, (const float*)x,
                   W, b, (float*)y, M, K, act)
}

// the fused head forward + signed column sum (N = 1, K % 8 == 0, K <= 4096)
bool skinny_fwd_cs_supported(int K) { return K > 0 && K % 8 == 0 && K <= 4096; }
static int skinny_cs_grid(int M) {
  const int64_t groups = ((int64_t)M + 4 * SK_ROWS - 1) / (4 * SK_ROWS);
  return (int)std::max<int64_t>(1, std::min<int64_t>(groups, (int64_t)device_cu_count() * 2));
}
size_t skinny_fwd_cs_workspace_floats(int M, int K) { return (size_t)skinny_cs_grid(M) * 4 * (K + 1); }

void launch_skinny_fwd_cs(int dt, const void* x, const float* W, const float* b, void* y, int M, int K, int split,
                          float wa, float wb, float* gW, float* gb, float* ws, hipStream_t s) {
  if (M <= 0) return;
  if (!skinny_fwd_cs_supported(K)) throw std::runtime_error("skinny_fwd_cs: K % 8 == 0 and K <= 4096");
  const int grid = skinny_cs_grid(M);
  const size_t sm = (size_t)K * sizeof(float);
  auto go = [&](auto kern, auto* xp, auto* yp) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), sm, s, xp, W, b, yp, M, K, split, wa, wb, ws);
  };
  const int kc = K / 8;
  if (dt == DT_BF16) {
    if (kc <= 320) go(skinny_fwd_cs_kernel<bf16_t, 5>, (const bf16_t*)x, (bf16_t*)y);
    else go(skinny_fwd_cs_kernel<bf16_t, 8>, (const bf16_t*)x, (bf16_t*)y);
  } else {
    if (kc <= 320) go(skinny_fwd_cs_kernel<float, 5>, (const float*)x, (float*)y);
    else go(skinny_fwd_cs_kernel<float, 8>, (const float*)x, (float*)y);
  }
  const int total = K + 1;
  hipLaunchKernelGGL(skinny_reduce_kernel, dim3((total + 63) / 64), dim3(1024), 0, s, ws, gW, gb, grid * 4, K, 1);
}

size_t skinny_wgrad_workspace_floats(int M, int K, int N) {
  const int splits = std::max(1, std::min(512, (M + 63) / 64));
  return (size_t)splits * (K + 1) * N;
}

void launch_skinny_wgrad(int dt, const void* x, const void* d, float* gW, float* gb, int M, int K, int N, float* ws,
                         hipStream_t s) {
  if (M <= 0) return;
  const int splits = std::max(1, std::min(512, (M + 63) / 64));
  const int rps = (M + splits - 1) / splits;
  const int threads = ((K / 8 + 63) / 64) * 64;
  if (dt == DT_BF16)
    HFREP_SKINNY_N(N, skinny_wgrad_kernel, bf16_t, dim3(splits), dim3(threads), 0, s, (const bf16_t*)x, (const bf16_t*)d,
                   ws, M, K, rps)
  else
    HFREP_SKINNY_N(N, skinny_wgrad_kernel, float, dim3(splits), dim3(threads), 0, s, (const float*)x, (const float*)d, ws,
                   M, K, rps)
  const int total = (K + 1) * N;
  hipLaunchKernelGGL(skinny_reduce_kernel, dim3((total + 63) / 64), dim3(1024), 0, s, ws, gW, gb, splits, K * N, N);
}

void launch_split_reduce(const float* slab, float* a, float* b, int splits, int na, int nb, hipStream_t s) {
  const int total = na + nb;
  hipLaunchKernelGGL(skinny_reduce_kernel, dim3((total + 63) / 64), dim3(1024), 0, s, slab, a, b, splits, na, nb);
}

void launch_skinny_dgrad(int dt, const void* d, const float* W, void* dx, int M, int K, int N, hipStream_t s) {
  if (M <= 0) return;
  const int64_t total = (int64_t)M * (K / 8);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, (int64_t)device_cu_count() * 16);
  if (dt == DT_BF16)
    HFREP_SKINNY_N(N, skinny_dgrad_kernel, bf16_t, dim3(grid), dim3(256), 0, s, (const bf16_t*)d, W, (bf16_t*)dx, M, K)
  else
    HFREP_SKINNY_N(N, skinny_dgrad_kernel, float, dim3(grid), dim3(256), 0, s, (const float*)d, W, (float*)dx, M, K)
}

}  // namespace hfrep
