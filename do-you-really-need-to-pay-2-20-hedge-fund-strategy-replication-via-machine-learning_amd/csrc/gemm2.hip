// GEMMs v2 (bf16, gfx950): LSTM weight-gradient GEMM with hardware-transposed LDS reads, and a
// wide-N linear kernel with vectorised staging.
//
// lstm_wgrad2: for one LSTM layer, ONE launch produces all three weight gradients
//     gW[K,N]  += sum_s X_s^T   dZ_s          (input kernel;   s = primal, tangent)
//     gU[Hd,N] += sum_s Hp_s^T  dZ_s          (recurrent kernel, Hp = h_{t-1} by index arithmetic)
//     gb[N]    += colsum(dZ_0)                 (bias: an all-ones row of the primal segment)
// i.e. C = A^T D with A = [X | H_{t-1} | 1] (M x Ktot) and the M = batch*T reduction split over
// workgroups.  A and D are staged into LDS exactly as they sit in HBM (row = data row m, 8-byte
// vector loads, no transpose on the way in); the MFMA operands need the reduction index m inside
// each lane's fragment, which gfx950's ds_read_b64_tr_b16 delivers directly (4 rows x 16 columns per
// 16-lane group, column-major) -- the transpose costs nothing.  v_mfma_f32_16x16x32_bf16 consumes
// the fragments (lane l holds A[l&15][8(l>>4)+j]).  v1 (gemm.hip wgrad) staged both operands with
// 2-byte transposing LDS writes and needed two launches (plus a reduce each) per layer.
//
// linear2: C[M,N] = act(A[M,K] . W + bias) with a 128 x 128 tile (each wave 32 rows x 128 cols), so
// the LSTM input gradients dZ.W^T (K = 400, N <= 128) read dZ exactly once.
#include "common.h"
#include "mfma.h"
#include "kernels.h"

namespace hfrep {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* tile, int LD, int k0, int col0, int lane) {
  // fragment for 16x16x32: lane l -> column col0 + (l & 15), rows k0 + 8*(l>>4) + 0..7
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const bf16_t* a0 = tile + (k0 + 8 * g + q) * LD + col0 + 4 * p;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * LD));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

constexpr int WG_I = 256, WG_J = 128, WG_M = 32;        // tile: i (A^T rows) x j (D cols), m chunk
constexpr int LDA2 = WG_I + 8, LDD2 = WG_J + 8;          // LDS row lengths (elements)

}  // namespace

__global__ void __launch_bounds__(512)
lstm_wgrad2_kernel(const bf16_t* __restrict__ X0, const bf16_t* __restrict__ H0, const bf16_t* __restrict__ D0,
                   const bf16_t* __restrict__ X1, const bf16_t* __restrict__ H1, const bf16_t* __restrict__ D1,
                   float* __restrict__ slab, int M, int K, int Hd, int N, int Tn, int nseg, int rows_per_split) {
  __shared__ __attribute__((aligned(16))) bf16_t As[WG_M * LDA2];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[WG_M * LDD2];
  const int Ktot = K + Hd + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntj = (N + WG_J - 1) / WG_J;
  const int tj = blockIdx.x % ntj, ti = blockIdx.x / ntj;
  const int i0 = ti * WG_I, j0 = tj * WG_J;
  const int z = blockIdx.y;
  const int mb = z * rows_per_split, me = min(M, mb + rows_per_split);
  const int wi0 = w * 32;                                    // this wave's 32 A^T rows (i)
  const bool active = (i0 + wi0) < Ktot;                     // wave-uniform
  f32x4 acc[2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s = 0; s < nseg; ++s) {
    const bf16_t* X = s ? X1 : X0;
    const bf16_t* Hh = s ? H1 : H0;
    const bf16_t* D = s ? D1 : D0;
    const float bias_one = (s == 0) ? 1.f : 0.f;
    for (int m0 = mb; m0 < me; m0 += WG_M) {
      __syncthreads();
      // ---- stage A = [X | H_{t-1} | 1] rows m0..m0+31, columns i0..i0+255 (4-element chunks)
      for (int e = tid; e < WG_M * (WG_I / 4); e += 512) {
        const int r = e / (WG_I / 4), c4 = (e % (WG_I / 4)) * 4;
        const int m = m0 + r, gi = i0 + c4;
        uint2 v = make_uint2(0, 0);
        if (m < me) {
          if (gi + 3 < K && (K & 3) == 0) {
            v = *reinterpret_cast<const uint2*>(X + (size_t)m * K + gi);
          } else if (gi >= K && gi + 3 < K + Hd && ((K | Hd) & 3) == 0) {
            if (m % Tn) v = *reinterpret_cast<const uint2*>(Hh + (size_t)(m - 1) * Hd + (gi - K));
          } else {
            uint16_t t4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int ii = gi + q;
              float x = 0.f;
              if (ii < K) x = bf2f(X[(size_t)m * K + ii]);
              else if (ii < K + Hd) x = (m % Tn) ? bf2f(Hh[(size_t)(m - 1) * Hd + (ii - K)]) : 0.f;
              else if (ii == K + Hd) x = bias_one;
              t4[q] = f2bf(x);
            }
            v = make_uint2((uint32_t)t4[0] | ((uint32_t)t4[1] << 16), (uint32_t)t4[2] | ((uint32_t)t4[3] << 16));
          }
        }
        *reinterpret_cast<uint2*>(As + r * LDA2 + c4) = v;
      }
      // ---- stage D rows m0..m0+31, columns j0..j0+127
      for (int e = tid; e < WG_M * (WG_J / 4); e += 512) {
        const int r = e / (WG_J / 4), c4 = (e % (WG_J / 4)) * 4;
        const int m = m0 + r, gj = j0 + c4;
        uint2 v = make_uint2(0, 0);
        if (m < me) {
          if (gj + 3 < N && (N & 3) == 0) {
            v = *reinterpret_cast<const uint2*>(D + (size_t)m * N + gj);
          } else {
            uint16_t t4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) t4[q] = (gj + q < N) ? D[(size_t)m * N + gj + q] : (uint16_t)0;
            v = make_uint2((uint32_t)t4[0] | ((uint32_t)t4[1] << 16), (uint32_t)t4[2] | ((uint32_t)t4[3] << 16));
          }
        }
        *reinterpret_cast<uint2*>(Ds + r * LDD2 + c4) = v;
      }
      __syncthreads();
      if (active) {
        const bf16x8 a0 = tr_frag(As, LDA2, 0, wi0, lane);
        const bf16x8 a1 = tr_frag(As, LDA2, 0, wi0 + 16, lane);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const bf16x8 bb = tr_frag(Ds, LDD2, 0, b * 16, lane);
          acc[0][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bb, acc[0][b], 0, 0, 0);
          acc[1][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bb, acc[1][b], 0, 0, 0);
        }
      }
    }
  }
  if (!active) return;
  // 16x16 accumulator: col = lane & 15, row = 4*(lane>>4) + reg
  float* out = slab + (size_t)z * Ktot * N;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wi0 + a * 16 + 4 * (lane >> 4) + r;
        const int j = j0 + b * 16 + (lane & 15);
        if (i < Ktot && j < N) out[(size_t)i * N + j] = acc[a][b][r];
      }
}

__global__ void __launch_bounds__(256)
lstm_wgrad2_reduce_kernel(const float* __restrict__ slab, float* __restrict__ gW, float* __restrict__ gU,
                          float* __restrict__ gb, int splits, int K, int Hd, int N, int Ks) {
  const int Ktot = Ks + Hd + 1;  // slab rows: Ks >= K input rows (rows K .. Ks - 1 padding, dropped)
  const int64_t total = (int64_t)Ktot * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // 4 independent chains: loads stay in flight
    int z = 0;
    for (; z + 3 < splits; z += 4) {
      s0 += slab[(size_t)z * total + e];
      s1 += slab[(size_t)(z + 1) * total + e];
      s2 += slab[(size_t)(z + 2) * total + e];
      s3 += slab[(size_t)(z + 3) * total + e];
    }
    for (; z < splits; ++z) s0 += slab[(size_t)z * total + e];
    const float s = (s0 + s1) + (s2 + s3);
    const int i = (int)(e / N), j = (int)(e % N);
    if (i < K) gW[(size_t)i * N + j] += s;
    else if (i < Ks) continue;
    else if (i < Ks + Hd) gU[(size_t)(i - Ks) * N + j] += s;
    else if (gb) gb[j] += s;
  }
}

static int wgrad2_splits(int M, int N) {
  // enough workgroups to occupy the chip even at the reference batch (M = 32 x 48 rows): one split
  // per 128 rows (4 chunks per workgroup), at most ~1024 workgroups in total
  const int ntj = (N + WG_J - 1) / WG_J;
  int splits = (M + 127) / 128;
  splits = std::max(1, std::min(splits, std::max(1, 1024 / ntj)));
  return splits;
}

size_t lstm_wgrad2_workspace_floats(int M, int K, int Hd, int N) {
  return (size_t)wgrad2_splits(M, N) * (size_t)(K + Hd + 1) * (size_t)N;
}

void launch_lstm_wgrad2(const void* X0, const void* H0, const void* D0, const void* X1, const void* H1, const void* D1,
                        float* gW, float* gU, float* gb, int M, int K, int Hd, int N, int Tn, float* ws, hipStream_t s) {
  if (M <= 0) return;
  const int Ktot = K + Hd + 1;
  const int splits = wgrad2_splits(M, N);
  int rps = (M + splits - 1) / splits;
  rps = (rps + WG_M - 1) / WG_M * WG_M;
  const int nti = (Ktot + WG_I - 1) / WG_I, ntj = (N + WG_J - 1) / WG_J;
  const int nseg = X1 ? 2 : 1;
  hipLaunchKernelGGL(lstm_wgrad2_kernel, dim3(nti * ntj, splits), dim3(512), 0, s, (const bf16_t*)X0,
                     (const bf16_t*)H0, (const bf16_t*)D0, (const bf16_t*)X1, (const bf16_t*)H1, (const bf16_t*)D1,
                     ws, M, K, Hd, N, Tn, nseg, rps);
  launch_lstm_wgrad2_reduce(ws, gW, gU, gb, splits, K, Hd, N, s);
}

void launch_lstm_wgrad2_reduce(const float* ws, float* gW, float* gU, float* gb, int splits, int K, int Hd, int N,
                               hipStream_t s, int Ks) {
  if (Ks < K) Ks = K;
  const int64_t total = (int64_t)(Ks + Hd + 1) * N;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(lstm_wgrad2_reduce_kernel, dim3(blocks), dim3(256), 0, s, ws, gW, gU, gb, splits, K, Hd, N, Ks);
}

// ---------------------------------------------------------------------------------------------
// linear2: 128 x 128 tile, 4 waves x (32 rows x 128 cols), 8-byte A staging (bf16)
// ---------------------------------------------------------------------------------------------
constexpr int L2M = 128, L2N = 128, L2K = 32, L2LD = L2K + 8;

__global__ void __launch_bounds__(256)
linear2_kernel(const bf16_t* __restrict__ A, const float* __restrict__ W, const float* __restrict__ bias,
               bf16_t* __restrict__ C, int M, int N, int K, int w_trans, int act) {
  using P = MF<bf16_t>;
  __shared__ __attribute__((aligned(16))) bf16_t As[L2M * L2LD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[L2N * L2LD];
  const int ntn = (N + L2N - 1) / L2N;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x % ntn;
  const int m0 = tm * L2M, n0 = tn * L2N;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool vecA = (K & 3) == 0;
  f32x16 acc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc[b] = zero16();
  for (int k0 = 0; k0 < K; k0 += L2K) {
    // A tile [128][32] in 4-element chunks (1024 chunks, 4 per thread)
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + it * 256, r = e >> 3, c4 = (e & 7) * 4;
      const int gm = m0 + r, gk = k0 + c4;
      uint2 v = make_uint2(0, 0);
      if (gm < M) {
        if (vecA && gk + 3 < K) {
          v = *reinterpret_cast<const uint2*>(A + (size_t)gm * K + gk);
        } else {
          uint16_t t4[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) t4[q] = (gk + q < K) ? A[(size_t)gm * K + gk + q] : (uint16_t)0;
          v = make_uint2((uint32_t)t4[0] | ((uint32_t)t4[1] << 16), (uint32_t)t4[2] | ((uint32_t)t4[3] << 16));
        }
      }
      *reinterpret_cast<uint2*>(As + r * L2LD + c4) = v;
    }
    // W tile as Bs[n][k] (fp32 -> bf16)
    if (!w_trans) {
#pragma unroll 4
      for (int it = 0; it < (L2N * L2K) / 256; ++it) {
        const int e = tid + it * 256, kk = e / L2N, n = e % L2N;
        const int gk = k0 + kk, gn = n0 + n;
        Bs[n * L2LD + kk] = f2bf((gk < K && gn < N) ? W[(size_t)gk * N + gn] : 0.f);
      }
    } else {
#pragma unroll 4
      for (int it = 0; it < (L2N * L2K) / 256; ++it) {
        const int e = tid + it * 256, n = e / L2K, kk = e % L2K;
        const int gk = k0 + kk, gn = n0 + n;
        Bs[n * L2LD + kk] = f2bf((gk < K && gn < N) ? W[(size_t)gn * K + gk] : 0.f);
      }
    }
    __syncthreads();
    const bf16_t* arow = As + (w * 32 + (lane & 31)) * L2LD;
#pragma unroll
    for (int ks = 0; ks < L2K / 16; ++ks) {
      const bf16x8 a = P::lda(arow, ks, lane);
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[b] = P::mma(a, P::lda(Bs + (b * 32 + (lane & 31)) * L2LD, ks, lane), acc[b]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int col = n0 + b * 32 + (lane & 31);
    const float bb = (bias && col < N) ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + w * 32 + acc32_row(r, lane);
      if (row < M && col < N) C[(size_t)row * N + col] = f2bf(act_f(act, acc[b][r] + bb));
    }
  }
}

void launch_linear2(const void* A, const float* W, const float* bias, void* C, int M, int N, int K, int w_trans, int act,
                    hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const int nwg = ((M + L2M - 1) / L2M) * ((N + L2N - 1) / L2N);
  hipLaunchKernelGGL(linear2_kernel, dim3(nwg), dim3(256), 0, s, (const bf16_t*)A, W, bias, (bf16_t*)C, M, N, K,
                     w_trans, act);
}

}  // namespace hfrep
