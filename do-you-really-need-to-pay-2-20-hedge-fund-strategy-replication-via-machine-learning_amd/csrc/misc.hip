// Bandwidth-bound kernels of the GAN training step (gfx950): activations, LayerNorm,
// gradient-penalty coefficient, interpolation, in-kernel Philox RNG and window sampling.
//
// LayerNorm follows Keras (axis -1, eps 1e-3: GAN/MTSS_WGAN_GP.py:225,228); the GP coefficient
// kernel is the per-sample ||dD/dx||_2 reduction of GAN/MTSS_WGAN_GP.py:201-216 fused with the
// derivative of lambda*mean((1-||g||)^2) w.r.t. g; interpolation is RandomWeightedAverage
// (GAN/MTSS_WGAN_GP.py:191-199) with a per-sample alpha of ANY batch size.
#include "common.h"
#include "kernels.h"
#include <algorithm>

namespace hfrep {

static inline int ew_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 4096));
}

// four consecutive values as one 16-byte (fp32) / 8-byte (bf16) store; same RNE conversion as st_f
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void st4(bf16_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(a, b), pk2bf(c, d));
}
__device__ __forceinline__ void ld4(const float* p, float (&x)[4]) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  x[0] = q.x; x[1] = q.y; x[2] = q.z; x[3] = q.w;
}
__device__ __forceinline__ void ld4(const bf16_t* p, float (&x)[4]) {
  const uint2 q = *reinterpret_cast<const uint2*>(p);
  x[0] = __uint_as_float(q.x << 16); x[1] = __uint_as_float(q.x & 0xffff0000u);
  x[2] = __uint_as_float(q.y << 16); x[3] = __uint_as_float(q.y & 0xffff0000u);
}


// ------------------------------------------------------------------ activations
template <typename T>
__global__ void __launch_bounds__(256) act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int act) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    st_f(y + i, act_f(act, ld_f(x + i)));
}
template <typename T>
__global__ void __launch_bounds__(256) act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx,
                                                      int64_t n, int act) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    st_f(dx + i, ld_f(dy + i) * act_dy(act, ld_f(y + i)));
}
template <typename T>
__global__ void __launch_bounds__(256) act_tbwd_kernel(const T* __restrict__ dyd, const T* __restrict__ y,
                                                       const T* __restrict__ zd, T* __restrict__ out, int64_t n, int act) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    st_f(out + i, ld_f(dyd + i) * act_d2y(act, ld_f(y + i)) * ld_f(zd + i));
}

void launch_act_fwd(int dt, const void* x, void* y, int64_t n, int act, hipStream_t s) {
  if (dt == DT_BF16)
    hipLaunchKernelGGL(act_fwd_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n, act);
  else
    hipLaunchKernelGGL(act_fwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, s, (const float*)x, (float*)y, n, act);
}
void launch_act_bwd(int dt, const void* dy, const void* y, void* dx, int64_t n, int act, hipStream_t s) {
  if (dt == DT_BF16)
    hipLaunchKernelGGL(act_bwd_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)y,
                       (bf16_t*)dx, n, act);
  else
    hipLaunchKernelGGL(act_bwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, s, (const float*)dy, (const float*)y,
                       (float*)dx, n, act);
}
void launch_act_tangent_bwd(int dt, const void* dyd, const void* y, const void* zd, void* out, int64_t n, int act,
                            hipStream_t s) {
  if (dt == DT_BF16)
    hipLaunchKernelGGL(act_tbwd_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)dyd,
                       (const bf16_t*)y, (const bf16_t*)zd, (bf16_t*)out, n, act);
  else
    hipLaunchKernelGGL(act_tbwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, s, (const float*)dyd, (const float*)y,
                       (const float*)zd, (float*)out, n, act);
}

// ------------------------------------------------------------------ LayerNorm (one wave per row)
// pre_alpha >= 0: the input is first passed through LeakyReLU(pre_alpha) and rounded to T, exactly
// as a separate activation kernel would store it (the generator's LReLU -> LN pairs)
template <typename T>
__device__ __forceinline__ float pre_lrelu(float v, float alpha) {
  return alpha < 0.f ? v : Cvt<T>::to_f(Cvt<T>::from_f(v >= 0.f ? v : alpha * v));
}

template <typename T>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, T* __restrict__ y,
                                                            T* __restrict__ xhat, float* __restrict__ rstd_out,
                                                            int64_t rows, int D, float eps, float pre_alpha) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += wstride) {
    const T* xr = x + row * D;
    float s = 0.f;
    for (int j = lane; j < D; j += 64) s += pre_lrelu<T>(ld_f(xr + j), pre_alpha);
    const float mu = wave_sum(s) / D;
    float v = 0.f;
    for (int j = lane; j < D; j += 64) { const float d = pre_lrelu<T>(ld_f(xr + j), pre_alpha) - mu; v += d * d; }
    const float rstd = rsqrtf(wave_sum(v) / D + eps);
    for (int j = lane; j < D; j += 64) {
      const float xh = (pre_lrelu<T>(ld_f(xr + j), pre_alpha) - mu) * rstd;
      if (xhat) st_f(xhat + row * D + j, xh);
      st_f(y + row * D + j, xh * gamma[j] + beta[j]);
    }
    if (lane == 0 && rstd_out) rstd_out[row] = rstd;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ xhat,
                                                            const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                            T* __restrict__ dx, float* __restrict__ slab,
                                                            int64_t rows, int D) {
  constexpr int MAXJ = 4;  // D <= 256
  __shared__ float red_g[4 * MAXJ * 64];
  __shared__ float red_b[4 * MAXJ * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float pg[MAXJ] = {0.f, 0.f, 0.f, 0.f}, pb[MAXJ] = {0.f, 0.f, 0.f, 0.f};
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wid; row < rows; row += wstride) {
    const T* dyr = dy + row * D;
    const T* xr = xhat + row * D;
    float sg = 0.f, sgx = 0.f;
    float gv[MAXJ], xv[MAXJ], dv[MAXJ];
#pragma unroll
    for (int q = 0; q < MAXJ; ++q) {
      const int j = lane + 64 * q;
      gv[q] = 0.f; xv[q] = 0.f; dv[q] = 0.f;
      if (j < D) {
        dv[q] = ld_f(dyr + j);
        xv[q] = ld_f(xr + j);
        gv[q] = dv[q] * gamma[j];
        sg += gv[q];
        sgx += gv[q] * xv[q];
        pg[q] += dv[q] * xv[q];
        pb[q] += dv[q];
      }
    }
    const float mg = wave_sum(sg) / D, mgx = wave_sum(sgx) / D;
    const float rs = rstd[row];
#pragma unroll
    for (int q = 0; q < MAXJ; ++q) {
      const int j = lane + 64 * q;
      if (j < D) st_f(dx + row * D + j, rs * (gv[q] - mg - xv[q] * mgx));
    }
  }
  if (slab == nullptr) return;
  // reduce the 4 waves' partials through LDS, then one slab row per workgroup (summed in a fixed
  // order by launch_split_reduce: bitwise run-to-run determinism, no float atomics)
#pragma unroll
  for (int q = 0; q < MAXJ; ++q) {
    red_g[(wid * MAXJ + q) * 64 + lane] = pg[q];
    red_b[(wid * MAXJ + q) * 64 + lane] = pb[q];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += 256) {
    const int q = j / 64, l = j % 64;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { a += red_g[(w * MAXJ + q) * 64 + l]; b += red_b[(w * MAXJ + q) * 64 + l]; }
    slab[(size_t)blockIdx.x * 2 * D + j] = a;
    slab[(size_t)blockIdx.x * 2 * D + D + j] = b;
  }
}
// D <= 128, D % 4 == 0 (bf16 or fp32): one row per half wave, 4 contiguous values per lane (one 8- /
// 16-byte load / store), mean and variance from registers (one read of x), and without SAVE (no-grad
// forwards: the generator in every critic step) no xhat / rstd traffic.  bf16: a fixed grid (8 workgroups
// per CU) strides over the rows, two rows per half wave per pass with both loads issued before either
// reduction (the one-pass-per-8-rows grid launched ~786 k workgroups per (262 144 x 24) call and moved
// 2.7-3.3 TB/s); fp32 keeps one row per half wave and pass, which its 16-byte lanes already stream at
// 4.4-5.3 TB/s (profiles/r05_ln).  The generic kernel above re-read x three times with
// 2-byte accesses (146 us per (16384 x 24) x 100 call, ~1.6 TB/s, profiles/r01_buf).
template <typename T>
struct LnIO;
template <>
struct LnIO<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, bool on, float (&v)[4]) {
    const uint2 r = on ? *reinterpret_cast<const uint2*>(p) : make_uint2(0, 0);
    v[0] = __uint_as_float(r.x << 16); v[1] = __uint_as_float(r.x & 0xffff0000u);
    v[2] = __uint_as_float(r.y << 16); v[3] = __uint_as_float(r.y & 0xffff0000u);
  }
  static __device__ __forceinline__ void store(bf16_t* p, float a, float b, float c, float d) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(a, b), pk2bf(c, d));
  }
};
template <>
struct LnIO<float> {
  static __device__ __forceinline__ void load(const float* p, bool on, float (&v)[4]) {
    const float4 r = on ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
  }
  static __device__ __forceinline__ void store(float* p, float a, float b, float c, float d) {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
  }
};
template <typename T, bool SAVE, bool PRE>
__device__ __forceinline__ void ln_row(float (&v)[4], int64_t row, int j, bool on, int D, float eps, float pre_alpha,
                                       const float4& g, const float4& b, T* __restrict__ y, T* __restrict__ xhat,
                                       float* __restrict__ rstd_out, int hl) {
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = pre_lrelu<T>(v[i], pre_alpha);
  }
  const float mu = halfwave_sum((v[0] + v[1]) + (v[2] + v[3])) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = on ? v[i] - mu : 0.f;
    q += v[i] * v[i];
  }
  const float rstd = rsqrtf(halfwave_sum(q) / D + eps);
  if (on) {
    const float h0 = v[0] * rstd, h1 = v[1] * rstd, h2 = v[2] * rstd, h3 = v[3] * rstd;
    LnIO<T>::store(y + row * D + j, h0 * g.x + b.x, h1 * g.y + b.y, h2 * g.z + b.z, h3 * g.w + b.w);
    if constexpr (SAVE) LnIO<T>::store(xhat + row * D + j, h0, h1, h2, h3);
  }
  if (SAVE && hl == 0) rstd_out[row] = rstd;
}
template <typename T, bool SAVE, bool PRE, int NR>
__global__ void __launch_bounds__(256) layernorm_fwd_x4_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, T* __restrict__ y,
                                                               T* __restrict__ xhat, float* __restrict__ rstd_out,
                                                               int64_t rows, int D, float eps, float pre_alpha) {
  static_assert(NR == 1 || NR == 2, "rows per half wave and pass");
  const int hl = threadIdx.x & 31;
  const int j = 4 * hl;
  const bool on = j < D;
  const float4 g = on ? *reinterpret_cast<const float4*>(gamma + j) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 b = on ? *reinterpret_cast<const float4*>(beta + j) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t stride = (int64_t)gridDim.x * 8 * NR;
  // (the row index is uniform over a half wave: every branch below keeps the half wave together, and the
  // reductions stay inside it)
  for (int64_t r0 = (int64_t)blockIdx.x * 8 * NR + (threadIdx.x >> 5); r0 < rows; r0 += stride) {
    float v0[4], v1[4];
    LnIO<T>::load(x + r0 * D + j, on, v0);
    if constexpr (NR == 2) {
      const int64_t r1 = r0 + 8;
      const bool two = r1 < rows;
      LnIO<T>::load(x + (two ? r1 : r0) * D + j, on && two, v1);
      ln_row<T, SAVE, PRE>(v0, r0, j, on, D, eps, pre_alpha, g, b, y, xhat, rstd_out, hl);
      if (two) ln_row<T, SAVE, PRE>(v1, r1, j, on, D, eps, pre_alpha, g, b, y, xhat, rstd_out, hl);
    } else {
      ln_row<T, SAVE, PRE>(v0, r0, j, on, D, eps, pre_alpha, g, b, y, xhat, rstd_out, hl);
    }
  }
}

void launch_layernorm_fwd(int dt, const void* x, const float* gamma, const float* beta, void* y, void* xhat,
                          float* rstd, int64_t rows, int D, float eps, float pre_alpha, hipStream_t s) {
  if ((dt == DT_F32 || dt == DT_BF16) && D <= 128 && D % 4 == 0) {
    const bool sv = xhat != nullptr, pre = pre_alpha >= 0.f;
    if (dt == DT_F32) {
      // fp32 (16-byte lanes): one row per half wave, one pass (4.4-5.3 TB/s; the bf16 form below measured
      // 4.1-4.4 here, scripts/bench_ln.py)
      const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 7) / 8, 1 << 30));
      auto k = sv ? (pre ? layernorm_fwd_x4_kernel<float, true, true, 1> : layernorm_fwd_x4_kernel<float, true, false, 1>)
                  : (pre ? layernorm_fwd_x4_kernel<float, false, true, 1> : layernorm_fwd_x4_kernel<float, false, false, 1>);
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s, (const float*)x, gamma, beta, (float*)y, (float*)xhat, rstd,
                         rows, D, eps, pre_alpha);
    } else {
      // bf16 (8-byte lanes): two rows per half wave and pass on a grid of 8 workgroups per CU (-30 % without
      // / -7 % with the saved xhat against one row per half wave and pass, 2.7 -> 3.9 TB/s)
      const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 15) / 16, (int64_t)device_cu_count() * 8));
      auto k = sv ? (pre ? layernorm_fwd_x4_kernel<bf16_t, true, true, 2> : layernorm_fwd_x4_kernel<bf16_t, true, false, 2>)
                  : (pre ? layernorm_fwd_x4_kernel<bf16_t, false, true, 2> : layernorm_fwd_x4_kernel<bf16_t, false, false, 2>);
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, gamma, beta, (bf16_t*)y, (bf16_t*)xhat, rstd,
                         rows, D, eps, pre_alpha);
    }
    return;
  }
  // one row per wave and no grid-stride loop: a wave's row is a dependent load -> reduce -> store
  // chain, so latency is hidden by having every row in flight at once, not by looping
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 1 << 30));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(layernorm_fwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, gamma, beta,
                       (bf16_t*)y, (bf16_t*)xhat, rstd, rows, D, eps, pre_alpha);
  else
    hipLaunchKernelGGL(layernorm_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, gamma, beta,
                       (float*)y, (float*)xhat, rstd, rows, D, eps, pre_alpha);
}

// D <= 128, D % 4 == 0: one row per half wave, 4 contiguous columns per lane (8- / 16-byte
// accesses), grid-stride; the per-column dgamma / dbeta partials stay in registers across rows and
// are reduced over the block's 8 half waves once.  The one-wave-per-row kernel above read 2-byte
// values with 4 lanes idle in every 64 (bf16: 1.63 ms per (262144 x 24) x 100 call, 2.3 TB/s).
template <typename T>
struct Vec4;
template <>
struct Vec4<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float (&v)[4]) {
    const uint2 r = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(r.x << 16); v[1] = __uint_as_float(r.x & 0xffff0000u);
    v[2] = __uint_as_float(r.y << 16); v[3] = __uint_as_float(r.y & 0xffff0000u);
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float (&v)[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(v[0], v[1]), pk2bf(v[2], v[3]));
  }
};
template <>
struct Vec4<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    const float4 r = *reinterpret_cast<const float4*>(p);
    v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};

template <typename T>
__global__ void __launch_bounds__(256) layernorm_bwd_x4_kernel(const T* __restrict__ dy, const T* __restrict__ xhat,
                                                               const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                               T* __restrict__ dx, float* __restrict__ slab, int64_t rows,
                                                               int D) {
  __shared__ float red[2][8][128];
  const int hl = threadIdx.x & 31, hw = threadIdx.x >> 5;
  const int j = 4 * hl;
  const bool on = j < D;
  float g[4] = {0.f, 0.f, 0.f, 0.f}, pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
  if (on) {
    const float4 gg = *reinterpret_cast<const float4*>(gamma + j);
    g[0] = gg.x; g[1] = gg.y; g[2] = gg.z; g[3] = gg.w;
  }
  const int64_t stride = (int64_t)gridDim.x * 8;
  for (int64_t row = (int64_t)blockIdx.x * 8 + hw; row < rows; row += stride) {
    float d[4] = {0.f, 0.f, 0.f, 0.f}, xh[4] = {0.f, 0.f, 0.f, 0.f};
    if (on) {
      Vec4<T>::load(dy + row * D + j, d);
      Vec4<T>::load(xhat + row * D + j, xh);
    }
    float gv[4], sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gv[i] = d[i] * g[i];
      sg += gv[i];
      sgx += gv[i] * xh[i];
      pg[i] += d[i] * xh[i];
      pb[i] += d[i];
    }
    const float mg = halfwave_sum(sg) / D, mgx = halfwave_sum(sgx) / D;
    const float rs = rstd[row];
    if (on) {
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = rs * (gv[i] - mg - xh[i] * mgx);
      Vec4<T>::store(dx + row * D + j, o);
    }
  }
  if (slab == nullptr) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[0][hw][j + i] = pg[i];
    red[1][hw][j + i] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int h = 0; h < 8; ++h) { a += red[0][h][c]; b += red[1][h][c]; }
    slab[(size_t)blockIdx.x * 2 * D + c] = a;
    slab[(size_t)blockIdx.x * 2 * D + D + c] = b;
  }
}

int layernorm_bwd_splits(int64_t rows) { return (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 2048)); }

void launch_layernorm_bwd(int dt, const void* dy, const void* xhat, const float* rstd, const float* gamma, void* dx,
                          float* ggamma, float* gbeta, float* ws, int64_t rows, int D, hipStream_t s) {
  float* slab = (ggamma || gbeta) ? ws : nullptr;
  if (D <= 128 && D % 4 == 0) {
    // grid <= layernorm_bwd_splits(rows): the workspace the caller sized holds its slabs
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 7) / 8, 2048));
    if (dt == DT_BF16)
      hipLaunchKernelGGL(layernorm_bwd_x4_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)dy,
                         (const bf16_t*)xhat, rstd, gamma, (bf16_t*)dx, slab, rows, D);
    else
      hipLaunchKernelGGL(layernorm_bwd_x4_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)dy,
                         (const float*)xhat, rstd, gamma, (float*)dx, slab, rows, D);
    if (slab) launch_split_reduce(slab, ggamma, gbeta, grid, D, D, s);
    return;
  }
  const int grid = layernorm_bwd_splits(rows);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(layernorm_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)dy,
                       (const bf16_t*)xhat, rstd, gamma, (bf16_t*)dx, slab, rows, D);
  else
    hipLaunchKernelGGL(layernorm_bwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)dy, (const float*)xhat,
                       rstd, gamma, (float*)dx, slab, rows, D);
  if (slab) launch_split_reduce(slab, ggamma, gbeta, grid, D, D, s);
}

// ------------------------------------------------------------------ LayerNorm tangents (GP critics)
// A gradient-penalty critic with LayerNorm (the lstm_critic_clip family) differentiates the LN's
// Jacobian-vector product: the reference gets it from nested tf.GradientTape
// (MTSS-GAN/mtss_gan.py:148-160); here it is two per-row kernels on the saved xhat / rstd.
// Per row (r = rstd, mean over D):
//   m = mean(xhat * xd),  xhatd = r (xd - mean(xd) - xhat m),  yd = gamma * xhatd
// and for the reverse of (y, yd) with seeds (dy, dyd), g = gamma dy, h = gamma dyd,
// S = sum(h xhat), P = sum(h xd):
//   dxd = r (h - mean(h) - xhat S / D)
//   G   = g - r m h - (r S / D) xd
//   dx  = r (G - mean(G) - xhat mean(G xhat)) - r^2 xhat (P - D mean(xd) mean(h) - m S) / D
//   dgamma += dy xhat + dyd xhatd,  dbeta += dy
// mean(G) and mean(G xhat) expand into the seven raw row sums below, so every row is one read of
// its four operands, one 7-way reduction and one write of dx / dxd.
template <typename T>
__global__ void __launch_bounds__(256) layernorm_tfwd_kernel(const T* __restrict__ xd, const T* __restrict__ xhat,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma, T* __restrict__ yd,
                                                             int64_t rows, int D) {
  constexpr int MAXJ = 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float dv[MAXJ], hv[MAXJ], sd = 0.f, sxd = 0.f;
#pragma unroll
  for (int q = 0; q < MAXJ; ++q) {
    const int j = lane + 64 * q;
    dv[q] = j < D ? ld_f(xd + row * D + j) : 0.f;
    hv[q] = j < D ? ld_f(xhat + row * D + j) : 0.f;
    sd += dv[q];
    sxd += dv[q] * hv[q];
  }
  const float mxd = wave_sum(sd) / D, m = wave_sum(sxd) / D, r = rstd[row];
#pragma unroll
  for (int q = 0; q < MAXJ; ++q) {
    const int j = lane + 64 * q;
    if (j < D) st_f(yd + row * D + j, gamma[j] * r * (dv[q] - mxd - hv[q] * m));
  }
}

template <typename T, bool HAS_DY, bool NEED_DX>
__global__ void __launch_bounds__(256) layernorm_tbwd_kernel(const T* __restrict__ dy, const T* __restrict__ dyd,
                                                             const T* __restrict__ xd, const T* __restrict__ xhat,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma, T* __restrict__ dx,
                                                             T* __restrict__ dxd, float* __restrict__ slab,
                                                             int64_t rows, int D) {
  constexpr int MAXJ = 4;  // D <= 256
  __shared__ float red_g[4 * MAXJ * 64];
  __shared__ float red_b[4 * MAXJ * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float pg[MAXJ] = {0.f, 0.f, 0.f, 0.f}, pb[MAXJ] = {0.f, 0.f, 0.f, 0.f};
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wid; row < rows; row += wstride) {
    const int64_t o = row * D;
    float yv[MAXJ], ev[MAXJ], hv[MAXJ], dv[MAXJ], xv[MAXJ];
    float s_d = 0.f, s_xd = 0.f, s_g = 0.f, s_gx = 0.f, s_h = 0.f, s_hx = 0.f, s_hd = 0.f;
#pragma unroll
    for (int q = 0; q < MAXJ; ++q) {
      const int j = lane + 64 * q;
      const bool on = j < D;
      const float ga = on ? gamma[j] : 0.f;
      yv[q] = (HAS_DY && on) ? ld_f(dy + o + j) : 0.f;
      ev[q] = on ? ld_f(dyd + o + j) : 0.f;
      hv[q] = ga * ev[q];  // h = gamma dyd
      dv[q] = on ? ld_f(xd + o + j) : 0.f;
      xv[q] = on ? ld_f(xhat + o + j) : 0.f;
      const float g = ga * yv[q];
      s_d += dv[q];
      s_xd += xv[q] * dv[q];
      s_g += g;
      s_gx += g * xv[q];
      s_h += hv[q];
      s_hx += hv[q] * xv[q];
      s_hd += hv[q] * dv[q];
    }
    const float invD = 1.f / D, r = rstd[row];
    const float mxd = wave_sum(s_d) * invD, m = wave_sum(s_xd) * invD;
    const float mh = wave_sum(s_h) * invD, S = wave_sum(s_hx), P = wave_sum(s_hd);
    const float c = r * S * invD;  // coefficient of xd in G (and of xhat in dxd, divided by r)
    float mG = 0.f, mGx = 0.f;
    if constexpr (NEED_DX) {
      mG = wave_sum(s_g) * invD - r * m * mh - c * mxd;
      mGx = wave_sum(s_gx) * invD - 2.f * r * m * S * invD;
    }
    const float kr = r * r * (P - D * mxd * mh - m * S) * invD;
#pragma unroll
    for (int q = 0; q < MAXJ; ++q) {
      const int j = lane + 64 * q;
      if (j < D) {
        const float ga = gamma[j];
        const float xhd = r * (dv[q] - mxd - xv[q] * m);
        pg[q] += (HAS_DY ? yv[q] * xv[q] : 0.f) + ev[q] * xhd;
        pb[q] += yv[q];
        if constexpr (NEED_DX) {
          const float G = ga * yv[q] - r * m * hv[q] - c * dv[q];
          st_f(dx + o + j, r * (G - mG - xv[q] * mGx) - kr * xv[q]);
          st_f(dxd + o + j, r * (hv[q] - mh) - c * xv[q]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAXJ; ++q) {
    red_g[(wid * MAXJ + q) * 64 + lane] = pg[q];
    red_b[(wid * MAXJ + q) * 64 + lane] = pb[q];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += 256) {
    const int q = j / 64, l = j % 64;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { a += red_g[(w * MAXJ + q) * 64 + l]; b += red_b[(w * MAXJ + q) * 64 + l]; }
    slab[(size_t)blockIdx.x * 2 * D + j] = a;
    slab[(size_t)blockIdx.x * 2 * D + D + j] = b;
  }
}

void launch_layernorm_tfwd(int dt, const void* xd, const void* xhat, const float* rstd, const float* gamma, void* yd,
                           int64_t rows, int D, hipStream_t s) {
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 1 << 30));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(layernorm_tfwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)xd,
                       (const bf16_t*)xhat, rstd, gamma, (bf16_t*)yd, rows, D);
  else
    hipLaunchKernelGGL(layernorm_tfwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)xd,
                       (const float*)xhat, rstd, gamma, (float*)yd, rows, D);
}

template <typename T>
static void tbwd_dispatch(const void* dy, const void* dyd, const void* xd, const void* xhat, const float* rstd,
                          const float* gamma, void* dx, void* dxd, float* slab, int64_t rows, int D, int grid,
                          hipStream_t s) {
#define HFREP_LNT(HD, ND)                                                                                       \
  hipLaunchKernelGGL((layernorm_tbwd_kernel<T, HD, ND>), dim3(grid), dim3(256), 0, s, (const T*)dy, (const T*)dyd, \
                     (const T*)xd, (const T*)xhat, rstd, gamma, (T*)dx, (T*)dxd, slab, rows, D)
  if (dy && dx) HFREP_LNT(true, true);
  else if (dy) HFREP_LNT(true, false);
  else if (dx) HFREP_LNT(false, true);
  else HFREP_LNT(false, false);
#undef HFREP_LNT
}

void launch_layernorm_tbwd(int dt, const void* dy, const void* dyd, const void* xd, const void* xhat,
                           const float* rstd, const float* gamma, void* dx, void* dxd, float* ggamma, float* gbeta,
                           float* ws, int64_t rows, int D, hipStream_t s) {
  const int grid = layernorm_bwd_splits(rows);
  if (dt == DT_BF16)
    tbwd_dispatch<bf16_t>(dy, dyd, xd, xhat, rstd, gamma, dx, dxd, ws, rows, D, grid, s);
  else
    tbwd_dispatch<float>(dy, dyd, xd, xhat, rstd, gamma, dx, dxd, ws, rows, D, grid, s);
  launch_split_reduce(ws, ggamma, gbeta, grid, D, D, s);
}

// ------------------------------------------------------------------ gradient penalty coefficient
// One wave per sample row: the per-row penalty term goes to its own slot and a single-workgroup
// reduce sums them (a per-row atomicAdd on one address serialised 16k adds: 212 us at B = 16384).
// one wave per row (grid-stride).  Rows with D % 4 == 0, D <= 1024 and aligned buffers are read once
// with 8-byte (bf16) / 16-byte (fp32) loads into registers (<= 16 values per lane) and scaled from there;
// other shapes take the scalar two-pass loop
template <typename T>
__global__ void __launch_bounds__(256) gp_coef_kernel(const T* __restrict__ g, T* __restrict__ v,
                                                      float* __restrict__ rowpen, int B, int64_t D, float weight) {
  const int lane = threadIdx.x & 63;
  const bool vec = (D & 3) == 0 && D <= 1024 && (reinterpret_cast<uintptr_t>(g) & (4 * sizeof(T) - 1)) == 0 &&
                   (reinterpret_cast<uintptr_t>(v) & (4 * sizeof(T) - 1)) == 0;
  for (int b = blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += gridDim.x * 4) {
    const T* gr = g + (int64_t)b * D;
    T* vr = v + (int64_t)b * D;
    float s = 0.f;
    if (vec) {
      float x[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t j = 4 * (lane + 64 * c);
        if (j < D) {
          ld4(gr + j, x[c]);
#pragma unroll
          for (int e = 0; e < 4; ++e) s = fmaf(x[c][e], x[c][e], s);
        }
      }
      const float nrm = sqrtf(wave_sum(s));
      const float one_m = 1.f - nrm;
      const float scale = -(2.f * weight / B) * one_m / fmaxf(nrm, 1e-30f);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t j = 4 * (lane + 64 * c);
        if (j < D) st4(vr + j, x[c][0] * scale, x[c][1] * scale, x[c][2] * scale, x[c][3] * scale);
      }
      if (lane == 0) rowpen[b] = one_m * one_m / B;
    } else {
      for (int64_t j = lane; j < D; j += 64) { const float x = ld_f(gr + j); s += x * x; }
      const float nrm = sqrtf(wave_sum(s));
      const float one_m = 1.f - nrm;
      const float scale = -(2.f * weight / B) * one_m / fmaxf(nrm, 1e-30f);
      for (int64_t j = lane; j < D; j += 64) st_f(vr + j, ld_f(gr + j) * scale);
      if (lane == 0) rowpen[b] = one_m * one_m / B;
    }
  }
}

// pen = sum of the row penalties (fixed order: bitwise reproducible); with w (the critic's two W terms)
// also the step's loss record pack = [w0 + w1 + weight pen, w0, w1, pen] (no torch glue on the step)
__global__ void __launch_bounds__(1024) gp_sum_kernel(const float* __restrict__ x, int n, float* __restrict__ out,
                                                      const float* __restrict__ w, float weight, float* __restrict__ pack) {
  __shared__ float red[16];
  // four independent 16-byte streams per thread (fixed order), then the scalar tail
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  const int n4 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? n / 4 : 0;
  for (int i = threadIdx.x; i < n4; i += 1024) {
    const float4 q = reinterpret_cast<const float4*>(x)[i];
    a0 += q.x; a1 += q.y; a2 += q.z; a3 += q.w;
  }
  for (int i = 4 * n4 + threadIdx.x; i < n; i += 1024) a0 += x[i];
  float s = (a0 + a1) + (a2 + a3);
  s = block_sum<16>(s, red);
  if (threadIdx.x == 0) {
    out[0] = s;
    if (pack) {
      pack[0] = w[0] + w[1] + weight * s;
      pack[1] = w[0];
      pack[2] = w[1];
      pack[3] = s;
    }
  }
}

// the loss record pack [w0 + w1 + weight pen, w0, w1, pen] from an already reduced penalty: the same
// arithmetic as gp_sum_kernel's pack (the concurrent small-batch critic step forms it after the join)
__global__ void gp_pack_kernel(const float* __restrict__ pen, const float* __restrict__ w, float weight,
                               float* __restrict__ pack) {
  if (threadIdx.x == 0) {
    const float s = pen[0];
    pack[0] = w[0] + w[1] + weight * s;
    pack[1] = w[0];
    pack[2] = w[1];
    pack[3] = s;
  }
}

void launch_gp_pack(const float* pen, const float* w, float weight, float* pack, hipStream_t s) {
  hipLaunchKernelGGL(gp_pack_kernel, dim3(1), dim3(64), 0, s, pen, w, weight, pack);
}

void launch_gp_coef(int dt, const void* g, void* v, float* pen, float* rowpen, int B, int64_t D, float weight,
                    hipStream_t s, const float* w, float* pack) {
  const int grid = std::max(1, std::min((B + 3) / 4, 8192));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gp_coef_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)g, (bf16_t*)v, rowpen, B, D,
                       weight);
  else
    hipLaunchKernelGGL(gp_coef_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)g, (float*)v, rowpen, B, D,
                       weight);
  hipLaunchKernelGGL(gp_sum_kernel, dim3(1), dim3(1024), 0, s, rowpen, B, pen, w, weight, pack);
}

// ------------------------------------------------------------------ GAN losses
// Value and gradient of the critic / generator losses in one pass over the scores p (N rows,
// flattened).  Elements [0, split) are segment 0 with label la, [split, n) segment 1 with label lb;
// each segment's loss is a mean over its own element count (the W terms on [real; fake] are one
// launch).  kind 0: Wasserstein, loss = label * p, grad = label.  kind 1: Keras binary
// cross-entropy on probabilities (clip to [eps, 1 - eps], log(o + eps); zero gradient where the
// clip is active).  Per-block partial sums, reduced in a fixed order: bitwise reproducible.
constexpr int LOSS_BLOCKS = 256;
template <typename T>
__global__ void __launch_bounds__(256) gan_loss_kernel(const T* __restrict__ p, int64_t n, int64_t split, float la,
                                                       float lb, int kind, T* __restrict__ grad,
                                                       float* __restrict__ partial) {
  __shared__ float red[4];
  constexpr float eps = 1e-7f;
  const float inv0 = split > 0 ? 1.f / (float)split : 0.f, inv1 = n > split ? 1.f / (float)(n - split) : 0.f;
  float s0 = 0.f, s1 = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const bool seg0 = i < split;
    const float y = seg0 ? la : lb, inv = seg0 ? inv0 : inv1;
    const float x = ld_f(p + i);
    float l, g;
    if (kind == 0) {
      l = y * x;
      g = y * inv;
    } else {
      const float o = fminf(fmaxf(x, eps), 1.f - eps);
      l = -(y * logf(o + eps) + (1.f - y) * logf(1.f - o + eps));
      const bool inside = x > eps && x < 1.f - eps;
      g = inside ? -(y / (o + eps) - (1.f - y) / (1.f - o + eps)) * inv : 0.f;
    }
    st_f(grad + i, g);
    if (seg0) s0 += l * inv;
    else s1 += l * inv;
  }
  s0 = block_sum<4>(s0, red);
  __syncthreads();
  s1 = block_sum<4>(s1, red);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = s0;
    partial[2 * blockIdx.x + 1] = s1;
  }
}
__global__ void __launch_bounds__(256) gan_loss_reduce_kernel(const float* __restrict__ partial, int nb,
                                                              float* __restrict__ out) {
  __shared__ float red[4];
  float s0 = 0.f, s1 = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) { s0 += partial[2 * i]; s1 += partial[2 * i + 1]; }
  s0 = block_sum<4>(s0, red);
  __syncthreads();
  s1 = block_sum<4>(s1, red);
  if (threadIdx.x == 0) { out[0] = s0; out[1] = s1; }
}
void launch_gan_loss(int dt, const void* p, int64_t n, int64_t split, float la, float lb, int kind, void* grad,
                     float* partial, float* out, hipStream_t s) {
  const int nb = (int)std::min<int64_t>(LOSS_BLOCKS, std::max<int64_t>(1, (n + 1023) / 1024));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gan_loss_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, (const bf16_t*)p, n, split, la, lb, kind,
                       (bf16_t*)grad, partial);
  else
    hipLaunchKernelGGL(gan_loss_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)p, n, split, la, lb, kind,
                       (float*)grad, partial);
  hipLaunchKernelGGL(gan_loss_reduce_kernel, dim3(1), dim3(256), 0, s, partial, nb, out);
}
int gan_loss_partials() { return LOSS_BLOCKS; }

// ------------------------------------------------------------------ interpolation
template <typename T>
__global__ void __launch_bounds__(256) interp_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                     const float* __restrict__ alpha, T* __restrict__ out, int64_t D,
                                                     int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float al = alpha[i / D];
    st_f(out + i, al * ld_f(a + i) + (1.f - al) * ld_f(b + i));
  }
}
void launch_interpolate(int dt, const void* real, const void* fake, const float* alpha, void* out, int B, int64_t D,
                        hipStream_t s) {
  const int64_t n = (int64_t)B * D;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(interp_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)real,
                       (const bf16_t*)fake, alpha, (bf16_t*)out, D, n);
  else
    hipLaunchKernelGGL(interp_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, s, (const float*)real,
                       (const float*)fake, alpha, (float*)out, D, n);
}

// ------------------------------------------------------------------ Philox RNG

template <typename T>
__global__ void __launch_bounds__(256) philox_fill_kernel(T* __restrict__ out, int64_t n, uint64_t seed,
                                                          const int64_t* __restrict__ ctr, int dist) {
  const uint64_t base = (uint64_t)ctr[0];
  const int64_t nq = (n + 3) / 4;
  const bool vec = (reinterpret_cast<uintptr_t>(out) & (4 * sizeof(T) - 1)) == 0;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
    const uint4 r = Philox::gen(seed, base + (uint64_t)q, 0x5EEDu);
    float v[4];
    const float u0 = u32_to_unit(r.x), u1 = u32_to_unit(r.y), u2 = u32_to_unit(r.z), u3 = u32_to_unit(r.w);
    if (dist == 1) {
      const float ra = sqrtf(-2.f * __logf(u0)), rb = sqrtf(-2.f * __logf(u2));
      float sa, ca, sb, cb;
      __sincosf(6.283185307179586f * u1, &sa, &ca);
      __sincosf(6.283185307179586f * u3, &sb, &cb);
      v[0] = ra * ca; v[1] = ra * sa; v[2] = rb * cb; v[3] = rb * sb;
    } else {
      v[0] = u0; v[1] = u1; v[2] = u2; v[3] = u3;
    }
    if (vec && q * 4 + 3 < n) {
      st4(out + q * 4, v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = q * 4 + k;
        if (i < n) st_f(out + i, v[k]);
      }
    }
  }
}

__global__ void ctr_advance_kernel(int64_t* ctr, int64_t by) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ctr[0] += by;
}

void launch_philox_fill(int dt, void* out, int64_t n, uint64_t seed, int64_t* ctr, int dist, hipStream_t s) {
  const int64_t nq = (n + 3) / 4;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(philox_fill_kernel<bf16_t>, dim3(ew_grid(nq)), dim3(256), 0, s, (bf16_t*)out, n, seed, ctr, dist);
  else
    hipLaunchKernelGGL(philox_fill_kernel<float>, dim3(ew_grid(nq)), dim3(256), 0, s, (float*)out, n, seed, ctr, dist);
  hipLaunchKernelGGL(ctr_advance_kernel, dim3(1), dim3(64), 0, s, ctr, nq);
}

// ------------------------------------------------------------------ batch sampling: out[b] = data[randint(N)]
// One wave per window (grid-stride; a window is D = T * F values, 768 at the bench shape), 16-byte
// loads and 16- / 8-byte stores when D % 4 == 0 and both buffers are aligned.  The window index of
// sample b is Philox(seed, ctr + b) as before, so the draws do not depend on the launch shape.
template <typename T>
__global__ void __launch_bounds__(256) sample_windows_kernel(const float* __restrict__ data, int64_t N, int64_t D,
                                                             T* __restrict__ out, int64_t B, uint64_t seed,
                                                             const int64_t* __restrict__ ctr) {
  const int lane = threadIdx.x & 63;
  const uint64_t c0 = (uint64_t)ctr[0];
  const bool vec = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & (4 * sizeof(T) - 1)) == 0;
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += (int64_t)gridDim.x * 4) {
    const uint4 r = Philox::gen(seed, c0 + (uint64_t)b, 0xB47Cu);
    const uint64_t idx = (((uint64_t)r.x << 32) | r.y) % (uint64_t)N;
    const float* src = data + (int64_t)idx * D;
    T* dst = out + b * D;
    if (vec) {
      for (int64_t j = 4 * lane; j < D; j += 256) {
        const float4 v = *reinterpret_cast<const float4*>(src + j);
        st4(dst + j, v.x, v.y, v.z, v.w);
      }
    } else {
      for (int64_t j = lane; j < D; j += 64) st_f(dst + j, src[j]);
    }
  }
}

void launch_sample_windows(int dt, const float* data, int64_t N, int64_t D, void* out, int B, uint64_t seed,
                           int64_t* ctr, hipStream_t s) {
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(((int64_t)B + 3) / 4, 8192));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(sample_windows_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, data, N, D, (bf16_t*)out, (int64_t)B,
                       seed, ctr);
  else
    hipLaunchKernelGGL(sample_windows_kernel<float>, dim3(grid), dim3(256), 0, s, data, N, D, (float*)out, (int64_t)B,
                       seed, ctr);
  hipLaunchKernelGGL(ctr_advance_kernel, dim3(1), dim3(64), 0, s, ctr, (int64_t)B);
}

// ------------------------------------------------------------------ dtype cast
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    st_f(out + i, ld_f(in + i));
}
void launch_cast(int dt_in, const void* in, int dt_out, void* out, int64_t n, hipStream_t s) {
  if (dt_in == DT_BF16 && dt_out == DT_F32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)in, (float*)out, n);
  else if (dt_in == DT_F32 && dt_out == DT_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), dim3(ew_grid(n)), dim3(256), 0, s, (const float*)in, (bf16_t*)out, n);
  else
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(ew_grid(n)), dim3(256), 0, s, (const float*)in, (float*)out, n);
}

// ------------------------------------------------------------------ causal dilated conv1d (im2col)
// cols[b, t, j*C + c] = x[b, t - (k-1-j)*dil, c] (0 before the start): the Conv1D layer is then a
// Dense GEMM over (k*C) columns (models/layers.py Conv1D); col2im is the matching GATHER (no
// atomics): dx[b, t, c] = sum_j dcols[b, t + (k-1-j)*dil, j*C + c].
template <typename T>
__global__ void __launch_bounds__(256) im2col_causal_kernel(const T* __restrict__ x, T* __restrict__ cols, int B, int Tn,
                                                            int C, int k, int dil) {
  const int64_t n = (int64_t)B * Tn * k * C;
  const int KC = k * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t bt = i / KC;
    const int jc = (int)(i - bt * KC), j = jc / C, c = jc - j * C;
    const int t = (int)(bt % Tn);
    const int src = t - (k - 1 - j) * dil;
    cols[i] = src >= 0 ? x[(bt - t + src) * C + c] : Cvt<T>::from_f(0.f);
  }
}
template <typename T>
__global__ void __launch_bounds__(256) col2im_causal_kernel(const T* __restrict__ dcols, T* __restrict__ dx, int B,
                                                            int Tn, int C, int k, int dil) {
  const int64_t n = (int64_t)B * Tn * C;
  const int KC = k * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t bt = i / C;
    const int c = (int)(i - bt * C), t = (int)(bt % Tn);
    float s = 0.f;
    for (int j = 0; j < k; ++j) {
      const int dst = t + (k - 1 - j) * dil;
      if (dst < Tn) s += ld_f(dcols + (bt - t + dst) * KC + j * C + c);
    }
    st_f(dx + i, s);
  }
}
void launch_im2col_causal(int dt, const void* x, void* cols, int B, int Tn, int C, int k, int dil, hipStream_t s) {
  const int64_t n = (int64_t)B * Tn * k * C;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(im2col_causal_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)x,
                       (bf16_t*)cols, B, Tn, C, k, dil);
  else
    hipLaunchKernelGGL(im2col_causal_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, s, (const float*)x, (float*)cols,
                       B, Tn, C, k, dil);
}
void launch_col2im_causal(int dt, const void* dcols, void* dx, int B, int Tn, int C, int k, int dil, hipStream_t s) {
  const int64_t n = (int64_t)B * Tn * C;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(col2im_causal_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, s, (const bf16_t*)dcols,
                       (bf16_t*)dx, B, Tn, C, k, dil);
  else
    hipLaunchKernelGGL(col2im_causal_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, s, (const float*)dcols,
                       (float*)dx, B, Tn, C, k, dil);
}

int device_cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    HFREP_CHECK_HIP(hipGetDevice(&dev));
    HFREP_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (cus <= 0) cus = 256;
  }
  return cus;
}

}  // namespace hfrep
