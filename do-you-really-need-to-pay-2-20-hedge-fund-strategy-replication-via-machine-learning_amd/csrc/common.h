// Shared device helpers for the hfrep gfx950 (CDNA4) kernel library.
//
// Everything here is written for MI355X only: wave64, MFMA 32x32 tiles, LDS.
// No CUDA shims and no dual-platform paths.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace hfrep {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// bf16 helpers (storage type is raw uint16_t so host code never needs hip_bf16)
// ---------------------------------------------------------------------------
typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even through the gfx950 conversion instruction (v_cvt_pk_bf16_f32: one VALU op
// per PAIR of values, NaN stays NaN); the integer-rounding form it replaces cost ~8 VALU per value
typedef __bf16 hw_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// two values -> packed bf16 pair (lo in bits 0..15)
__device__ __forceinline__ uint32_t pk2bf(float lo, float hi) {
  const hw_bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};
template <typename T> __device__ __forceinline__ float ld_f(const T* p) { return Cvt<T>::to_f(*p); }
template <typename T> __device__ __forceinline__ void st_f(T* p, float v) { *p = Cvt<T>::from_f(v); }

// ---------------------------------------------------------------------------
// activations (Keras semantics).  act codes shared with the host side:
//   0 = linear, 1 = sigmoid, 2 = tanh, 3 = leaky_relu(0.2), 4 = relu
// ---------------------------------------------------------------------------
enum Act : int { ACT_LINEAR = 0, ACT_SIGMOID = 1, ACT_TANH = 2, ACT_LRELU = 3, ACT_RELU = 4 };

// The LSTM cell evaluates 3 sigmoids + 2 tanh per unit per step; with IEEE division (a ~10
// instruction div_scale/div_fmas/div_fixup sequence each) these were ~2.4k VALU instructions per
// step per wave, the single largest cost of the recurrent kernels.  v_exp_f32 + v_rcp_f32 (1 ulp
// each) is 4-5 instructions per activation and far below bf16 storage precision.
__device__ __forceinline__ float rcpf_(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sigmoidf_(float x) { return rcpf_(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  // tanh(|x|) = (1 - e) / (1 + e), e = exp(-2|x|) in (0, 1]: no overflow, saturates cleanly
  const float e = __expf(-2.0f * fabsf(x));
  return copysignf((1.0f - e) * rcpf_(1.0f + e), x);
}

__device__ __forceinline__ float act_f(int act, float x) {
  switch (act) {
    case ACT_SIGMOID: return sigmoidf_(x);
    case ACT_TANH: return tanhf_(x);
    case ACT_LRELU: return x >= 0.f ? x : 0.2f * x;
    case ACT_RELU: return x > 0.f ? x : 0.f;
    default: return x;
  }
}
// ---------------------------------------------------------------------------
// Packed gate math for the recurrent step loops (VALU-issue bound: lstm_fwd4 spent ~1.8k VALU
// issue cycles per wave per step against 1k of MFMA).  Pairs of values go through v_pk_add /
// v_pk_mul / v_pk_fma_f32 (two fp32 lanes per instruction), and the pre-activations arrive
// PRE-SCALED by the weights (W, U and b multiplied by -log2 e, or -2 log2 e for a tanh gate), so
// a sigmoid is exp2 + add + rcp and a tanh is one more fma: no per-element scale, no abs /
// copysign.  exp2 of a large argument is +inf and rcp(inf) = 0, so both saturate cleanly.
// ---------------------------------------------------------------------------
typedef float f2_t __attribute__((ext_vector_type(2)));
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ f2_t ex2_2(f2_t x) { return f2_t{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])}; }
__device__ __forceinline__ f2_t rcp_2(f2_t x) { return f2_t{__builtin_amdgcn_rcpf(x[0]), __builtin_amdgcn_rcpf(x[1])}; }
// sigmoid(z) from s = -log2(e) z
__device__ __forceinline__ f2_t sig_s2(f2_t s) { return rcp_2(1.f + ex2_2(s)); }
// tanh(z) from s = -2 log2(e) z
__device__ __forceinline__ f2_t tanh_s2(f2_t s) { return 2.f * sig_s2(s) - 1.f; }
// pre-scale of an activation's argument (1 for the piecewise-linear ones)
template <int ACT>
__device__ constexpr float act_prescale() {
  return ACT == ACT_TANH ? -2.f * kLog2e : ACT == ACT_SIGMOID ? -kLog2e : 1.f;
}
// act(z) from the pre-scaled s = act_prescale<ACT>() z
template <int ACT>
__device__ __forceinline__ f2_t act_s2(f2_t s) {
  if constexpr (ACT == ACT_TANH) return tanh_s2(s);
  else if constexpr (ACT == ACT_SIGMOID) return sig_s2(s);
  else return f2_t{act_f(ACT, s[0]), act_f(ACT, s[1])};
}

// derivative expressed through the activation OUTPUT y (all supported acts allow it)
__device__ __forceinline__ float act_dy(int act, float y) {
  switch (act) {
    case ACT_SIGMOID: return y * (1.f - y);
    case ACT_TANH: return 1.f - y * y;
    case ACT_LRELU: return y >= 0.f ? 1.f : 0.2f;
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}
// act_dy on a pair, compile-time act (packed-fp32 cell math)
template <int ACT>
__device__ __forceinline__ f2_t act_dy2(f2_t y) {
  if constexpr (ACT == ACT_TANH) return 1.f - y * y;
  else if constexpr (ACT == ACT_SIGMOID) return y - y * y;
  else return f2_t{act_dy(ACT, y[0]), act_dy(ACT, y[1])};
}
// second derivative expressed through y: needed by the tangent (double-backward) LSTM
__device__ __forceinline__ float act_d2y(int act, float y) {
  switch (act) {
    case ACT_SIGMOID: return y * (1.f - y) * (1.f - 2.f * y);
    case ACT_TANH: return -2.f * y * (1.f - y * y);
    default: return 0.f;
  }
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup-scope release fence
// + s_barrier, and the fence waits for every outstanding global STORE (vmcnt(0)): in the
// recurrent kernels that exposed the full write latency of each step's tape / h stores at every
// step barrier (70% of wave cycles parked in lstm_fwd2).  Here only LDS traffic is drained; global
// stores retire in the background and nothing in the kernel reads them back.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------
// wave / block reductions (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
// sum over the 32 lanes of one half-wave (lanes l and l^k for k<32)
__device__ __forceinline__ float halfwave_sum(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int NWAVES>
__device__ __forceinline__ float block_sum(float v, float* red /* LDS, >= NWAVES floats */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) s += red[i];
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------
// MFMA fragment types
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// 32x32 accumulator row index of register r for lane l (dtype independent on gfx950)
__device__ __forceinline__ int acc32_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ---------------------------------------------------------------------------
// Philox4x32-10 counter RNG (device side).  Deterministic in (seed, offset).
// ---------------------------------------------------------------------------
struct Philox {
  __device__ __forceinline__ static void round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                               uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  __device__ __forceinline__ static uint4 gen(uint64_t seed, uint64_t ctr_hi, uint32_t ctr_lo) {
    uint32_t c0 = ctr_lo, c1 = 0, c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      round(c0, c1, c2, c3, k0, k1);
      k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
  }
};
__device__ __forceinline__ float u32_to_unit(uint32_t x) {  // (0,1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

}  // namespace hfrep

#define HFREP_CHECK_HIP(expr)                                                                  \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
    }                                                                                          \
  } while (0)
