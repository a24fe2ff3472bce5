// Fused MLP-GAN passes for gfx950: BASELINE configs 3 / 4 (vanilla GAN, GAN/GAN.py:127-204, and the
// MLP WGAN-GP, GAN/WGAN_GP.py:221-288) as one kernel per pass instead of one kernel per layer.
//
// The layer-by-layer engine (models/layers.py) round-tripped every (B*T, 100) activation and adjoint
// through HBM: 607 GB per bf16 WGAN-GP iteration at 2.3 TB/s (profiles/r06_mlp/baseline).  Here a
// wave owns 32 rows and carries them through every layer of the pass in registers:
//
//  * transposed orientation: a layer output is held as Y^T (features x rows) in f32x16 accumulators,
//    32 features per tile, row = lane & 31; register q of lane half h is feature 8(q>>2) + 4h + (q&3).
//    The next layer sums over that feature index, so the accumulator IS its B operand (CDNA4 guide
//    §3 "An accumulator tile as the next MFMA's operand"): bf16 packs registers 8s..8s+7 into the
//    k-step s fragment of v_mfma_f32_32x32x16_bf16, fp32 feeds register r straight into k-step r of the
//    exact v_mfma_f32_32x32x2_f32.  No LDS round trip between layers.
//  * the weights live in LDS as pre-permuted A-fragment images (one ds_read_b128 / b32 per MFMA, lane
//    linear, conflict free), built per workgroup from the fp32 master weights in the prologue: a
//    forward image A[o][k = i] and, where the pass goes backwards, a dgrad image A[i][k = o], both with
//    the k order of the accumulator map above.
//  * LayerNorm, bias, sigmoid / LeakyReLU and the per-row head dot are register epilogues: a row's
//    features sit in one lane's registers plus its lane ^ 32 partner, so every row reduction is 16
//    in-lane adds and one cross-half swap.
//  * only the pass's inputs and outputs touch HBM: noise / windows in, fake windows, the weight-
//    gradient operands (consumed by the streaming wgrad kernels) and per-wave loss partials out.
//
// The WGAN-GP critic of WGAN_GP.py (Dense(100) -> Dense(100) -> Flatten -> Dense(1), all linear) gets a
// specialised step kernel (mlp_wgp_*): for an affine critic the W-terms on real / fake and the
// reverse-over-tangent of the gradient penalty all have adjoints along the same head vector w3_t, so
// their weight-gradient operands are summed per row before they leave the kernel (X2c, X1c, Y3c
// below) and each weight gets ONE streaming wgrad instead of three.
#include "common.h"
#include "kernels.h"
#include "mfma.h"
#include "mlp.h"

#include <algorithm>
#include <stdexcept>

namespace hfrep {

// fp32 storage with the products on the bf16 matrix pipe: every operand as three exact bf16 planes
// (hi / mid / lo by truncation, 8 mantissa bits each) and 6 of the 9 plane products (the dropped ones
// are < 2^-24 of the product) on v_mfma_f32_32x32x16_bf16 -- the LSTM fp32 kernels' split (lstm_f32.hip
// split3; error within 2x the exact kernel's vs fp64).  Policy tag f32s_t: k-step geometry of bf16.
struct f32s_t {};
struct F3 {
  bf16x8 h, m, l;
};
template <> struct MF<f32s_t> {
  typedef F3 frag;
  // small terms first: the fp32 accumulator rounds them before the large ones arrive
  __device__ __forceinline__ static f32x16 mma(const frag& a, const frag& b, f32x16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, c, 0, 0, 0);
  }
};
__device__ __forceinline__ F3 split_f3(const float (&v)[8]) {
  F3 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float a = v[j];  // (a scalar copy first: tests/test_isa_hazards.py bit_cast lint)
    const uint32_t u = __builtin_bit_cast(uint32_t, a), hb = u & 0xffff0000u;
    const float r1 = a - __builtin_bit_cast(float, hb);
    const uint32_t mb = __builtin_bit_cast(uint32_t, r1) & 0xffff0000u;
    const float r2 = r1 - __builtin_bit_cast(float, mb);
    f.h[j] = (short)(hb >> 16);
    f.m[j] = (short)(mb >> 16);
    f.l[j] = (short)(__builtin_bit_cast(uint32_t, r2) >> 16);
  }
  return f;
}

namespace {

constexpr int MLP_WAVES = 4;  // waves per workgroup (one per SIMD; up to 512 registers per wave)
constexpr int MLP_THREADS = 64 * MLP_WAVES;
constexpr int VEC = 128;      // padded length of every per-feature vector in LDS
constexpr float LN_EPS_F = 1e-3f, LRELU_ALPHA_F = 0.2f, KERAS_EPS_F = 1e-7f;

__device__ __forceinline__ int featq(int q, int h) { return 8 * (q >> 2) + 4 * h + (q & 3); }

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------------
// precision policies: k-step structure of the two MFMA forms over the accumulator feature map
// ---------------------------------------------------------------------------------------------------
template <typename T> struct MP;

template <> struct MP<bf16_t> {
  typedef bf16x8 frag;
  static constexpr int steps(int K) { return (K + 15) / 16; }
  // input feature of element e (0..7) of k-step s, lane half h
  __device__ __forceinline__ static int feat(int s, int e, int h) { return 32 * (s >> 1) + featq(8 * (s & 1) + e, h); }
  __device__ __forceinline__ static frag bop(const f32x16* a, int s) {
    const f32x16& t = a[s >> 1];
    const int o = 8 * (s & 1);
    const u32x4_t u = {pk2bf(t[o], t[o + 1]), pk2bf(t[o + 2], t[o + 3]), pk2bf(t[o + 4], t[o + 5]),
                       pk2bf(t[o + 6], t[o + 7])};
    return __builtin_bit_cast(frag, u);
  }
  template <class G> __device__ __forceinline__ static frag make(G get) {
    const u32x4_t u = {pk2bf(get(0), get(1)), pk2bf(get(2), get(3)), pk2bf(get(4), get(5)), pk2bf(get(6), get(7))};
    return __builtin_bit_cast(frag, u);
  }
};

template <> struct MP<float> {
  typedef float frag;
  // k-steps over K features: whole 32-feature tiles take 16, the last partial tile the prefix of
  // registers whose lane-half-0 feature is < K (featq(r, 0) increases with r)
  static constexpr int steps(int K) {
    int n = 16 * (K / 32);
    const int rem = K % 32;
    for (int r = 0; r < 16; ++r)
      if (rem && 8 * (r >> 2) + (r & 3) < rem) ++n;
    return n;
  }
  __device__ __forceinline__ static int feat(int s, int /*e*/, int h) { return 32 * (s >> 4) + featq(s & 15, h); }
  __device__ __forceinline__ static frag bop(const f32x16* a, int s) { return a[s >> 4][s & 15]; }
  template <class G> __device__ __forceinline__ static frag make(G get) { return get(0); }
};

template <> struct MP<f32s_t> {
  typedef F3 frag;
  static constexpr int steps(int K) { return (K + 15) / 16; }
  __device__ __forceinline__ static int feat(int s, int e, int h) { return MP<bf16_t>::feat(s, e, h); }
  __device__ __forceinline__ static frag bop(const f32x16* a, int s) {
    const f32x16& t = a[s >> 1];
    const int o = 8 * (s & 1);
    const float v[8] = {t[o], t[o + 1], t[o + 2], t[o + 3], t[o + 4], t[o + 5], t[o + 6], t[o + 7]};
    return split_f3(v);
  }
  template <class G> __device__ __forceinline__ static frag make(G get) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = get(j);
    return split_f3(v);
  }
};

// ---------------------------------------------------------------------------------------------------
// LDS images (built by the whole workgroup in the prologue)
// ---------------------------------------------------------------------------------------------------
// forward image of W (K x N, row-major fp32): entry (t, s) = A fragment rows o = 32 t .. +31, k-step s
template <typename T, int K, int N>
__device__ void build_fwd(typename MP<T>::frag* img, const float* __restrict__ W) {
  constexpr int S = MP<T>::steps(K), NT = (N + 31) / 32;
  for (int e = threadIdx.x; e < NT * S * 64; e += blockDim.x) {
    const int lane = e & 63, idx = e >> 6, t = idx / S, s = idx - t * S;
    const int o = 32 * t + (lane & 31), h = lane >> 5;
    img[e] = MP<T>::make([&](int j) {
      const int i = MP<T>::feat(s, j, h);
      return (i < K && o < N) ? W[i * N + o] : 0.f;
    });
  }
}
// dgrad image of W (K x N): entry (t, s) = A fragment rows i = 32 t .. +31 (input features), k-step s
// over the N output features
template <typename T, int K, int N>
__device__ void build_dgrad(typename MP<T>::frag* img, const float* __restrict__ W) {
  constexpr int S = MP<T>::steps(N), NT = (K + 31) / 32;
  for (int e = threadIdx.x; e < NT * S * 64; e += blockDim.x) {
    const int lane = e & 63, idx = e >> 6, t = idx / S, s = idx - t * S;
    const int i = 32 * t + (lane & 31), h = lane >> 5;
    img[e] = MP<T>::make([&](int j) {
      const int o = MP<T>::feat(s, j, h);
      return (i < K && o < N) ? W[i * N + o] : 0.f;
    });
  }
}
template <typename T, int K, int N> constexpr int fwd_entries() { return ((N + 31) / 32) * MP<T>::steps(K); }
template <typename T, int K, int N> constexpr int dgrad_entries() { return ((K + 31) / 32) * MP<T>::steps(N); }
template <typename T> constexpr int frag_bytes() { return 64 * (int)sizeof(typename MP<T>::frag); }

__device__ void load_vec(float* dst, const float* __restrict__ src, int n) {
  for (int i = threadIdx.x; i < VEC; i += blockDim.x) dst[i] = (src && i < n) ? src[i] : 0.f;
}

// ---------------------------------------------------------------------------------------------------
// register-level building blocks
// ---------------------------------------------------------------------------------------------------
// out[t] = sum over the KIN input features of img (t, s) x in: one output tile per 32 features of NOUT
// The A fragments of step s + 1 are read while step s's MFMAs issue; the scheduling barrier per step
// keeps hipcc from hoisting the whole image into registers (it did: 208 VGPRs for the fp32 100 x 100
// layer, and spills everywhere).
template <typename T, int KIN, int NOUT>
__device__ __forceinline__ void dense(const f32x16* in, f32x16* out, const typename MP<T>::frag* img, int lane) {
  constexpr int S = MP<T>::steps(KIN), NT = (NOUT + 31) / 32;
  typedef typename MP<T>::frag Fr;
  Fr cur[NT], nxt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    out[t] = zero16();
    cur[t] = img[(t * S) * 64 + lane];
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) {
#pragma unroll
      for (int t = 0; t < NT; ++t) nxt[t] = img[(t * S + s + 1) * 64 + lane];
    }
    const Fr b = MP<T>::bop(in, s);
#pragma unroll
    for (int t = 0; t < NT; ++t) out[t] = MF<T>::mma(cur[t], b, out[t]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NT; ++t) cur[t] = nxt[t];
  }
}

// 4 consecutive elements of a row (feature f0 .. f0 + 3), as floats
template <typename T> struct Q4;
template <> struct Q4<bf16_t> {
  __device__ __forceinline__ static float4 ld(const bf16_t* p) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                       __uint_as_float(v.y & 0xffff0000u));
  }
  __device__ __forceinline__ static void st(bf16_t* p, float a, float b, float c, float d) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(a, b), pk2bf(c, d));
  }
};
template <> struct Q4<float> {
  __device__ __forceinline__ static float4 ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ __forceinline__ static void st(float* p, float a, float b, float c, float d) {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
  }
};

// rows (M x K row-major) -> accumulator layout (zeros past M / K)
template <typename T, int K>
__device__ __forceinline__ void load_rows(f32x16* a, const T* __restrict__ x, int64_t row, int64_t M, int h) {
  constexpr int NT = (K + 31) / 32;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < M && f0 < K) v = Q4<T>::ld(x + row * K + f0);
      a[t][4 * g] = v.x; a[t][4 * g + 1] = v.y; a[t][4 * g + 2] = v.z; a[t][4 * g + 3] = v.w;
    }
}
template <typename T, int N>
__device__ __forceinline__ void store_rows(T* __restrict__ y, int64_t row, int64_t M, const f32x16* a, int h) {
  constexpr int NT = (N + 31) / 32;
  if (row >= M) return;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      if (f0 < N) Q4<T>::st(y + row * N + f0, a[t][4 * g], a[t][4 * g + 1], a[t][4 * g + 2], a[t][4 * g + 3]);
    }
}
// a per-row head vector (w: this row's N weights, fp32) scaled by `sc`, in accumulator layout
template <int N>
__device__ __forceinline__ void head_rows(f32x16* a, const float* __restrict__ w, float sc, bool ok, int h) {
  constexpr int NT = (N + 31) / 32;
  const float* wh = w + 4 * h;  // lane-half base: the per-(t, g) offsets below fold into immediates
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok && f0 < N) v = *reinterpret_cast<const float4*>(wh + 32 * t + 8 * g);
      a[t][4 * g] = sc * v.x; a[t][4 * g + 1] = sc * v.y; a[t][4 * g + 2] = sc * v.z; a[t][4 * g + 3] = sc * v.w;
    }
}
// sum_f a[row, f] * w[f] for this lane's row (both lane halves get the total)
template <int N>
__device__ __forceinline__ float rowdot(const f32x16* a, const float* __restrict__ w, bool ok, int h) {
  constexpr int NT = (N + 31) / 32;
  const float* wh = w + 4 * h;
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      if (ok && f0 < N) {
        const float4 v = *reinterpret_cast<const float4*>(wh + 32 * t + 8 * g);
        s = fmaf(a[t][4 * g], v.x, s); s = fmaf(a[t][4 * g + 1], v.y, s);
        s = fmaf(a[t][4 * g + 2], v.z, s); s = fmaf(a[t][4 * g + 3], v.w, s);
      }
    }
  return s + __shfl_xor(s, 32, 64);
}
// a = act(a + b) on features < N, 0 past N (b: LDS vector)
template <int N>
__device__ __forceinline__ void bias_act(f32x16* a, const float* b, int act, int h) {
  constexpr int NT = (N + 31) / 32;
  const float* bh = b + 4 * h;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      const float4 bv = *reinterpret_cast<const float4*>(bh + 32 * t + 8 * g);
      const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = a[t][4 * g + e] + bb[e];
        v = act == ACT_SIGMOID ? sigmoidf_(v) : v;
        a[t][4 * g + e] = f0 + e < N ? v : 0.f;
      }
    }
}
template <int N>
__device__ __forceinline__ void axpy(f32x16* y, float s, const f32x16* x) {
#pragma unroll
  for (int t = 0; t < (N + 31) / 32; ++t) y[t] += s * x[t];
}
__device__ __forceinline__ float lrelu(float v) { return v >= 0.f ? v : LRELU_ALPHA_F * v; }

// LeakyReLU then LayerNorm (eps 1e-3, biased variance) of this lane's row, in place; a holds the
// activation outputs with zeros past N.  Returns the row statistics.
template <int N>
__device__ __forceinline__ void lrelu_ln(f32x16* a, const float* gam, const float* bet, int h, float& mean,
                                         float& rstd) {
  constexpr int NT = (N + 31) / 32;
  const float *gh = gam + 4 * h, *beh = bet + 4 * h;
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      a[t][q] = lrelu(a[t][q]);
      s += a[t][q];
    }
  s += __shfl_xor(s, 32, 64);
  mean = s * (1.f / N);
  float v = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float d = 32 * t + featq(q, h) < N ? a[t][q] - mean : 0.f;
      v = fmaf(d, d, v);
    }
  v += __shfl_xor(v, 32, 64);
  rstd = 1.f / sqrtf(v * (1.f / N) + LN_EPS_F);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      const float4 gv = *reinterpret_cast<const float4*>(gh + 32 * t + 8 * g),
                   bv = *reinterpret_cast<const float4*>(beh + 32 * t + 8 * g);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w}, bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u = (a[t][4 * g + e] - mean) * rstd * gg[e] + bb[e];
        a[t][4 * g + e] = f0 + e < N ? u : 0.f;
      }
    }
}

// Sum over the 32 rows of one lane half of every feature of tile v (transpose-reduce butterfly: 16
// shuffles instead of 80).  Lane l ends with the column sum of register q(l) = 8 b4 + 4 b3 + 2 b2 + b1
// (bk = bit k of l), i.e. feature featq(q(l), h); lanes l and l ^ 1 hold the same value.
// The element reads go through an empty asm: otherwise InstCombine folds select(b, v[8 + i], v[i]) into
// a DYNAMIC extractelement v[b ? 8 + i : i], which the backend lowers as a 16-way v_cmp / v_cndmask
// chain per element (16 live lane masks, spilled to VGPR lanes: 100 VALU per MFMA in mlp_gen_bwd_w).
__device__ __forceinline__ float opaque(float x) {
  asm("" : "+v"(x));
  return x;
}
__device__ __forceinline__ float colsum(const f32x16& v, int lane) {
  float a8[8], a4[4], a2[2];
  bool b = lane & 16;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float lo = opaque(v[i]), hi = opaque(v[8 + i]);
    a8[i] = (b ? hi : lo) + __shfl_xor(b ? lo : hi, 16, 64);
  }
  b = lane & 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) a4[i] = (b ? a8[4 + i] : a8[i]) + __shfl_xor(b ? a8[i] : a8[4 + i], 8, 64);
  b = lane & 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) a2[i] = (b ? a4[2 + i] : a4[i]) + __shfl_xor(b ? a4[i] : a4[2 + i], 4, 64);
  b = lane & 2;
  float a1 = (b ? a2[1] : a2[0]) + __shfl_xor(b ? a2[0] : a2[1], 2, 64);
  return a1 + __shfl_xor(a1, 1, 64);
}
__device__ __forceinline__ int colsum_q(int lane) {
  return (((lane >> 4) & 1) << 3) | (((lane >> 3) & 1) << 2) | (((lane >> 2) & 1) << 1) | ((lane >> 1) & 1);
}

// per-wave partial sums -> slab row of this wave
__device__ __forceinline__ void slab_put(float* slab, int L, int k, float v) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) slab[((int64_t)blockIdx.x * MLP_WAVES + (threadIdx.x >> 6)) * L + k] = v;
}

// Keras binary cross-entropy on a probability p with label y, its p-gradient scaled by inv
// (zero where the [eps, 1 - eps] clip is active): the gan_loss kind-1 contract (ops/reference.py)
__device__ __forceinline__ void bce(float p, float y, float inv, float& lo, float& g) {
  const float o = fminf(fmaxf(p, KERAS_EPS_F), 1.f - KERAS_EPS_F);
  lo = -(y * __logf(o + KERAS_EPS_F) + (1.f - y) * __logf(1.f - o + KERAS_EPS_F));
  const bool inside = p > KERAS_EPS_F && p < 1.f - KERAS_EPS_F;
  g = inside ? -(y / (o + KERAS_EPS_F) - (1.f - y) / (1.f - o + KERAS_EPS_F)) * inv : 0.f;
}

#define MLP_LOOP                                                                                               \
  const int lane = threadIdx.x & 63, h = lane >> 5;                                                            \
  const int64_t ntile = (M + 31) / 32;                                                                         \
  for (int64_t tile = (int64_t)blockIdx.x * MLP_WAVES + (threadIdx.x >> 6); tile < ntile;                      \
       tile += (int64_t)gridDim.x * MLP_WAVES)

}  // namespace

// ===================================================================================================
// generator forward: noise -> fake (GAN/WGAN_GP.py:221-236 build_generator)
// ===================================================================================================
// P: the product policy (T, or f32s_t for fp32 storage on the split bf16 path)
template <typename T, int F, int H, typename P = T>
__global__ void __launch_bounds__(MLP_THREADS) mlp_gen_fwd_kernel(const T* __restrict__ z, MlpGen g,
                                                                  T* __restrict__ out, int64_t M) {
  using Fr = typename MP<P>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* i1 = reinterpret_cast<Fr*>(lds);
  Fr* i2 = i1 + fwd_entries<P, F, H>() * 64;
  Fr* i3 = i2 + fwd_entries<P, H, H>() * 64;
  float* vec = reinterpret_cast<float*>(i3 + fwd_entries<P, H, F>() * 64);
  build_fwd<P, F, H>(i1, g.W1);
  build_fwd<P, H, H>(i2, g.W2);
  build_fwd<P, H, F>(i3, g.W3);
  load_vec(vec + 0 * VEC, g.b1, H); load_vec(vec + 1 * VEC, g.g1, H); load_vec(vec + 2 * VEC, g.be1, H);
  load_vec(vec + 3 * VEC, g.b2, H); load_vec(vec + 4 * VEC, g.g2, H); load_vec(vec + 5 * VEC, g.be2, H);
  load_vec(vec + 6 * VEC, g.b3, F);
  __syncthreads();
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    f32x16 x[NTF], a[NTH], b[NTH];
    float mean, rstd;
    load_rows<T, F>(x, z, row, M, h);
    dense<P, F, H>(x, a, i1, lane);
    bias_act<H>(a, vec + 0 * VEC, ACT_SIGMOID, h);
    lrelu_ln<H>(a, vec + 1 * VEC, vec + 2 * VEC, h, mean, rstd);
    dense<P, H, H>(a, b, i2, lane);
    bias_act<H>(b, vec + 3 * VEC, ACT_SIGMOID, h);
    lrelu_ln<H>(b, vec + 4 * VEC, vec + 5 * VEC, h, mean, rstd);
    dense<P, H, F>(b, x, i3, lane);
    bias_act<F>(x, vec + 6 * VEC, ACT_LINEAR, h);
    store_rows<T, F>(out, row, M, x, h);
  }
}

// ===================================================================================================
// WGAN-GP critic (GAN/WGAN_GP.py:238-253): D(x) = sum_t ((x_t W1 + b1) W2 + b2) . w3_t + b3
// ===================================================================================================
// First-order GP pass: g = dD/dx at every row (for an affine critic it does not depend on x:
// dh2 = w3_t, dh1 = W2 dh2, g = W1 dh1) and its squared norm per row.
template <typename T, int F, int H>
__global__ void __launch_bounds__(MLP_THREADS) mlp_wgp_norm_kernel(MlpCritic c, float* __restrict__ gsq, int64_t M,
                                                                   int Tn) {
  using Fr = typename MP<T>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* d2 = reinterpret_cast<Fr*>(lds);
  Fr* d1 = d2 + dgrad_entries<T, H, H>() * 64;
  build_dgrad<T, H, H>(d2, c.W2);
  build_dgrad<T, F, H>(d1, c.W1);
  __syncthreads();
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    const bool ok = row < M;
    const int tr = ok ? (int)(row % Tn) : 0;
    f32x16 a[NTH], b[NTH], gg[NTF];
    head_rows<H>(a, c.w3 + (int64_t)tr * H, 1.f, ok, h);
    dense<T, H, H>(a, b, d2, lane);
    dense<T, H, F>(b, gg, d1, lane);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NTF; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) s = fmaf(gg[t][q], gg[t][q], s);
    s += __shfl_xor(s, 32, 64);
    if (ok && h == 0) gsq[row] = s;
  }
}

// per sample: |g_b| from the T row norms, c_b = -(2 lam / B)(1 - |g_b|) / |g_b| (the gp_coef adjoint,
// ops/reference.py); epart[block] = sum over the block's samples of (1 - |g_b|)^2 (fixed order)
__global__ void __launch_bounds__(256) mlp_wgp_coef_kernel(const float* __restrict__ gsq, int Tn, int64_t B, float lam,
                                                           float* __restrict__ c, float* __restrict__ epart) {
  __shared__ float red[4];
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float e = 0.f;
  if (b < B) {
    float s = 0.f;
    for (int t = 0; t < Tn; ++t) s += gsq[b * Tn + t];
    const float n = sqrtf(s);
    c[b] = -(2.f * lam / (float)B) * (1.f - n) / fmaxf(n, 1e-30f);
    e = (1.f - n) * (1.f - n);
  }
  e = wave_sum(e);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) epart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// One GP critic update's device work per row (b, t):
//   W terms: dL/ds_b = -1/B (real), +1/B (fake)  ->  dh2 = +-w3_t / B, dh1 = +-W2 w3_t / B
//   GP term (reverse over the tangent along v = c_b g): zd1 = v W1, zd2 = zd1 W2; seeds dzd2 = w3_t,
//   dzd1 = W2 w3_t
// Every adjoint of layer 2 is along w3_t and every adjoint of layer 1 along dh1' = W2 w3_t, so each
// weight needs one product with a per-row combined operand:
//   gW2 += X2c^T dY2,  X2c = (h1_fake - h1_real) / B + zd1,  dY2 = w3_t
//   gW1 += X1c^T dY1,  X1c = (x_fake - x_real) / B + v,      dY1 = dh1' = W2 w3_t
//   gw3_t += sum_b Y3c,  Y3c = (h2_fake - h2_real) / B + zd2 = X2c W2   (the b2 terms cancel)
// The bias gradients cancel exactly (-1/B and +1/B per row pair; the tangent has none).  slab: per-wave
// sums of h2 . w3_t over the real and the fake rows (the two W losses).
template <typename T, int F, int H>
__global__ void __launch_bounds__(MLP_THREADS) mlp_wgp_critic_kernel(
    const T* __restrict__ real, const T* __restrict__ fake, const float* __restrict__ cvec, MlpCritic c,
    T* __restrict__ X2c, T* __restrict__ dY2, T* __restrict__ X1c, T* __restrict__ dY1, T* __restrict__ Y3c,
    float* __restrict__ slab, int64_t M, int Tn, float invB) {
  using Fr = typename MP<T>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d2 = f2 + fwd_entries<T, H, H>() * 64;
  Fr* d1 = d2 + dgrad_entries<T, H, H>() * 64;
  float* vec = reinterpret_cast<float*>(d1 + dgrad_entries<T, F, H>() * 64);
  build_fwd<T, F, H>(f1, c.W1);
  build_fwd<T, H, H>(f2, c.W2);
  build_dgrad<T, H, H>(d2, c.W2);
  build_dgrad<T, F, H>(d1, c.W1);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  __syncthreads();
  float sr = 0.f, sf = 0.f;
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    const bool ok = row < M;
    const int64_t bidx = ok ? row / Tn : 0;
    const float* w3t = c.w3 + (int64_t)(ok ? row - bidx * Tn : 0) * H;
    f32x16 A[NTH], Bv[NTH], X2[NTH], X1[NTF], x[NTF];
    // ---- GP tangent stream
    head_rows<H>(A, w3t, 1.f, ok, h);
    store_rows<T, H>(dY2, row, M, A, h);
    dense<T, H, H>(A, Bv, d2, lane);           // dh1' = W2 w3_t
    store_rows<T, H>(dY1, row, M, Bv, h);
    dense<T, H, F>(Bv, X1, d1, lane);          // g = W1 dh1'
    const float cb = ok ? cvec[bidx] : 0.f;
#pragma unroll
    for (int t = 0; t < NTF; ++t) X1[t] *= cb;  // v
    dense<T, F, H>(X1, X2, f1, lane);          // zd1 = v W1
    // ---- W terms: real (-1/B) then fake (+1/B)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const float sg = pass ? invB : -invB;
      load_rows<T, F>(x, pass ? fake : real, row, M, h);
      axpy<F>(X1, sg, x);
      dense<T, F, H>(x, A, f1, lane);
      bias_act<H>(A, vec, ACT_LINEAR, h);      // h1
      axpy<H>(X2, sg, A);
      dense<T, H, H>(A, Bv, f2, lane);
      bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);  // h2
      const float sc = rowdot<H>(Bv, w3t, ok, h);
      if (ok && h == 0) {
        if (pass) sf += sc;
        else sr += sc;
      }
    }
    store_rows<T, F>(X1c, row, M, X1, h);
    store_rows<T, H>(X2c, row, M, X2, h);
    dense<T, H, H>(X2, A, f2, lane);           // Y3c = X2c W2
    store_rows<T, H>(Y3c, row, M, A, h);
  }
  slab_put(slab, 2, 0, sr);
  slab_put(slab, 2, 1, sf);
}

// ---------------------------------------------------------------------------------------------------
// The same critic update with the weight gradients taken in the kernel by per-t column sums (any dtype;
// the fp32 path, whose weight images leave no LDS for mlp_wgp_critic_w's staging).
//
// Rows are walked t-major: wave wid owns t = wid % Tn and takes 32-SAMPLE tiles (rows b T + t,
// b = 32 bt + lane) of that t only.  Every adjoint of such a tile lies along the same vectors (w3_t
// for layer 2, dh1'_t = W2 w3_t for layer 1), so
//   gW2 = sum_t S2[t] (x) w3_t,  gW1 = sum_t S1[t] (x) dh1'_t,  gw3_t = S3[t],
//   S1[t] = sum_b X1c[b, t],  S2[t] = sum_b X2c[b, t],  S3[t] = sum_b Y3c[b, t]
// (X1c, X2c, Y3c the per-row operands of mlp_wgp_critic, computed here in registers as there).  Each
// tile adds its transpose-reduce column sums to ~10 per-lane registers; a wave writes one slab row
// [S1 F | S2 H | S3 H] for its t at the end, and mlp_wgp_tsum_finish reduces the rows of each t in a
// fixed order and forms the outer products.  No per-row operand leaves the kernel.
// ---------------------------------------------------------------------------------------------------
template <typename T, int F, int H>
__global__ void __launch_bounds__(MLP_THREADS) mlp_wgp_critic_t_kernel(
    const T* __restrict__ real, const T* __restrict__ fake, const float* __restrict__ cvec, MlpCritic c,
    float* __restrict__ tslab, float* __restrict__ slab, int64_t Bn, int Tn, int kper, float invB) {
  using Fr = typename MP<T>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d2 = f2 + fwd_entries<T, H, H>() * 64;
  Fr* d1 = d2 + dgrad_entries<T, H, H>() * 64;
  float* vec = reinterpret_cast<float*>(d1 + dgrad_entries<T, F, H>() * 64);
  build_fwd<T, F, H>(f1, c.W1);
  build_fwd<T, H, H>(f2, c.W2);
  build_dgrad<T, H, H>(d2, c.W2);
  build_dgrad<T, F, H>(d1, c.W1);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wid = blockIdx.x * MLP_WAVES + (threadIdx.x >> 6);
  const int tt = wid % Tn, j = wid / Tn;  // this wave's t and its index among the kper waves of that t
  const float* w3t = c.w3 + (int64_t)tt * H;
  float s1[NTF], s2[NTH], s3[NTH];
#pragma unroll
  for (int i = 0; i < NTF; ++i) s1[i] = 0.f;
#pragma unroll
  for (int i = 0; i < NTH; ++i) s2[i] = s3[i] = 0.f;
  float sr = 0.f, sf = 0.f;
  const int64_t nbt = (Bn + 31) / 32;
  for (int64_t bt = j; j < kper && bt < nbt; bt += kper) {
    const int64_t b = bt * 32 + (lane & 31);
    const bool ok = b < Bn;
    const int64_t row = ok ? b * Tn + tt : 0;
    const int64_t M = ok ? row + 1 : 0;  // load_rows' bound: the lane's own row only
    f32x16 A[NTH], Bv[NTH], X2[NTH], X1[NTF], x[NTF];
    head_rows<H>(A, w3t, 1.f, true, h);
    dense<T, H, H>(A, Bv, d2, lane);            // dh1' = W2 w3_t
    dense<T, H, F>(Bv, X1, d1, lane);           // g = W1 dh1'
    const float cb = ok ? cvec[b] : 0.f;
#pragma unroll
    for (int i = 0; i < NTF; ++i) X1[i] *= cb;  // v
    dense<T, F, H>(X1, X2, f1, lane);           // zd1 = v W1
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const float sg = pass ? invB : -invB;
      load_rows<T, F>(x, pass ? fake : real, row, M, h);
      axpy<F>(X1, sg, x);
      dense<T, F, H>(x, A, f1, lane);
      bias_act<H>(A, vec, ACT_LINEAR, h);       // h1
      axpy<H>(X2, sg, A);
      dense<T, H, H>(A, Bv, f2, lane);
      bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);  // h2
      const float sc = rowdot<H>(Bv, w3t, ok, h);
      if (ok && h == 0) {
        if (pass) sf += sc;
        else sr += sc;
      }
    }
    if (!ok) {  // samples past B contribute nothing
#pragma unroll
      for (int i = 0; i < NTH; ++i) X2[i] = zero16();
#pragma unroll
      for (int i = 0; i < NTF; ++i) X1[i] = zero16();
    }
    dense<T, H, H>(X2, A, f2, lane);            // Y3c = X2c W2
#pragma unroll
    for (int i = 0; i < NTF; ++i) s1[i] += colsum(X1[i], lane);
#pragma unroll
    for (int i = 0; i < NTH; ++i) {
      s2[i] += colsum(X2[i], lane);
      s3[i] += colsum(A[i], lane);
    }
  }
  // this wave's per-t partial sums (lanes l, l ^ 1 hold the same column): row wid of tslab
  constexpr int L = F + 2 * H;
  float* out = tslab + (int64_t)wid * L;
  const int fq = featq(colsum_q(lane), h);
  if ((lane & 1) == 0) {
#pragma unroll
    for (int i = 0; i < NTF; ++i)
      if (32 * i + fq < F) out[32 * i + fq] = s1[i];
#pragma unroll
    for (int i = 0; i < NTH; ++i)
      if (32 * i + fq < H) {
        out[F + 32 * i + fq] = s2[i];
        out[F + H + 32 * i + fq] = s3[i];
      }
  }
  slab_put(slab, 2, 0, sr);
  slab_put(slab, 2, 1, sf);
}

// (1) S[t][col] = the fixed-order sum of the kper slab rows of t (rows wid = t + Tn j), and
// D[t][o] = dh1'_t[o] = sum_k W2[o][k] w3_t[k]: tsum = [Tn][L = F + 2 H] then [Tn][H]
__global__ void __launch_bounds__(256) mlp_wgp_tsum_prep_kernel(const float* __restrict__ tslab, MlpCritic c, int F,
                                                                int H, int Tn, int kper, float* __restrict__ tsum) {
  const int L = F + 2 * H;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < Tn * L) {
    const int t = e / L, col = e - t * L;
    float a = 0.f;
    for (int jj = 0; jj < kper; ++jj) a += tslab[(int64_t)(t + Tn * jj) * L + col];
    tsum[e] = a;
  } else if (e < Tn * L + Tn * H) {
    const int q = e - Tn * L, t = q / H, o = q - t * H;
    float d = 0.f;
    for (int k = 0; k < H; ++k) d = fmaf(c.W2[o * H + k], c.w3[t * H + k], d);
    tsum[e] = d;
  }
}
// (2) gW1 += sum_t S1[t] (x) D[t], gW2 += sum_t S2[t] (x) w3_t, gw3_t += S3[t]: one output per thread
__global__ void __launch_bounds__(256) mlp_wgp_tsum_finish_kernel(const float* __restrict__ tsum, MlpCritic c, int F,
                                                                  int H, int Tn, float* __restrict__ gW1,
                                                                  float* __restrict__ gW2, float* __restrict__ gw3) {
  const int L = F + 2 * H;
  const float* D = tsum + Tn * L;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int n1 = F * H, n2 = H * H, n3 = Tn * H;
  if (e < n1) {
    const int i = e / H, o = e - i * H;
    float acc = 0.f;
    for (int t = 0; t < Tn; ++t) acc = fmaf(tsum[t * L + i], D[t * H + o], acc);
    gW1[e] += acc;
  } else if (e < n1 + n2) {
    const int q = e - n1, i = q / H, o = q - i * H;
    float acc = 0.f;
    for (int t = 0; t < Tn; ++t) acc = fmaf(tsum[t * L + F + i], c.w3[t * H + o], acc);
    gW2[q] += acc;
  } else if (e < n1 + n2 + n3) {
    const int q = e - n1 - n2, t = q / H, o = q - t * H;
    gw3[q] += tsum[t * L + F + H + o];
  }
}

// ---------------------------------------------------------------------------------------------------
// The affine critic's update from batch sums (mlp_wgp_affine, default; GAN/WGAN_GP.py:238-253, loop
// :255-288).  D(x) = sum_t ((x_t W1 + b1) W2 + b2) . w3_t + b3 is affine in x, so
//   * its input gradient g_t = W1 W2 w3_t is a function of t alone: every sample has the same |g|, the
//     same GP coefficient c = -(2 lam / B)(1 - |g|) / |g| and the same tangent v_t = c g_t;
//   * the per-row operands of mlp_wgp_critic_t enter the gradients only through their sums over the
//     batch, and those are linear in the per-t sums of the inputs (sum_b (x_b W) = (sum_b x_b) W):
//       S1[t] = d_t / B + B v_t,  d_t = sum_b (fake - real)[b, t]
//       S2[t] = S1[t] W1                       (= (d_t W1) / B + B v_t W1: b1 cancels in d)
//       S3[t] = S2[t] W2
//     and the W-loss score sums are sum_t (s_t W1 + B b1) . (W2 w3_t) + B b2 . w3_t.
// So the update reads each input once (mlp_bt_colsum: per-t column sums, HBM-bound) and finishes in
// fp32 in one workgroup; mlp_wgp_tsum_finish forms the T outer products as for mlp_wgp_critic_t.  Same
// gradient and loss pack as the per-row path up to fp32 summation order (and without its bf16 rounding
// of h1 / h2 in the bf16 build).  mode 1 is the generator step's critic input gradient: the per-t
// dfake row -g_t / B (broadcast over the batch by mlp_bcast_rows) and the fake score sum.
// ---------------------------------------------------------------------------------------------------

// part[p][k][col] = sum over rows r = p, p + P, ... < B of y_k[r][col]; y_0 = x0, y_1 = x1 - x0 (the
// difference is formed per row: no cancellation between two large sums).  col < C = T F, 16-byte
// vectors; thread (p, column group) walks its rows with independent loads in flight.
template <typename T>
__global__ void __launch_bounds__(256) mlp_bt_colsum_kernel(const T* __restrict__ x0, const T* __restrict__ x1,
                                                            int64_t B, int C, int P, float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  const int G = C / V;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)G * P) return;
  const int cg = (int)(gid % G), p = (int)(gid / G);
  float a0[V], a1[V];
#pragma unroll
  for (int j = 0; j < V; ++j) a0[j] = a1[j] = 0.f;
  auto unpack = [](const uint4& u, float* f) {
    if constexpr (sizeof(T) == 4) {
      f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y); f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
    } else {
      const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[2 * j] = __uint_as_float(w4[j] << 16);
        f[2 * j + 1] = __uint_as_float(w4[j] & 0xFFFF0000u);
      }
    }
  };
  const int64_t c0 = (int64_t)cg * V;
#pragma unroll 4
  for (int64_t r = p; r < B; r += P) {
    const uint4 u0 = *reinterpret_cast<const uint4*>(x0 + r * C + c0);
    float f0[V];
    unpack(u0, f0);
    if (x1) {
      const uint4 u1 = *reinterpret_cast<const uint4*>(x1 + r * C + c0);
      float f1[V];
      unpack(u1, f1);
#pragma unroll
      for (int j = 0; j < V; ++j) a1[j] += f1[j] - f0[j];
    }
#pragma unroll
    for (int j = 0; j < V; ++j) a0[j] += f0[j];
  }
  const int nk = x1 ? 2 : 1;
  float* o = part + (int64_t)p * nk * C + c0;
#pragma unroll
  for (int j = 0; j < V; j += 4) *reinterpret_cast<f32x4*>(o + j) = f32x4{a0[j], a0[j + 1], a0[j + 2], a0[j + 3]};
  if (x1) {
#pragma unroll
    for (int j = 0; j < V; j += 4)
      *reinterpret_cast<f32x4*>(o + C + j) = f32x4{a1[j], a1[j + 1], a1[j + 2], a1[j + 3]};
  }
}

// One workgroup (1024 threads).  sums: [nk][Tn][F] from mlp_bt_colsum (mode 0: k = 0 real, 1 fake - real;
// mode 1: k = 0 fake).  W1, W2 (row pitch AFP = 101: odd, so the strided reads are bank-conflict free),
// w3 and the per-t tables live in LDS (mlp_affine_lds_bytes; Tn <= mlp_affine_max_t).  D = the (Tn, H)
// table W2 w3_t (also written to the D block of tsum in mode 0).  Mode 0 writes tsum's S1 / S2 / S3 rows,
// slab[0..1] = the real / fake score sums (without b3) and e[0] = B (1 - |g|)^2 (the penalty's sum over
// samples); mode 1 writes gdx = -g / B and slab = {fake score sum, 0}.
constexpr int AFP = 101;
__host__ __device__ constexpr size_t mlp_affine_lds_floats(int F, int H, int Tn) {
  return (size_t)F * AFP + (size_t)H * AFP + (size_t)Tn * (3 * H + F);
}
__global__ void __launch_bounds__(1024) mlp_wgp_affine_kernel(const float* __restrict__ sums, MlpCritic c, int F, int H,
                                                             int Tn, float Bf, float lam, int mode, float* __restrict__ Dg,
                                                             float* __restrict__ tsum, float* __restrict__ slab,
                                                             float* __restrict__ e, float* __restrict__ gdx) {
  extern __shared__ __attribute__((aligned(16))) float als[];
  __shared__ float red[16];
  float* W1 = als;                    // [F][AFP]
  float* W2 = W1 + F * AFP;           // [H][AFP]
  float* w3 = W2 + H * AFP;           // [Tn][H]
  float* D = w3 + Tn * H;             // [Tn][H]
  float* S2 = D + Tn * H;             // [Tn][H]
  float* g = S2 + Tn * H;             // [Tn][F]
  const int tid = threadIdx.x, NT = blockDim.x, L = F + 2 * H;
  for (int q = tid; q < F * H; q += NT) W1[(q / H) * AFP + q % H] = c.W1[q];
  for (int q = tid; q < H * H; q += NT) W2[(q / H) * AFP + q % H] = c.W2[q];
  for (int q = tid; q < Tn * H; q += NT) w3[q] = c.w3[q];
  __syncthreads();
  const float* s0 = sums;           // mode 0: real, mode 1: fake
  const float* sd = sums + Tn * F;  // mode 0: fake - real
  // (A) D[t][o] = sum_k W2[o][k] w3_t[k]
  for (int q = tid; q < Tn * H; q += NT) {
    const int t = q / H, o = q - t * H;
    float d = 0.f;
    for (int k = 0; k < H; ++k) d = fmaf(W2[o * AFP + k], w3[t * H + k], d);
    D[q] = d;
    if (Dg) Dg[q] = d;
  }
  __syncthreads();
  // (B) g[t][i] = sum_o W1[i][o] D[t][o] and |g|^2
  float gs = 0.f;
  for (int q = tid; q < Tn * F; q += NT) {
    const int t = q / F, i = q - t * F;
    float a = 0.f;
    for (int o = 0; o < H; ++o) a = fmaf(W1[i * AFP + o], D[t * H + o], a);
    g[q] = a;
    gs = fmaf(a, a, gs);
    if (mode == 1) gdx[q] = a * (-1.f / Bf);
  }
  const float gsq = block_sum<16>(gs, red);  // (barriers inside: g complete)
  const float n = sqrtf(gsq);
  const float cc = -(2.f * lam / Bf) * (1.f - n) / fmaxf(n, 1e-30f);
  // (C) S1, S2 and the score sums
  float scr = 0.f, scf = 0.f;
  for (int q = tid; q < Tn * H; q += NT) {
    const int t = q / H, o = q - t * H;
    float z = 0.f, dw = 0.f, h0 = 0.f;
    for (int i = 0; i < F; ++i) {
      const float wv = W1[i * AFP + o];
      h0 = fmaf(s0[t * F + i], wv, h0);
      if (mode == 0) {
        z = fmaf(g[t * F + i], wv, z);
        dw = fmaf(sd[t * F + i], wv, dw);
      }
    }
    const float hb = Bf * c.b1[o], tb = Bf * c.b2[o] * w3[q];
    scr += fmaf(h0 + hb, D[q], tb);
    if (mode == 0) {
      const float s2 = dw / Bf + Bf * (cc * z);
      S2[q] = s2;
      tsum[t * L + F + o] = s2;
      scf += fmaf(h0 + dw + hb, D[q], tb);
    }
  }
  if (mode == 0)
    for (int q = tid; q < Tn * F; q += NT) {
      const int t = q / F, i = q - t * F;
      tsum[t * L + i] = sd[q] / Bf + Bf * (cc * g[q]);
    }
  const float sr = block_sum<16>(scr, red);  // (barriers inside: S2 complete)
  const float sf = block_sum<16>(scf, red);
  if (tid == 0) {
    slab[0] = sr;
    slab[1] = mode == 0 ? sf : 0.f;
    if (mode == 0) e[0] = Bf * (1.f - n) * (1.f - n);
  }
  if (mode != 0) return;
  // (D) S3[t][k] = sum_o S2[t][o] W2[o][k]
  for (int q = tid; q < Tn * H; q += NT) {
    const int t = q / H, k = q - t * H;
    float a = 0.f;
    for (int o = 0; o < H; ++o) a = fmaf(S2[t * H + o], W2[o * AFP + k], a);
    tsum[t * L + F + H + k] = a;
  }
}

// out[b][col] = row[col] for every b < B (C = T F columns): thread (p, column group) packs its 16 bytes
// once and stores them to rows p, p + P, ...
template <typename T>
__global__ void __launch_bounds__(256) mlp_bcast_rows_kernel(const float* __restrict__ row, int C, int64_t B, int P,
                                                             T* __restrict__ out) {
  constexpr int V = 16 / (int)sizeof(T);
  const int G = C / V;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)G * P) return;
  const int cg = (int)(gid % G), p = (int)(gid / G), col = cg * V;
  uint4 u;
  if constexpr (sizeof(T) == 4) {
    u = make_uint4(__float_as_uint(row[col]), __float_as_uint(row[col + 1]), __float_as_uint(row[col + 2]),
                   __float_as_uint(row[col + 3]));
  } else {
    u = make_uint4(pk2bf(row[col], row[col + 1]), pk2bf(row[col + 2], row[col + 3]), pk2bf(row[col + 4], row[col + 5]),
                   pk2bf(row[col + 6], row[col + 7]));
  }
#pragma unroll 4
  for (int64_t r = p; r < B; r += P) *reinterpret_cast<uint4*>(out + r * C + col) = u;
}

// ---------------------------------------------------------------------------------------------------
// The same critic update with the three weight gradients accumulated in the kernel (bf16).
//
// mlp_wgp_critic writes 5 per-row operands (872 B a row at F = 36) that linear_wgrad_ reads back:
// ~11 GB of HBM traffic per update at B*T = 6.3 M rows.  Here the 4 waves of a workgroup walk 128-row
// block tiles together.  After the per-row chain (unchanged) each wave stages its 32 rows of X2c, X1c and
// Y3c in LDS, TRANSPOSED (feature-major [f][row], bf16, pitch WQ), and the block's 128 rows become the
// k dimension of three small GEMMs on v_mfma_f32_32x32x16_bf16, wave w owning output columns
// o = 32 w .. 32 w + 31:
//   gW2[i][o] += sum_r X2c[r][i] w3_{t(r)}[o]     A: one ds_read_b128 of img2 row i, B: gathered from
//   gW1[i][o] += sum_r X1c[r][i] dh1'_{t(r)}[o]        the per-t tables (w3_t and dh1'_t = W2 w3_t are
//   gw3[t][o] += sum_r [t(r) = t] Y3c[r][o]             functions of t only: built once per workgroup)
// (A: the one-hot of t(r), built in registers; B: one ds_read_b128 of img3 row o.)  The 8-row runs the
// fragments need are contiguous in the transposed images, so every MFMA operand is one 16-byte read;
// WQ = 136 bf16 makes those reads conflict-free (272 B row stride = 68 dwords: 16 lanes hit 16 distinct
// 4-bank groups).  The per-workgroup partial gradients go to one fp32 slab row per workgroup, summed in
// a fixed order by mlp_slab_sum.  Two barriers per block tile: before the staging writes (the previous
// tile's readers are done) and before the reads.
// ---------------------------------------------------------------------------------------------------
constexpr int WQ = 136;  // pitch (bf16) of a transposed staging row: 128 rows + 8

template <int F, int H> constexpr size_t wgpw_images() {
  return (size_t)(fwd_entries<bf16_t, F, H>() + fwd_entries<bf16_t, H, H>() + dgrad_entries<bf16_t, H, H>() +
                  dgrad_entries<bf16_t, F, H>()) *
             frag_bytes<bf16_t>() +
         2 * VEC * 4;
}
// byte offsets: [images][img2: H x WQ][img3: H x WQ][img1: F x WQ][toff: 128 ints][w3 table][dh1' table]
template <int F, int H> constexpr size_t wgpw_off_img2() { return wgpw_images<F, H>(); }
template <int F, int H> constexpr size_t wgpw_off_img3() { return wgpw_off_img2<F, H>() + (size_t)H * WQ * 2; }
template <int F, int H> constexpr size_t wgpw_off_img1() { return wgpw_off_img3<F, H>() + (size_t)H * WQ * 2; }
template <int F, int H> constexpr size_t wgpw_off_toff() { return wgpw_off_img1<F, H>() + (size_t)F * WQ * 2; }
template <int F, int H> constexpr size_t wgpw_off_tab() { return wgpw_off_toff<F, H>() + 128 * 4; }
// tables: w3_t fp32 [Tn][128] (head_rows / rowdot / the gW2 gathers), then dh1'_t bf16 [Tn][128]
template <int F, int H> constexpr size_t wgpw_lds(int Tn) { return wgpw_off_tab<F, H>() + (size_t)Tn * 128 * (4 + 2); }
static_assert(wgpw_off_img3<36, 100>() % 16 == 0 && wgpw_off_toff<36, 100>() % 16 == 0, "16-byte aligned images");
static_assert(wgpw_off_img3<32, 100>() % 16 == 0 && wgpw_off_toff<32, 100>() % 16 == 0, "16-byte aligned images");

__device__ __forceinline__ float dpp_xor1(float v) {
  // quad_perm [1, 0, 3, 2]: the value of lane ^ 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
// this lane's row rr (block-local, 0..127) of accumulator tiles a -> img[f][rr] for f < N.  The
// (even, odd) row pair of a feature is one dword: both lanes of the pair write it (same address, same
// value; the odd lane's halves are rotated into place by one v_alignbit), so there is no per-store
// exec mask.  Feature validity is compile-time except the last tile's features fb .. fb + 3 < N <=
// fb + 7, which only lane half 0 holds (one masked group).
template <int N>
__device__ __forceinline__ void stage_t(unsigned short* img, const f32x16* a, int rr, int h) {
  constexpr int NT = (N + 31) / 32, REM = N - 32 * (NT - 1);
  unsigned short* base = img + (rr & ~1) + 4 * h * WQ;
  const uint32_t rot = (rr & 1) * 16;
  uint32_t part[4];
  int pf[4], np = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int fb = 8 * (q >> 2) + (q & 3);  // feature (in the tile) of this register in lane half 0
      if (t == NT - 1 && fb >= REM) continue;
      const float v = a[t][q];
      const float p = dpp_xor1(v);
      const uint32_t w0 = pk2bf(v, p);
      const uint32_t w = __builtin_amdgcn_alignbit(w0, w0, rot);
      if (t < NT - 1 || fb + 4 < REM) {
        *reinterpret_cast<uint32_t*>(base + (32 * t + fb) * WQ) = w;
      } else {
        pf[np & 3] = fb;  // at most 4 such features (REM - 4 .. REM - 1)
        part[np++ & 3] = w;
      }
    }
  if (np && h == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < np) *reinterpret_cast<uint32_t*>(base + (32 * (NT - 1) + pf[q]) * WQ) = part[q];
  }
}
// a per-t table row (bf16, 128 features) from accumulator tiles; zeros past N come from a
template <int N>
__device__ __forceinline__ void table_put(unsigned short* row, const f32x16* a, int h) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      const float4 v = t < (N + 31) / 32 ? make_float4(a[t][4 * g], a[t][4 * g + 1], a[t][4 * g + 2], a[t][4 * g + 3])
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<uint2*>(row + f0) = make_uint2(pk2bf(v.x, v.y), pk2bf(v.z, v.w));
    }
}
// B fragment gathered from a per-t table: element j = tab[ofs[j] + col]
__device__ __forceinline__ bf16x8 gather8(const unsigned short* tab, const int* ofs, int col) {
  u32x4_t u;
#pragma unroll
  for (int e = 0; e < 4; ++e) u[e] = (uint32_t)tab[ofs[2 * e] + col] | ((uint32_t)tab[ofs[2 * e + 1] + col] << 16);
  return __builtin_bit_cast(bf16x8, u);
}
__device__ __forceinline__ bf16x8 gather8(const float* tab, const int* ofs, int col) {
  u32x4_t u;
#pragma unroll
  for (int e = 0; e < 4; ++e) u[e] = pk2bf(tab[ofs[2 * e] + col], tab[ofs[2 * e + 1] + col]);
  return __builtin_bit_cast(bf16x8, u);
}
// raw bf16 rows (4 features per (tile, g) as one uint2), loaded ahead of their use
template <int K> struct RawRows {
  uint2 v[(K + 31) / 32 * 4];
};
template <int K>
__device__ __forceinline__ void load_raw(RawRows<K>& r, const bf16_t* __restrict__ x, int64_t row, int64_t M, int h) {
#pragma unroll
  for (int t = 0; t < (K + 31) / 32; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * t + 8 * g + 4 * h;
      r.v[4 * t + g] = (row < M && f0 < K) ? *reinterpret_cast<const uint2*>(x + row * K + f0) : make_uint2(0u, 0u);
    }
}
template <int K>
__device__ __forceinline__ void raw_to_acc(f32x16* a, const RawRows<K>& r) {
#pragma unroll
  for (int t = 0; t < (K + 31) / 32; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint2 v = r.v[4 * t + g];
      a[t][4 * g] = __uint_as_float(v.x << 16);
      a[t][4 * g + 1] = __uint_as_float(v.x & 0xffff0000u);
      a[t][4 * g + 2] = __uint_as_float(v.y << 16);
      a[t][4 * g + 3] = __uint_as_float(v.y & 0xffff0000u);
    }
}

template <int F, int H, int NTT>
__global__ void __launch_bounds__(MLP_THREADS) mlp_wgp_critic_w_kernel(
    const bf16_t* __restrict__ real, const bf16_t* __restrict__ fake, const float* __restrict__ cvec, MlpCritic c,
    float* __restrict__ gslab, float* __restrict__ slab, int64_t M, int Tn, float invB) {
  using T = bf16_t;
  using Fr = bf16x8;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d2 = f2 + fwd_entries<T, H, H>() * 64;
  Fr* d1 = d2 + dgrad_entries<T, H, H>() * 64;
  float* vec = reinterpret_cast<float*>(d1 + dgrad_entries<T, F, H>() * 64);
  unsigned short* img2 = reinterpret_cast<unsigned short*>(lds + wgpw_off_img2<F, H>());
  unsigned short* img3 = reinterpret_cast<unsigned short*>(lds + wgpw_off_img3<F, H>());
  unsigned short* img1 = reinterpret_cast<unsigned short*>(lds + wgpw_off_img1<F, H>());
  int* toff = reinterpret_cast<int*>(lds + wgpw_off_toff<F, H>());
  float* tabw = reinterpret_cast<float*>(lds + wgpw_off_tab<F, H>());
  unsigned short* tabd = reinterpret_cast<unsigned short*>(tabw + Tn * 128);
  build_fwd<T, F, H>(f1, c.W1);
  build_fwd<T, H, H>(f2, c.W2);
  build_dgrad<T, H, H>(d2, c.W2);
  build_dgrad<T, F, H>(d1, c.W1);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  for (int e = threadIdx.x; e < Tn * 128; e += blockDim.x) {  // w3_t, fp32, 128 wide (zeros past H)
    const int t = e >> 7, o = e & 127;
    tabw[e] = o < H ? c.w3[t * H + o] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, w = threadIdx.x >> 6, cl = lane & 31;
  // dh1' table: wave w < NTT computes t = 32 w + lane (the chain's own head_rows / dense, so the table
  // holds exactly the bf16 values the operand path stored per row)
  if (w < NTT) {
    const int t = 32 * w + cl;
    const bool ok = t < Tn;
    f32x16 A[NTH], Bv[NTH];
    head_rows<H>(A, tabw + (ok ? t : 0) * 128, 1.f, ok, h);
    dense<T, H, H>(A, Bv, d2, lane);
    if (ok) table_put<H>(tabd + t * 128, Bv, h);
  }
  f32x16 gW2[NTH], gW1[NTF], gw3[NTT];
#pragma unroll
  for (int i = 0; i < NTH; ++i) gW2[i] = zero16();
#pragma unroll
  for (int i = 0; i < NTF; ++i) gW1[i] = zero16();
#pragma unroll
  for (int i = 0; i < NTT; ++i) gw3[i] = zero16();
  float sr = 0.f, sf = 0.f;
  const int rr = 32 * w + cl;  // this lane's block-local row
  const int64_t nbt = (M + 127) / 128;
  for (int64_t bt = blockIdx.x; bt < nbt; bt += gridDim.x) {
    const int64_t row = bt * 128 + rr;
    const bool ok = row < M;
    const int64_t bidx = ok ? row / Tn : 0;
    const int tr = ok ? (int)(row - bidx * Tn) : 0;
    const float* w3t = tabw + tr * 128;
    RawRows<F> xr, xf;  // this tile's windows, loaded first: the head chain below hides their latency
    load_raw<F>(xr, real, row, M, h);
    load_raw<F>(xf, fake, row, M, h);
    f32x16 A[NTH], Bv[NTH], X2[NTH], X1[NTF], x[NTF];
    head_rows<H>(A, w3t, 1.f, ok, h);
    dense<T, H, H>(A, Bv, d2, lane);            // dh1' = W2 w3_t
    dense<T, H, F>(Bv, X1, d1, lane);           // g = W1 dh1'
    const float cb = ok ? cvec[bidx] : 0.f;
#pragma unroll
    for (int t = 0; t < NTF; ++t) X1[t] *= cb;  // v
    dense<T, F, H>(X1, X2, f1, lane);           // zd1 = v W1
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const float sg = pass ? invB : -invB;
      raw_to_acc<F>(x, pass ? xf : xr);
      axpy<F>(X1, sg, x);
      dense<T, F, H>(x, A, f1, lane);
      bias_act<H>(A, vec, ACT_LINEAR, h);       // h1
      axpy<H>(X2, sg, A);
      dense<T, H, H>(A, Bv, f2, lane);
      bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);  // h2
      const float sc = rowdot<H>(Bv, w3t, ok, h);
      if (ok && h == 0) {
        if (pass) sf += sc;
        else sr += sc;
      }
    }
    // rows past M contribute nothing (their operands are exactly what the zero inputs give, up to an
    // fma residue of b1 / B - b1 / B: zeroed explicitly)
    if (!ok) {
#pragma unroll
      for (int t = 0; t < NTH; ++t) X2[t] = zero16();
#pragma unroll
      for (int t = 0; t < NTF; ++t) X1[t] = zero16();
    }
    dense<T, H, H>(X2, A, f2, lane);            // Y3c = X2c W2
    __syncthreads();  // the previous block tile's wgrad reads are done
    stage_t<H>(img2, X2, rr, h);
    stage_t<H>(img3, A, rr, h);
    stage_t<F>(img1, X1, rr, h);
    if (h == 0) toff[rr] = tr * 128;
    __syncthreads();
#pragma unroll 2
    for (int ks = 0; ks < 8; ++ks) {
      const int r0 = 16 * ks + 8 * h;
      const int4 oa = *reinterpret_cast<const int4*>(toff + r0), ob = *reinterpret_cast<const int4*>(toff + r0 + 4);
      const int ofs[8] = {oa.x, oa.y, oa.z, oa.w, ob.x, ob.y, ob.z, ob.w};
      const int col = 32 * w + cl;
      const Fr bw = gather8(tabw, ofs, col), bd = gather8(tabd, ofs, col);
#pragma unroll
      for (int it = 0; it < NTH; ++it) {
        const int i = min(32 * it + cl, H - 1);
        gW2[it] = MF<T>::mma(*reinterpret_cast<const Fr*>(img2 + i * WQ + r0), bw, gW2[it]);
      }
#pragma unroll
      for (int it = 0; it < NTF; ++it) {
        const int i = min(32 * it + cl, F - 1);
        gW1[it] = MF<T>::mma(*reinterpret_cast<const Fr*>(img1 + i * WQ + r0), bd, gW1[it]);
      }
      const Fr b3 = *reinterpret_cast<const Fr*>(img3 + min(col, H - 1) * WQ + r0);
#pragma unroll
      for (int tt = 0; tt < NTT; ++tt) {
        const int want = (32 * tt + cl) * 128;
        u32x4_t u;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          u[e] = (ofs[2 * e] == want ? 0x3F80u : 0u) | (ofs[2 * e + 1] == want ? 0x3F800000u : 0u);
        gw3[tt] = MF<T>::mma(__builtin_bit_cast(Fr, u), b3, gw3[tt]);
      }
    }
  }
  // this workgroup's partial gradients: [gW2 H x H][gW1 F x H][gw3 Tn x H], wave w writes columns 32 w ..
  const int64_t L = (int64_t)(H + F + Tn) * H;
  float* g = gslab + (int64_t)blockIdx.x * L;
  const int o = 32 * w + cl;
  if (o < H) {
#pragma unroll
    for (int it = 0; it < NTH; ++it)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 32 * it + featq(q, h);
        if (i < H) g[i * H + o] = gW2[it][q];
      }
#pragma unroll
    for (int it = 0; it < NTF; ++it)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 32 * it + featq(q, h);
        if (i < F) g[(H + i) * H + o] = gW1[it][q];
      }
#pragma unroll
    for (int tt = 0; tt < NTT; ++tt)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int t = 32 * tt + featq(q, h);
        if (t < Tn) g[(H + F + t) * H + o] = gw3[tt][q];
      }
  }
  slab_put(slab, 2, 0, sr);
  slab_put(slab, 2, 1, sf);
}

// ===================================================================================================
// critic input gradient for the generator step (and its loss): head 0 = the linear WGAN-GP critic
// with W(fake, -1) (GAN/WGAN_GP.py:178-189), head 1 = the GAN discriminator Dense -> Dense ->
// Dense(1, sigmoid) per row with BCE(label) (GAN/GAN.py:144-158, 195-198)
// ===================================================================================================
template <typename T, int F, int H, int HEAD>
__global__ void __launch_bounds__(MLP_THREADS) mlp_critic_dx_kernel(const T* __restrict__ x, MlpCritic c, float label,
                                                                    T* __restrict__ dx, float* __restrict__ slab,
                                                                    int64_t M, int Tn, float inv) {
  using Fr = typename MP<T>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d2 = f2 + fwd_entries<T, H, H>() * 64;
  Fr* d1 = d2 + dgrad_entries<T, H, H>() * 64;
  float* vec = reinterpret_cast<float*>(d1 + dgrad_entries<T, F, H>() * 64);
  build_fwd<T, F, H>(f1, c.W1);
  build_fwd<T, H, H>(f2, c.W2);
  build_dgrad<T, H, H>(d2, c.W2);
  build_dgrad<T, F, H>(d1, c.W1);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  __syncthreads();
  const float b3 = c.b3 ? c.b3[0] : 0.f;
  float acc = 0.f;
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    const bool ok = row < M;
    const float* w3t = HEAD == 0 ? c.w3 + (int64_t)(ok ? row % Tn : 0) * H : c.w3;
    f32x16 A[NTH], Bv[NTH], X[NTF];
    load_rows<T, F>(X, x, row, M, h);
    dense<T, F, H>(X, A, f1, lane);
    bias_act<H>(A, vec, ACT_LINEAR, h);
    dense<T, H, H>(A, Bv, f2, lane);
    bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);
    const float sc = rowdot<H>(Bv, w3t, ok, h);
    float dz;
    if (HEAD == 0) {
      if (ok && h == 0) acc += sc;
      dz = -inv;  // d W(fake, -1) / d s_b = -1 / B
    } else {
      const float p = sigmoidf_(sc + b3);
      float lo, gp;
      bce(p, label, inv, lo, gp);
      if (ok && h == 0) acc += lo;
      dz = gp * p * (1.f - p);
    }
    head_rows<H>(A, w3t, dz, ok, h);  // dh2
    dense<T, H, H>(A, Bv, d2, lane);  // dh1
    dense<T, H, F>(Bv, X, d1, lane);  // dx
    store_rows<T, F>(dx, row, M, X, h);
  }
  slab_put(slab, 2, 0, acc);
  slab_put(slab, 2, 1, 0.f);
}

// The generator step's input gradient through the GAN discriminator (head 1), rank-1 form: the hidden
// layers are linear (Dense -> Dense -> Dense(1, sigmoid); _critic_lists checks it), so every row's
// adjoint is dx = dz_row g with ONE vector g = W1 W2 w3 -- computed once per workgroup in the prologue
// instead of two dgrad MFMA passes per row (mlp_critic_dx_kernel<HEAD = 1>).  No dgrad images: the
// forward images alone leave LDS room for fp32 on the split bf16 products (P = f32s_t).
template <typename T, int F, int H, typename P = T>
__global__ void __launch_bounds__(MLP_THREADS) mlp_gan_dx_kernel(const T* __restrict__ x, MlpCritic c, float label,
                                                                 T* __restrict__ dx, float* __restrict__ slab, int64_t M,
                                                                 float inv) {
  using Fr = typename MP<P>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<P, F, H>() * 64;
  float* vec = reinterpret_cast<float*>(f2 + fwd_entries<P, H, H>() * 64);  // b1 | b2 | w3 | D | g
  build_fwd<P, F, H>(f1, c.W1);
  build_fwd<P, H, H>(f2, c.W2);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  load_vec(vec + 2 * VEC, c.w3, H);
  for (int o = threadIdx.x; o < VEC; o += blockDim.x) {  // D = W2 w3
    float d = 0.f;
    if (o < H)
      for (int k = 0; k < H; ++k) d = fmaf(c.W2[o * H + k], c.w3[k], d);
    vec[3 * VEC + o] = d;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < VEC; i += blockDim.x) {  // g = W1 D
    float a = 0.f;
    if (i < F)
      for (int o = 0; o < H; ++o) a = fmaf(c.W1[i * H + o], vec[3 * VEC + o], a);
    vec[4 * VEC + i] = a;
  }
  __syncthreads();
  const float b3 = c.b3 ? c.b3[0] : 0.f;
  const float* gh = vec + 4 * VEC + 4 * ((threadIdx.x & 63) >> 5);  // lane-half base (see head_rows)
  float acc = 0.f;
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    const bool ok = row < M;
    f32x16 A[NTH], Bv[NTH], X[NTF];
    load_rows<T, F>(X, x, row, M, h);
    dense<P, F, H>(X, A, f1, lane);
    bias_act<H>(A, vec, ACT_LINEAR, h);
    dense<P, H, H>(A, Bv, f2, lane);
    bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);
    const float sc = rowdot<H>(Bv, vec + 2 * VEC, ok, h);
    const float p = sigmoidf_(sc + b3);
    float lo, gp;
    bce(p, label, inv, lo, gp);
    if (ok && h == 0) acc += lo;
    const float dz = gp * p * (1.f - p);
#pragma unroll
    for (int t = 0; t < NTF; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 gv = *reinterpret_cast<const float4*>(gh + 32 * t + 8 * g);
        X[t][4 * g] = dz * gv.x; X[t][4 * g + 1] = dz * gv.y; X[t][4 * g + 2] = dz * gv.z; X[t][4 * g + 3] = dz * gv.w;
      }
    store_rows<T, F>(dx, row, M, X, h);
  }
  slab_put(slab, 2, 0, acc);
  slab_put(slab, 2, 1, 0.f);
}

// ===================================================================================================
// vanilla GAN discriminator update (GAN/GAN.py:187-189): forward, BCE(label) per row, reverse to the
// weight-gradient operands
// ===================================================================================================
template <typename T, int F, int H>
__global__ void __launch_bounds__(MLP_THREADS) mlp_gan_critic_kernel(const T* __restrict__ x, MlpCritic c, float label,
                                                                     T* __restrict__ h1o, T* __restrict__ dh2o,
                                                                     T* __restrict__ dh1o, T* __restrict__ h2o,
                                                                     T* __restrict__ dz3o, float* __restrict__ slab,
                                                                     int64_t M, float inv) {
  using Fr = typename MP<T>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d2 = f2 + fwd_entries<T, H, H>() * 64;
  float* vec = reinterpret_cast<float*>(d2 + dgrad_entries<T, H, H>() * 64);
  build_fwd<T, F, H>(f1, c.W1);
  build_fwd<T, H, H>(f2, c.W2);
  build_dgrad<T, H, H>(d2, c.W2);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  __syncthreads();
  const float b3 = c.b3 ? c.b3[0] : 0.f;
  float acc = 0.f;
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    const bool ok = row < M;
    f32x16 A[NTH], Bv[NTH], X[NTF];
    load_rows<T, F>(X, x, row, M, h);
    dense<T, F, H>(X, A, f1, lane);
    bias_act<H>(A, vec, ACT_LINEAR, h);
    store_rows<T, H>(h1o, row, M, A, h);
    dense<T, H, H>(A, Bv, f2, lane);
    bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);
    store_rows<T, H>(h2o, row, M, Bv, h);
    const float p = sigmoidf_(rowdot<H>(Bv, c.w3, ok, h) + b3);
    float lo, gp;
    bce(p, label, inv, lo, gp);
    const float dz = gp * p * (1.f - p);
    if (ok && h == 0) {
      acc += lo;
      dz3o[row] = Cvt<T>::from_f(dz);
    }
    head_rows<H>(A, c.w3, dz, ok, h);
    store_rows<T, H>(dh2o, row, M, A, h);
    dense<T, H, H>(A, Bv, d2, lane);
    store_rows<T, H>(dh1o, row, M, Bv, h);
  }
  slab_put(slab, 2, 0, acc);
  slab_put(slab, 2, 1, 0.f);
}

// LayerNorm -> LeakyReLU -> sigmoid reverse of one row (the generator's Dense(sigmoid) + LReLU + LN
// blocks): g = dL/du (LN output gradient), y = the sigmoid outputs, (mean, rstd) of lrelu(y); writes
// dL/dz into out (may alias g or y: element-wise after the row sums) and adds the gamma-gradient
// column sums (sum_r g * xhat) into pg
template <int N>
__device__ __forceinline__ void ln_reverse(const f32x16* g, const f32x16* y, f32x16* out, const float* gam, float mean,
                                           float rstd, int h, int lane, float* pg) {
  constexpr int NT = (N + 31) / 32;
  const float* gh = gam + 4 * h;
  float m1 = 0.f, m2 = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int f0 = 32 * t + 8 * gq + 4 * h;
      const float4 gv = *reinterpret_cast<const float4*>(gh + 32 * t + 8 * gq);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = 4 * gq + e;
        const bool in = f0 + e < N;
        const float xh = in ? (lrelu(y[t][q]) - mean) * rstd : 0.f;
        const float gd = in ? g[t][q] * gg[e] : 0.f;
        m1 += gd;
        m2 = fmaf(gd, xh, m2);
      }
    }
  m1 += __shfl_xor(m1, 32, 64);
  m2 += __shfl_xor(m2, 32, 64);
  m1 *= 1.f / N;
  m2 *= 1.f / N;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f32x16 px;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int f0 = 32 * t + 8 * gq + 4 * h;
      const float4 gv = *reinterpret_cast<const float4*>(gh + 32 * t + 8 * gq);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = 4 * gq + e;
        const bool in = f0 + e < N;
        const float yv = y[t][q];
        const float xh = in ? (lrelu(yv) - mean) * rstd : 0.f;
        const float dv = in ? g[t][q] : 0.f;
        px[q] = dv * xh;
        float dl = rstd * (dv * gg[e] - m1 - xh * m2);
        dl *= yv >= 0.f ? 1.f : LRELU_ALPHA_F;
        out[t][q] = in ? dl * yv * (1.f - yv) : 0.f;
      }
    }
    pg[t] += colsum(px, lane);
  }
}

// ---------------------------------------------------------------------------------------------------
// The same discriminator update with its six parameter gradients taken in the kernel.  The hidden
// layers are linear, so every adjoint of a row is that row's scalar dz times a fixed vector:
//   dh2 = dz w3,  dh1 = dz u (u = W2 w3)
// and each weight gradient factorises into a dz-weighted column sum of the layer's own input:
//   gW1 = s1 (x) u,  gW2 = s2 (x) w3,  gw3 = s3,  gb1 = S u,  gb2 = S w3,  gb3 = S
//   s1 = sum_r dz_r x_r,  s2 = sum_r dz_r h1_r,  s3 = sum_r dz_r h2_r,  S = sum_r dz_r.
// Each lane accumulates dz * (x, h1, h2) of its rows in registers over all its tiles (fp32); one
// transpose-reduce butterfly per tile set at the end gives the wave's column sums (slab row of the
// wave: [s1 F | s2 H | s3 H | S]); mlp_gan_grad_finish reduces the slab in a fixed order and forms
// the outer products.  The per-row forward and BCE are the same as mlp_gan_critic's.
// ---------------------------------------------------------------------------------------------------
template <typename T, int F, int H, typename P = T>  // P: product policy (f32s_t: fp32 on split bf16)
__global__ void __launch_bounds__(MLP_THREADS) mlp_gan_critic_g_kernel(const T* __restrict__ x, MlpCritic c, float label,
                                                                       float* __restrict__ gslab,
                                                                       float* __restrict__ slab, int64_t M, float inv) {
  using Fr = typename MP<P>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<P, F, H>() * 64;
  float* vec = reinterpret_cast<float*>(f2 + fwd_entries<P, H, H>() * 64);
  build_fwd<P, F, H>(f1, c.W1);
  build_fwd<P, H, H>(f2, c.W2);
  load_vec(vec, c.b1, H);
  load_vec(vec + VEC, c.b2, H);
  load_vec(vec + 2 * VEC, c.w3, H);
  __syncthreads();
  const float b3 = c.b3 ? c.b3[0] : 0.f;
  float acc = 0.f, sdz = 0.f;
  f32x16 ax[NTF], a1[NTH], a2[NTH];
#pragma unroll
  for (int t = 0; t < NTF; ++t) ax[t] = zero16();
#pragma unroll
  for (int t = 0; t < NTH; ++t) a1[t] = a2[t] = zero16();
  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    const bool ok = row < M;
    f32x16 A[NTH], Bv[NTH], X[NTF];
    load_rows<T, F>(X, x, row, M, h);
    dense<P, F, H>(X, A, f1, lane);
    bias_act<H>(A, vec, ACT_LINEAR, h);         // h1
    dense<P, H, H>(A, Bv, f2, lane);
    bias_act<H>(Bv, vec + VEC, ACT_LINEAR, h);  // h2
    const float p = sigmoidf_(rowdot<H>(Bv, vec + 2 * VEC, true, h) + b3);
    float lo, gp;
    bce(p, label, inv, lo, gp);
    const float dz = ok ? gp * p * (1.f - p) : 0.f;
    if (ok && h == 0) {
      acc += lo;
      sdz += dz;
    }
#pragma unroll
    for (int t = 0; t < NTF; ++t) ax[t] += dz * X[t];
#pragma unroll
    for (int t = 0; t < NTH; ++t) {
      a1[t] += dz * A[t];
      a2[t] += dz * Bv[t];
    }
  }
  constexpr int L = F + 2 * H + 1;
  float* out = gslab + ((int64_t)blockIdx.x * MLP_WAVES + (threadIdx.x >> 6)) * L;
  const int fq = featq(colsum_q(lane), h);
#pragma unroll
  for (int t = 0; t < NTF; ++t) {
    const float v = colsum(ax[t], lane);
    if ((lane & 1) == 0 && 32 * t + fq < F) out[32 * t + fq] = v;
  }
#pragma unroll
  for (int t = 0; t < NTH; ++t) {
    const float v1 = colsum(a1[t], lane), v2 = colsum(a2[t], lane);
    if ((lane & 1) == 0 && 32 * t + fq < H) {
      out[F + 32 * t + fq] = v1;
      out[F + H + 32 * t + fq] = v2;
    }
  }
  sdz = wave_sum(sdz);
  if ((threadIdx.x & 63) == 0) out[F + 2 * H] = sdz;
  slab_put(slab, 2, 0, acc);
  slab_put(slab, 2, 1, 0.f);
}

// the six gradients from the reduced sums v = [s1 F | s2 H | s3 H | S] (one workgroup, fp32)
__global__ void __launch_bounds__(256) mlp_gan_grad_finish_kernel(const float* __restrict__ v, MlpCritic c, int F, int H,
                                                                  float* __restrict__ gW1, float* __restrict__ gb1,
                                                                  float* __restrict__ gW2, float* __restrict__ gb2,
                                                                  float* __restrict__ gw3, float* __restrict__ gb3) {
  __shared__ float u[128], w3[128];
  const float* s1 = v;
  const float* s2 = v + F;
  const float* s3 = v + F + H;
  const float S = v[F + 2 * H];
  for (int i = threadIdx.x; i < H; i += blockDim.x) {
    float a = 0.f;
    for (int o = 0; o < H; ++o) a = fmaf(c.W2[i * H + o], c.w3[o], a);  // u = W2 w3
    u[i] = a;
    w3[i] = c.w3[i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < F * H; e += blockDim.x) gW1[e] += s1[e / H] * u[e % H];
  for (int e = threadIdx.x; e < H * H; e += blockDim.x) gW2[e] += s2[e / H] * w3[e % H];
  for (int o = threadIdx.x; o < H; o += blockDim.x) {
    gb1[o] += S * u[o];
    gb2[o] += S * w3[o];
    gw3[o] += s3[o];
  }
  if (threadIdx.x == 0) gb3[0] += S;
}

// ===================================================================================================
// generator reverse pass (GAN/WGAN_GP.py:178-189 / GAN/GAN.py:195-198: the combined model's update)
// from dfake = dL/dG(z): recomputes the forward in registers and writes the weight-gradient operands
// ===================================================================================================
template <typename T, int F, int H>
__global__ void __launch_bounds__(MLP_THREADS) mlp_gen_bwd_kernel(const T* __restrict__ z, const T* __restrict__ dfake,
                                                                  MlpGen g, T* __restrict__ dz1o, T* __restrict__ u1o,
                                                                  T* __restrict__ dz2o, T* __restrict__ u2o,
                                                                  float* __restrict__ lnslab, int64_t M) {
  using Fr = typename MP<T>::frag;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d3 = f2 + fwd_entries<T, H, H>() * 64;
  Fr* d2 = d3 + dgrad_entries<T, H, F>() * 64;
  float* vec = reinterpret_cast<float*>(d2 + dgrad_entries<T, H, H>() * 64);
  build_fwd<T, F, H>(f1, g.W1);
  build_fwd<T, H, H>(f2, g.W2);
  build_dgrad<T, H, F>(d3, g.W3);
  build_dgrad<T, H, H>(d2, g.W2);
  load_vec(vec + 0 * VEC, g.b1, H); load_vec(vec + 1 * VEC, g.g1, H); load_vec(vec + 2 * VEC, g.be1, H);
  load_vec(vec + 3 * VEC, g.b2, H); load_vec(vec + 4 * VEC, g.g2, H); load_vec(vec + 5 * VEC, g.be2, H);
  __syncthreads();
  const float* gam1 = vec + 1 * VEC;
  const float* gam2 = vec + 4 * VEC;
  float pg1[NTH], pb1[NTH], pg2[NTH], pb2[NTH];  // per-lane column sums (see colsum)
#pragma unroll
  for (int t = 0; t < NTH; ++t) pg1[t] = pb1[t] = pg2[t] = pb2[t] = 0.f;


  MLP_LOOP {
    const int64_t row = tile * 32 + (lane & 31);
    f32x16 x[NTF], a[NTH], y2[NTH], d[NTH];
    float mean1, rstd1, mean2, rstd2;
    // ---- forward (u1, u2 out; y2 and the row statistics kept)
    load_rows<T, F>(x, z, row, M, h);
    dense<T, F, H>(x, a, f1, lane);
    bias_act<H>(a, vec + 0 * VEC, ACT_SIGMOID, h);
    lrelu_ln<H>(a, vec + 1 * VEC, vec + 2 * VEC, h, mean1, rstd1);
    store_rows<T, H>(u1o, row, M, a, h);
    dense<T, H, H>(a, y2, f2, lane);
    bias_act<H>(y2, vec + 3 * VEC, ACT_SIGMOID, h);
#pragma unroll
    for (int t = 0; t < NTH; ++t) a[t] = y2[t];
    lrelu_ln<H>(a, vec + 4 * VEC, vec + 5 * VEC, h, mean2, rstd2);
    store_rows<T, H>(u2o, row, M, a, h);
    // ---- reverse: du2 = dfake W3^T, LN2 / LReLU / sigmoid reverse -> dz2
    load_rows<T, F>(x, dfake, row, M, h);
    dense<T, F, H>(x, d, d3, lane);
#pragma unroll
    for (int t = 0; t < NTH; ++t) pb2[t] += colsum(d[t], lane);
    ln_reverse<H>(d, y2, d, gam2, mean2, rstd2, h, lane, pg2);
    store_rows<T, H>(dz2o, row, M, d, h);
    // ---- du1 = dz2 W2^T; recompute y1; LN1 / LReLU / sigmoid reverse -> dz1
    dense<T, H, H>(d, y2, d2, lane);  // y2 now holds du1
#pragma unroll
    for (int t = 0; t < NTH; ++t) pb1[t] += colsum(y2[t], lane);
    load_rows<T, F>(x, z, row, M, h);
    dense<T, F, H>(x, a, f1, lane);
    bias_act<H>(a, vec + 0 * VEC, ACT_SIGMOID, h);  // y1
    ln_reverse<H>(y2, a, a, gam1, mean1, rstd1, h, lane, pg1);
    store_rows<T, H>(dz1o, row, M, a, h);
  }
  // per-wave LN partials: lanes with bit 0 clear own feature featq(colsum_q(lane), h) of every tile
  float* out = lnslab + ((int64_t)blockIdx.x * MLP_WAVES + (threadIdx.x >> 6)) * 4 * H;
  if ((lane & 1) == 0) {
#pragma unroll
    for (int t = 0; t < NTH; ++t) {
      const int f = 32 * t + featq(colsum_q(lane), h);
      if (f < H) {
        out[f] = pg1[t];
        out[H + f] = pb1[t];
        out[2 * H + f] = pg2[t];
        out[3 * H + f] = pb2[t];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// The generator reverse with its six parameter gradients (W1, b1, W2, b2, W3, b3) accumulated in the
// kernel (bf16), the scheme of mlp_wgp_critic_w: 4 waves walk 128-row block tiles together, stage the
// X / dY operands of each weight transposed in LDS and run the block's rows as the k dimension of
// gW = X^T dY on v_mfma_f32_32x32x16_bf16.  The bias gradients come out of the same MFMAs: every X
// image has a row of ones after its last feature (written once), so C row K of gW is sum_r dY[r].
// Four staging buffers, reused as the chain produces operands (two barriers per weight):
//   A: u1 -> dz1     B: u2 -> dz2     C: dfake     D: noise
//   gW3 (+ gb3): X = u2 (B), dY = dfake (C); wave w owns input tile w, every output tile
//   gW2 (+ gb2): X = u1 (A), dY = dz2 (B);   wave w owns output tile w
//   gW1 (+ gb1): X = noise (D), dY = dz1 (A); wave w owns output tile w
// LayerNorm parameter gradients stay the per-wave colsum partials of mlp_gen_bwd (lnslab).
// ---------------------------------------------------------------------------------------------------
template <int F, int H> constexpr size_t gbw_images() {
  return (size_t)(fwd_entries<bf16_t, F, H>() + fwd_entries<bf16_t, H, H>() + dgrad_entries<bf16_t, H, F>() +
                  dgrad_entries<bf16_t, H, H>()) *
             frag_bytes<bf16_t>() +
         6 * VEC * 4;
}
template <int F, int H> constexpr size_t gbw_off_a() { return gbw_images<F, H>(); }
template <int F, int H> constexpr size_t gbw_off_b() { return gbw_off_a<F, H>() + (size_t)(H + 1) * WQ * 2; }
template <int F, int H> constexpr size_t gbw_off_c() { return gbw_off_b<F, H>() + (size_t)(H + 1) * WQ * 2; }
template <int F, int H> constexpr size_t gbw_off_d() { return gbw_off_c<F, H>() + (size_t)F * WQ * 2; }
template <int F, int H> constexpr size_t gbw_lds() { return gbw_off_d<F, H>() + (size_t)(F + 1) * WQ * 2; }
static_assert(gbw_lds<36, 100>() <= 160 * 1024, "generator reverse staging exceeds LDS");
static_assert(gbw_off_b<36, 100>() % 16 == 0 && gbw_off_c<36, 100>() % 16 == 0 && gbw_off_d<36, 100>() % 16 == 0,
              "16-byte aligned staging images");
static_assert(gbw_off_b<32, 100>() % 16 == 0 && gbw_off_c<32, 100>() % 16 == 0 && gbw_off_d<32, 100>() % 16 == 0,
              "16-byte aligned staging images");

// rows past M stage zeros
template <int N>
__device__ __forceinline__ void stage_t_ok(unsigned short* img, f32x16* a, int rr, int h, bool ok) {
  if (!ok) {
#pragma unroll
    for (int t = 0; t < (N + 31) / 32; ++t) a[t] = zero16();
  }
  stage_t<N>(img, a, rr, h);
}
// gW[tile] += X^T dY over the block's 128 rows: A = rows of the X image (clamped to row KX: the ones
// row or a discarded one), B = row `col` of the dY image
template <int NI>
__device__ __forceinline__ void wgrad_block(f32x16* acc, const unsigned short* X, int i0, int KX,
                                            const unsigned short* Y, int col, int cl, int h) {
#pragma unroll 2
  for (int ks = 0; ks < 8; ++ks) {
    const int r0 = 16 * ks + 8 * h;
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(Y + col * WQ + r0);
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int i = min(i0 + 32 * it + cl, KX);
      acc[it] = MF<bf16_t>::mma(*reinterpret_cast<const bf16x8*>(X + i * WQ + r0), b, acc[it]);
    }
  }
}

// acc[ot] += X^T dY for ONE input row i of X and NO output tiles (B = rows 32 ot + lane of the dY
// image, clamped to KY - 1)
template <int NO>
__device__ __forceinline__ void wgrad_block_out(f32x16* acc, const unsigned short* X, int i, const unsigned short* Y,
                                                int KY, int cl, int h) {
#pragma unroll 2
  for (int ks = 0; ks < 8; ++ks) {
    const int r0 = 16 * ks + 8 * h;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(X + i * WQ + r0);
#pragma unroll
    for (int ot = 0; ot < NO; ++ot) {
      const int o = min(32 * ot + cl, KY - 1);
      acc[ot] = MF<bf16_t>::mma(a, *reinterpret_cast<const bf16x8*>(Y + o * WQ + r0), acc[ot]);
    }
  }
}

template <int F, int H>
__global__ void __launch_bounds__(MLP_THREADS) mlp_gen_bwd_w_kernel(const bf16_t* __restrict__ z,
                                                                    const bf16_t* __restrict__ dfake, MlpGen g,
                                                                    float* __restrict__ gslab,
                                                                    float* __restrict__ lnslab, int64_t M) {
  using T = bf16_t;
  using Fr = bf16x8;
  constexpr int NTH = (H + 31) / 32, NTF = (F + 31) / 32, NX1 = (F + 1 + 31) / 32;
  static_assert((H + 1 + 31) / 32 == NTH, "the ones row of the H-wide images fits the last input tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  Fr* f1 = reinterpret_cast<Fr*>(lds);
  Fr* f2 = f1 + fwd_entries<T, F, H>() * 64;
  Fr* d3 = f2 + fwd_entries<T, H, H>() * 64;
  Fr* d2 = d3 + dgrad_entries<T, H, F>() * 64;
  float* vec = reinterpret_cast<float*>(d2 + dgrad_entries<T, H, H>() * 64);
  unsigned short* bA = reinterpret_cast<unsigned short*>(lds + gbw_off_a<F, H>());
  unsigned short* bB = reinterpret_cast<unsigned short*>(lds + gbw_off_b<F, H>());
  unsigned short* bC = reinterpret_cast<unsigned short*>(lds + gbw_off_c<F, H>());
  unsigned short* bD = reinterpret_cast<unsigned short*>(lds + gbw_off_d<F, H>());
  build_fwd<T, F, H>(f1, g.W1);
  build_fwd<T, H, H>(f2, g.W2);
  build_dgrad<T, H, F>(d3, g.W3);
  build_dgrad<T, H, H>(d2, g.W2);
  load_vec(vec + 0 * VEC, g.b1, H); load_vec(vec + 1 * VEC, g.g1, H); load_vec(vec + 2 * VEC, g.be1, H);
  load_vec(vec + 3 * VEC, g.b2, H); load_vec(vec + 4 * VEC, g.g2, H); load_vec(vec + 5 * VEC, g.be2, H);
  for (int r = threadIdx.x; r < 128; r += blockDim.x) {  // the ones rows (bf16 1.0)
    bA[H * WQ + r] = 0x3F80;
    bB[H * WQ + r] = 0x3F80;
    bD[F * WQ + r] = 0x3F80;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, w = threadIdx.x >> 6, cl = lane & 31;
  const int rr = 32 * w + cl;
  const float* gam1 = vec + 1 * VEC;
  const float* gam2 = vec + 4 * VEC;
  float pg1[NTH], pb1[NTH], pg2[NTH], pb2[NTH];
#pragma unroll
  for (int t = 0; t < NTH; ++t) pg1[t] = pb1[t] = pg2[t] = pb2[t] = 0.f;
  f32x16 gW3[NTF], gW2[NTH], gW1[NX1];
#pragma unroll
  for (int i = 0; i < NTF; ++i) gW3[i] = zero16();
#pragma unroll
  for (int i = 0; i < NTH; ++i) gW2[i] = zero16();
#pragma unroll
  for (int i = 0; i < NX1; ++i) gW1[i] = zero16();
  const int64_t nbt = (M + 127) / 128;
  for (int64_t bt = blockIdx.x; bt < nbt; bt += gridDim.x) {
    const int64_t row = bt * 128 + rr;
    const bool ok = row < M;
    f32x16 x[NTF], a[NTH], y2[NTH], d[NTH];
    float mean1, rstd1, mean2, rstd2;
    __syncthreads();  // S0: the previous block tile's gW1 reads (A, D) are done
    load_rows<T, F>(x, z, row, M, h);
    stage_t_ok<F>(bD, x, rr, h, ok);
    dense<T, F, H>(x, a, f1, lane);
    bias_act<H>(a, vec + 0 * VEC, ACT_SIGMOID, h);
    lrelu_ln<H>(a, vec + 1 * VEC, vec + 2 * VEC, h, mean1, rstd1);  // u1
    dense<T, H, H>(a, y2, f2, lane);
    stage_t_ok<H>(bA, a, rr, h, ok);
    bias_act<H>(y2, vec + 3 * VEC, ACT_SIGMOID, h);
#pragma unroll
    for (int t = 0; t < NTH; ++t) a[t] = y2[t];
    lrelu_ln<H>(a, vec + 4 * VEC, vec + 5 * VEC, h, mean2, rstd2);  // u2
    stage_t_ok<H>(bB, a, rr, h, ok);
    load_rows<T, F>(x, dfake, row, M, h);  // zeros past M
    stage_t<F>(bC, x, rr, h);
    dense<T, F, H>(x, d, d3, lane);        // du2 = dfake W3^T
#pragma unroll
    for (int t = 0; t < NTH; ++t) pb2[t] += colsum(d[t], lane);
    ln_reverse<H>(d, y2, d, gam2, mean2, rstd2, h, lane, pg2);  // dz2 (y2 dead from here)
    __syncthreads();  // S1: u1, u2, dfake, noise staged
    __builtin_amdgcn_sched_barrier(0);
    wgrad_block_out<NTF>(gW3, bB, min(32 * w + cl, H), bC, F, cl, h);  // gW3[i in tile w][o = 32 ot + cl]
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // S2: the gW3 reads of B are done
    stage_t_ok<H>(bB, d, rr, h, ok);
    dense<T, H, H>(d, y2, d2, lane);  // y2 now holds du1
    __syncthreads();  // S2b: dz2 staged
    __builtin_amdgcn_sched_barrier(0);
    wgrad_block<NTH>(gW2, bA, 0, H, bB, min(32 * w + cl, H - 1), cl, h);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NTH; ++t) pb1[t] += colsum(y2[t], lane);
    load_rows<T, F>(x, z, row, M, h);
    dense<T, F, H>(x, a, f1, lane);
    bias_act<H>(a, vec + 0 * VEC, ACT_SIGMOID, h);  // y1
    ln_reverse<H>(y2, a, a, gam1, mean1, rstd1, h, lane, pg1);  // dz1
    __syncthreads();  // S3: the gW2 reads of A are done
    stage_t_ok<H>(bA, a, rr, h, ok);
    __syncthreads();  // S3b: dz1 staged
    __builtin_amdgcn_sched_barrier(0);
    wgrad_block<NX1>(gW1, bD, 0, F, bA, min(32 * w + cl, H - 1), cl, h);
    __builtin_amdgcn_sched_barrier(0);
  }
  // partial gradients of this workgroup: [W1 F x H][b1 H][W2 H x H][b2 H][W3 H x F][b3 F]
  constexpr int oB1 = F * H, oW2 = oB1 + H, oB2 = oW2 + H * H, oW3 = oB2 + H, oB3 = oW3 + H * F, L = oB3 + F;
  float* gs = gslab + (int64_t)blockIdx.x * L;
  {
    const int o = 32 * w + cl;  // gW2 / gW1 output column
    if (o < H) {
#pragma unroll
      for (int it = 0; it < NTH; ++it)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = 32 * it + featq(q, h);
          if (i < H) gs[oW2 + i * H + o] = gW2[it][q];
          else if (i == H) gs[oB2 + o] = gW2[it][q];
        }
#pragma unroll
      for (int it = 0; it < NX1; ++it)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = 32 * it + featq(q, h);
          if (i < F) gs[i * H + o] = gW1[it][q];
          else if (i == F) gs[oB1 + o] = gW1[it][q];
        }
    }
#pragma unroll
    for (int ot = 0; ot < NTF; ++ot) {
      const int o3 = 32 * ot + cl;
      if (o3 < F) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = 32 * w + featq(q, h);
          if (i < H) gs[oW3 + i * F + o3] = gW3[ot][q];
          else if (i == H) gs[oB3 + o3] = gW3[ot][q];
        }
      }
    }
  }
  float* out = lnslab + ((int64_t)blockIdx.x * MLP_WAVES + w) * 4 * H;
  if ((lane & 1) == 0) {
#pragma unroll
    for (int t = 0; t < NTH; ++t) {
      const int f = 32 * t + featq(colsum_q(lane), h);
      if (f < H) {
        out[f] = pg1[t];
        out[H + f] = pb1[t];
        out[2 * H + f] = pg2[t];
        out[3 * H + f] = pb2[t];
      }
    }
  }
}

// ===================================================================================================
// fixed-order reductions
// ===================================================================================================
__global__ void __launch_bounds__(256) mlp_finish_kernel(const float* __restrict__ slab, int P,
                                                         const float* __restrict__ e, int64_t ne, int mode, float invB,
                                                         const float* __restrict__ b3p, float lam,
                                                         float* __restrict__ out) {
  __shared__ float red[3][4];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < P; i += 256) {
    s0 += slab[2 * i];
    s1 += slab[2 * i + 1];
  }
  for (int64_t i = threadIdx.x; i < ne; i += 256) s2 += e[i];
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s0;
    red[1][w] = s1;
    red[2][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b3 = b3p ? b3p[0] : 0.f;
    const float a = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    const float b = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const float c = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
    if (mode == 0) {
      const float wr = -(a * invB + b3), wf = b * invB + b3, pen = c * invB;
      out[0] = wr + wf + lam * pen;
      out[1] = wr;
      out[2] = wf;
      out[3] = pen;
    } else if (mode == 1) {  // generator W loss on the fake rows: W(fake, -1) = -mean s
      out[0] = -(a * invB + b3);
      out[1] = out[2] = out[3] = 0.f;
    } else {  // BCE: the slab holds the per-row losses; invB = 1 / rows gives their mean
      out[0] = a * invB;
      out[1] = out[2] = out[3] = 0.f;
    }
  }
}

// out[k][j] += sum_p slab[p][k L + j] for the nseg segments: 64 elements per workgroup, the 16 waves
// split the P rows (4 partial sums each so loads overlap), combined in a fixed order (deterministic)
// (slab rows have `stride` floats; the summed columns start at col0)
__global__ void __launch_bounds__(1024) mlp_slab_sum_kernel(const float* __restrict__ slab, int P, int64_t stride,
                                                            int col0, int L, int nseg, float* __restrict__ o0,
                                                            float* __restrict__ o1, float* __restrict__ o2,
                                                            float* __restrict__ o3) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane, n = nseg * L;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n) {
    const float* col = slab + col0 + i;
    int p = wv;
    for (; p + 48 < P; p += 64) {
      s0 += col[(int64_t)p * stride];
      s1 += col[(int64_t)(p + 16) * stride];
      s2 += col[(int64_t)(p + 32) * stride];
      s3 += col[(int64_t)(p + 48) * stride];
    }
    for (; p < P; p += 16) s0 += col[(int64_t)p * stride];
  }
  part[wv][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wv == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += part[w][lane];
    const int k = i / L, j = i - k * L;
    float* o = k == 0 ? o0 : k == 1 ? o1 : k == 2 ? o2 : o3;
    if (o) o[j] += t;
  }
}

// ===================================================================================================
// host launchers
// ===================================================================================================
bool mlp_supported(int F, int H) { return H == 100 && (F == 32 || F == 36); }

namespace {

template <typename KER>
int mlp_grid(KER kern, size_t lds, int64_t M) {
  static_assert(sizeof(KER) > 0, "");
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), MLP_THREADS, lds) !=
          hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t ntile = (M + 31) / 32;
  const int64_t want = (ntile + MLP_WAVES - 1) / MLP_WAVES;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)device_cu_count() * std::min(per_cu, 2)));
}

template <typename KER>
void set_lds(KER kern, size_t lds) {
  if (lds > 64 * 1024)
    HFREP_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)lds));
}

template <typename T, int F, int H> constexpr size_t lds_gen_fwd() {
  return (size_t)(fwd_entries<T, F, H>() + fwd_entries<T, H, H>() + fwd_entries<T, H, F>()) * frag_bytes<T>() +
         7 * VEC * 4;
}
template <typename T, int F, int H> constexpr size_t lds_wgp_norm() {
  return (size_t)(dgrad_entries<T, H, H>() + dgrad_entries<T, F, H>()) * frag_bytes<T>();
}
template <typename T, int F, int H> constexpr size_t lds_critic4() {
  return (size_t)(fwd_entries<T, F, H>() + fwd_entries<T, H, H>() + dgrad_entries<T, H, H>() +
                  dgrad_entries<T, F, H>()) *
             frag_bytes<T>() +
         2 * VEC * 4;
}
template <typename T, int F, int H> constexpr size_t lds_gan_critic() {
  return (size_t)(fwd_entries<T, F, H>() + fwd_entries<T, H, H>() + dgrad_entries<T, H, H>()) * frag_bytes<T>() +
         2 * VEC * 4;
}
template <typename T, int F, int H> constexpr size_t lds_gen_bwd() {
  return (size_t)(fwd_entries<T, F, H>() + fwd_entries<T, H, H>() + dgrad_entries<T, H, F>() +
                  dgrad_entries<T, H, H>()) *
             frag_bytes<T>() +
         6 * VEC * 4;
}
static_assert(lds_critic4<float, 36, 100>() <= 160 * 1024, "fp32 critic images exceed LDS");
static_assert(lds_gen_bwd<float, 36, 100>() <= 160 * 1024, "fp32 generator reverse images exceed LDS");

// dispatch over (dtype, F) with H = 100
#define MLP_DISPATCH(dt, F, ...)                      \
  do {                                                 \
    if (dt == DT_BF16) {                               \
      using T = bf16_t;                                \
      if (F == 32) { constexpr int FF = 32; __VA_ARGS__ }     \
      else { constexpr int FF = 36; __VA_ARGS__ }             \
    } else {                                           \
      using T = float;                                 \
      if (F == 32) { constexpr int FF = 32; __VA_ARGS__ }     \
      else { constexpr int FF = 36; __VA_ARGS__ }             \
    }                                                  \
  } while (0)

}  // namespace

int mlp_slab_rows(int64_t M) {
  const int64_t ntile = (M + 31) / 32;
  const int64_t want = (ntile + MLP_WAVES - 1) / MLP_WAVES;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)device_cu_count() * 2)) * MLP_WAVES;
}

void launch_mlp_gen_fwd(int dt, const void* noise, const MlpGen& g, void* out, int64_t M, int F, int H,
                        hipStream_t s) {
  if (M <= 0) return;
  // fp32 at F = 32: the split bf16 products (the three weight planes fit LDS: 136 KB; F = 36 needs 166)
  if (dt == DT_F32 && F == 32 && !fp32_exact_mode()) {
    auto k = mlp_gen_fwd_kernel<float, 32, 100, f32s_t>;
    constexpr size_t lds = lds_gen_fwd<f32s_t, 32, 100>();
    static_assert(lds <= 160 * 1024, "split generator images exceed LDS");
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(mlp_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const float*)noise, g, (float*)out, M);
    return;
  }
  MLP_DISPATCH(dt, F, {
    auto k = mlp_gen_fwd_kernel<T, FF, 100>;
    constexpr size_t lds = lds_gen_fwd<T, FF, 100>();
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(mlp_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)noise, g, (T*)out, M);
  });
  (void)H;
}

void launch_mlp_wgp_norm(int dt, const MlpCritic& c, float* gsq, int64_t M, int Tn, int F, int H, hipStream_t s) {
  if (M <= 0) return;
  MLP_DISPATCH(dt, F, {
    auto k = mlp_wgp_norm_kernel<T, FF, 100>;
    constexpr size_t lds = lds_wgp_norm<T, FF, 100>();
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(mlp_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, c, gsq, M, Tn);
  });
  (void)H;
}

int mlp_wgp_coef_parts(int64_t B) { return (int)((B + 255) / 256); }

void launch_mlp_wgp_coef(const float* gsq, int Tn, int64_t B, float lam, float* c, float* e, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(mlp_wgp_coef_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, gsq, Tn, B, lam, c, e);
}

// the slab-writing launchers must use exactly mlp_slab_rows(M) / MLP_WAVES workgroups
template <typename KER>
static int slab_grid(KER kern, size_t lds, int64_t M) {
  (void)kern;
  (void)lds;
  return mlp_slab_rows(M) / MLP_WAVES;
}

void launch_mlp_wgp_critic(int dt, const void* real, const void* fake, const float* c, const MlpCritic& cr,
                           void* X2c, void* dY2, void* X1c, void* dY1, void* Y3c, float* slab, int64_t M, int Tn,
                           int F, int H, hipStream_t s) {
  if (M <= 0) return;
  const float invB = (float)Tn / (float)M;
  MLP_DISPATCH(dt, F, {
    auto k = mlp_wgp_critic_kernel<T, FF, 100>;
    constexpr size_t lds = lds_critic4<T, FF, 100>();
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)real, (const T*)fake, c, cr,
                       (T*)X2c, (T*)dY2, (T*)X1c, (T*)dY1, (T*)Y3c, slab, M, Tn, invB);
  });
  (void)H;
}

void launch_mlp_critic_dx(int dt, int head, const void* x, const MlpCritic& cr, float label, void* dx, float* slab,
                          int64_t M, int Tn, int F, int H, hipStream_t s) {
  if (M <= 0) return;
  // head 0: d/ds_b of the W loss = -1/B (B = M / T samples); head 1: BCE mean over the M rows
  const float inv = head == 0 ? (float)Tn / (float)M : 1.f / (float)M;
  if (head == 1) {  // rank-1 input gradient (mlp_gan_dx_kernel); fp32 on the split bf16 products
    constexpr size_t vecb = 5 * VEC * 4;
    if (dt == DT_F32 && !fp32_exact_mode()) {
      MLP_DISPATCH(dt, F, {
        auto k = mlp_gan_dx_kernel<float, FF, 100, f32s_t>;
        constexpr size_t lds =
            (size_t)(fwd_entries<f32s_t, FF, 100>() + fwd_entries<f32s_t, 100, 100>()) * frag_bytes<f32s_t>() + vecb;
        static_assert(lds <= 160 * 1024, "split discriminator images exceed LDS");
        set_lds(k, lds);
        hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const float*)x, cr, label,
                           (float*)dx, slab, M, inv);
      });
    } else {
      MLP_DISPATCH(dt, F, {
        auto k = mlp_gan_dx_kernel<T, FF, 100>;
        constexpr size_t lds = (size_t)(fwd_entries<T, FF, 100>() + fwd_entries<T, 100, 100>()) * frag_bytes<T>() + vecb;
        set_lds(k, lds);
        hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)x, cr, label, (T*)dx,
                           slab, M, inv);
      });
    }
    (void)H;
    return;
  }
  MLP_DISPATCH(dt, F, {
    constexpr size_t lds = lds_critic4<T, FF, 100>();
    if (head == 0) {
      auto k = mlp_critic_dx_kernel<T, FF, 100, 0>;
      set_lds(k, lds);
      hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)x, cr, label, (T*)dx, slab,
                         M, Tn, inv);
    } else {
      auto k = mlp_critic_dx_kernel<T, FF, 100, 1>;
      set_lds(k, lds);
      hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)x, cr, label, (T*)dx, slab,
                         M, Tn, inv);
    }
  });
  (void)H;
}

void launch_mlp_gan_critic(int dt, const void* x, const MlpCritic& cr, float label, void* h1, void* dh2, void* dh1,
                           void* h2, void* dz3, float* slab, int64_t M, int F, int H, hipStream_t s) {
  if (M <= 0) return;
  MLP_DISPATCH(dt, F, {
    auto k = mlp_gan_critic_kernel<T, FF, 100>;
    constexpr size_t lds = lds_gan_critic<T, FF, 100>();
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)x, cr, label, (T*)h1,
                       (T*)dh2, (T*)dh1, (T*)h2, (T*)dz3, slab, M, 1.f / (float)M);
  });
  (void)H;
}

void launch_mlp_gen_bwd(int dt, const void* noise, const void* dfake, const MlpGen& g, void* dz1, void* u1,
                        void* dz2, void* u2, float* lnslab, int64_t M, int F, int H, hipStream_t s) {
  if (M <= 0) return;
  MLP_DISPATCH(dt, F, {
    auto k = mlp_gen_bwd_kernel<T, FF, 100>;
    constexpr size_t lds = lds_gen_bwd<T, FF, 100>();
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)noise, (const T*)dfake, g,
                       (T*)dz1, (T*)u1, (T*)dz2, (T*)u2, lnslab, M);
  });
  (void)H;
}

void launch_mlp_finish(const float* slab, int P, const float* e, int64_t n_e, int mode, float invB, const float* b3,
                       float lam, float* out, hipStream_t s) {
  hipLaunchKernelGGL(mlp_finish_kernel, dim3(1), dim3(256), 0, s, slab, P, e, n_e, mode, invB, b3, lam, out);
}

void launch_mlp_slab_sum(const float* slab, int P, int L, float* out, hipStream_t s) {
  hipLaunchKernelGGL(mlp_slab_sum_kernel, dim3((L + 63) / 64), dim3(1024), 0, s, slab, P, (int64_t)L, 0, L, 1, out,
                     nullptr, nullptr, nullptr);
}

void launch_mlp_slab_sum4(const float* slab, int P, int L, float* o0, float* o1, float* o2, float* o3, hipStream_t s) {
  hipLaunchKernelGGL(mlp_slab_sum_kernel, dim3((4 * L + 63) / 64), dim3(1024), 0, s, slab, P, (int64_t)4 * L, 0, L, 4,
                     o0, o1, o2, o3);
}

void launch_mlp_slab_sum_cols(const float* slab, int P, int64_t stride, int col0, int L, float* out, hipStream_t s) {
  hipLaunchKernelGGL(mlp_slab_sum_kernel, dim3((L + 63) / 64), dim3(1024), 0, s, slab, P, stride, col0, L, 1, out,
                     nullptr, nullptr, nullptr);
}

// ---- GAN discriminator update with in-kernel gradients (both dtypes) ----
void launch_mlp_gan_critic_g(int dt, const void* x, const MlpCritic& cr, float label, float* gslab, float* slab,
                             int64_t M, int F, hipStream_t s) {
  if (M <= 0) return;
  if (dt == DT_F32 && !fp32_exact_mode()) {  // fp32 on the split bf16 products (images: 108 / 117 KB)
    MLP_DISPATCH(dt, F, {
      auto k = mlp_gan_critic_g_kernel<float, FF, 100, f32s_t>;
      constexpr size_t lds =
          (size_t)(fwd_entries<f32s_t, FF, 100>() + fwd_entries<f32s_t, 100, 100>()) * frag_bytes<f32s_t>() + 3 * VEC * 4;
      static_assert(lds <= 160 * 1024, "split discriminator images exceed LDS");
      set_lds(k, lds);
      hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const float*)x, cr, label, gslab,
                         slab, M, 1.f / (float)M);
    });
    return;
  }
  MLP_DISPATCH(dt, F, {
    auto k = mlp_gan_critic_g_kernel<T, FF, 100>;
    constexpr size_t lds = (size_t)(fwd_entries<T, FF, 100>() + fwd_entries<T, 100, 100>()) * frag_bytes<T>() +
                           3 * VEC * 4;
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(slab_grid(k, lds, M)), dim3(MLP_THREADS), lds, s, (const T*)x, cr, label, gslab, slab, M,
                       1.f / (float)M);
  });
}

void launch_mlp_gan_grad_finish(const float* v, const MlpCritic& cr, int F, int H, float* gW1, float* gb1, float* gW2,
                                float* gb2, float* gw3, float* gb3, hipStream_t s) {
  hipLaunchKernelGGL(mlp_gan_grad_finish_kernel, dim3(1), dim3(256), 0, s, v, cr, F, H, gW1, gb1, gW2, gb2, gw3, gb3);
}

// ---- GP critic update with per-t column-sum gradients (fp32 / bf16) ----
int mlp_wgpt_waves_per_t(int Tn) { return std::max(1, device_cu_count() * 2 * MLP_WAVES / std::max(1, Tn)); }
int mlp_wgpt_blocks(int Tn) { return (mlp_wgpt_waves_per_t(Tn) * Tn + MLP_WAVES - 1) / MLP_WAVES; }
size_t mlp_wgpt_tsum_floats(int F, int Tn) { return (size_t)Tn * (F + 3 * 100); }

void launch_mlp_wgp_critic_t(int dt, const void* real, const void* fake, const float* c, const MlpCritic& cr,
                             float* tslab, float* tsum, float* slab, int64_t Bn, int Tn, int F, float* gW1, float* gW2,
                             float* gw3, hipStream_t s) {
  if (Bn <= 0) return;
  const int kper = mlp_wgpt_waves_per_t(Tn), P = mlp_wgpt_blocks(Tn);
  const float invB = 1.f / (float)Bn;
  MLP_DISPATCH(dt, F, {
    auto k = mlp_wgp_critic_t_kernel<T, FF, 100>;
    constexpr size_t lds = lds_critic4<T, FF, 100>();
    set_lds(k, lds);
    hipLaunchKernelGGL(k, dim3(P), dim3(MLP_THREADS), lds, s, (const T*)real, (const T*)fake, c, cr, tslab, slab, Bn, Tn,
                       kper, invB);
  });
  const int H = 100, L = F + 2 * H;
  const int np = Tn * (L + H), nf = F * H + H * H + Tn * H;
  hipLaunchKernelGGL(mlp_wgp_tsum_prep_kernel, dim3((np + 255) / 256), dim3(256), 0, s, tslab, cr, F, H, Tn, kper, tsum);
  hipLaunchKernelGGL(mlp_wgp_tsum_finish_kernel, dim3((nf + 255) / 256), dim3(256), 0, s, tsum, cr, F, H, Tn, gW1, gW2,
                     gw3);
}

// ---- the affine critic's update from batch sums (both dtypes) ----
// the finish kernel keeps W1, W2, w3 and its per-t tables in LDS
static constexpr int kAffineLdsMax = 160 * 1024 - 1024;
bool mlp_affine_supported(int F, int Tn) {
  return mlp_supported(F, 100) && Tn > 0 && (Tn * F) % 8 == 0 &&
         mlp_affine_lds_floats(F, 100, Tn) * sizeof(float) <= (size_t)kAffineLdsMax;
}

// row partitions of mlp_bt_colsum over the C / V column groups: ~1024 threads per CU for bf16, 512 for
// fp32 (measured on config 4: bf16 206 -> 140 us per call at 1024, 2048 no better; fp32 best at 512;
// profiles/r06_affine/colsum_ab)
static int colsum_parts(int dt, int64_t B, int C) {
  const int V = dt == DT_BF16 ? 8 : 4, G = C / V, tpc = dt == DT_BF16 ? 1024 : 512;
  const int64_t want = ((int64_t)device_cu_count() * tpc + G - 1) / G;
  return (int)std::max<int64_t>(1, std::min<int64_t>(B, want));
}
size_t mlp_affine_ws_floats(int dt, int64_t Bn, int Tn, int F) {
  const int H = 100, C = Tn * F;
  // part | sums | tsum (S rows + D) | g   (mode 1 needs less: part | sums | D | g | gdx)
  return (size_t)colsum_parts(dt, Bn, C) * 2 * C + 2 * (size_t)C + (size_t)Tn * (F + 3 * H) + (size_t)Tn * F;
}
// sums[k][col] = sum_b y_k[b][col] (y_0 = x0, y_1 = x1 - x0), fixed order
static void bt_colsum(int dt, const void* x0, const void* x1, int64_t B, int C, float* part, float* sums, hipStream_t s) {
  const int P = colsum_parts(dt, B, C), V = dt == DT_BF16 ? 8 : 4, nk = x1 ? 2 : 1;
  const int grid = (int)(((int64_t)(C / V) * P + 255) / 256);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(mlp_bt_colsum_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x0, (const bf16_t*)x1, B,
                       C, P, part);
  else
    hipLaunchKernelGGL(mlp_bt_colsum_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x0, (const float*)x1, B, C,
                       P, part);
  (void)hipMemsetAsync(sums, 0, sizeof(float) * nk * C, s);
  launch_mlp_slab_sum_cols(part, P, (int64_t)nk * C, 0, nk * C, sums, s);
}

void launch_mlp_wgp_affine(int dt, const void* real, const void* fake, const MlpCritic& cr, int64_t Bn, int Tn, int F,
                           float lam, float* ws, float* slab, float* e, float* gW1, float* gW2, float* gw3, hipStream_t s) {
  if (Bn <= 0) return;
  const int H = 100, C = Tn * F, L = F + 2 * H;
  float* part = ws;
  float* sums = part + (size_t)colsum_parts(dt, Bn, C) * 2 * C;
  float* tsum = sums + 2 * C;
  float* g = tsum + (size_t)Tn * (L + H);
  (void)g;
  bt_colsum(dt, real, fake, Bn, C, part, sums, s);
  const size_t lds = mlp_affine_lds_floats(F, H, Tn) * sizeof(float);
  set_lds(mlp_wgp_affine_kernel, lds);
  hipLaunchKernelGGL(mlp_wgp_affine_kernel, dim3(1), dim3(1024), lds, s, sums, cr, F, H, Tn, (float)Bn, lam, 0,
                     tsum + (size_t)Tn * L, tsum, slab, e, (float*)nullptr);
  const int nf = F * H + H * H + Tn * H;
  hipLaunchKernelGGL(mlp_wgp_tsum_finish_kernel, dim3((nf + 255) / 256), dim3(256), 0, s, tsum, cr, F, H, Tn, gW1, gW2,
                     gw3);
}

void launch_mlp_critic_dx_affine(int dt, const void* fake, const MlpCritic& cr, int64_t Bn, int Tn, int F, float* ws,
                                 float* slab, void* dx, hipStream_t s) {
  if (Bn <= 0) return;
  const int H = 100, C = Tn * F;
  float* part = ws;
  float* sums = part + (size_t)colsum_parts(dt, Bn, C) * C;
  float* D = sums + C;
  float* g = D + (size_t)Tn * H;
  float* gdx = g + (size_t)Tn * F;
  (void)D; (void)g;
  bt_colsum(dt, fake, nullptr, Bn, C, part, sums, s);
  const size_t lds = mlp_affine_lds_floats(F, H, Tn) * sizeof(float);
  set_lds(mlp_wgp_affine_kernel, lds);
  hipLaunchKernelGGL(mlp_wgp_affine_kernel, dim3(1), dim3(1024), lds, s, sums, cr, F, H, Tn, (float)Bn, 0.f, 1,
                     (float*)nullptr, (float*)nullptr, slab, (float*)nullptr, gdx);
  const int P = colsum_parts(dt, Bn, C), V = dt == DT_BF16 ? 8 : 4;
  const int grid = (int)(((int64_t)(C / V) * P + 255) / 256);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(mlp_bcast_rows_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, gdx, C, Bn, P, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(mlp_bcast_rows_kernel<float>, dim3(grid), dim3(256), 0, s, gdx, C, Bn, P, (float*)dx);
}

// ---- generator reverse with in-kernel parameter gradients (bf16) ----
int mlp_gbw_blocks(int64_t M) { return mlp_wgpw_blocks(M); }

void launch_mlp_gen_bwd_w(const void* noise, const void* dfake, const MlpGen& g, float* gslab, float* lnslab, int64_t M,
                          int F, hipStream_t s) {
  if (M <= 0) return;
  const int P = mlp_gbw_blocks(M);
  auto go = [&](auto kern, size_t lds) {
    set_lds(kern, lds);
    hipLaunchKernelGGL(kern, dim3(P), dim3(MLP_THREADS), lds, s, (const bf16_t*)noise, (const bf16_t*)dfake, g, gslab,
                       lnslab, M);
  };
  if (F == 32) go(mlp_gen_bwd_w_kernel<32, 100>, gbw_lds<32, 100>());
  else if (F == 36) go(mlp_gen_bwd_w_kernel<36, 100>, gbw_lds<36, 100>());
  else throw std::runtime_error("mlp_gen_bwd_w: F in {32, 36}");
}

// ---- GP critic update with in-kernel weight gradients (bf16) ----
bool mlp_wgpw_supported(int F, int Tn) {
  if (Tn < 1 || Tn > 64 || !(F == 32 || F == 36)) return false;
  const size_t lds = F == 32 ? wgpw_lds<32, 100>(Tn) : wgpw_lds<36, 100>(Tn);
  return lds <= 160 * 1024;
}

int mlp_wgpw_blocks(int64_t M) {
  const int64_t nbt = (M + 127) / 128;
  return (int)std::max<int64_t>(1, std::min<int64_t>(nbt, (int64_t)device_cu_count()));
}

void launch_mlp_wgp_critic_w(const void* real, const void* fake, const float* c, const MlpCritic& cr, float* gslab,
                             float* slab, int64_t M, int Tn, int F, hipStream_t s) {
  if (M <= 0) return;
  if (!mlp_wgpw_supported(F, Tn))
    throw std::runtime_error("mlp_wgp_critic_w: (F, T) outside the in-kernel weight-gradient variant");
  const float invB = (float)Tn / (float)M;
  const int P = mlp_wgpw_blocks(M);
  auto go = [&](auto kern, size_t lds) {
    set_lds(kern, lds);
    hipLaunchKernelGGL(kern, dim3(P), dim3(MLP_THREADS), lds, s, (const bf16_t*)real, (const bf16_t*)fake, c, cr, gslab,
                       slab, M, Tn, invB);
  };
  if (F == 32) {
    if (Tn <= 32) go(mlp_wgp_critic_w_kernel<32, 100, 1>, wgpw_lds<32, 100>(Tn));
    else go(mlp_wgp_critic_w_kernel<32, 100, 2>, wgpw_lds<32, 100>(Tn));
  } else {  // F = 36: the LDS plan leaves room for T <= 27 tables only (one t tile)
    go(mlp_wgp_critic_w_kernel<36, 100, 1>, wgpw_lds<36, 100>(Tn));
  }
}

}  // namespace hfrep
