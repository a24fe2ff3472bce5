// Persistent LSTM recurrence kernels for gfx950: forward, BPTT, tangent forward, tangent reverse.
//
// Keras LSTM semantics (implementation 2, gate order [i, f, c, o], recurrent activation sigmoid,
// cell activation act in {tanh, sigmoid, linear}); see GAN/MTSS_WGAN_GP.py:224-243 for the models.
// Each workgroup owns 32 batch rows for ALL T steps (one launch per layer and direction):
//
//   * one wave per 32-unit tile (H=100 -> 4 waves, 256 threads); the wave keeps its slice of the
//     recurrent kernel U (H x 4H) -- all four gates -- resident in REGISTERS as MFMA B fragments,
//     so the per-step recurrent GEMM reads nothing from memory except the previous state;
//   * the previous state h_{t-1} (or dz_{t+1} in the reverse kernels) lives in LDS, double
//     buffered, as the MFMA A operand, padded so the fragment reads are bank-conflict free;
//   * the four gate accumulators of a (row, unit) land in the SAME lane (the 32x32 accumulator puts
//     the unit on the lane and rows in registers), so gate math, the cell state c (kept in
//     registers for all T) and the stores are lane-local: no shuffles, no extra LDS traffic.
//
// The tangent kernels implement d/dtheta <v, dD/dx> for the WGAN-GP critic as reverse-over-
// tangent (see ops/reference.py lstm_seq_tfwd / lstm_seq_tbwd for the exact contracts).
#include "common.h"
#include "mfma.h"
#include "kernels.h"

namespace hfrep {

template <int H>
constexpr int lstm_threads = ((H + 31) / 32) * 64;

template <typename T, int H>
struct LstmGeom {
  using P = MF<T>;
  static constexpr int NW = (H + 31) / 32;                 // waves per WG (unit tiles)
  static constexpr int G = 4 * H;
  static constexpr int NKH = (H + P::KS - 1) / P::KS;      // k-steps over H   (h . U)
  static constexpr int NKG = (G + P::KS - 1) / P::KS;      // k-steps over 4H  (dz . U^T)
  static constexpr int LH = NKH * P::KS + P::LDS_PAD;      // LDS row length for h tiles
  static constexpr int LG = NKG * P::KS + P::LDS_PAD;      // LDS row length for dz tiles
  static constexpr int THREADS = NW * 64;
};

// ------------------------------------------------------------------------------------------
// forward:  z_t = zx_t + h_{t-1} U ;  gates ; c_t ; h_t
// ------------------------------------------------------------------------------------------
template <typename T, int H>
__global__ void __launch_bounds__(lstm_threads<H>)
lstm_fwd_kernel(const T* __restrict__ zx, const float* __restrict__ U, T* __restrict__ hs, T* __restrict__ gates,
                T* __restrict__ cs, int B, int Tn, int act) {
  using Gm = LstmGeom<T, H>;
  using P = MF<T>;
  constexpr int G = Gm::G, NKH = Gm::NKH, LH = Gm::LH, KPAD = NKH * P::KS;
  __shared__ __attribute__((aligned(16))) T hb[2][32 * LH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int row0 = blockIdx.x * 32;

  typename P::frag ub[4][NKH];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks)
      ub[q][ks] = P::make([&](int k) { return (uok && k < H) ? U[k * G + q * H + u] : 0.f; }, ks, lane);

  for (int i = threadIdx.x; i < 2 * 32 * LH; i += blockDim.x) (&hb[0][0])[i] = Cvt<T>::from_f(0.f);
  float c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  __syncthreads();

  for (int t = 0; t < Tn; ++t) {
    const T* arow = hb[t & 1] + (lane & 31) * LH;
    T* hn = hb[(t + 1) & 1];
    f32x16 acc[4];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + acc32_row(r, lane);
      const bool ok = uok && row < B;
      const size_t b4 = ((size_t)row * Tn + t) * G + u;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q][r] = ok ? ld_f(zx + b4 + q * H) : 0.f;
    }
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks) {
      const typename P::frag a = P::lda(arow, ks, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = P::mma(a, ub[q][ks], acc[q]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc32_row(r, lane);
      const int row = row0 + rr;
      const float ig = sigmoidf_(acc[0][r]), fg = sigmoidf_(acc[1][r]);
      const float gg = act_f(act, acc[2][r]), og = sigmoidf_(acc[3][r]);
      float cn = fg * c[r] + ig * gg;
      float h = og * act_f(act, cn);
      if (!uok) { cn = 0.f; h = 0.f; }
      c[r] = cn;
      if (u < KPAD) hn[rr * LH + u] = Cvt<T>::from_f(h);
      if (uok && row < B) {
        const size_t b1 = ((size_t)row * Tn + t) * H + u;
        st_f(hs + b1, h);
        if (gates) {
          const size_t b4 = ((size_t)row * Tn + t) * G + u;
          st_f(gates + b4, ig);
          st_f(gates + b4 + H, fg);
          st_f(gates + b4 + 2 * H, gg);
          st_f(gates + b4 + 3 * H, og);
        }
        if (cs) st_f(cs + b1, cn);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// BPTT: dZ_t = dL/dz_t given dH (adjoint of every h_t) and the saved gates / cells
// ------------------------------------------------------------------------------------------
template <typename T, int H>
__global__ void __launch_bounds__(lstm_threads<H>)
lstm_bwd_kernel(const T* __restrict__ dH, const T* __restrict__ gates, const T* __restrict__ cs,
                const float* __restrict__ U, T* __restrict__ dZ, int B, int Tn, int act) {
  using Gm = LstmGeom<T, H>;
  using P = MF<T>;
  constexpr int G = Gm::G, NKG = Gm::NKG, LG = Gm::LG;
  __shared__ __attribute__((aligned(16))) T zb[2][32 * LG];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int row0 = blockIdx.x * 32;

  typename P::frag ut[NKG];  // B[k][n] = U[n][k]  (U^T), n = this lane's unit
#pragma unroll
  for (int ks = 0; ks < NKG; ++ks)
    ut[ks] = P::make([&](int k) { return (uok && k < G) ? U[u * G + k] : 0.f; }, ks, lane);

  for (int i = threadIdx.x; i < 2 * 32 * LG; i += blockDim.x) (&zb[0][0])[i] = Cvt<T>::from_f(0.f);
  float dc[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) dc[r] = 0.f;
  __syncthreads();

  for (int t = Tn - 1; t >= 0; --t) {
    const int rb = t & 1, wb = rb ^ 1;
    f32x16 acc = zero16();
    if (t < Tn - 1) {
      const T* arow = zb[rb] + (lane & 31) * LG;
#pragma unroll
      for (int ks = 0; ks < NKG; ++ks) acc = P::mma(P::lda(arow, ks, lane), ut[ks], acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc32_row(r, lane);
      const int row = row0 + rr;
      float dz0 = 0.f, dz1 = 0.f, dz2 = 0.f, dz3 = 0.f;
      if (uok && row < B) {
        const size_t b1 = ((size_t)row * Tn + t) * H + u;
        const size_t b4 = ((size_t)row * Tn + t) * G + u;
        const float ig = ld_f(gates + b4), fg = ld_f(gates + b4 + H);
        const float gg = ld_f(gates + b4 + 2 * H), og = ld_f(gates + b4 + 3 * H);
        const float c = ld_f(cs + b1);
        const float cp = t > 0 ? ld_f(cs + b1 - H) : 0.f;
        const float dht = (dH ? ld_f(dH + b1) : 0.f) + acc[r];
        const float ca = act_f(act, c);
        const float dov = dht * ca;
        const float dct = dc[r] + dht * og * act_dy(act, ca);
        dc[r] = dct * fg;
        dz0 = dct * gg * ig * (1.f - ig);
        dz1 = dct * cp * fg * (1.f - fg);
        dz2 = dct * ig * act_dy(act, gg);
        dz3 = dov * og * (1.f - og);
        st_f(dZ + b4, dz0);
        st_f(dZ + b4 + H, dz1);
        st_f(dZ + b4 + 2 * H, dz2);
        st_f(dZ + b4 + 3 * H, dz3);
      }
      if (uok) {
        T* zr = zb[wb] + rr * LG + u;
        zr[0] = Cvt<T>::from_f(dz0);
        zr[H] = Cvt<T>::from_f(dz1);
        zr[2 * H] = Cvt<T>::from_f(dz2);
        zr[3 * H] = Cvt<T>::from_f(dz3);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// tangent forward at a saved primal point:  zdot_t = dzx_t + hdot_{t-1} U
// ------------------------------------------------------------------------------------------
template <typename T, int H>
__global__ void __launch_bounds__(lstm_threads<H>)
lstm_tfwd_kernel(const T* __restrict__ dzx, const T* __restrict__ gates, const T* __restrict__ cs,
                 const float* __restrict__ U, T* __restrict__ hds, T* __restrict__ zds, T* __restrict__ cds, int B,
                 int Tn, int act) {
  using Gm = LstmGeom<T, H>;
  using P = MF<T>;
  constexpr int G = Gm::G, NKH = Gm::NKH, LH = Gm::LH, KPAD = NKH * P::KS;
  __shared__ __attribute__((aligned(16))) T hb[2][32 * LH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int row0 = blockIdx.x * 32;

  typename P::frag ub[4][NKH];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks)
      ub[q][ks] = P::make([&](int k) { return (uok && k < H) ? U[k * G + q * H + u] : 0.f; }, ks, lane);

  for (int i = threadIdx.x; i < 2 * 32 * LH; i += blockDim.x) (&hb[0][0])[i] = Cvt<T>::from_f(0.f);
  float cd[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) cd[r] = 0.f;
  __syncthreads();

  for (int t = 0; t < Tn; ++t) {
    const T* arow = hb[t & 1] + (lane & 31) * LH;
    T* hn = hb[(t + 1) & 1];
    f32x16 acc[4];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + acc32_row(r, lane);
      const bool ok = uok && row < B;
      const size_t b4 = ((size_t)row * Tn + t) * G + u;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q][r] = ok ? ld_f(dzx + b4 + q * H) : 0.f;
    }
#pragma unroll
    for (int ks = 0; ks < NKH; ++ks) {
      const typename P::frag a = P::lda(arow, ks, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = P::mma(a, ub[q][ks], acc[q]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc32_row(r, lane);
      const int row = row0 + rr;
      float hd = 0.f;
      if (uok && row < B) {
        const size_t b1 = ((size_t)row * Tn + t) * H + u;
        const size_t b4 = ((size_t)row * Tn + t) * G + u;
        const float ig = ld_f(gates + b4), fg = ld_f(gates + b4 + H);
        const float gg = ld_f(gates + b4 + 2 * H), og = ld_f(gates + b4 + 3 * H);
        const float c = ld_f(cs + b1);
        const float cp = t > 0 ? ld_f(cs + b1 - H) : 0.f;
        const float idot = ig * (1.f - ig) * acc[0][r];
        const float fdot = fg * (1.f - fg) * acc[1][r];
        const float gdot = act_dy(act, gg) * acc[2][r];
        const float odot = og * (1.f - og) * acc[3][r];
        const float cdn = fdot * cp + fg * cd[r] + idot * gg + ig * gdot;
        cd[r] = cdn;
        const float ca = act_f(act, c);
        hd = odot * ca + og * act_dy(act, ca) * cdn;
        st_f(hds + b1, hd);
        st_f(cds + b1, cdn);
        st_f(zds + b4, acc[0][r]);
        st_f(zds + b4 + H, acc[1][r]);
        st_f(zds + b4 + 2 * H, acc[2][r]);
        st_f(zds + b4 + 3 * H, acc[3][r]);
      }
      if (u < KPAD) hn[rr * LH + u] = Cvt<T>::from_f(hd);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// reverse of the tangent system: adjoints (dZ, dZdot) from (dH, dHdot) and the saved tapes
// ------------------------------------------------------------------------------------------
template <typename T, int H, int NB>
__global__ void __launch_bounds__(lstm_threads<H>)
lstm_tbwd_kernel(const T* __restrict__ dH, const T* __restrict__ dHd, const T* __restrict__ gates,
                 const T* __restrict__ cs, const T* __restrict__ zds, const T* __restrict__ cds,
                 const float* __restrict__ U, T* __restrict__ dZ, T* __restrict__ dZd, int B, int Tn, int act) {
  using Gm = LstmGeom<T, H>;
  using P = MF<T>;
  constexpr int G = Gm::G, NKG = Gm::NKG, LG = Gm::LG;
  __shared__ __attribute__((aligned(16))) T zb[NB][32 * LG];
  __shared__ __attribute__((aligned(16))) T zdb[NB][32 * LG];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int u = w * 32 + (lane & 31);
  const bool uok = u < H;
  const int row0 = blockIdx.x * 32;

  typename P::frag ut[NKG];
#pragma unroll
  for (int ks = 0; ks < NKG; ++ks)
    ut[ks] = P::make([&](int k) { return (uok && k < G) ? U[u * G + k] : 0.f; }, ks, lane);

  for (int i = threadIdx.x; i < NB * 32 * LG; i += blockDim.x) {
    (&zb[0][0])[i] = Cvt<T>::from_f(0.f);
    (&zdb[0][0])[i] = Cvt<T>::from_f(0.f);
  }
  float ac[16], acd[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) { ac[r] = 0.f; acd[r] = 0.f; }
  __syncthreads();

  for (int t = Tn - 1; t >= 0; --t) {
    const int rb = (NB == 2) ? (t & 1) : 0, wb = (NB == 2) ? (rb ^ 1) : 0;
    f32x16 ah = zero16(), ahd = zero16();
    if (t < Tn - 1) {
      const T* arow = zb[rb] + (lane & 31) * LG;
      const T* drow = zdb[rb] + (lane & 31) * LG;
#pragma unroll
      for (int ks = 0; ks < NKG; ++ks) {
        ah = P::mma(P::lda(arow, ks, lane), ut[ks], ah);
        ahd = P::mma(P::lda(drow, ks, lane), ut[ks], ahd);
      }
    }
    if (NB == 1) __syncthreads();  // single buffer: every wave has read before anyone overwrites
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = acc32_row(r, lane);
      const int row = row0 + rr;
      float z0 = 0.f, z1 = 0.f, z2 = 0.f, z3 = 0.f, d0 = 0.f, d1v = 0.f, d2v = 0.f, d3 = 0.f;
      if (uok && row < B) {
        const size_t b1 = ((size_t)row * Tn + t) * H + u;
        const size_t b4 = ((size_t)row * Tn + t) * G + u;
        const float ig = ld_f(gates + b4), fg = ld_f(gates + b4 + H);
        const float gg = ld_f(gates + b4 + 2 * H), og = ld_f(gates + b4 + 3 * H);
        const float c = ld_f(cs + b1);
        const float cp = t > 0 ? ld_f(cs + b1 - H) : 0.f;
        const float cd = ld_f(cds + b1);
        const float cdp = t > 0 ? ld_f(cds + b1 - H) : 0.f;
        const float zdi = ld_f(zds + b4), zdf = ld_f(zds + b4 + H);
        const float zdg = ld_f(zds + b4 + 2 * H), zdo = ld_f(zds + b4 + 3 * H);
        const float si = ig * (1.f - ig), sf = fg * (1.f - fg), so = og * (1.f - og);
        const float sg = act_dy(act, gg);
        const float idot = si * zdi, fdot = sf * zdf, gdot = sg * zdg, odot = so * zdo;
        const float ca = act_f(act, c);
        const float e1 = act_dy(act, ca), e2 = act_d2y(act, ca);
        const float a_h = (dH ? ld_f(dH + b1) : 0.f) + ah[r];
        const float a_hd = ld_f(dHd + b1) + ahd[r];
        const float a_od = a_hd * ca;
        const float a_o = a_h * ca + a_hd * e1 * cd;
        const float a_cd = acd[r] + a_hd * og * e1;
        const float a_c = ac[r] + a_h * og * e1 + a_hd * (odot * e1 + og * e2 * cd);
        const float a_fd = a_cd * cp, a_id = a_cd * gg, a_gd = a_cd * ig;
        const float a_f = a_c * cp + a_cd * cdp;
        const float a_i = a_c * gg + a_cd * gdot;
        const float a_g = a_c * ig + a_cd * idot;
        ac[r] = a_c * fg + a_cd * fdot;
        acd[r] = a_cd * fg;
        const float s2i = si * (1.f - 2.f * ig), s2f = sf * (1.f - 2.f * fg), s2o = so * (1.f - 2.f * og);
        const float s2g = act_d2y(act, gg);
        d0 = a_id * si; d1v = a_fd * sf; d2v = a_gd * sg; d3 = a_od * so;
        z0 = a_i * si + a_id * s2i * zdi;
        z1 = a_f * sf + a_fd * s2f * zdf;
        z2 = a_g * sg + a_gd * s2g * zdg;
        z3 = a_o * so + a_od * s2o * zdo;
        st_f(dZ + b4, z0); st_f(dZ + b4 + H, z1); st_f(dZ + b4 + 2 * H, z2); st_f(dZ + b4 + 3 * H, z3);
        st_f(dZd + b4, d0); st_f(dZd + b4 + H, d1v); st_f(dZd + b4 + 2 * H, d2v); st_f(dZd + b4 + 3 * H, d3);
      }
      if (uok) {
        T* zr = zb[wb] + rr * LG + u;
        T* dr = zdb[wb] + rr * LG + u;
        zr[0] = Cvt<T>::from_f(z0); zr[H] = Cvt<T>::from_f(z1); zr[2 * H] = Cvt<T>::from_f(z2); zr[3 * H] = Cvt<T>::from_f(z3);
        dr[0] = Cvt<T>::from_f(d0); dr[H] = Cvt<T>::from_f(d1v); dr[2 * H] = Cvt<T>::from_f(d2v); dr[3 * H] = Cvt<T>::from_f(d3);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// host dispatch
// ------------------------------------------------------------------------------------------
#define HFREP_LSTM_H_LIST(X) X(100) X(64) X(32)

template <typename T>
static bool lstm_fwd_dispatch(const void* zx, const float* U, void* hs, void* gates, void* cs, int B, int Tn, int H,
                              int act, hipStream_t s) {
  const dim3 grid((B + 31) / 32);
#define CASE(HH)                                                                                                  \
  if (H == HH) {                                                                                                  \
    hipLaunchKernelGGL((lstm_fwd_kernel<T, HH>), grid, dim3(LstmGeom<T, HH>::THREADS), 0, s, (const T*)zx, U,    \
                       (T*)hs, (T*)gates, (T*)cs, B, Tn, act);                                                     \
    return true;                                                                                                  \
  }
  HFREP_LSTM_H_LIST(CASE)
#undef CASE
  return false;
}

template <typename T>
static bool lstm_bwd_dispatch(const void* dH, const void* gates, const void* cs, const float* U, void* dZ, int B,
                              int Tn, int H, int act, hipStream_t s) {
  const dim3 grid((B + 31) / 32);
#define CASE(HH)                                                                                               \
  if (H == HH) {                                                                                               \
    hipLaunchKernelGGL((lstm_bwd_kernel<T, HH>), grid, dim3(LstmGeom<T, HH>::THREADS), 0, s, (const T*)dH,    \
                       (const T*)gates, (const T*)cs, U, (T*)dZ, B, Tn, act);                                   \
    return true;                                                                                               \
  }
  HFREP_LSTM_H_LIST(CASE)
#undef CASE
  return false;
}

template <typename T>
static bool lstm_tfwd_dispatch(const void* dzx, const void* gates, const void* cs, const float* U, void* hds,
                               void* zds, void* cds, int B, int Tn, int H, int act, hipStream_t s) {
  const dim3 grid((B + 31) / 32);
#define CASE(HH)                                                                                                 \
  if (H == HH) {                                                                                                 \
    hipLaunchKernelGGL((lstm_tfwd_kernel<T, HH>), grid, dim3(LstmGeom<T, HH>::THREADS), 0, s, (const T*)dzx,    \
                       (const T*)gates, (const T*)cs, U, (T*)hds, (T*)zds, (T*)cds, B, Tn, act);                  \
    return true;                                                                                                 \
  }
  HFREP_LSTM_H_LIST(CASE)
#undef CASE
  return false;
}

template <typename T>
static bool lstm_tbwd_dispatch(const void* dH, const void* dHd, const void* gates, const void* cs, const void* zds,
                               const void* cds, const float* U, void* dZ, void* dZd, int B, int Tn, int H, int act,
                               hipStream_t s) {
  const dim3 grid((B + 31) / 32);
  // fp32 double buffers would need 2 x 2 x 51 KB of LDS for H=100: single-buffer there
  constexpr int NB = sizeof(T) == 2 ? 2 : 1;
#define CASE(HH)                                                                                                  \
  if (H == HH) {                                                                                                  \
    hipLaunchKernelGGL((lstm_tbwd_kernel<T, HH, NB>), grid, dim3(LstmGeom<T, HH>::THREADS), 0, s, (const T*)dH, \
                       (const T*)dHd, (const T*)gates, (const T*)cs, (const T*)zds, (const T*)cds, U, (T*)dZ,     \
                       (T*)dZd, B, Tn, act);                                                                      \
    return true;                                                                                                  \
  }
  HFREP_LSTM_H_LIST(CASE)
#undef CASE
  return false;
}

bool launch_lstm_fwd(int dt, const void* zx, const float* U, void* hs, void* gates, void* cs, int B, int Tn, int H,
                     int act, hipStream_t s) {
  return dt == DT_BF16 ? lstm_fwd_dispatch<bf16_t>(zx, U, hs, gates, cs, B, Tn, H, act, s)
                       : lstm_fwd_dispatch<float>(zx, U, hs, gates, cs, B, Tn, H, act, s);
}
bool launch_lstm_bwd(int dt, const void* dH, const void* gates, const void* cs, const float* U, void* dZ, int B,
                     int Tn, int H, int act, hipStream_t s) {
  return dt == DT_BF16 ? lstm_bwd_dispatch<bf16_t>(dH, gates, cs, U, dZ, B, Tn, H, act, s)
                       : lstm_bwd_dispatch<float>(dH, gates, cs, U, dZ, B, Tn, H, act, s);
}
bool launch_lstm_tfwd(int dt, const void* dzx, const void* gates, const void* cs, const float* U, void* hds,
                      void* zds, void* cds, int B, int Tn, int H, int act, hipStream_t s) {
  return dt == DT_BF16 ? lstm_tfwd_dispatch<bf16_t>(dzx, gates, cs, U, hds, zds, cds, B, Tn, H, act, s)
                       : lstm_tfwd_dispatch<float>(dzx, gates, cs, U, hds, zds, cds, B, Tn, H, act, s);
}
bool launch_lstm_tbwd(int dt, const void* dH, const void* dHd, const void* gates, const void* cs, const void* zds,
                      const void* cds, const float* U, void* dZ, void* dZd, int B, int Tn, int H, int act,
                      hipStream_t s) {
  return dt == DT_BF16 ? lstm_tbwd_dispatch<bf16_t>(dH, dHd, gates, cs, zds, cds, U, dZ, dZd, B, Tn, H, act, s)
                       : lstm_tbwd_dispatch<float>(dH, dHd, gates, cs, zds, cds, U, dZ, dZd, B, Tn, H, act, s);
}

}  // namespace hfrep
