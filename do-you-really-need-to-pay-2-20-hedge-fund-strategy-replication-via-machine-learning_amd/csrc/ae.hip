// Factor-autoencoder training in ONE launch (gfx950): the whole Keras `fit` of
// Autoencoder_encapsulate.py:72-105 -- MSE loss, Nadam, batch 48, the last 25 % of rows as the
// validation set, EarlyStopping(val_loss, patience) -- runs inside one persistent workgroup, and a
// launch carries any number of independent fits (one workgroup each: a whole latent sweep, or every
// (seed, latent) pair of a study, trains side by side across the CUs).
//
// The model is tiny (22 -> k -> 22, no bias, k <= 21: <= 924 weights) and one epoch is 3 batches of
// <= 48 rows, so the eager engine was launch-bound: ~15 kernel launches and a loss copy per batch
// (gather, two Dense + LeakyReLU forwards, the MSE value and gradient in torch elementwise kernels,
// the reverse pass, Nadam, the step counter) and a host sync per epoch for the EarlyStopping
// decision.  Here every epoch, batch and decision stays on the CU: the batch is gathered into LDS by
// the host-drawn permutation (numpy RandomState, the same draws as the eager trainer), the forward,
// the fused MSE value + gradient, the reverse pass and the Keras 2.7 Nadam update (momentum-cache
// schedule, optim.hip's formula) run between workgroup barriers, the validation loss is a fixed-order
// fp64 reduction, and EarlyStopping is decided by thread 0.  The per-epoch train / validation losses
// go to a history buffer, the number of epochs run to a counter.
//
// Numerics follow the explicit engine (models/autoencoder.py): with BF = true every activation is
// rounded to bf16 where the engine stores a bf16 tensor (inputs, Dense outputs, LeakyReLU outputs,
// y - x, the MSE gradient, the reverse-pass adjoints), products are exact bf16 x bf16 products summed
// in fp32 (the bf16 MFMA's arithmetic), and master weights, gradients and optimizer slots are fp32.
#include "common.h"
#include "kernels.h"

namespace hfrep {

namespace {

// (LDS: 5 activation tiles of 64 x 32 floats + 4 weight images of 32 x 32 = 56 KiB)
constexpr int AE_MAXA = 32, AE_MAXK = 32, AE_MAXB = 64, AE_THREADS = 256;

template <bool BF>
__device__ __forceinline__ float rnd(float v) {
  if constexpr (BF) return bf2f(f2bf(v));
  else return v;
}
__device__ __forceinline__ float lrelu(float x) { return x >= 0.f ? x : 0.2f * x; }
__device__ __forceinline__ float lrelu_dy(float y) { return y >= 0.f ? 1.f : 0.2f; }

// fixed-order block sum of one double per thread (tree over LDS): every thread gets the total
__device__ double block_sum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
#pragma unroll
  for (int s = AE_THREADS / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// z = lrelu(x W) for `nr` rows: x (nr, na) in LDS, W (na, nb) in LDS; out (nr, nb); pre-activation
// rounded to the activation dtype before the LeakyReLU (Dense then LeakyReLU layer)
template <bool BF>
__device__ __forceinline__ void dense_lrelu(const float* x, int na, const float* W, int nb, float* out, int nr) {
  for (int e = threadIdx.x; e < nr * nb; e += AE_THREADS) {
    const int r = e / nb, j = e - r * nb;
    float s = 0.f;
    for (int a = 0; a < na; ++a) s = fmaf(x[r * na + a], W[a * nb + j], s);
    out[e] = rnd<BF>(lrelu(rnd<BF>(s)));
  }
}

}  // namespace

template <bool BF>
__global__ void __launch_bounds__(AE_THREADS, 1)
ae_fit_kernel(const AeFitJob* __restrict__ jobs, int batch, float lr, float b1, float b2, float eps, int A) {
  // one workgroup per fit: every (latent size, seed, panel) of a study trains side by side, each on
  // its own CU (the fits are independent; their per-fit state lives in the job record)
  const AeFitJob& J = jobs[blockIdx.x];
  const float* __restrict__ Xt = J.Xt;
  const float* __restrict__ Xv = J.Xv;
  const int* __restrict__ order = J.order;
  float* __restrict__ We = J.We;
  float* __restrict__ Wd = J.Wd;
  float* __restrict__ mWe = J.mWe;
  float* __restrict__ vWe = J.vWe;
  float* __restrict__ mWd = J.mWd;
  float* __restrict__ vWd = J.vWd;
  float* __restrict__ step = J.step;
  float* __restrict__ m_cache = J.m_cache;
  double* __restrict__ hist = J.hist;
  int* __restrict__ nep = J.nep;
  const int nt = J.nt, nv = J.nv, epochs = J.epochs, patience = J.patience, k = J.k;
  static_assert(AE_MAXK <= AE_MAXA, "zb / dzb share the activation tile size");
  __shared__ float xb[AE_MAXB * AE_MAXA], zb[AE_MAXB * AE_MAXK], yb[AE_MAXB * AE_MAXA];
  __shared__ float dyb[AE_MAXB * AE_MAXA], dzb[AE_MAXB * AE_MAXK];
  __shared__ float we[AE_MAXA * AE_MAXK], wd[AE_MAXK * AE_MAXA];  // bf16-rounded copies in BF mode
  __shared__ float ge[AE_MAXA * AE_MAXK], gd[AE_MAXK * AE_MAXA];
  __shared__ double red[AE_THREADS];
  __shared__ int stop_flag;
  const int tid = threadIdx.x;
  const int nW = A * k;
  float st = step[0], mc = m_cache[0];  // (uniform: every thread tracks the shared counters)
  double best = 1e300;
  int wait = 0, ep = 0;
  for (; ep < epochs; ++ep) {
    double tot = 0.0;  // thread-partial of sum over batches of (batch loss * rows); only thread 0's is used
    const int* ord = order + (size_t)ep * nt;
    for (int s0 = 0; s0 < nt; s0 += batch) {
      const int nr = min(batch, nt - s0);
      // operands of this batch: the gathered rows and the weights as the MFMA sees them
      for (int e = tid; e < nr * A; e += AE_THREADS) {
        const int r = e / A, a = e - r * A;
        xb[e] = rnd<BF>(Xt[(size_t)ord[s0 + r] * A + a]);
      }
      for (int e = tid; e < nW; e += AE_THREADS) {
        we[e] = rnd<BF>(We[e]);
        wd[e] = rnd<BF>(Wd[e]);
      }
      __syncthreads();
      dense_lrelu<BF>(xb, A, we, k, zb, nr);
      __syncthreads();
      dense_lrelu<BF>(zb, k, wd, A, yb, nr);
      __syncthreads();
      // fused MSE value + gradient: loss = mean((y - x)^2), dL/dy = 2 (y - x) / n, times the LeakyReLU
      // slope (the adjoint of the decoder's pre-activation)
      double part = 0.0;
      const float gs = 2.f / (float)(nr * A);
      for (int e = tid; e < nr * A; e += AE_THREADS) {
        const float d = rnd<BF>(yb[e] - xb[e]);
        part += (double)d * (double)d;
        dyb[e] = rnd<BF>(rnd<BF>(gs * d) * lrelu_dy(yb[e]));
      }
      const double lsum = block_sum(part, red);  // (barrier inside: dyb complete)
      tot += (lsum / (double)(nr * A)) * (double)nr;
      // reverse pass: gWd = z^T dy', dz' = (dy' Wd^T) * slope(z), gWe = x^T dz'
      for (int e = tid; e < nW; e += AE_THREADS) {
        const int j = e / A, a = e - j * A;  // gd[j][a]
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s = fmaf(zb[r * k + j], dyb[r * A + a], s);
        gd[e] = s;
      }
      for (int e = tid; e < nr * k; e += AE_THREADS) {
        const int r = e / k, j = e - r * k;
        float s = 0.f;
        for (int a = 0; a < A; ++a) s = fmaf(dyb[r * A + a], wd[j * A + a], s);
        dzb[e] = rnd<BF>(rnd<BF>(s) * lrelu_dy(zb[e]));
      }
      __syncthreads();
      for (int e = tid; e < nW; e += AE_THREADS) {
        const int a = e / k, j = e - a * k;  // ge[a][j]
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s = fmaf(xb[r * A + a], dzb[r * k + j], s);
        ge[e] = s;
      }
      __syncthreads();
      // Keras 2.7 Nadam, one iteration tick for both layers (csrc/optim.hip nadam_kernel)
      const float local_step = st + 1.f, next_step = st + 2.f;
      const float mt = b1 * (1.f - 0.5f * powf(0.96f, 0.004f * local_step));
      const float mt1 = b1 * (1.f - 0.5f * powf(0.96f, 0.004f * next_step));
      const float sched_new = mc * mt, sched_next = sched_new * mt1;
      const float vden = 1.f - powf(b2, local_step);
      for (int e = tid; e < 2 * nW; e += AE_THREADS) {
        const bool enc = e < nW;
        const int i = enc ? e : e - nW;
        float* p = enc ? We : Wd;
        float* m = enc ? mWe : mWd;
        float* v = enc ? vWe : vWd;
        const float gk = enc ? ge[i] : gd[i];
        const float gprime = gk / (1.f - sched_new);
        const float mk = b1 * m[i] + (1.f - b1) * gk;
        const float vk = b2 * v[i] + (1.f - b2) * gk * gk;
        m[i] = mk;
        v[i] = vk;
        const float mprime = mk / (1.f - sched_next), vprime = vk / vden;
        const float mbar = (1.f - mt) * gprime + mt1 * mprime;
        p[i] = p[i] - lr * mbar / (sqrtf(vprime) + eps);
      }
      mc *= mt;
      st += 1.f;
      __syncthreads();  // (the next batch stages the updated weights)
    }
    // validation loss: mean((AE(xv) - xv)^2) over all nv x A values, fixed-order fp64 sum
    double vpart = 0.0;
    if (nv > 0) {
      for (int e = tid; e < nW; e += AE_THREADS) {
        we[e] = rnd<BF>(We[e]);
        wd[e] = rnd<BF>(Wd[e]);
      }
      for (int v0 = 0; v0 < nv; v0 += AE_MAXB) {
        const int nr = min(AE_MAXB, nv - v0);
        for (int e = tid; e < nr * A; e += AE_THREADS) xb[e] = rnd<BF>(Xv[(size_t)v0 * A + e]);
        __syncthreads();
        dense_lrelu<BF>(xb, A, we, k, zb, nr);
        __syncthreads();
        dense_lrelu<BF>(zb, k, wd, A, yb, nr);
        __syncthreads();
        for (int e = tid; e < nr * A; e += AE_THREADS) {
          const double d = (double)yb[e] - (double)xb[e];
          vpart += d * d;
        }
        __syncthreads();
      }
    }
    const double vl = block_sum(vpart, red) / (double)max(1, nv * A);
    if (tid == 0) {
      hist[2 * ep] = tot / (double)nt;
      hist[2 * ep + 1] = vl;
      int stop = 0;
      if (nv > 0) {
        if (vl < best) { best = vl; wait = 0; }
        else if (++wait >= patience) stop = 1;
      }
      stop_flag = stop;
    }
    __syncthreads();
    if (stop_flag) { ++ep; break; }
  }
  if (tid == 0) {
    nep[0] = ep;
    step[0] = st;
    m_cache[0] = mc;
  }
}

bool ae_fit_supported(int A, int k, int batch) {
  return A >= 1 && A <= AE_MAXA && k >= 1 && k <= AE_MAXK && batch >= 1 && batch <= AE_MAXB;
}

void launch_ae_fit(bool bf16, const AeFitJob* jobs, int njobs, int batch, float lr, float b1, float b2, float eps, int A,
                   hipStream_t s) {
  if (njobs <= 0) return;
  if (bf16)
    hipLaunchKernelGGL(ae_fit_kernel<true>, dim3(njobs), dim3(AE_THREADS), 0, s, jobs, batch, lr, b1, b2, eps, A);
  else
    hipLaunchKernelGGL(ae_fit_kernel<false>, dim3(njobs), dim3(AE_THREADS), 0, s, jobs, batch, lr, b1, b2, eps, A);
}

}  // namespace hfrep
