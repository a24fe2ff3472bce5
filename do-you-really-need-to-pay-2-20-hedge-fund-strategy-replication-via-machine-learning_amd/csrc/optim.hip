// Fused, flat-buffer Keras-exact optimizers (RMSprop / Adam / Nadam) + weight clipping.
//
// One launch updates every parameter of a model: params, grads and slots are single flat
// fp32 buffers (the same flat grad buffer is the data-parallel all-reduce bucket), so the
// reference's per-variable `apply_gradients` (Keras 2.7, e.g. GAN/MTSS_WGAN_GP.py:128
// RMSprop(5e-5), GAN/GAN.py:100 Adam(2e-4,.5), Autoencoder_encapsulate.py:80 Nadam())
// becomes one bandwidth-bound pass over ~140k floats.
//
// Step-dependent coefficients (Adam bias correction, Nadam momentum schedule) are computed
// ON DEVICE from a device-resident step counter so the launch can sit inside a hipGraph
// that is replayed every training iteration.  The counter is advanced by the caller with
// `hfrep_step_increment` (one tiny launch, also graph-capturable); Keras shares one
// `iterations` counter between the critic and combined models, which callers reproduce by
// sharing the counter tensor.
#include "common.h"
#include "kernels.h"

namespace hfrep {

// grid-stride, float4-vectorised when aligned
__global__ void __launch_bounds__(256) rmsprop_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ ms, int64_t n, float lr, float rho,
                                                      float eps, float clip, float gscale, int vec) {
  const int64_t n4 = vec ? (n >> 2) : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(ms);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = p4[i], gv = g4[i], mv = m4[i];
    float* pp = reinterpret_cast<float*>(&pv);
    float* gg = reinterpret_cast<float*>(&gv);
    float* mm = reinterpret_cast<float*>(&mv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gg[k] * gscale;
      float m = rho * mm[k] + (1.f - rho) * gk * gk;
      mm[k] = m;
      float np = pp[k] - lr * gk / (sqrtf(m) + eps);
      if (clip > 0.f) np = fminf(fmaxf(np, -clip), clip);
      pp[k] = np;
    }
    p4[i] = pv;
    m4[i] = mv;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gk = g[i] * gscale;
    float m = rho * ms[i] + (1.f - rho) * gk * gk;
    ms[i] = m;
    float np = p[i] - lr * gk / (sqrtf(m) + eps);
    if (clip > 0.f) np = fminf(fmaxf(np, -clip), clip);
    p[i] = np;
  }
}

// Keras Adam (epsilon-hat form): lr_t = lr*sqrt(1-b2^t)/(1-b1^t); p -= lr_t*m/(sqrt(v)+eps)
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const float* __restrict__ step_ctr, float lr, float b1,
                                                   float b2, float eps, float clip, float gscale) {
  const float t = step_ctr[0] + 1.0f;
  const float lr_t = lr * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gk = g[i] * gscale;
    float mk = b1 * m[i] + (1.f - b1) * gk;
    float vk = b2 * v[i] + (1.f - b2) * gk * gk;
    m[i] = mk;
    v[i] = vk;
    float np = p[i] - lr_t * mk / (sqrtf(vk) + eps);
    if (clip > 0.f) np = fminf(fmaxf(np, -clip), clip);
    p[i] = np;
  }
}

// Keras 2.7 Nadam (momentum-cache schedule, decay base 0.96, cache decay 0.004).
// m_cache (device scalar) holds the running product of momentum schedules; the caller's
// increment kernel advances it together with the step counter (see nadam_advance below).
__global__ void __launch_bounds__(256) nadam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    const float* __restrict__ step_ctr,
                                                    const float* __restrict__ m_cache, float lr, float b1,
                                                    float b2, float eps, float gscale) {
  const float local_step = step_ctr[0] + 1.f, next_step = step_ctr[0] + 2.f;
  const float mt = b1 * (1.f - 0.5f * powf(0.96f, 0.004f * local_step));
  const float mt1 = b1 * (1.f - 0.5f * powf(0.96f, 0.004f * next_step));
  const float sched_new = m_cache[0] * mt;
  const float sched_next = sched_new * mt1;
  const float vden = 1.f - powf(b2, local_step);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gk = g[i] * gscale;
    float gprime = gk / (1.f - sched_new);
    float mk = b1 * m[i] + (1.f - b1) * gk;
    float vk = b2 * v[i] + (1.f - b2) * gk * gk;
    m[i] = mk;
    v[i] = vk;
    float mprime = mk / (1.f - sched_next);
    float vprime = vk / vden;
    float mbar = (1.f - mt) * gprime + mt1 * mprime;
    p[i] = p[i] - lr * mbar / (sqrtf(vprime) + eps);
  }
}

// advance the shared step counter; for Nadam also fold the new schedule into m_cache
__global__ void step_advance_kernel(float* step_ctr, float* m_cache, float b1) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (m_cache) {
      const float local_step = step_ctr[0] + 1.f;
      const float mt = b1 * (1.f - 0.5f * powf(0.96f, 0.004f * local_step));
      m_cache[0] = m_cache[0] * mt;
    }
    step_ctr[0] += 1.f;
  }
}

__global__ void __launch_bounds__(256) clip_kernel(float* __restrict__ p, int64_t n, float c) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    p[i] = fminf(fmaxf(p[i], -c), c);
}

static inline int grid_for(int64_t n, int per_thread = 1) {
  int64_t blocks = (n / per_thread + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  return (int)blocks;
}

void launch_rmsprop(float* p, const float* g, float* ms, int64_t n, float lr, float rho, float eps, float clip,
                    float gscale, hipStream_t s) {
  const int vec = ((uintptr_t)p % 16 == 0) && ((uintptr_t)g % 16 == 0) && ((uintptr_t)ms % 16 == 0);
  hipLaunchKernelGGL(rmsprop_kernel, dim3(grid_for(n, vec ? 4 : 1)), dim3(256), 0, s, p, g, ms, n, lr, rho, eps,
                     clip, gscale, vec);
}

void launch_adam(float* p, const float* g, float* m, float* v, int64_t n, const float* step, float lr, float b1,
                 float b2, float eps, float clip, float gscale, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, g, m, v, n, step, lr, b1, b2, eps, clip,
                     gscale);
}

void launch_nadam(float* p, const float* g, float* m, float* v, int64_t n, const float* step, const float* m_cache,
                  float lr, float b1, float b2, float eps, float gscale, hipStream_t s) {
  hipLaunchKernelGGL(nadam_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, g, m, v, n, step, m_cache, lr, b1, b2,
                     eps, gscale);
}

void launch_step_advance(float* step, float* m_cache, float b1, hipStream_t s) {
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, s, step, m_cache, b1);
}

void launch_clip(float* p, int64_t n, float c, hipStream_t s) {
  hipLaunchKernelGGL(clip_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, n, c);
}

}  // namespace hfrep
