// Host-side launcher declarations of the hfrep gfx950 kernel library.
// Kernel translation units (*.hip) define these; bindings.cpp exposes them as torch ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hfrep {

// ---- optim.hip ----
void launch_rmsprop(float* p, const float* g, float* ms, int64_t n, float lr, float rho, float eps, float clip,
                    float gscale, hipStream_t s);
void launch_adam(float* p, const float* g, float* m, float* v, int64_t n, const float* step, float lr, float b1,
                 float b2, float eps, float clip, float gscale, hipStream_t s);
void launch_nadam(float* p, const float* g, float* m, float* v, int64_t n, const float* step, const float* m_cache,
                  float lr, float b1, float b2, float eps, float gscale, hipStream_t s);
void launch_step_advance(float* step, float* m_cache, float b1, hipStream_t s);
void launch_clip(float* p, int64_t n, float c, hipStream_t s);

}  // namespace hfrep
