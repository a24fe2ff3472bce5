// torch op registrations for the hfrep gfx950 kernel library (namespace torch.ops.hfrep).
//
// Every op validates device/dtype/contiguity on the host, then launches on the current
// HIP stream of the tensor's device, so ops are capturable into hipGraphs and compose with
// torch's stream semantics.  Only the CUDA (=HIP on ROCm) dispatch key is implemented: on a
// CPU tensor the op raises, which is how the Python layer guarantees the native path is the
// one that runs on a GPU box (it never silently falls back).
#include <torch/extension.h>
#include <torch/library.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels.h"

namespace {

inline hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

#define CHECK_F32(t) TORCH_CHECK((t).is_cuda() && (t).scalar_type() == at::kFloat && (t).is_contiguous(), #t " must be a contiguous fp32 GPU tensor")

void rmsprop_(at::Tensor p, at::Tensor g, at::Tensor ms, double lr, double rho, double eps, double clip,
              double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(ms);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == ms.numel(), "rmsprop_: size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  hfrep::launch_rmsprop(p.data_ptr<float>(), g.data_ptr<float>(), ms.data_ptr<float>(), p.numel(), (float)lr,
                        (float)rho, (float)eps, (float)clip, (float)gscale, cur_stream(p));
}

void adam_(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor step, double lr, double b1, double b2,
           double eps, double clip, double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(step);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam_: size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  hfrep::launch_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.numel(),
                     step.data_ptr<float>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)clip, (float)gscale,
                     cur_stream(p));
}

void nadam_(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor step, at::Tensor m_cache, double lr,
            double b1, double b2, double eps, double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(step); CHECK_F32(m_cache);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  hfrep::launch_nadam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.numel(),
                      step.data_ptr<float>(), m_cache.data_ptr<float>(), (float)lr, (float)b1, (float)b2, (float)eps,
                      (float)gscale, cur_stream(p));
}

void step_advance_(at::Tensor step, c10::optional<at::Tensor> m_cache, double b1) {
  CHECK_F32(step);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(step.device());
  float* mc = nullptr;
  if (m_cache.has_value()) { CHECK_F32(*m_cache); mc = m_cache->data_ptr<float>(); }
  hfrep::launch_step_advance(step.data_ptr<float>(), mc, (float)b1, cur_stream(step));
}

void clip_(at::Tensor p, double c) {
  CHECK_F32(p);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  hfrep::launch_clip(p.data_ptr<float>(), p.numel(), (float)c, cur_stream(p));
}

}  // namespace

TORCH_LIBRARY(hfrep, m) {
  m.def("rmsprop_(Tensor(a!) p, Tensor g, Tensor(b!) ms, float lr, float rho, float eps, float clip, float gscale) -> ()");
  m.def("adam_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor step, float lr, float b1, float b2, float eps, float clip, float gscale) -> ()");
  m.def("nadam_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor step, Tensor m_cache, float lr, float b1, float b2, float eps, float gscale) -> ()");
  m.def("step_advance_(Tensor(a!) step, Tensor(b!)? m_cache, float b1) -> ()");
  m.def("clip_(Tensor(a!) p, float c) -> ()");
}

TORCH_LIBRARY_IMPL(hfrep, CUDA, m) {
  m.impl("rmsprop_", &rmsprop_);
  m.impl("adam_", &adam_);
  m.impl("nadam_", &nadam_);
  m.impl("step_advance_", &step_advance_);
  m.impl("clip_", &clip_);
}
