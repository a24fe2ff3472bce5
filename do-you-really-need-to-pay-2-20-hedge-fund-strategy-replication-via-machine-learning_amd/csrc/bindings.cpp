// torch op registrations for the hfrep gfx950 kernel library (namespace torch.ops.hfrep).
//
// Every op validates device/dtype/contiguity/shape on the host, allocates outputs through the
// torch caching allocator (graph-capture safe) and launches on the current HIP stream of the
// tensor's device, so ops are capturable into hipGraphs and compose with torch stream semantics.
// Only the CUDA (=HIP on ROCm) dispatch key is implemented: a CPU tensor raises, which is how the
// Python layer guarantees the native path is the one that runs on a GPU box (no silent fallback).
#include <torch/extension.h>
#include <torch/library.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels.h"

#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace {

using at::Tensor;
using c10::optional;

inline hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

#define GUARD(t) c10::hip::HIPGuardMasqueradingAsCUDA _guard((t).device())
#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda() && (t).is_contiguous(), #t " must be a contiguous GPU tensor")
#define CHECK_F32(t) TORCH_CHECK((t).is_cuda() && (t).scalar_type() == at::kFloat && (t).is_contiguous(), #t " must be a contiguous fp32 GPU tensor")

inline int dt_of(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return hfrep::DT_BF16;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "hfrep kernels support float32 and bfloat16 activations, got ",
              t.scalar_type());
  return hfrep::DT_F32;
}
inline void same_dt(const Tensor& a, const Tensor& b) {
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "dtype mismatch: ", a.scalar_type(), " vs ", b.scalar_type());
}
inline const void* ptr_or_null(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// Debug poison mode (HFREP_POISON=1 or set_debug_poison(True)): every op output / workspace is
// allocated filled with NaN instead of uninitialised, so an element a kernel fails to write shows
// up as a non-finite loss or gradient (tests/test_gpu_runtime.py).  Off by default (it costs a
// fill per output).  Tapes are exempt: their padded unit lanes are unwritten by design and never
// read.
std::atomic<bool>& poison_flag() {
  static std::atomic<bool> f{[] {
    const char* e = getenv("HFREP_POISON");
    return e && e[0] == '1';
  }()};
  return f;
}
inline Tensor out_empty(at::IntArrayRef sizes, const at::TensorOptions& o) {
  return poison_flag().load(std::memory_order_relaxed) ? at::full(sizes, NAN, o) : at::empty(sizes, o);
}
inline Tensor out_empty_like(const Tensor& t) {
  return poison_flag().load(std::memory_order_relaxed) ? at::full_like(t, NAN) : at::empty_like(t);
}
bool set_debug_poison(bool on) { return poison_flag().exchange(on); }

// ------------------------------------------------------------------------------------ GEMM
// out (optional): a contiguous (M, N) destination of x's dtype, e.g. a row slice of a larger buffer
// (the generator writes its fake batch straight into the critic's [real; fake] input)
Tensor linear(Tensor x, Tensor W, optional<Tensor> b, int64_t act, optional<Tensor> out) {
  CHECK_GPU(x); CHECK_F32(W);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && x.size(1) == W.size(0), "linear: shape mismatch");
  if (b.has_value()) { CHECK_F32(*b); TORCH_CHECK(b->numel() == W.size(1), "linear: bias size"); }
  GUARD(x);
  const int M = x.size(0), K = x.size(1), N = W.size(1);
  if (out.has_value())
    TORCH_CHECK(out->is_cuda() && out->device() == x.device() && out->is_contiguous() &&
                    out->scalar_type() == x.scalar_type() && out->numel() == (int64_t)M * N,
                "linear: out must be a contiguous (M, N) tensor of x's dtype on x's device");
  Tensor y = out.has_value() ? out->view({M, N}) : out_empty({M, N}, x.options());
  if (hfrep::skinny_supported(K, N))
    hfrep::launch_skinny_fwd(dt_of(x), x.data_ptr(), W.data_ptr<float>(), b.has_value() ? b->data_ptr<float>() : nullptr,
                             y.data_ptr(), M, K, N, (int)act, cur_stream(x));
  else if (dt_of(x) == hfrep::DT_F32 && hfrep::narrowf_supported(K, N))
    hfrep::launch_narrowf(x.data_ptr<float>(), W.data_ptr<float>(), N, 1, b.has_value() ? b->data_ptr<float>() : nullptr,
                          y.data_ptr<float>(), M, K, N, (int)act, cur_stream(x));
  else if (dt_of(x) == hfrep::DT_F32 && hfrep::widef_supported(K, N))
    hfrep::launch_widef(x.data_ptr<float>(), W.data_ptr<float>(), N, 1, b.has_value() ? b->data_ptr<float>() : nullptr,
                        y.data_ptr<float>(), M, K, N, (int)act, cur_stream(x));
  else if (dt_of(x) == hfrep::DT_BF16 && hfrep::narrow_supported(K, N))
    hfrep::launch_narrow_fwd(x.data_ptr(), W.data_ptr<float>(), b.has_value() ? b->data_ptr<float>() : nullptr,
                             y.data_ptr(), M, K, N, (int)act, cur_stream(x));
  else if (dt_of(x) == hfrep::DT_BF16 && N > 64)
    hfrep::launch_linear2(x.data_ptr(), W.data_ptr<float>(), b.has_value() ? b->data_ptr<float>() : nullptr,
                          y.data_ptr(), M, N, K, 0, (int)act, cur_stream(x));
  else
    hfrep::launch_linear(dt_of(x), x.data_ptr(), W.data_ptr<float>(), b.has_value() ? b->data_ptr<float>() : nullptr,
                         y.data_ptr(), M, N, K, 0, (int)act, cur_stream(x));
  return y;
}

// linear Dense(1) head forward + its weight gradient for a known per-row loss gradient (wa for the
// first `split` rows, wb after): y = x W + b, gW += sum_r ds_r x_r, gb += sum_r ds_r in one pass over x
Tensor linear_head_cs(Tensor x, Tensor W, optional<Tensor> b, int64_t split, double wa, double wb, Tensor gW,
                      optional<Tensor> gb) {
  CHECK_GPU(x); CHECK_F32(W); CHECK_F32(gW);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && x.size(1) == W.size(0) && W.size(1) == 1, "linear_head_cs: (M, K) x (K, 1)");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous() && gW.is_contiguous() && gW.numel() == W.numel() &&
                  gW.device() == x.device(),
              "linear_head_cs: contiguous operands, gW like W on x's device");
  if (b.has_value()) { CHECK_F32(*b); TORCH_CHECK(b->numel() == 1, "linear_head_cs: bias size"); }
  if (gb.has_value()) {
    CHECK_F32(*gb);
    TORCH_CHECK(gb->numel() == 1 && gb->device() == x.device(), "linear_head_cs: gb size");
  }
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(hfrep::skinny_fwd_cs_supported(K), "linear_head_cs: K % 8 == 0 and K <= 4096");
  GUARD(x);
  Tensor y = out_empty({M, 1}, x.options());
  Tensor ws = out_empty({(int64_t)hfrep::skinny_fwd_cs_workspace_floats(M, K)}, x.options().dtype(at::kFloat));
  hfrep::launch_skinny_fwd_cs(dt_of(x), x.data_ptr(), W.data_ptr<float>(), b.has_value() ? b->data_ptr<float>() : nullptr,
                              y.data_ptr(), M, K, (int)split, (float)wa, (float)wb, gW.data_ptr<float>(),
                              gb.has_value() ? gb->data_ptr<float>() : nullptr, ws.data_ptr<float>(), cur_stream(x));
  return y;
}
bool linear_head_cs_supported(int64_t K) { return hfrep::skinny_fwd_cs_supported((int)K); }

Tensor linear_dgrad(Tensor dz, Tensor W) {
  CHECK_GPU(dz); CHECK_F32(W);
  TORCH_CHECK(dz.dim() == 2 && W.dim() == 2 && dz.size(1) == W.size(1), "linear_dgrad: shape mismatch");
  GUARD(dz);
  const int M = dz.size(0), K = dz.size(1), N = W.size(0);
  Tensor dx = out_empty({M, N}, dz.options());
  // dx = dz . W^T : W stored (N, K) row-major -> w_trans
  if (hfrep::skinny_supported(N, K))
    hfrep::launch_skinny_dgrad(dt_of(dz), dz.data_ptr(), W.data_ptr<float>(), dx.data_ptr(), M, N, K, cur_stream(dz));
  else if (dt_of(dz) == hfrep::DT_F32 && hfrep::narrowf_supported(K, N))  // B[k][n] = W[n][k]
    hfrep::launch_narrowf(dz.data_ptr<float>(), W.data_ptr<float>(), 1, K, nullptr, dx.data_ptr<float>(), M, K, N, 0,
                          cur_stream(dz));
  else if (dt_of(dz) == hfrep::DT_F32 && hfrep::widef_supported(K, N))  // B[k][n] = W[n][k]
    hfrep::launch_widef(dz.data_ptr<float>(), W.data_ptr<float>(), 1, K, nullptr, dx.data_ptr<float>(), M, K, N, 0,
                        cur_stream(dz));
  else if (dt_of(dz) == hfrep::DT_BF16 && N > 64)
    hfrep::launch_linear2(dz.data_ptr(), W.data_ptr<float>(), nullptr, dx.data_ptr(), M, N, K, 1, 0, cur_stream(dz));
  else
    hfrep::launch_linear(dt_of(dz), dz.data_ptr(), W.data_ptr<float>(), nullptr, dx.data_ptr(), M, N, K, 1, 0,
                         cur_stream(dz));
  return dx;
}

void linear_wgrad_(Tensor x, Tensor dz, Tensor gW, optional<Tensor> gb, int64_t shiftT) {
  CHECK_GPU(x); CHECK_GPU(dz); same_dt(x, dz);
  TORCH_CHECK(gW.is_cuda() && gW.scalar_type() == at::kFloat && gW.is_contiguous(), "gW must be contiguous fp32");
  TORCH_CHECK(x.dim() == 2 && dz.dim() == 2 && x.size(0) == dz.size(0), "wgrad: rows mismatch");
  TORCH_CHECK(gW.numel() == x.size(1) * dz.size(1), "wgrad: gW size");
  if (gb.has_value()) { CHECK_F32(*gb); TORCH_CHECK(gb->numel() == dz.size(1), "wgrad: gb size"); }
  GUARD(x);
  const int M = x.size(0), K = x.size(1), N = dz.size(1);
  if (shiftT == 0 && hfrep::skinny_supported(K, N)) {
    Tensor ws = out_empty({(int64_t)hfrep::skinny_wgrad_workspace_floats(M, K, N)}, x.options().dtype(at::kFloat));
    hfrep::launch_skinny_wgrad(dt_of(x), x.data_ptr(), dz.data_ptr(), gW.data_ptr<float>(),
                               gb.has_value() ? gb->data_ptr<float>() : nullptr, M, K, N, ws.data_ptr<float>(),
                               cur_stream(x));
    return;
  }
  Tensor ws = out_empty({(int64_t)hfrep::wgrad_workspace_floats(M, K, N)}, x.options().dtype(at::kFloat));
  hfrep::launch_wgrad(dt_of(x), x.data_ptr(), dz.data_ptr(), gW.data_ptr<float>(),
                      gb.has_value() ? gb->data_ptr<float>() : nullptr, M, K, N, (int)shiftT, ws.data_ptr<float>(),
                      cur_stream(x));
}

// fused LSTM weight gradients (bf16): gW += X^T dZ (+ Xd^T dZd), gU += Hprev^T dZ (+ Hdprev^T dZd), gb += sum dZ
void lstm_wgrad_(Tensor x, Tensor hs, Tensor dZ, Tensor gW, Tensor gU, optional<Tensor> gb, optional<Tensor> xd,
                 optional<Tensor> hds, optional<Tensor> dZd, int64_t impl) {
  CHECK_GPU(x); CHECK_GPU(hs); CHECK_GPU(dZ); same_dt(x, dZ); same_dt(hs, dZ);
  const bool f32 = x.scalar_type() == at::kFloat;
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || (f32 && hfrep::lstmf_wgrad_supported(x.size(2), hs.size(2), dZ.size(2))),
              "lstm_wgrad_: bf16, or fp32 with K in {32, 36, 100}, H = 100");
  TORCH_CHECK(x.dim() == 3 && hs.dim() == 3 && dZ.dim() == 3, "lstm_wgrad_: (B,T,*) tensors");
  const int B = x.size(0), Tn = x.size(1), K = x.size(2), Hd = hs.size(2), N = dZ.size(2);
  TORCH_CHECK(hs.size(0) == B && dZ.size(0) == B && hs.size(1) == Tn && dZ.size(1) == Tn, "lstm_wgrad_: B/T");
  CHECK_F32(gW); CHECK_F32(gU);
  TORCH_CHECK(gW.numel() == (int64_t)K * N && gU.numel() == (int64_t)Hd * N, "lstm_wgrad_: grad sizes");
  if (gb.has_value()) { CHECK_F32(*gb); TORCH_CHECK(gb->numel() == N, "gb size"); }
  const bool tangent = xd.has_value();
  if (tangent) {
    TORCH_CHECK(hds.has_value() && dZd.has_value(), "tangent segment needs xd, hds, dZd");
    CHECK_GPU(*xd); CHECK_GPU(*hds); CHECK_GPU(*dZd);
    // the fp32 launcher takes untyped pointers: a bf16 tangent beside an fp32 primal would be read as fp32
    same_dt(*xd, x); same_dt(*hds, hs); same_dt(*dZd, dZ);
    TORCH_CHECK(xd->sizes() == x.sizes() && hds->sizes() == hs.sizes() && dZd->sizes() == dZ.sizes(), "tangent shapes");
  }
  GUARD(x);
  const int M = B * Tn;
  const void* X1 = tangent ? xd->data_ptr() : nullptr;
  const void* H1 = tangent ? hds->data_ptr() : nullptr;
  const void* D1 = tangent ? dZd->data_ptr() : nullptr;
  float* gbp = gb.has_value() ? gb->data_ptr<float>() : nullptr;
  if (f32) {
    // impl (fp32): 0 = default, 1 = exact-fp32 MFMA kernel, 2 = three-term bf16 split kernel
    Tensor ws = out_empty({(int64_t)hfrep::lstmf_wgrad_workspace_floats(M, K, (int)impl)}, x.options());
    hfrep::launch_lstmf_wgrad(x.data_ptr(), hs.data_ptr(), dZ.data_ptr(),
                              X1, H1, D1, gW.data_ptr<float>(), gU.data_ptr<float>(), gbp,
                              M, K, Tn, ws.data_ptr<float>(), cur_stream(x), (int)impl);
    return;
  }
  // impl: 0 = auto (LDS-DMA streaming v3 where supported), 2 = force v2 (tests / A-B)
  if (impl != 2 && hfrep::lstm_wgrad3_supported(M, K, Hd, N)) {
    Tensor ws = out_empty({(int64_t)hfrep::lstm_wgrad3_workspace_floats(K, Hd, N)}, x.options().dtype(at::kFloat));
    if (hfrep::launch_lstm_wgrad3(x.data_ptr(), hs.data_ptr(), dZ.data_ptr(), X1, H1, D1, gW.data_ptr<float>(),
                                  gU.data_ptr<float>(), gbp, M, K, Hd, N, Tn, ws.data_ptr<float>(), cur_stream(x)))
      return;
  }
  Tensor ws = out_empty({(int64_t)hfrep::lstm_wgrad2_workspace_floats(M, K, Hd, N)}, x.options().dtype(at::kFloat));
  hfrep::launch_lstm_wgrad2(x.data_ptr(), hs.data_ptr(), dZ.data_ptr(), tangent ? xd->data_ptr() : nullptr,
                            tangent ? hds->data_ptr() : nullptr, tangent ? dZd->data_ptr() : nullptr,
                            gW.data_ptr<float>(), gU.data_ptr<float>(), gb.has_value() ? gb->data_ptr<float>() : nullptr,
                            M, K, Hd, N, Tn, ws.data_ptr<float>(), cur_stream(x));
}

// ------------------------------------------------------------------------------------ elementwise
Tensor act_fwd(Tensor x, int64_t act) {
  CHECK_GPU(x); GUARD(x);
  Tensor y = out_empty_like(x);
  hfrep::launch_act_fwd(dt_of(x), x.data_ptr(), y.data_ptr(), x.numel(), (int)act, cur_stream(x));
  return y;
}
Tensor act_bwd(Tensor dy, Tensor y, int64_t act) {
  CHECK_GPU(dy); CHECK_GPU(y); same_dt(dy, y);
  TORCH_CHECK(dy.numel() == y.numel(), "act_bwd: size");
  GUARD(dy);
  Tensor dx = out_empty_like(dy);
  hfrep::launch_act_bwd(dt_of(dy), dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(), (int)act, cur_stream(dy));
  return dx;
}
Tensor act_tangent_bwd(Tensor dyd, Tensor y, Tensor zd, int64_t act) {
  CHECK_GPU(dyd); CHECK_GPU(y); CHECK_GPU(zd); same_dt(dyd, y); same_dt(dyd, zd);
  TORCH_CHECK(dyd.numel() == y.numel() && y.numel() == zd.numel(), "act_tangent_bwd: size");
  GUARD(dyd);
  Tensor out = out_empty_like(dyd);
  hfrep::launch_act_tangent_bwd(dt_of(dyd), dyd.data_ptr(), y.data_ptr(), zd.data_ptr(), out.data_ptr(), dyd.numel(),
                                (int)act, cur_stream(dyd));
  return out;
}

// ------------------------------------------------------------------------------------ LSTM
void check_lstm_U(const Tensor& U, int64_t H) {
  CHECK_F32(U);
  TORCH_CHECK(U.dim() == 2 && U.size(0) == H && U.size(1) == 4 * H, "recurrent kernel must be (H, 4H)");
}

std::tuple<Tensor, Tensor, Tensor> lstm_fwd(Tensor zx, Tensor U, int64_t act, bool save) {
  CHECK_GPU(zx);
  TORCH_CHECK(zx.dim() == 3 && zx.size(2) % 4 == 0, "zx must be (B, T, 4H)");
  const int B = zx.size(0), Tn = zx.size(1), H = zx.size(2) / 4;
  check_lstm_U(U, H);
  GUARD(zx);
  Tensor hs = out_empty({B, Tn, H}, zx.options());
  Tensor gates = save ? out_empty({B, Tn, 4 * H}, zx.options()) : out_empty({0}, zx.options());
  Tensor cs = save ? out_empty({B, Tn, H}, zx.options()) : out_empty({0}, zx.options());
  const bool ok = hfrep::launch_lstm_fwd(dt_of(zx), zx.data_ptr(), U.data_ptr<float>(), hs.data_ptr(),
                                         save ? gates.data_ptr() : nullptr, save ? cs.data_ptr() : nullptr, B, Tn, H,
                                         (int)act, cur_stream(zx));
  TORCH_CHECK(ok, "lstm_fwd: hidden size ", H, " not instantiated (supported: 100, 64, 32)");
  return {hs, gates, cs};
}

Tensor lstm_bwd(Tensor dH, Tensor gates, Tensor cs, Tensor U, int64_t act) {
  CHECK_GPU(dH); CHECK_GPU(gates); CHECK_GPU(cs); same_dt(dH, gates); same_dt(dH, cs);
  const int B = gates.size(0), Tn = gates.size(1), H = gates.size(2) / 4;
  TORCH_CHECK(dH.sizes() == cs.sizes() && cs.size(2) == H, "lstm_bwd: shapes");
  check_lstm_U(U, H);
  GUARD(dH);
  Tensor dZ = out_empty_like(gates);
  const bool ok = hfrep::launch_lstm_bwd(dt_of(dH), dH.data_ptr(), gates.data_ptr(), cs.data_ptr(),
                                         U.data_ptr<float>(), dZ.data_ptr(), B, Tn, H, (int)act, cur_stream(dH));
  TORCH_CHECK(ok, "lstm_bwd: hidden size ", H, " not instantiated");
  return dZ;
}

std::tuple<Tensor, Tensor, Tensor> lstm_tfwd(Tensor dzx, Tensor gates, Tensor cs, Tensor U, int64_t act) {
  CHECK_GPU(dzx); CHECK_GPU(gates); CHECK_GPU(cs); same_dt(dzx, gates); same_dt(dzx, cs);
  TORCH_CHECK(dzx.sizes() == gates.sizes(), "lstm_tfwd: shapes");
  const int B = gates.size(0), Tn = gates.size(1), H = gates.size(2) / 4;
  check_lstm_U(U, H);
  GUARD(dzx);
  Tensor hds = out_empty({B, Tn, H}, dzx.options());
  Tensor zds = out_empty_like(gates);
  Tensor cds = out_empty({B, Tn, H}, dzx.options());
  const bool ok = hfrep::launch_lstm_tfwd(dt_of(dzx), dzx.data_ptr(), gates.data_ptr(), cs.data_ptr(),
                                          U.data_ptr<float>(), hds.data_ptr(), zds.data_ptr(), cds.data_ptr(), B, Tn,
                                          H, (int)act, cur_stream(dzx));
  TORCH_CHECK(ok, "lstm_tfwd: hidden size ", H, " not instantiated");
  return {hds, zds, cds};
}

std::tuple<Tensor, Tensor> lstm_tbwd(optional<Tensor> dH, Tensor dHd, Tensor gates, Tensor cs, Tensor zds, Tensor cds,
                                     Tensor U, int64_t act) {
  CHECK_GPU(dHd); CHECK_GPU(gates); CHECK_GPU(cs); CHECK_GPU(zds); CHECK_GPU(cds);
  same_dt(dHd, gates); same_dt(dHd, zds); same_dt(dHd, cds);
  if (dH.has_value()) { CHECK_GPU(*dH); same_dt(*dH, dHd); }
  const int B = gates.size(0), Tn = gates.size(1), H = gates.size(2) / 4;
  check_lstm_U(U, H);
  GUARD(dHd);
  Tensor dZ = out_empty_like(gates), dZd = out_empty_like(gates);
  const bool ok = hfrep::launch_lstm_tbwd(dt_of(dHd), ptr_or_null(dH), dHd.data_ptr(), gates.data_ptr(),
                                          cs.data_ptr(), zds.data_ptr(), cds.data_ptr(), U.data_ptr<float>(),
                                          dZ.data_ptr(), dZd.data_ptr(), B, Tn, H, (int)act, cur_stream(dHd));
  TORCH_CHECK(ok, "lstm_tbwd: hidden size ", H, " not instantiated");
  return {dZ, dZd};
}

// ------------------------------------------------------------------------------------ LSTM fp32 fused
bool lstmf_supported(int64_t H, int64_t K, int64_t act) { return hfrep::lstmf_supported((int)H, (int)K, (int)act); }
bool narrowf_supported(int64_t K, int64_t N) { return hfrep::narrowf_supported((int)K, (int)N); }
int64_t set_lstmf_fwd_impl(int64_t v) { return hfrep::set_lstmf_fwd_impl((int)v); }
int64_t set_lstmf_bwd_impl(int64_t v) { return hfrep::set_lstmf_bwd_impl((int)v); }

std::tuple<Tensor, Tensor> lstmf_fwd(Tensor x, Tensor W, optional<Tensor> b, Tensor U, int64_t act, bool save) {
  CHECK_F32(x); CHECK_F32(W);
  TORCH_CHECK(x.dim() == 3, "x must be (B, T, K)");
  const int B = x.size(0), Tn = x.size(1), K = x.size(2), H = U.size(0);
  check_lstm_U(U, H);
  TORCH_CHECK(W.size(0) == K && W.size(1) == 4 * H, "W must be (K, 4H)");
  if (b.has_value()) { CHECK_F32(*b); TORCH_CHECK(b->numel() == 4 * H, "bias size"); }
  TORCH_CHECK(hfrep::lstmf_supported(H, K, (int)act), "lstmf_fwd: unsupported H/K/act");
  GUARD(x);
  Tensor hs = out_empty({B, Tn, H}, x.options());
  Tensor tape = at::empty({save ? (int64_t)hfrep::lstmf_tape_elems(B, Tn) : 0}, x.options());  // (padding slots unwritten)
  const bool ok = hfrep::launch_lstmf_fwd(x.data_ptr<float>(), W.data_ptr<float>(),
                                          b.has_value() ? b->data_ptr<float>() : nullptr, U.data_ptr<float>(),
                                          hs.data_ptr<float>(), save ? tape.data_ptr<float>() : nullptr, B, Tn, K, H,
                                          (int)act, cur_stream(x));
  TORCH_CHECK(ok, "lstmf_fwd: launch failed");
  return {hs, tape};
}

std::tuple<Tensor, Tensor> lstmf_tfwd(Tensor xd, Tensor W, Tensor U, Tensor tape, int64_t act) {
  CHECK_F32(xd); CHECK_F32(W); CHECK_F32(tape);
  TORCH_CHECK(xd.dim() == 3, "xd must be (B, T, K)");
  const int B = xd.size(0), Tn = xd.size(1), K = xd.size(2), H = U.size(0);
  check_lstm_U(U, H);
  TORCH_CHECK(W.size(0) == K && W.size(1) == 4 * H, "W must be (K, 4H)");
  TORCH_CHECK(tape.numel() == (int64_t)hfrep::lstmf_tape_elems(B, Tn), "lstmf_tfwd: tape size");
  TORCH_CHECK(hfrep::lstmf_supported(H, K, (int)act), "lstmf_tfwd: unsupported H/K/act");
  GUARD(xd);
  Tensor hds = out_empty({B, Tn, H}, xd.options());
  Tensor ttape = at::empty_like(tape);
  const bool ok = hfrep::launch_lstmf_tfwd(xd.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                                           tape.data_ptr<float>(), hds.data_ptr<float>(), ttape.data_ptr<float>(), B, Tn,
                                           K, H, (int)act, cur_stream(xd));
  TORCH_CHECK(ok, "lstmf_tfwd: launch failed");
  return {hds, ttape};
}

// the critic head's outer-product adjoint (d (B) x w (Tn H)) as kernel operands: fp32, on the tape's device
static void check_head(const optional<Tensor>& d, const optional<Tensor>& w, const Tensor& like, int64_t B, int64_t n) {
  if (d.has_value()) {
    CHECK_F32(*d);
    TORCH_CHECK(d->numel() == B && d->device() == like.device(), "head adjoint factor: B fp32 values");
  }
  if (w.has_value()) {
    CHECK_F32(*w);
    TORCH_CHECK(w->numel() == n && w->device() == like.device(), "head weight: Tn H fp32 values");
  }
}

Tensor lstmf_bwd(optional<Tensor> dH, Tensor tape, Tensor U, int64_t act, int64_t B, int64_t Tn, optional<Tensor> hd,
                 optional<Tensor> hw) {
  CHECK_F32(tape);
  const int H = U.size(0);
  check_lstm_U(U, H);
  TORCH_CHECK(tape.numel() == (int64_t)hfrep::lstmf_tape_elems(B, Tn), "lstmf_bwd: tape size");
  if (dH.has_value()) { CHECK_F32(*dH); TORCH_CHECK(dH->numel() == B * Tn * H, "lstmf_bwd: dH shape"); }
  TORCH_CHECK(hd.has_value() == hw.has_value() && !(hd.has_value() && dH.has_value()),
              "lstmf_bwd: dH or the head factors (hd, hw)");
  check_head(hd, hw, tape, B, Tn * H);
  GUARD(tape);
  Tensor dZ = out_empty({B, Tn, 4 * H}, tape.options());
  Tensor dHm;
  if (hd.has_value() && !hfrep::lstmf_head_supported()) {  // exact-fp32 BPTT: materialise hd (x) hw
    dHm = out_empty({B, Tn * H}, tape.options());
    // (M rows, K = Tn H input features, N = 1 head column): linear_dgrad's skinny call for this head
    hfrep::launch_skinny_dgrad(hfrep::DT_F32, hd->data_ptr<float>(), hw->data_ptr<float>(), dHm.data_ptr(), B,
                               (int)(Tn * H), 1, cur_stream(tape));
  }
  const bool head = hd.has_value() && !dHm.defined();
  const float* dhp = dHm.defined() ? dHm.data_ptr<float>() : dH.has_value() ? dH->data_ptr<float>() : nullptr;
  const bool ok = hfrep::launch_lstmf_bwd(dhp, tape.data_ptr<float>(), U.data_ptr<float>(), dZ.data_ptr<float>(), B, Tn,
                                          H, (int)act, cur_stream(tape), head ? hd->data_ptr<float>() : nullptr,
                                          head ? hw->data_ptr<float>() : nullptr);
  TORCH_CHECK(ok, "lstmf_bwd: unsupported H / act");
  return dZ;
}

std::tuple<Tensor, Tensor> lstmf_tbwd(optional<Tensor> dH, optional<Tensor> dHd, Tensor tape, Tensor ttape, Tensor U,
                                      int64_t act, int64_t B, int64_t Tn, optional<Tensor> hd, optional<Tensor> hdd,
                                      optional<Tensor> hw) {
  CHECK_F32(tape); CHECK_F32(ttape);
  const int H = U.size(0);
  check_lstm_U(U, H);
  TORCH_CHECK(tape.numel() == (int64_t)hfrep::lstmf_tape_elems(B, Tn) && ttape.numel() == tape.numel(), "tape size");
  for (const auto* d : {&dH, &dHd})
    if (d->has_value()) { CHECK_F32(**d); TORCH_CHECK((*d)->numel() == B * Tn * H, "lstmf_tbwd: adjoint shape"); }
  const bool head = hw.has_value();
  TORCH_CHECK(!head || (!dH.has_value() && !dHd.has_value()), "lstmf_tbwd: adjoints (dH, dHd) or head factors, not both");
  check_head(hd, hw, tape, B, Tn * H);
  check_head(hdd, {}, tape, B, Tn * H);
  GUARD(tape);
  Tensor dZ = out_empty({B, Tn, 4 * H}, tape.options()), dZd = out_empty({B, Tn, 4 * H}, tape.options());
  const bool ok = hfrep::launch_lstmf_tbwd(dH.has_value() ? dH->data_ptr<float>() : nullptr,
                                           dHd.has_value() ? dHd->data_ptr<float>() : nullptr, tape.data_ptr<float>(),
                                           ttape.data_ptr<float>(), U.data_ptr<float>(), dZ.data_ptr<float>(),
                                           dZd.data_ptr<float>(), B, Tn, H, (int)act, cur_stream(tape),
                                           head && hd.has_value() ? hd->data_ptr<float>() : nullptr,
                                           head && hdd.has_value() ? hdd->data_ptr<float>() : nullptr,
                                           head ? hw->data_ptr<float>() : nullptr);
  TORCH_CHECK(ok, "lstmf_tbwd: unsupported H / act");
  return {dZ, dZd};
}

Tensor lstmf_dgrad(Tensor dz, Tensor W, int64_t impl) {
  CHECK_F32(dz); CHECK_F32(W);
  TORCH_CHECK(dz.dim() == 2 && dz.is_contiguous() && W.dim() == 2 && W.is_contiguous() && W.size(1) == dz.size(1),
              "lstmf_dgrad: dz (M, N) and W (KO, N), contiguous");
  TORCH_CHECK(hfrep::lstmf_dgrad_supported(dz.size(1), W.size(0)), "lstmf_dgrad: N must be 400 and KO <= 112");
  GUARD(dz);
  Tensor x = out_empty({dz.size(0), W.size(0)}, dz.options());
  if (dz.size(0) == 0) return x;
  const bool ok = hfrep::launch_lstmf_dgrad(dz.data_ptr<float>(), W.data_ptr<float>(), x.data_ptr<float>(), dz.size(0),
                                            dz.size(1), W.size(0), cur_stream(dz), (int)impl);
  TORCH_CHECK(ok, "lstmf_dgrad: launch failed");
  return x;
}

// ---- FP3 planes: an fp32 tensor (..., C) as its three exact bf16 split planes (..., 3, C) ----
bool is_fp3(const Tensor& t) { return t.scalar_type() == at::kBFloat16 && t.dim() >= 2 && t.size(-2) == 3; }

Tensor fp3_split(Tensor x, bool interleave) {
  CHECK_F32(x);
  TORCH_CHECK(x.is_contiguous() && x.dim() >= 1, "fp3_split: a contiguous fp32 tensor");
  const int64_t C = x.size(-1), M = C ? x.numel() / C : 0;
  auto sz = x.sizes().vec();
  sz.insert(sz.end() - 1, 3);
  GUARD(x);
  Tensor p = out_empty(sz, x.options().dtype(at::kBFloat16));
  hfrep::launch_fp3_split(x.data_ptr<float>(), reinterpret_cast<uint16_t*>(p.data_ptr()), M, (int)C, interleave,
                          cur_stream(x));
  return p;
}

Tensor fp3_join(Tensor p, bool interleave) {
  CHECK_GPU(p);
  TORCH_CHECK(is_fp3(p) && p.is_contiguous(), "fp3_join: contiguous bf16 planes (..., 3, C)");
  const int64_t C = p.size(-1), M = C ? p.numel() / (3 * C) : 0;
  auto sz = p.sizes().vec();
  sz.erase(sz.end() - 2);
  GUARD(p);
  Tensor x = out_empty(sz, p.options().dtype(at::kFloat));
  hfrep::launch_fp3_join(reinterpret_cast<const uint16_t*>(p.data_ptr()), x.data_ptr<float>(), M, (int)C, interleave,
                         cur_stream(p));
  return x;
}

// fp32 LSTM weight gradients with any of x (B,T,K) / hs (B,T,H) / dZ (B,T,400) given as FP3 planes
// ((B,T,3,C) bf16; dZ in the interleaved gate order); the tangent segment's operands mirror the primal's
void lstmf_wgrad_p_(Tensor x, Tensor hs, Tensor dZ, Tensor gW, Tensor gU, optional<Tensor> gb, optional<Tensor> xd,
                    optional<Tensor> hds, optional<Tensor> dZd, int64_t impl) {
  CHECK_GPU(x); CHECK_GPU(hs); CHECK_GPU(dZ);
  const int pm = (is_fp3(x) ? 1 : 0) | (is_fp3(hs) ? 2 : 0) | (is_fp3(dZ) ? 4 : 0);
  for (const Tensor* t : {&x, &hs, &dZ})
    TORCH_CHECK(t->is_contiguous() && (is_fp3(*t) ? t->dim() == 4 : (t->scalar_type() == at::kFloat && t->dim() == 3)),
                "lstmf_wgrad_p_: fp32 (B,T,C) or FP3 planes (B,T,3,C), contiguous");
  const int B = x.size(0), Tn = x.size(1), K = x.size(-1), Hd = hs.size(-1), N = dZ.size(-1);
  TORCH_CHECK(hs.size(0) == B && dZ.size(0) == B && hs.size(1) == Tn && dZ.size(1) == Tn, "lstmf_wgrad_p_: B/T");
  TORCH_CHECK(hfrep::lstmf_wgrad_supported(K, Hd, N) && (pm == 0 || K == 32 || K == 100), "lstmf_wgrad_p_: K / H / N");
  CHECK_F32(gW); CHECK_F32(gU);
  TORCH_CHECK(gW.numel() == (int64_t)K * N && gU.numel() == (int64_t)Hd * N, "lstmf_wgrad_p_: grad sizes");
  if (gb.has_value()) { CHECK_F32(*gb); TORCH_CHECK(gb->numel() == N, "gb size"); }
  const bool tangent = xd.has_value();
  if (tangent) {
    TORCH_CHECK(hds.has_value() && dZd.has_value(), "tangent segment needs xd, hds, dZd");
    TORCH_CHECK(xd->sizes() == x.sizes() && hds->sizes() == hs.sizes() && dZd->sizes() == dZ.sizes() &&
                xd->scalar_type() == x.scalar_type() && hds->scalar_type() == hs.scalar_type() &&
                dZd->scalar_type() == dZ.scalar_type() && xd->is_contiguous() && hds->is_contiguous() &&
                dZd->is_contiguous(), "lstmf_wgrad_p_: tangent operands must mirror the primal ones");
  }
  GUARD(x);
  const int M = B * Tn;
  Tensor ws = out_empty({(int64_t)hfrep::lstmf_wgrad_workspace_floats(M, K, (int)impl)}, gW.options());
  hfrep::launch_lstmf_wgrad(x.data_ptr(), hs.data_ptr(), dZ.data_ptr(), tangent ? xd->data_ptr() : nullptr,
                            tangent ? hds->data_ptr() : nullptr, tangent ? dZd->data_ptr() : nullptr, gW.data_ptr<float>(),
                            gU.data_ptr<float>(), gb.has_value() ? gb->data_ptr<float>() : nullptr, M, K, Tn,
                            ws.data_ptr<float>(), cur_stream(x), (int)impl, pm);
}

// dX (M, KO) = dZ W^T with dZ as FP3 planes (M, 3, 400) in the interleaved gate order
Tensor lstmf_dgrad_p(Tensor dzp, Tensor W, int64_t impl) {
  CHECK_GPU(dzp); CHECK_F32(W);
  TORCH_CHECK(is_fp3(dzp) && dzp.dim() == 3 && dzp.is_contiguous() && W.dim() == 2 && W.is_contiguous() &&
              W.size(1) == dzp.size(2), "lstmf_dgrad_p: planes (M, 3, N) and W (KO, N), contiguous");
  TORCH_CHECK(hfrep::lstmf_dgrad_supported(dzp.size(2), W.size(0)), "lstmf_dgrad_p: N must be 400 and KO <= 112");
  GUARD(dzp);
  Tensor x = out_empty({dzp.size(0), W.size(0)}, W.options());
  if (dzp.size(0) == 0) return x;
  const bool ok = hfrep::launch_lstmf_dgrad(dzp.data_ptr(), W.data_ptr<float>(), x.data_ptr<float>(), dzp.size(0),
                                            dzp.size(2), W.size(0), cur_stream(dzp), (int)impl, true);
  TORCH_CHECK(ok, "lstmf_dgrad_p: launch failed");
  return x;
}

// ------------------------------------------------------------------------------------ LSTM v2 (bf16 fused)
void check_lstm2(const Tensor& x, const Tensor& U, int64_t H) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "lstm2 kernels are bf16-only");
  check_lstm_U(U, H);
  TORCH_CHECK(hfrep::lstm2_supported((int)H, (int)x.size(2)), "lstm2: unsupported H/K (H must be 100, K <= 128)");
}

std::tuple<Tensor, Tensor> lstm2_fwd(Tensor x, Tensor W, optional<Tensor> b, Tensor U, int64_t act, bool save) {
  CHECK_GPU(x); CHECK_F32(W);
  TORCH_CHECK(x.dim() == 3, "x must be (B, T, K)");
  const int B = x.size(0), Tn = x.size(1), K = x.size(2), H = U.size(0);
  check_lstm2(x, U, H);
  TORCH_CHECK(W.size(0) == K && W.size(1) == 4 * H, "W must be (K, 4H)");
  if (b.has_value()) { CHECK_F32(*b); TORCH_CHECK(b->numel() == 4 * H, "bias size"); }
  GUARD(x);
  Tensor hs = out_empty({B, Tn, H}, x.options());
  Tensor tape = at::empty({save ? (int64_t)hfrep::lstm2_tape_elems(B, Tn) : 0}, x.options());  // (not poisoned: padded lanes)
  hfrep::launch_lstm2_fwd(x.data_ptr(), W.data_ptr<float>(), b.has_value() ? b->data_ptr<float>() : nullptr,
                          U.data_ptr<float>(), hs.data_ptr(), save ? tape.data_ptr() : nullptr, B, Tn, K, H, (int)act,
                          cur_stream(x));
  return {hs, tape};
}


// W given: also returns dX = dZ W^T (B, T, K) from the same launch; otherwise dX is empty
static int check_dx_W(const optional<Tensor>& W, int H) {
  if (!W.has_value()) return 0;
  CHECK_F32(*W);
  TORCH_CHECK(W->dim() == 2 && W->size(1) == 4 * H && W->size(0) >= 1 && W->size(0) <= 128,
              "fused dX: W must be (K <= 128, 4H)");
  return (int)W->size(0);
}

// Flatten -> Dense(1) critic-head adjoint: dH[b, t, h] = head_d[b] * head_w[t H + h] (head_d (B, 1) bf16,
// head_w (T H) fp32 = the Dense kernel), generated inside the reverse kernels with the skinny-dgrad
// rounding (bf16(float(d) * w)): the (B, T, H) tensor is never materialised.
static void check_head(const optional<Tensor>& d, const Tensor& w, const Tensor& like, int64_t B, int64_t Tn, int64_t H) {
  if (!d.has_value()) return;
  CHECK_GPU(*d); same_dt(*d, like);
  TORCH_CHECK(d->numel() == B && d->is_contiguous(), "head adjoint: d must be (B, 1) contiguous");
  CHECK_F32(w);
  TORCH_CHECK(w.numel() == Tn * H && w.is_contiguous(), "head adjoint: w must hold T * H floats");
}

std::tuple<Tensor, Tensor> lstm2_bwd(optional<Tensor> dH_, Tensor tape, Tensor U, int64_t act, optional<Tensor> W,
                                     bool need_dz, optional<Tensor> head_d, optional<Tensor> head_w) {
  CHECK_GPU(tape);
  const int H = U.size(0);
  TORCH_CHECK(dH_.has_value() != (head_d.has_value() && head_w.has_value()), "lstm2_bwd: dH xor (head_d, head_w)");
  const int B = dH_ ? dH_->size(0) : head_d->size(0);
  const int Tn = dH_ ? dH_->size(1) : head_w->numel() / H;
  check_lstm_U(U, H);
  if (dH_) { CHECK_GPU(*dH_); same_dt(*dH_, tape); TORCH_CHECK(dH_->size(2) == H, "dH shape"); }
  else check_head(head_d, *head_w, tape, B, Tn, H);
  TORCH_CHECK(tape.numel() == (int64_t)hfrep::lstm2_tape_elems(B, Tn), "lstm2_bwd: tape size");
  const int K = check_dx_W(W, H);
  GUARD(tape);
  TORCH_CHECK(need_dz || K, "lstm2_bwd: nothing to compute (need_dz=False without W)");
  const bool gen = !dH_;
  Tensor dZ = out_empty({need_dz ? B : 0, Tn, 4 * H}, tape.options());
  Tensor dX = out_empty({K ? B : 0, Tn, K}, tape.options());
  hfrep::launch_lstm2_bwd(gen ? nullptr : dH_->data_ptr(), tape.data_ptr(), U.data_ptr<float>(),
                          need_dz ? dZ.data_ptr() : nullptr, K ? W->data_ptr<float>() : nullptr,
                          K ? dX.data_ptr() : nullptr, K, B, Tn, H, (int)act, cur_stream(tape),
                          gen ? head_d->data_ptr() : nullptr, gen ? head_w->data_ptr<float>() : nullptr);
  return {dZ, dX};
}

std::tuple<Tensor, Tensor> lstm2_tfwd(Tensor xd, Tensor W, Tensor U, Tensor tape, int64_t act) {
  CHECK_GPU(xd); CHECK_F32(W); CHECK_GPU(tape); same_dt(xd, tape);
  const int B = xd.size(0), Tn = xd.size(1), K = xd.size(2), H = U.size(0);
  check_lstm2(xd, U, H);
  TORCH_CHECK(W.size(0) == K && W.size(1) == 4 * H, "W must be (K, 4H)");
  TORCH_CHECK(tape.numel() == (int64_t)hfrep::lstm2_tape_elems(B, Tn), "lstm2_tfwd: tape size");
  GUARD(xd);
  Tensor hds = out_empty({B, Tn, H}, xd.options());
  Tensor ttape = at::empty_like(tape);  // (not poisoned: padded lanes)
  hfrep::launch_lstm2_tfwd(xd.data_ptr(), W.data_ptr<float>(), U.data_ptr<float>(), tape.data_ptr(), hds.data_ptr(),
                           ttape.data_ptr(), B, Tn, K, H, (int)act, cur_stream(xd));
  return {hds, ttape};
}

// dH / dHd: tensors, or (with head_w) the outer products head_d / head_dd x head_w (either may be
// absent = zeros); the two forms are not mixed in one call
std::tuple<Tensor, Tensor, Tensor, Tensor> lstm2_tbwd(optional<Tensor> dH, optional<Tensor> dHd_, Tensor tape,
                                                      Tensor ttape, Tensor U, int64_t act, optional<Tensor> W,
                                                      optional<Tensor> head_d, optional<Tensor> head_dd,
                                                      optional<Tensor> head_w) {
  CHECK_GPU(tape); CHECK_GPU(ttape); same_dt(tape, ttape);
  const int H = U.size(0);
  const bool head = head_w.has_value();
  TORCH_CHECK(head ? (!dH && !dHd_ && (head_d || head_dd)) : (dHd_.has_value() && !head_d && !head_dd),
              "lstm2_tbwd: (dH?, dHd) tensors xor (head_d?, head_dd?, head_w)");
  const int B = head ? (head_d ? head_d->size(0) : head_dd->size(0)) : dHd_->size(0);
  const int Tn = head ? head_w->numel() / H : dHd_->size(1);
  check_lstm_U(U, H);
  if (!head) {
    CHECK_GPU(*dHd_); same_dt(*dHd_, tape);
    if (dH.has_value()) { CHECK_GPU(*dH); same_dt(*dH, *dHd_); TORCH_CHECK(dH->sizes() == dHd_->sizes(), "dH shape"); }
  } else {
    check_head(head_d, *head_w, tape, B, Tn, H);
    check_head(head_dd, *head_w, tape, B, Tn, H);
  }
  TORCH_CHECK(tape.numel() == (int64_t)hfrep::lstm2_tape_elems(B, Tn) && ttape.numel() == tape.numel(), "tape size");
  GUARD(tape);
  const int K = check_dx_W(W, H);
  // the in-kernel generated head adjoint, with or without the fused input gradient (DX + GEN was parked
  // in r01-r02 for run-to-run drift; the cause was the cross-opcode MFMA SrcC hazard fixed in r03,
  // profiles/r03_race/README.md)
  const bool gen = head;
  Tensor dZ = out_empty({B, Tn, 4 * H}, tape.options()), dZd = out_empty({B, Tn, 4 * H}, tape.options());
  Tensor dX = out_empty({K ? B : 0, Tn, K}, tape.options()), dXd = out_empty({K ? B : 0, Tn, K}, tape.options());
  hfrep::launch_lstm2_tbwd(gen ? nullptr : ptr_or_null(dH), gen ? nullptr : dHd_->data_ptr(), tape.data_ptr(),
                           ttape.data_ptr(), U.data_ptr<float>(), dZ.data_ptr(), dZd.data_ptr(),
                           K ? W->data_ptr<float>() : nullptr, K ? dX.data_ptr() : nullptr, K ? dXd.data_ptr() : nullptr,
                           K, B, Tn, H, (int)act, cur_stream(tape), gen ? ptr_or_null(head_d) : nullptr,
                           gen ? ptr_or_null(head_dd) : nullptr, gen ? head_w->data_ptr<float>() : nullptr);
  return {dZ, dZd, dX, dXd};
}

// ------------------------------------------------------------------------------------ LayerNorm
// save == false (no-grad forward): xhat and rstd come back empty and are never written
// pre_lrelu >= 0: LayerNorm(LeakyReLU(x, pre_lrelu)) in one pass (the activation never hits HBM)
std::tuple<Tensor, Tensor, Tensor> layernorm_fwd(Tensor x, Tensor gamma, Tensor beta, double eps, bool save,
                                                 double pre_lrelu) {
  CHECK_GPU(x); CHECK_F32(gamma); CHECK_F32(beta);
  const int D = x.size(-1);
  TORCH_CHECK(D <= 256 && gamma.numel() == D && beta.numel() == D, "layernorm: D <= 256 and param sizes");
  GUARD(x);
  const int64_t rows = x.numel() / D;
  Tensor y = out_empty_like(x), xhat = save ? out_empty_like(x) : out_empty({0}, x.options());
  std::vector<int64_t> rs(x.sizes().begin(), x.sizes().end() - 1);
  rs.push_back(1);
  Tensor rstd = save ? out_empty(rs, x.options().dtype(at::kFloat)) : out_empty({0}, x.options().dtype(at::kFloat));
  hfrep::launch_layernorm_fwd(dt_of(x), x.data_ptr(), gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(),
                              save ? xhat.data_ptr() : nullptr, save ? rstd.data_ptr<float>() : nullptr, rows, D,
                              (float)eps, (float)pre_lrelu, cur_stream(x));
  return {y, xhat, rstd};
}

Tensor layernorm_bwd_(Tensor dy, Tensor xhat, Tensor rstd, Tensor gamma, optional<Tensor> ggamma,
                      optional<Tensor> gbeta) {
  CHECK_GPU(dy); CHECK_GPU(xhat); same_dt(dy, xhat); CHECK_F32(rstd); CHECK_F32(gamma);
  const int D = dy.size(-1);
  TORCH_CHECK(D <= 256, "layernorm: D <= 256");
  float* gg = nullptr; float* gbp = nullptr;
  if (ggamma.has_value()) { CHECK_F32(*ggamma); gg = ggamma->data_ptr<float>(); }
  if (gbeta.has_value()) { CHECK_F32(*gbeta); gbp = gbeta->data_ptr<float>(); }
  GUARD(dy);
  Tensor dx = out_empty_like(dy);
  const int64_t rows = dy.numel() / D;
  Tensor ws = out_empty({(gg || gbp) ? (int64_t)hfrep::layernorm_bwd_splits(rows) * 2 * D : 0},
                        dy.options().dtype(at::kFloat));
  hfrep::launch_layernorm_bwd(dt_of(dy), dy.data_ptr(), xhat.data_ptr(), rstd.data_ptr<float>(),
                              gamma.data_ptr<float>(), dx.data_ptr(), gg, gbp, (gg || gbp) ? ws.data_ptr<float>() : nullptr,
                              rows, D, cur_stream(dy));
  return dx;
}

Tensor layernorm_tfwd(Tensor xd, Tensor xhat, Tensor rstd, Tensor gamma) {
  CHECK_GPU(xd); CHECK_GPU(xhat); same_dt(xd, xhat); CHECK_F32(rstd); CHECK_F32(gamma);
  const int D = xd.size(-1);
  TORCH_CHECK(D <= 256 && gamma.numel() == D && xhat.numel() == xd.numel() && rstd.numel() * D == xd.numel(),
              "layernorm_tfwd: D <= 256 and matching xd / xhat / rstd");
  GUARD(xd);
  xd = xd.contiguous();
  Tensor yd = out_empty_like(xd);
  hfrep::launch_layernorm_tfwd(dt_of(xd), xd.data_ptr(), xhat.data_ptr(), rstd.data_ptr<float>(),
                               gamma.data_ptr<float>(), yd.data_ptr(), xd.numel() / D, D, cur_stream(xd));
  return yd;
}

// (dx, dxd); need_dx == false returns two empty tensors and only accumulates ggamma / gbeta
std::tuple<Tensor, Tensor> layernorm_tbwd_(optional<Tensor> dy, Tensor dyd, Tensor xd, Tensor xhat, Tensor rstd,
                                           Tensor gamma, Tensor ggamma, Tensor gbeta, bool need_dx) {
  CHECK_GPU(dyd); CHECK_GPU(xd); CHECK_GPU(xhat); same_dt(dyd, xd); same_dt(dyd, xhat);
  CHECK_F32(rstd); CHECK_F32(gamma); CHECK_F32(ggamma); CHECK_F32(gbeta);
  const int D = dyd.size(-1);
  const int64_t n = dyd.numel();
  TORCH_CHECK(D <= 256 && gamma.numel() == D && ggamma.numel() == D && gbeta.numel() == D && xd.numel() == n &&
                  xhat.numel() == n && rstd.numel() * D == n,
              "layernorm_tbwd: D <= 256 and matching operand sizes");
  Tensor dyc;
  if (dy.has_value()) {
    CHECK_GPU(*dy); same_dt(*dy, dyd);
    TORCH_CHECK(dy->numel() == n, "layernorm_tbwd: dy size");
    dyc = dy->contiguous();
  }
  GUARD(dyd);
  dyd = dyd.contiguous(); xd = xd.contiguous();
  const int64_t rows = n / D;
  Tensor dx = need_dx ? out_empty_like(dyd) : out_empty({0}, dyd.options());
  Tensor dxd = need_dx ? out_empty_like(dyd) : out_empty({0}, dyd.options());
  Tensor ws = out_empty({(int64_t)hfrep::layernorm_bwd_splits(rows) * 2 * D}, dyd.options().dtype(at::kFloat));
  hfrep::launch_layernorm_tbwd(dt_of(dyd), dy.has_value() ? dyc.data_ptr() : nullptr, dyd.data_ptr(), xd.data_ptr(),
                               xhat.data_ptr(), rstd.data_ptr<float>(), gamma.data_ptr<float>(),
                               need_dx ? dx.data_ptr() : nullptr, need_dx ? dxd.data_ptr() : nullptr,
                               ggamma.data_ptr<float>(), gbeta.data_ptr<float>(), ws.data_ptr<float>(), rows, D,
                               cur_stream(dyd));
  return {dx, dxd};
}

// ------------------------------------------------------------------------------------ conv1d (causal)
Tensor im2col_causal(Tensor x, int64_t k, int64_t dil) {
  CHECK_GPU(x);
  TORCH_CHECK(x.dim() == 3 && k >= 1 && dil >= 1, "im2col_causal: (B,T,C), k, dil");
  GUARD(x);
  const int B = x.size(0), Tn = x.size(1), C = x.size(2);
  Tensor cols = out_empty({B, Tn, k * C}, x.options());
  hfrep::launch_im2col_causal(dt_of(x), x.data_ptr(), cols.data_ptr(), B, Tn, C, (int)k, (int)dil, cur_stream(x));
  return cols;
}
Tensor col2im_causal(Tensor dcols, int64_t k, int64_t dil, int64_t C) {
  CHECK_GPU(dcols);
  TORCH_CHECK(dcols.dim() == 3 && dcols.size(2) == k * C, "col2im_causal: (B,T,k*C)");
  GUARD(dcols);
  const int B = dcols.size(0), Tn = dcols.size(1);
  Tensor dx = out_empty({B, Tn, C}, dcols.options());
  hfrep::launch_col2im_causal(dt_of(dcols), dcols.data_ptr(), dx.data_ptr(), B, Tn, (int)C, (int)k, (int)dil,
                              cur_stream(dcols));
  return dx;
}

// ------------------------------------------------------------------------------------ WGAN-GP helpers
std::tuple<Tensor, Tensor> gp_coef(Tensor g, double weight) {
  CHECK_GPU(g); GUARD(g);
  const int B = g.size(0);
  const int64_t D = g.numel() / B;
  Tensor v = out_empty_like(g);
  Tensor pen = out_empty({}, g.options().dtype(at::kFloat));
  Tensor rowpen = out_empty({B}, g.options().dtype(at::kFloat));
  hfrep::launch_gp_coef(dt_of(g), g.data_ptr(), v.data_ptr(), pen.data_ptr<float>(), rowpen.data_ptr<float>(), B, D,
                        (float)weight, cur_stream(g));
  return {pen, v};
}

// (pack [w0 + w1 + weight pen, w0, w1, pen] fp32, v): gp_coef plus the critic step's loss record, from
// the W terms w [2] (fp32) of the same step
std::tuple<Tensor, Tensor> gp_coef_pack(Tensor g, double weight, Tensor w) {
  CHECK_GPU(g); GUARD(g);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.numel() == 2 && w.is_contiguous() && w.device() == g.device(),
              "gp_coef_pack: w = the two fp32 W terms on g's device");
  const int B = g.size(0);
  const int64_t D = g.numel() / B;
  Tensor v = out_empty_like(g);
  Tensor pen = out_empty({}, g.options().dtype(at::kFloat));
  Tensor pack = out_empty({4}, g.options().dtype(at::kFloat));
  Tensor rowpen = out_empty({B}, g.options().dtype(at::kFloat));
  hfrep::launch_gp_coef(dt_of(g), g.data_ptr(), v.data_ptr(), pen.data_ptr<float>(), rowpen.data_ptr<float>(), B, D,
                        (float)weight, cur_stream(g), w.data_ptr<float>(), pack.data_ptr<float>());
  return {pack, v};
}

// pack [w0 + w1 + weight pen, w0, w1, pen] from gp_coef's penalty and the W terms (gp_coef_pack's record)
Tensor gp_pack(Tensor pen, double weight, Tensor w) {
  CHECK_GPU(pen); GUARD(pen);
  TORCH_CHECK(pen.scalar_type() == at::kFloat && pen.numel() == 1 && w.scalar_type() == at::kFloat && w.numel() == 2 &&
              w.is_contiguous() && w.device() == pen.device(), "gp_pack: fp32 penalty [1] and W terms [2]");
  Tensor pack = out_empty({4}, pen.options());
  hfrep::launch_gp_pack(pen.data_ptr<float>(), w.data_ptr<float>(), (float)weight, pack.data_ptr<float>(),
                        cur_stream(pen));
  return pack;
}

// (segment losses [2] fp32, dL/dp like p): see csrc/misc.hip gan_loss_kernel
std::tuple<Tensor, Tensor> gan_loss(Tensor p, int64_t split, double la, double lb, int64_t kind) {
  CHECK_GPU(p); GUARD(p);
  TORCH_CHECK(p.is_contiguous(), "gan_loss: contiguous scores");
  TORCH_CHECK(kind == 0 || kind == 1, "gan_loss: kind 0 (wasserstein) or 1 (bce)");
  const int64_t n = p.numel();
  TORCH_CHECK(split >= 0 && split <= n, "gan_loss: split");
  Tensor grad = out_empty_like(p);
  Tensor out = out_empty({2}, p.options().dtype(at::kFloat));
  Tensor partial = at::empty({2 * hfrep::gan_loss_partials()}, p.options().dtype(at::kFloat));
  hfrep::launch_gan_loss(dt_of(p), p.data_ptr(), n, split, (float)la, (float)lb, (int)kind, grad.data_ptr(),
                         partial.data_ptr<float>(), out.data_ptr<float>(), cur_stream(p));
  return {out, grad};
}

Tensor interpolate(Tensor real, Tensor fake, Tensor alpha) {
  CHECK_GPU(real); CHECK_GPU(fake); same_dt(real, fake); CHECK_F32(alpha);
  TORCH_CHECK(real.sizes() == fake.sizes() && alpha.numel() == real.size(0), "interpolate: shapes");
  GUARD(real);
  Tensor out = out_empty_like(real);
  const int B = real.size(0);
  hfrep::launch_interpolate(dt_of(real), real.data_ptr(), fake.data_ptr(), alpha.data_ptr<float>(), out.data_ptr(), B,
                            real.numel() / B, cur_stream(real));
  return out;
}

// ------------------------------------------------------------------------------------ RNG / sampling
void philox_fill_(Tensor out, int64_t seed, Tensor ctr, int64_t dist) {
  CHECK_GPU(out);
  TORCH_CHECK(ctr.is_cuda() && ctr.scalar_type() == at::kLong && ctr.numel() == 1, "ctr must be a 1-element int64 GPU tensor");
  GUARD(out);
  hfrep::launch_philox_fill(dt_of(out), out.data_ptr(), out.numel(), (uint64_t)seed, ctr.data_ptr<int64_t>(), (int)dist,
                            cur_stream(out));
}

Tensor sample_windows(Tensor data, int64_t batch, int64_t seed, Tensor ctr, at::ScalarType out_dtype,
                      optional<Tensor> dst) {
  CHECK_F32(data);
  TORCH_CHECK(ctr.is_cuda() && ctr.scalar_type() == at::kLong && ctr.numel() == 1, "ctr must be a 1-element int64 GPU tensor");
  GUARD(data);
  std::vector<int64_t> shape(data.sizes().begin(), data.sizes().end());
  shape[0] = batch;
  if (dst.has_value())
    TORCH_CHECK(dst->is_cuda() && dst->device() == data.device() && dst->is_contiguous() && dst->scalar_type() == out_dtype &&
                    dst->sizes() == at::IntArrayRef(shape),
                "sample_windows: dst must be a contiguous (batch, ...) tensor of out_dtype on data's device");
  Tensor out = dst.has_value() ? *dst : out_empty(shape, data.options().dtype(out_dtype));
  const int64_t N = data.size(0), D = data.numel() / N;
  hfrep::launch_sample_windows(dt_of(out), data.data_ptr<float>(), N, D, out.data_ptr(), (int)batch, (uint64_t)seed,
                               ctr.data_ptr<int64_t>(), cur_stream(data));
  return out;
}

// ------------------------------------------------------------------------------------ autoencoder
// The whole fit of the factor autoencoder (Autoencoder_encapsulate.py:72-105) in one launch: Xt (nt, A)
// and Xv (nv, A) fp32 (MinMax-scaled), order (epochs, nt) int32 batch permutations, We (A, k) / Wd (k, A)
// fp32 weights and their Nadam slots, the shared step counter / momentum cache.  Returns the per-epoch
// (train loss, val loss) history (epochs, 2) fp64 and the number of epochs run (int32 scalar tensor).
bool ae_fit_supported(int64_t A, int64_t k, int64_t batch) { return hfrep::ae_fit_supported((int)A, (int)k, (int)batch); }

// every fit of the lists trains in ONE launch (one workgroup per fit, csrc/ae.hip); shared: A (the
// inputs' width), batch, the Nadam hyper-parameters and the dtype.  Returns hist (n, max epochs, 2)
// fp64 and the epochs each fit ran (n,) int32.
std::tuple<Tensor, Tensor> ae_fit(at::TensorList Xt, at::TensorList Xv, at::TensorList order, at::TensorList We,
                                  at::TensorList Wd, at::TensorList mWe, at::TensorList vWe, at::TensorList mWd,
                                  at::TensorList vWd, at::TensorList step, at::TensorList m_cache, at::IntArrayRef patience, double lr, double b1, double b2, double eps,
                                  int64_t batch, bool bf16) {
  const size_t n = Xt.size();
  TORCH_CHECK(n >= 1, "ae_fit: at least one fit");
  for (at::TensorList l : {Xv, order, We, Wd, mWe, vWe, mWd, vWd, step, m_cache})
    TORCH_CHECK(l.size() == n, "ae_fit: every per-fit list needs ", n, " entries");
  TORCH_CHECK(patience.size() == n, "ae_fit: one patience per fit");
  const auto dev = Xt[0].device();
  TORCH_CHECK(Xt[0].is_cuda() && Xt[0].dim() == 2, "ae_fit: Xt (nt, A) on the GPU");
  const int A = Xt[0].size(1);
  int max_ep = 0;
  std::vector<hfrep::AeFitJob> jobs(n);
  for (size_t i = 0; i < n; ++i) {
    for (const Tensor* t : {&Xt[i], &Xv[i], &We[i], &Wd[i], &mWe[i], &vWe[i], &mWd[i], &vWd[i], &step[i], &m_cache[i]}) {
      CHECK_F32(*t);
      TORCH_CHECK(t->is_contiguous() && t->device() == dev, "ae_fit: contiguous fp32 tensors on one device");
    }
    const Tensor& o = order[i];
    TORCH_CHECK(o.device() == dev && o.scalar_type() == at::kInt && o.is_contiguous() && o.dim() == 2,
                "ae_fit: order must be a contiguous (epochs, nt) int32 tensor");
    TORCH_CHECK(Xt[i].dim() == 2 && Xv[i].dim() == 2 && Xt[i].size(1) == A && Xv[i].size(1) == A,
                "ae_fit: Xt (nt, A), Xv (nv, A) with one A for every fit");
    const int nt = Xt[i].size(0), k = We[i].numel() / A, epochs = o.size(0);
    TORCH_CHECK(o.size(1) == nt && nt > 0 && epochs > 0, "ae_fit: order shape");
    TORCH_CHECK(We[i].numel() == (int64_t)A * k && Wd[i].numel() == We[i].numel() && mWe[i].numel() == We[i].numel() &&
                    vWe[i].numel() == We[i].numel() && mWd[i].numel() == We[i].numel() && vWd[i].numel() == We[i].numel(),
                "ae_fit: weight / slot sizes");
    TORCH_CHECK(step[i].numel() == 1 && m_cache[i].numel() == 1, "ae_fit: scalar counters");
    TORCH_CHECK(hfrep::ae_fit_supported(A, k, (int)batch) && patience[i] >= 1, "ae_fit: A, k <= 32 and batch <= 64");
    max_ep = std::max(max_ep, epochs);
    hfrep::AeFitJob& J = jobs[i];
    J.Xt = Xt[i].data_ptr<float>();
    J.Xv = Xv[i].data_ptr<float>();
    J.order = o.data_ptr<int>();
    J.We = We[i].data_ptr<float>(); J.Wd = Wd[i].data_ptr<float>();
    J.mWe = mWe[i].data_ptr<float>(); J.vWe = vWe[i].data_ptr<float>();
    J.mWd = mWd[i].data_ptr<float>(); J.vWd = vWd[i].data_ptr<float>();
    J.step = step[i].data_ptr<float>(); J.m_cache = m_cache[i].data_ptr<float>();
    J.nt = nt; J.nv = Xv[i].size(0); J.epochs = epochs; J.patience = (int)patience[i]; J.k = k; J.pad_ = 0;
  }
  GUARD(Xt[0]);
  const auto fopt = Xt[0].options();
  Tensor hist = at::zeros({(int64_t)n, max_ep, 2}, fopt.dtype(at::kDouble));
  Tensor nep = at::zeros({(int64_t)n}, fopt.dtype(at::kInt));
  for (size_t i = 0; i < n; ++i) {
    jobs[i].hist = hist.data_ptr<double>() + i * (size_t)max_ep * 2;
    jobs[i].nep = nep.data_ptr<int>() + i;
  }
  // the job records: host bytes -> device (ordered on the current stream before the launch)
  const int64_t bytes = (int64_t)(n * sizeof(hfrep::AeFitJob));
  Tensor host = at::empty({bytes}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), jobs.data(), bytes);
  Tensor dj = host.to(dev);
  hfrep::launch_ae_fit(bf16, reinterpret_cast<const hfrep::AeFitJob*>(dj.data_ptr()), (int)n, (int)batch, (float)lr,
                       (float)b1, (float)b2, (float)eps, A, cur_stream(Xt[0]));
  const hipError_t err = hipGetLastError();
  TORCH_CHECK(err == hipSuccess, "ae_fit: launch failed: ", hipGetErrorString(err));
  return {hist, nep};
}

// ------------------------------------------------------------------------------------ optimizers
void rmsprop_(Tensor p, Tensor g, Tensor ms, double lr, double rho, double eps, double clip, double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(ms);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == ms.numel(), "rmsprop_: size mismatch");
  GUARD(p);
  hfrep::launch_rmsprop(p.data_ptr<float>(), g.data_ptr<float>(), ms.data_ptr<float>(), p.numel(), (float)lr,
                        (float)rho, (float)eps, (float)clip, (float)gscale, cur_stream(p));
}

void adam_(Tensor p, Tensor g, Tensor m, Tensor v, Tensor step, double lr, double b1, double b2, double eps,
           double clip, double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(step);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam_: size mismatch");
  GUARD(p);
  hfrep::launch_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.numel(),
                     step.data_ptr<float>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)clip, (float)gscale,
                     cur_stream(p));
}

void nadam_(Tensor p, Tensor g, Tensor m, Tensor v, Tensor step, Tensor m_cache, double lr, double b1, double b2,
            double eps, double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(step); CHECK_F32(m_cache);
  GUARD(p);
  hfrep::launch_nadam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.numel(),
                      step.data_ptr<float>(), m_cache.data_ptr<float>(), (float)lr, (float)b1, (float)b2, (float)eps,
                      (float)gscale, cur_stream(p));
}

void step_advance_(Tensor step, optional<Tensor> m_cache, double b1) {
  CHECK_F32(step);
  GUARD(step);
  float* mc = nullptr;
  if (m_cache.has_value()) { CHECK_F32(*m_cache); mc = m_cache->data_ptr<float>(); }
  hfrep::launch_step_advance(step.data_ptr<float>(), mc, (float)b1, cur_stream(step));
}

void clip_(Tensor p, double c) {
  CHECK_F32(p);
  GUARD(p);
  hfrep::launch_clip(p.data_ptr<float>(), p.numel(), (float)c, cur_stream(p));
}

// ------------------------------------------------------------------------------------ p2p all-reduce
// The buffer is a uint8 tensor over the hipExtMallocWithFlags allocation (freed by its deleter);
// its data_ptr is the allocation base, which is what an IPC handle names.
Tensor p2p_buffer(int64_t cap, int64_t device) {
  TORCH_CHECK(cap > 0, "p2p_buffer: cap must be positive");
  bool fine = false;
  void* p = hfrep::p2p_alloc(cap, (int)device, &fine);
  auto opts = at::TensorOptions().dtype(at::kByte).device(at::Device(at::kCUDA, (int)device));
  return torch::from_blob(p, {(int64_t)hfrep::p2p_buffer_bytes(cap)}, [](void* q) { hfrep::p2p_free(q); }, opts);
}

std::vector<int64_t> p2p_handle(Tensor buf) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kByte, "p2p_handle: a p2p_buffer tensor");
  uint8_t h[64];
  hfrep::p2p_ipc_handle(buf.data_ptr(), h);
  return std::vector<int64_t>(h, h + 64);
}

int64_t p2p_open(std::vector<int64_t> handle, int64_t device) {
  TORCH_CHECK(handle.size() == 64, "p2p_open: a 64-byte IPC handle");
  uint8_t h[64];
  for (int i = 0; i < 64; ++i) h[i] = (uint8_t)handle[i];
  return (int64_t)reinterpret_cast<intptr_t>(hfrep::p2p_ipc_open(h, (int)device));
}

void p2p_close(int64_t ptr) { hfrep::p2p_ipc_close(reinterpret_cast<void*>((intptr_t)ptr)); }

void p2p_allreduce_(Tensor x, Tensor buf, std::vector<int64_t> peers, int64_t rank, int64_t cap, double scale,
                    double timeout_s) {
  CHECK_F32(x);
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kByte && buf.device() == x.device(),
              "p2p_allreduce_: buf must be this device's p2p_buffer");
  const int world = (int)peers.size();
  TORCH_CHECK(world >= 1 && world <= hfrep::kP2PMaxRanks && rank >= 0 && rank < world, "p2p_allreduce_: 1 <= world <= 8");
  TORCH_CHECK(x.numel() <= cap && buf.numel() >= (int64_t)hfrep::p2p_buffer_bytes(cap), "p2p_allreduce_: x exceeds cap");
  TORCH_CHECK(peers[rank] == (int64_t)reinterpret_cast<intptr_t>(buf.data_ptr()), "p2p_allreduce_: peers[rank] must be buf");
  hfrep::P2PPeers pp{};
  for (int r = 0; r < world; ++r) pp.base[r] = reinterpret_cast<char*>((intptr_t)peers[r]);
  TORCH_CHECK(timeout_s > 0, "p2p_allreduce_: timeout_s must be positive");
  GUARD(x);
  // the tick rate is per device and fixed: query it once per (device, timeout)
  static thread_local int s_dev = -1;
  static thread_local double s_sec = -1;
  static thread_local uint64_t s_ticks = 0;
  if (s_dev != x.get_device() || s_sec != timeout_s) {
    s_ticks = hfrep::p2p_timeout_ticks(timeout_s, x.get_device());
    s_dev = x.get_device();
    s_sec = timeout_s;
  }
  hfrep::launch_p2p_allreduce(x.data_ptr<float>(), x.numel(), pp, (int)rank, world, cap, (float)scale, s_ticks,
                              cur_stream(x));
}

int64_t p2p_error(Tensor buf) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kByte, "p2p_error: a p2p_buffer tensor");
  GUARD(buf);
  return hfrep::p2p_read_error(buf.data_ptr());
}

}  // namespace

TORCH_LIBRARY(hfrep, m) {
  m.def("linear(Tensor x, Tensor W, Tensor? b, int act, Tensor(a!)? out=None) -> Tensor");  // writes into out when given
  m.def("linear_dgrad(Tensor dz, Tensor W) -> Tensor");
  m.def("linear_wgrad_(Tensor x, Tensor dz, Tensor(a!) gW, Tensor(b!)? gb, int shiftT=0) -> ()");
  m.def("fp3_split(Tensor x, bool interleave=False) -> Tensor");
  m.def("fp3_join(Tensor p, bool interleave=False) -> Tensor");
  m.def("lstmf_wgrad_p_(Tensor x, Tensor hs, Tensor dZ, Tensor(a!) gW, Tensor(b!) gU, Tensor(c!)? gb, Tensor? xd=None, Tensor? hds=None, Tensor? dZd=None, int impl=0) -> ()");
  m.def("lstmf_dgrad_p(Tensor dzp, Tensor W, int impl=0) -> Tensor");
  m.def("lstm_wgrad_(Tensor x, Tensor hs, Tensor dZ, Tensor(a!) gW, Tensor(b!) gU, Tensor(c!)? gb, Tensor? xd=None, Tensor? hds=None, Tensor? dZd=None, int impl=0) -> ()");
  m.def("act_fwd(Tensor x, int act) -> Tensor");
  m.def("act_bwd(Tensor dy, Tensor y, int act) -> Tensor");
  m.def("act_tangent_bwd(Tensor dyd, Tensor y, Tensor zd, int act) -> Tensor");
  m.def("lstm_fwd(Tensor zx, Tensor U, int act, bool save) -> (Tensor, Tensor, Tensor)");
  m.def("lstm_bwd(Tensor dH, Tensor gates, Tensor cs, Tensor U, int act) -> Tensor");
  m.def("lstm_tfwd(Tensor dzx, Tensor gates, Tensor cs, Tensor U, int act) -> (Tensor, Tensor, Tensor)");
  m.def("lstm_tbwd(Tensor? dH, Tensor dHd, Tensor gates, Tensor cs, Tensor zds, Tensor cds, Tensor U, int act) -> (Tensor, Tensor)");
  m.def("lstmf_supported(int H, int K, int act) -> bool", &lstmf_supported);  // no tensor inputs: catch-all kernel
  m.def("narrowf_supported(int K, int N) -> bool", &narrowf_supported);
  m.def("set_lstmf_fwd_impl(int v) -> int", &set_lstmf_fwd_impl);
  m.def("set_lstmf_bwd_impl(int v) -> int", &set_lstmf_bwd_impl);
  m.def("lstmf_fwd(Tensor x, Tensor W, Tensor? b, Tensor U, int act, bool save) -> (Tensor, Tensor)");
  m.def("linear_head_cs(Tensor x, Tensor W, Tensor? b, int split, float wa, float wb, Tensor(a!) gW, Tensor(b!)? gb) -> Tensor");
  m.def("linear_head_cs_supported(int K) -> bool", &linear_head_cs_supported);
  m.def("lstmf_bwd(Tensor? dH, Tensor tape, Tensor U, int act, int B, int T, Tensor? hd=None, Tensor? hw=None) -> Tensor");
  m.def("lstmf_tbwd(Tensor? dH, Tensor? dHd, Tensor tape, Tensor ttape, Tensor U, int act, int B, int T, Tensor? hd=None, "
        "Tensor? hdd=None, Tensor? hw=None) -> (Tensor, Tensor)");
  m.def("lstmf_tfwd(Tensor xd, Tensor W, Tensor U, Tensor tape, int act) -> (Tensor, Tensor)");
  m.def("lstmf_dgrad(Tensor dz, Tensor W, int impl=0) -> Tensor");
  m.def("lstm2_fwd(Tensor x, Tensor W, Tensor? b, Tensor U, int act, bool save) -> (Tensor, Tensor)");
  m.def("lstm2_bwd(Tensor? dH, Tensor tape, Tensor U, int act, Tensor? W=None, bool need_dz=True, Tensor? head_d=None, "
        "Tensor? head_w=None) -> (Tensor, Tensor)");
  m.def("lstm2_tfwd(Tensor xd, Tensor W, Tensor U, Tensor tape, int act) -> (Tensor, Tensor)");
  m.def("lstm2_tbwd(Tensor? dH, Tensor? dHd, Tensor tape, Tensor ttape, Tensor U, int act, Tensor? W=None, "
        "Tensor? head_d=None, Tensor? head_dd=None, Tensor? head_w=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("set_debug_poison(bool on) -> bool", &set_debug_poison);  // no tensor inputs: catch-all kernel
  m.def("layernorm_fwd(Tensor x, Tensor gamma, Tensor beta, float eps, bool save=True, float pre_lrelu=-1.0) -> "
        "(Tensor, Tensor, Tensor)");
  m.def("layernorm_bwd_(Tensor dy, Tensor xhat, Tensor rstd, Tensor gamma, Tensor(a!)? ggamma, Tensor(b!)? gbeta) -> Tensor");
  m.def("layernorm_tfwd(Tensor xd, Tensor xhat, Tensor rstd, Tensor gamma) -> Tensor");
  m.def("layernorm_tbwd_(Tensor? dy, Tensor dyd, Tensor xd, Tensor xhat, Tensor rstd, Tensor gamma, "
        "Tensor(a!) ggamma, Tensor(b!) gbeta, bool need_dx) -> (Tensor, Tensor)");
  m.def("gp_coef(Tensor g, float weight) -> (Tensor, Tensor)");
  m.def("gp_coef_pack(Tensor g, float weight, Tensor w) -> (Tensor, Tensor)");
  m.def("gp_pack(Tensor pen, float weight, Tensor w) -> Tensor");
  m.def("gan_loss(Tensor p, int split, float la, float lb, int kind) -> (Tensor, Tensor)");
  m.def("im2col_causal(Tensor x, int k, int dil) -> Tensor");
  m.def("col2im_causal(Tensor dcols, int k, int dil, int C) -> Tensor");
  m.def("interpolate(Tensor real, Tensor fake, Tensor alpha) -> Tensor");
  m.def("philox_fill_(Tensor(a!) out, int seed, Tensor(b!) ctr, int dist) -> ()");
  m.def("sample_windows(Tensor data, int batch, int seed, Tensor(a!) ctr, ScalarType out_dtype, Tensor(b!)? dst=None) -> Tensor");
  m.def("ae_fit_supported(int A, int k, int batch) -> bool", &ae_fit_supported);  // no tensor inputs: catch-all kernel
  m.def("ae_fit(Tensor[] Xt, Tensor[] Xv, Tensor[] order, Tensor(a!)[] We, Tensor(b!)[] Wd, Tensor(c!)[] mWe, "
        "Tensor(d!)[] vWe, Tensor(e!)[] mWd, Tensor(f!)[] vWd, Tensor(g!)[] step, Tensor(h!)[] m_cache, int[] patience, "
        "float lr, float b1, float b2, float eps, int batch, bool bf16) -> (Tensor, Tensor)");
  m.def("rmsprop_(Tensor(a!) p, Tensor g, Tensor(b!) ms, float lr, float rho, float eps, float clip, float gscale) -> ()");
  m.def("adam_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor step, float lr, float b1, float b2, float eps, float clip, float gscale) -> ()");
  m.def("nadam_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor step, Tensor m_cache, float lr, float b1, float b2, float eps, float gscale) -> ()");
  m.def("step_advance_(Tensor(a!) step, Tensor(b!)? m_cache, float b1) -> ()");
  m.def("clip_(Tensor(a!) p, float c) -> ()");
  m.def("p2p_buffer(int cap, int device) -> Tensor", &p2p_buffer);  // no tensor inputs: catch-all kernel
  m.def("p2p_handle(Tensor buf) -> int[]");
  m.def("p2p_open(int[] handle, int device) -> int", &p2p_open);
  m.def("p2p_close(int ptr) -> ()", &p2p_close);
  m.def("p2p_allreduce_(Tensor(a!) x, Tensor buf, int[] peers, int rank, int cap, float scale, float timeout_s) -> ()");
  m.def("p2p_error(Tensor buf) -> int");
}

TORCH_LIBRARY_IMPL(hfrep, CUDA, m) {
  m.impl("linear", &linear);
  m.impl("p2p_handle", &p2p_handle);
  m.impl("p2p_allreduce_", &p2p_allreduce_);
  m.impl("p2p_error", &p2p_error);
  m.impl("linear_dgrad", &linear_dgrad);
  m.impl("linear_wgrad_", &linear_wgrad_);
  m.impl("lstm_wgrad_", &lstm_wgrad_);
  m.impl("act_fwd", &act_fwd);
  m.impl("act_bwd", &act_bwd);
  m.impl("act_tangent_bwd", &act_tangent_bwd);
  m.impl("lstm_fwd", &lstm_fwd);
  m.impl("lstmf_fwd", &lstmf_fwd);
  m.impl("lstmf_tfwd", &lstmf_tfwd);
  m.impl("linear_head_cs", &linear_head_cs);
  m.impl("lstmf_bwd", &lstmf_bwd);
  m.impl("lstmf_tbwd", &lstmf_tbwd);
  m.impl("lstmf_dgrad", &lstmf_dgrad);
  m.impl("fp3_split", &fp3_split);
  m.impl("fp3_join", &fp3_join);
  m.impl("lstmf_wgrad_p_", &lstmf_wgrad_p_);
  m.impl("lstmf_dgrad_p", &lstmf_dgrad_p);
  m.impl("lstm_bwd", &lstm_bwd);
  m.impl("lstm_tfwd", &lstm_tfwd);
  m.impl("lstm_tbwd", &lstm_tbwd);
  m.impl("lstm2_fwd", &lstm2_fwd);
  m.impl("lstm2_bwd", &lstm2_bwd);
  m.impl("lstm2_tfwd", &lstm2_tfwd);
  m.impl("lstm2_tbwd", &lstm2_tbwd);
  m.impl("layernorm_fwd", &layernorm_fwd);
  m.impl("layernorm_bwd_", &layernorm_bwd_);
  m.impl("layernorm_tfwd", &layernorm_tfwd);
  m.impl("layernorm_tbwd_", &layernorm_tbwd_);
  m.impl("gp_coef", &gp_coef);
  m.impl("gp_coef_pack", &gp_coef_pack);
  m.impl("gp_pack", &gp_pack);
  m.impl("gan_loss", &gan_loss);
  m.impl("im2col_causal", &im2col_causal);
  m.impl("col2im_causal", &col2im_causal);
  m.impl("interpolate", &interpolate);
  m.impl("philox_fill_", &philox_fill_);
  m.impl("sample_windows", &sample_windows);
  m.impl("ae_fit", &ae_fit);
  m.impl("rmsprop_", &rmsprop_);
  m.impl("adam_", &adam_);
  m.impl("nadam_", &nadam_);
  m.impl("step_advance_", &step_advance_);
  m.impl("clip_", &clip_);
}
