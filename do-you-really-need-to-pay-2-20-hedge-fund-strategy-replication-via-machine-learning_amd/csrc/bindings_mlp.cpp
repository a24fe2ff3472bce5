// torch op registrations of the fused MLP-GAN passes (csrc/mlp.hip), a fragment of the hfrep library
// (bindings.cpp holds the rest).  Same conventions: host-side validation, outputs through the caching
// allocator, launches on the tensor's current HIP stream (graph-capturable), CUDA dispatch key only.
//
// Activations are (B, T, F) / (B, T, H) tensors of one dtype (fp32 or bf16); weights are the fp32
// master views of the flat parameter buffer, passed as a list in model order:
//   generator gp = [W1 (F,H), b1, gamma1, beta1, W2 (H,H), b2, gamma2, beta2, W3 (H,F), b3]
//   critic    cp = [W1 (F,H), b1, W2 (H,H), b2, w3 (T*H or H, 1), b3 (1)]
#include <torch/extension.h>
#include <torch/library.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels.h"
#include "mlp.h"

#include <tuple>
#include <vector>

namespace {

using at::Tensor;
using c10::optional;

inline hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}
#define GUARD(t) c10::hip::HIPGuardMasqueradingAsCUDA _guard((t).device())

inline int act_dt(const Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "mlp ops: activations must be contiguous GPU tensors");
  if (t.scalar_type() == at::kBFloat16) return hfrep::DT_BF16;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "mlp ops: float32 or bfloat16 activations");
  return hfrep::DT_F32;
}
inline const float* w(const Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == numel,
              "mlp ops: ", what, " must be a contiguous fp32 GPU tensor of ", numel, " elements");
  return t.data_ptr<float>();
}
// (B, T, F) activations: returns M = B T, checks the feature count
inline int64_t rows_of(const Tensor& x, int64_t feat, const char* what) {
  TORCH_CHECK(x.dim() == 3 && x.size(2) == feat, "mlp ops: ", what, " must be (B, T, ", feat, ")");
  return x.size(0) * x.size(1);
}

hfrep::MlpGen gen_of(const std::vector<Tensor>& p, int64_t F, int64_t H) {
  TORCH_CHECK(p.size() == 10, "mlp ops: generator weights [W1, b1, g1, be1, W2, b2, g2, be2, W3, b3]");
  return hfrep::MlpGen{w(p[0], F * H, "W1"), w(p[1], H, "b1"), w(p[2], H, "gamma1"), w(p[3], H, "beta1"),
                       w(p[4], H * H, "W2"), w(p[5], H, "b2"), w(p[6], H, "gamma2"), w(p[7], H, "beta2"),
                       w(p[8], H * F, "W3"), w(p[9], F, "b3")};
}
hfrep::MlpCritic critic_of(const std::vector<Tensor>& p, int64_t F, int64_t H, int64_t head_len) {
  TORCH_CHECK(p.size() == 6, "mlp ops: critic weights [W1, b1, W2, b2, w3, b3]");
  return hfrep::MlpCritic{w(p[0], F * H, "W1"), w(p[1], H, "b1"), w(p[2], H * H, "W2"), w(p[3], H, "b2"),
                          w(p[4], head_len, "w3"), w(p[5], 1, "b3")};
}
inline int64_t hidden_of(const std::vector<Tensor>& p, int64_t F) {
  TORCH_CHECK(!p.empty() && p[0].dim() == 2 && p[0].size(0) == F, "mlp ops: W1 must be (F, H)");
  const int64_t H = p[0].size(1);
  TORCH_CHECK(hfrep::mlp_supported((int)F, (int)H), "mlp ops: (F, H) = (", F, ", ", H, ") not instantiated");
  return H;
}
inline Tensor slab_new(const Tensor& like, int64_t M, int64_t L) {
  // every wave of the launch writes its whole row (also waves without a tile): no fill needed
  return at::empty({(int64_t)hfrep::mlp_slab_rows(M), L}, like.options().dtype(at::kFloat));
}

bool mlp_supported_op(int64_t F, int64_t H) { return hfrep::mlp_supported((int)F, (int)H); }

Tensor mlp_gen_fwd(Tensor noise, std::vector<Tensor> gp, optional<Tensor> out) {
  const int dt = act_dt(noise);
  const int64_t F = noise.size(-1), H = hidden_of(gp, F), M = rows_of(noise, F, "noise");
  const auto g = gen_of(gp, F, H);
  GUARD(noise);
  if (out.has_value())
    TORCH_CHECK(out->is_cuda() && out->is_contiguous() && out->scalar_type() == noise.scalar_type() &&
                    out->numel() == noise.numel() && out->device() == noise.device(),
                "mlp_gen_fwd: out must be a contiguous tensor like noise");
  Tensor y = out.has_value() ? out->view(noise.sizes()) : at::empty_like(noise);
  hfrep::launch_mlp_gen_fwd(dt, noise.data_ptr(), g, y.data_ptr(), M, (int)F, (int)H, cur_stream(noise));
  return y;
}

Tensor mlp_wgp_norm(Tensor like, std::vector<Tensor> cp) {
  const int dt = act_dt(like);
  const int64_t F = like.size(-1), H = hidden_of(cp, F), M = rows_of(like, F, "like"), T = like.size(1);
  const auto c = critic_of(cp, F, H, T * H);
  GUARD(like);
  Tensor gsq = at::empty({like.size(0), T}, like.options().dtype(at::kFloat));
  hfrep::launch_mlp_wgp_norm(dt, c, gsq.data_ptr<float>(), M, (int)T, (int)F, (int)H, cur_stream(like));
  return gsq;
}

std::tuple<Tensor, Tensor> mlp_wgp_coef(Tensor gsq, double lam) {
  TORCH_CHECK(gsq.is_cuda() && gsq.scalar_type() == at::kFloat && gsq.is_contiguous() && gsq.dim() == 2,
              "mlp_wgp_coef: gsq (B, T) fp32");
  GUARD(gsq);
  const int64_t B = gsq.size(0), T = gsq.size(1);
  Tensor c = at::empty({B}, gsq.options()), e = at::empty({hfrep::mlp_wgp_coef_parts(B)}, gsq.options());
  hfrep::launch_mlp_wgp_coef(gsq.data_ptr<float>(), (int)T, B, (float)lam, c.data_ptr<float>(), e.data_ptr<float>(),
                             cur_stream(gsq));
  return {c, e};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> mlp_wgp_critic(Tensor real, Tensor fake, Tensor c,
                                                                          std::vector<Tensor> cp) {
  const int dt = act_dt(real);
  TORCH_CHECK(fake.scalar_type() == real.scalar_type() && fake.sizes() == real.sizes(), "mlp_wgp_critic: fake like real");
  act_dt(fake);
  const int64_t F = real.size(-1), H = hidden_of(cp, F), M = rows_of(real, F, "real"), B = real.size(0), T = real.size(1);
  const auto cr = critic_of(cp, F, H, T * H);
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kFloat && c.is_contiguous() && c.numel() == B,
              "mlp_wgp_critic: c (B) fp32");
  GUARD(real);
  Tensor X2c = at::empty({B, T, H}, real.options()), dY2 = at::empty({B, T, H}, real.options());
  Tensor X1c = at::empty({B, T, F}, real.options()), dY1 = at::empty({B, T, H}, real.options());
  Tensor Y3c = at::empty({B, T, H}, real.options());
  Tensor slab = slab_new(real, M, 2);
  hfrep::launch_mlp_wgp_critic(dt, real.data_ptr(), fake.data_ptr(), c.data_ptr<float>(), cr, X2c.data_ptr(),
                               dY2.data_ptr(), X1c.data_ptr(), dY1.data_ptr(), Y3c.data_ptr(), slab.data_ptr<float>(), M,
                               (int)T, (int)F, (int)H, cur_stream(real));
  return {X2c, dY2, X1c, dY1, Y3c, slab};
}

bool mlp_wgpw_supported_op(int64_t F, int64_t T) { return hfrep::mlp_wgpw_supported((int)F, (int)T); }

// the GP critic update with per-t column-sum weight gradients (fp32 / bf16): adds gW1, gW2, gw3 into the
// fp32 gradient views and returns the W-loss slab
Tensor mlp_wgp_critic_t(Tensor real, Tensor fake, Tensor c, std::vector<Tensor> cp, Tensor gW1, Tensor gW2, Tensor gw3) {
  const int dt = act_dt(real);
  TORCH_CHECK(fake.scalar_type() == real.scalar_type() && fake.sizes() == real.sizes(), "mlp_wgp_critic_t: fake like real");
  act_dt(fake);
  const int64_t F = real.size(-1), H = hidden_of(cp, F), B = real.size(0), T = real.size(1);
  rows_of(real, F, "real");
  const auto cr = critic_of(cp, F, H, T * H);
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kFloat && c.is_contiguous() && c.numel() == B,
              "mlp_wgp_critic_t: c (B) fp32");
  for (const Tensor* g : {&gW1, &gW2, &gw3})
    TORCH_CHECK(g->device() == real.device(), "mlp_wgp_critic_t: gradients on the activations' device");
  float* pW1 = const_cast<float*>(w(gW1, F * H, "gW1"));
  float* pW2 = const_cast<float*>(w(gW2, H * H, "gW2"));
  float* pw3 = const_cast<float*>(w(gw3, T * H, "gw3"));
  GUARD(real);
  const int P = hfrep::mlp_wgpt_blocks((int)T);
  auto f32 = real.options().dtype(at::kFloat);
  // every tslab / slab row is written by its wave (waves without a tile write zeros)
  Tensor tslab = at::empty({4 * (int64_t)P, F + 2 * H}, f32);
  Tensor tsum = at::empty({(int64_t)hfrep::mlp_wgpt_tsum_floats((int)F, (int)T)}, f32);
  Tensor slab = at::empty({4 * (int64_t)P, 2}, f32);
  hfrep::launch_mlp_wgp_critic_t(dt, real.data_ptr(), fake.data_ptr(), c.data_ptr<float>(), cr, tslab.data_ptr<float>(),
                                 tsum.data_ptr<float>(), slab.data_ptr<float>(), B, (int)T, (int)F, pW1, pW2, pw3,
                                 cur_stream(real));
  return slab;
}

bool mlp_affine_supported_op(int64_t F, int64_t T) { return hfrep::mlp_affine_supported((int)F, (int)T); }

inline void check_affine(const Tensor& x, const char* what) {
  TORCH_CHECK(hfrep::mlp_affine_supported((int)x.size(2), (int)x.size(1)), what, ": T F must be a multiple of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, what, ": 16-byte aligned rows");
}

// the affine critic's GP update from batch sums (fp32 / bf16): adds gW1, gW2, gw3 into the fp32 gradient
// views, returns the score slab (1, 2) and the penalty sum e (1) for mlp_finish
std::tuple<Tensor, Tensor> mlp_wgp_affine(Tensor real, Tensor fake, std::vector<Tensor> cp, double lam, Tensor gW1,
                                          Tensor gW2, Tensor gw3) {
  const int dt = act_dt(real);
  TORCH_CHECK(fake.scalar_type() == real.scalar_type() && fake.sizes() == real.sizes(), "mlp_wgp_affine: fake like real");
  act_dt(fake);
  const int64_t F = real.size(-1), H = hidden_of(cp, F), B = real.size(0), T = real.size(1);
  rows_of(real, F, "real");
  check_affine(real, "mlp_wgp_affine");
  check_affine(fake, "mlp_wgp_affine");
  const auto cr = critic_of(cp, F, H, T * H);
  for (const Tensor* g : {&gW1, &gW2, &gw3})
    TORCH_CHECK(g->device() == real.device(), "mlp_wgp_affine: gradients on the activations' device");
  float* pW1 = const_cast<float*>(w(gW1, F * H, "gW1"));
  float* pW2 = const_cast<float*>(w(gW2, H * H, "gW2"));
  float* pw3 = const_cast<float*>(w(gw3, T * H, "gw3"));
  GUARD(real);
  auto f32 = real.options().dtype(at::kFloat);
  Tensor ws = at::empty({(int64_t)hfrep::mlp_affine_ws_floats(dt, B, (int)T, (int)F)}, f32);
  Tensor slab = at::empty({1, 2}, f32), e = at::empty({1}, f32);
  hfrep::launch_mlp_wgp_affine(dt, real.data_ptr(), fake.data_ptr(), cr, B, (int)T, (int)F, (float)lam,
                               ws.data_ptr<float>(), slab.data_ptr<float>(), e.data_ptr<float>(), pW1, pW2, pw3,
                               cur_stream(real));
  return {slab, e};
}

// the affine critic's input gradient for the generator step: dfake (B, T, F) = -g_t / B per row, and
// the fake score slab (1, 2) for mlp_finish mode 1
std::tuple<Tensor, Tensor> mlp_critic_dx_affine(Tensor fake, std::vector<Tensor> cp) {
  const int dt = act_dt(fake);
  const int64_t F = fake.size(-1), H = hidden_of(cp, F), B = fake.size(0), T = fake.size(1);
  rows_of(fake, F, "fake");
  check_affine(fake, "mlp_critic_dx_affine");
  const auto cr = critic_of(cp, F, H, T * H);
  GUARD(fake);
  auto f32 = fake.options().dtype(at::kFloat);
  Tensor ws = at::empty({(int64_t)hfrep::mlp_affine_ws_floats(dt, B, (int)T, (int)F)}, f32);
  Tensor slab = at::empty({1, 2}, f32), dx = at::empty_like(fake);
  hfrep::launch_mlp_critic_dx_affine(dt, fake.data_ptr(), cr, B, (int)T, (int)F, ws.data_ptr<float>(),
                                     slab.data_ptr<float>(), dx.data_ptr(), cur_stream(fake));
  return {dx, slab};
}

// the GP critic update with in-kernel weight gradients (bf16): adds gW1, gW2, gw3 into the given fp32
// gradient views (bias gradients cancel, as in mlp_wgp_critic) and returns the W-loss slab
Tensor mlp_wgp_critic_w(Tensor real, Tensor fake, Tensor c, std::vector<Tensor> cp, Tensor gW1, Tensor gW2,
                        Tensor gw3) {
  TORCH_CHECK(act_dt(real) == hfrep::DT_BF16, "mlp_wgp_critic_w: bf16 activations");
  TORCH_CHECK(fake.scalar_type() == real.scalar_type() && fake.sizes() == real.sizes(), "mlp_wgp_critic_w: fake like real");
  act_dt(fake);
  const int64_t F = real.size(-1), H = hidden_of(cp, F), M = rows_of(real, F, "real"), B = real.size(0), T = real.size(1);
  TORCH_CHECK(hfrep::mlp_wgpw_supported((int)F, (int)T), "mlp_wgp_critic_w: (F, T) = (", F, ", ", T,
              ") outside the in-kernel weight-gradient variant");
  const auto cr = critic_of(cp, F, H, T * H);
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kFloat && c.is_contiguous() && c.numel() == B,
              "mlp_wgp_critic_w: c (B) fp32");
  for (const Tensor* g : {&gW1, &gW2, &gw3})
    TORCH_CHECK(g->device() == real.device(), "mlp_wgp_critic_w: gradients on the activations' device");
  float* pW1 = const_cast<float*>(w(gW1, F * H, "gW1"));
  float* pW2 = const_cast<float*>(w(gW2, H * H, "gW2"));
  float* pw3 = const_cast<float*>(w(gw3, T * H, "gw3"));
  GUARD(real);
  const int P = hfrep::mlp_wgpw_blocks(M);
  const int64_t L = (H + F + T) * H;
  Tensor gslab = at::empty({P, L}, real.options().dtype(at::kFloat));
  Tensor slab = at::empty({4 * (int64_t)P, 2}, real.options().dtype(at::kFloat));
  const hipStream_t s = cur_stream(real);
  hfrep::launch_mlp_wgp_critic_w(real.data_ptr(), fake.data_ptr(), c.data_ptr<float>(), cr, gslab.data_ptr<float>(),
                                 slab.data_ptr<float>(), M, (int)T, (int)F, s);
  hfrep::launch_mlp_slab_sum_cols(gslab.data_ptr<float>(), P, L, 0, (int)(H * H), pW2, s);
  hfrep::launch_mlp_slab_sum_cols(gslab.data_ptr<float>(), P, L, (int)(H * H), (int)(F * H), pW1, s);
  hfrep::launch_mlp_slab_sum_cols(gslab.data_ptr<float>(), P, L, (int)((H + F) * H), (int)(T * H), pw3, s);
  return slab;
}

// the generator reverse with in-kernel parameter gradients (bf16): adds the gradients of
// [W1, b1, gamma1, beta1, W2, b2, gamma2, beta2, W3, b3] into the fp32 views gg
void mlp_gen_bwd_w(Tensor noise, Tensor dfake, std::vector<Tensor> gp, std::vector<Tensor> gg) {
  TORCH_CHECK(act_dt(noise) == hfrep::DT_BF16, "mlp_gen_bwd_w: bf16 activations");
  act_dt(dfake);
  TORCH_CHECK(dfake.scalar_type() == noise.scalar_type() && dfake.sizes() == noise.sizes(), "mlp_gen_bwd_w: dfake like noise");
  const int64_t F = noise.size(-1), H = hidden_of(gp, F), M = rows_of(noise, F, "noise");
  const auto g = gen_of(gp, F, H);
  TORCH_CHECK(gg.size() == 10, "mlp_gen_bwd_w: 10 gradient views");
  const int64_t n[10] = {F * H, H, H, H, H * H, H, H, H, H * F, F};
  float* p[10];
  for (int i = 0; i < 10; ++i) {
    TORCH_CHECK(gg[i].device() == noise.device(), "mlp_gen_bwd_w: gradients on the activations' device");
    p[i] = const_cast<float*>(w(gg[i], n[i], "generator gradient"));
  }
  GUARD(noise);
  const int P = hfrep::mlp_gbw_blocks(M);
  const int64_t L = F * H + H + H * H + H + H * F + F;
  Tensor gslab = at::empty({P, L}, noise.options().dtype(at::kFloat));
  Tensor lnslab = at::empty({4 * (int64_t)P, 4 * H}, noise.options().dtype(at::kFloat));
  const hipStream_t s = cur_stream(noise);
  hfrep::launch_mlp_gen_bwd_w(noise.data_ptr(), dfake.data_ptr(), g, gslab.data_ptr<float>(), lnslab.data_ptr<float>(), M,
                              (int)F, s);
  // slab segments in the order [W1][b1][W2][b2][W3][b3]
  const int seg[6] = {0, 1, 4, 5, 8, 9};
  int64_t col = 0;
  for (int k : seg) {
    hfrep::launch_mlp_slab_sum_cols(gslab.data_ptr<float>(), P, L, (int)col, (int)n[k], p[k], s);
    col += n[k];
  }
  hfrep::launch_mlp_slab_sum4(lnslab.data_ptr<float>(), 4 * P, (int)H, p[2], p[3], p[6], p[7], s);
}

// the GAN discriminator update with its six gradients in the kernel (fp32 / bf16): adds them into the
// fp32 views cg = [gW1, gb1, gW2, gb2, gw3, gb3] and returns the loss slab
Tensor mlp_gan_critic_g(Tensor x, std::vector<Tensor> cp, double label, std::vector<Tensor> cg) {
  const int dt = act_dt(x);
  const int64_t F = x.size(-1), H = hidden_of(cp, F), M = rows_of(x, F, "x");
  const auto cr = critic_of(cp, F, H, H);
  TORCH_CHECK(cg.size() == 6, "mlp_gan_critic_g: 6 gradient views");
  const int64_t n[6] = {F * H, H, H * H, H, H, 1};
  float* p[6];
  for (int i = 0; i < 6; ++i) {
    TORCH_CHECK(cg[i].device() == x.device(), "mlp_gan_critic_g: gradients on the activations' device");
    p[i] = const_cast<float*>(w(cg[i], n[i], "critic gradient"));
  }
  GUARD(x);
  const int64_t L = F + 2 * H + 1;
  Tensor gslab = slab_new(x, M, L), slab = slab_new(x, M, 2);
  Tensor v = at::zeros({L}, x.options().dtype(at::kFloat));
  const hipStream_t s = cur_stream(x);
  hfrep::launch_mlp_gan_critic_g(dt, x.data_ptr(), cr, (float)label, gslab.data_ptr<float>(), slab.data_ptr<float>(), M,
                                 (int)F, s);
  hfrep::launch_mlp_slab_sum(gslab.data_ptr<float>(), (int)gslab.size(0), (int)L, v.data_ptr<float>(), s);
  hfrep::launch_mlp_gan_grad_finish(v.data_ptr<float>(), cr, (int)F, (int)H, p[0], p[1], p[2], p[3], p[4], p[5], s);
  return slab;
}

std::tuple<Tensor, Tensor> mlp_critic_dx(Tensor x, std::vector<Tensor> cp, int64_t head, double label) {
  const int dt = act_dt(x);
  TORCH_CHECK(head == 0 || head == 1, "mlp_critic_dx: head 0 (flatten, W loss) or 1 (per-row sigmoid, BCE)");
  const int64_t F = x.size(-1), H = hidden_of(cp, F), M = rows_of(x, F, "x"), T = x.size(1);
  const auto cr = critic_of(cp, F, H, head == 0 ? T * H : H);
  GUARD(x);
  Tensor dx = at::empty_like(x);
  Tensor slab = slab_new(x, M, 2);
  hfrep::launch_mlp_critic_dx(dt, (int)head, x.data_ptr(), cr, (float)label, dx.data_ptr(), slab.data_ptr<float>(), M,
                              (int)T, (int)F, (int)H, cur_stream(x));
  return {dx, slab};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> mlp_gan_critic(Tensor x, std::vector<Tensor> cp,
                                                                          double label) {
  const int dt = act_dt(x);
  const int64_t F = x.size(-1), H = hidden_of(cp, F), M = rows_of(x, F, "x"), B = x.size(0), T = x.size(1);
  const auto cr = critic_of(cp, F, H, H);
  GUARD(x);
  Tensor h1 = at::empty({B, T, H}, x.options()), dh2 = at::empty({B, T, H}, x.options());
  Tensor dh1 = at::empty({B, T, H}, x.options()), h2 = at::empty({B, T, H}, x.options());
  Tensor dz3 = at::empty({B, T, 1}, x.options());
  Tensor slab = slab_new(x, M, 2);
  hfrep::launch_mlp_gan_critic(dt, x.data_ptr(), cr, (float)label, h1.data_ptr(), dh2.data_ptr(), dh1.data_ptr(),
                               h2.data_ptr(), dz3.data_ptr(), slab.data_ptr<float>(), M, (int)F, (int)H, cur_stream(x));
  return {h1, dh2, dh1, h2, dz3, slab};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> mlp_gen_bwd(Tensor noise, Tensor dfake, std::vector<Tensor> gp) {
  const int dt = act_dt(noise);
  act_dt(dfake);
  TORCH_CHECK(dfake.scalar_type() == noise.scalar_type() && dfake.sizes() == noise.sizes(), "mlp_gen_bwd: dfake like noise");
  const int64_t F = noise.size(-1), H = hidden_of(gp, F), M = rows_of(noise, F, "noise"), B = noise.size(0),
                T = noise.size(1);
  const auto g = gen_of(gp, F, H);
  GUARD(noise);
  Tensor dz1 = at::empty({B, T, H}, noise.options()), u1 = at::empty({B, T, H}, noise.options());
  Tensor dz2 = at::empty({B, T, H}, noise.options()), u2 = at::empty({B, T, H}, noise.options());
  Tensor lnslab = slab_new(noise, M, 4 * H);
  hfrep::launch_mlp_gen_bwd(dt, noise.data_ptr(), dfake.data_ptr(), g, dz1.data_ptr(), u1.data_ptr(), dz2.data_ptr(),
                            u2.data_ptr(), lnslab.data_ptr<float>(), M, (int)F, (int)H, cur_stream(noise));
  return {dz1, u1, dz2, u2, lnslab};
}

Tensor mlp_finish(Tensor slab, optional<Tensor> e, int64_t mode, double invB, optional<Tensor> b3, double lam) {
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.is_contiguous() && slab.dim() == 2 &&
                  slab.size(1) == 2,
              "mlp_finish: slab (P, 2) fp32");
  if (e.has_value()) TORCH_CHECK(e->is_cuda() && e->scalar_type() == at::kFloat && e->is_contiguous(), "mlp_finish: e fp32");
  const float* b3p = b3.has_value() ? w(*b3, 1, "b3") : nullptr;
  GUARD(slab);
  Tensor out = at::empty({4}, slab.options());
  hfrep::launch_mlp_finish(slab.data_ptr<float>(), (int)slab.size(0), e.has_value() ? e->data_ptr<float>() : nullptr,
                           e.has_value() ? e->numel() : 0, (int)mode, (float)invB, b3p, (float)lam, out.data_ptr<float>(),
                           cur_stream(slab));
  return out;
}

// slab (P, nseg * L): out_k += column sums of segment k (fixed order)
void mlp_slab_sum_(Tensor slab, int64_t L, optional<Tensor> o0, optional<Tensor> o1, optional<Tensor> o2,
                   optional<Tensor> o3) {
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.is_contiguous() && slab.dim() == 2,
              "mlp_slab_sum_: slab (P, nseg L) fp32");
  const int64_t nseg = slab.size(1) / L;
  TORCH_CHECK(nseg * L == slab.size(1) && (nseg == 1 || nseg == 4), "mlp_slab_sum_: 1 or 4 segments of L");
  auto p = [&](const optional<Tensor>& o) -> float* {
    return o.has_value() ? const_cast<float*>(w(*o, L, "slab_sum output")) : nullptr;
  };
  GUARD(slab);
  if (nseg == 1)
    hfrep::launch_mlp_slab_sum(slab.data_ptr<float>(), (int)slab.size(0), (int)L, p(o0), cur_stream(slab));
  else
    hfrep::launch_mlp_slab_sum4(slab.data_ptr<float>(), (int)slab.size(0), (int)L, p(o0), p(o1), p(o2), p(o3),
                                cur_stream(slab));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(hfrep, m) {
  m.def("mlp_supported(int F, int H) -> bool", &mlp_supported_op);  // no tensor inputs: catch-all kernel
  m.def("mlp_gen_fwd(Tensor noise, Tensor[] gp, Tensor(a!)? out=None) -> Tensor");
  m.def("mlp_wgp_norm(Tensor like, Tensor[] cp) -> Tensor");
  m.def("mlp_wgp_coef(Tensor gsq, float lam) -> (Tensor, Tensor)");
  m.def("mlp_wgp_critic(Tensor real, Tensor fake, Tensor c, Tensor[] cp) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("mlp_wgpw_supported(int F, int T) -> bool", &mlp_wgpw_supported_op);
  m.def("mlp_affine_supported(int F, int T) -> bool", &mlp_affine_supported_op);
  m.def("mlp_wgp_affine(Tensor real, Tensor fake, Tensor[] cp, float lam, Tensor(a!) gW1, Tensor(b!) gW2, "
        "Tensor(c!) gw3) -> (Tensor, Tensor)");
  m.def("mlp_critic_dx_affine(Tensor fake, Tensor[] cp) -> (Tensor, Tensor)");
  m.def("mlp_wgp_critic_t(Tensor real, Tensor fake, Tensor c, Tensor[] cp, Tensor(a!) gW1, Tensor(b!) gW2, "
        "Tensor(c!) gw3) -> Tensor");
  m.def("mlp_wgp_critic_w(Tensor real, Tensor fake, Tensor c, Tensor[] cp, Tensor(a!) gW1, Tensor(b!) gW2, "
        "Tensor(c!) gw3) -> Tensor");
  m.def("mlp_gen_bwd_w(Tensor noise, Tensor dfake, Tensor[] gp, Tensor(a!)[] gg) -> ()");
  m.def("mlp_gan_critic_g(Tensor x, Tensor[] cp, float label, Tensor(a!)[] cg) -> Tensor");
  m.def("mlp_critic_dx(Tensor x, Tensor[] cp, int head, float label) -> (Tensor, Tensor)");
  m.def("mlp_gan_critic(Tensor x, Tensor[] cp, float label) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("mlp_gen_bwd(Tensor noise, Tensor dfake, Tensor[] gp) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("mlp_finish(Tensor slab, Tensor? e, int mode, float invB, Tensor? b3, float lam) -> Tensor");
  m.def("mlp_slab_sum_(Tensor slab, int L, Tensor(a!)? o0, Tensor(b!)? o1=None, Tensor(c!)? o2=None, "
        "Tensor(d!)? o3=None) -> ()");
}

TORCH_LIBRARY_IMPL(hfrep, CUDA, m) {
  m.impl("mlp_gen_fwd", &mlp_gen_fwd);
  m.impl("mlp_wgp_critic_w", &mlp_wgp_critic_w);
  m.impl("mlp_wgp_critic_t", &mlp_wgp_critic_t);
  m.impl("mlp_wgp_affine", &mlp_wgp_affine);
  m.impl("mlp_critic_dx_affine", &mlp_critic_dx_affine);
  m.impl("mlp_gen_bwd_w", &mlp_gen_bwd_w);
  m.impl("mlp_gan_critic_g", &mlp_gan_critic_g);
  m.impl("mlp_wgp_norm", &mlp_wgp_norm);
  m.impl("mlp_wgp_coef", &mlp_wgp_coef);
  m.impl("mlp_wgp_critic", &mlp_wgp_critic);
  m.impl("mlp_critic_dx", &mlp_critic_dx);
  m.impl("mlp_gan_critic", &mlp_gan_critic);
  m.impl("mlp_gen_bwd", &mlp_gen_bwd);
  m.impl("mlp_finish", &mlp_finish);
  m.impl("mlp_slab_sum_", &mlp_slab_sum_);
}
