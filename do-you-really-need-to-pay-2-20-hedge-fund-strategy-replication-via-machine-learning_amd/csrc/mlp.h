// Fused MLP-GAN passes (csrc/mlp.hip): host launchers for BASELINE configs 3 / 4 (the vanilla GAN of
// GAN/GAN.py and the MLP WGAN-GP of GAN/WGAN_GP.py).  Included only by mlp.hip and bindings.cpp.
//
// Every launcher takes the fp32 master weights (Keras layout: kernel (in, out), row-major) and
// activations of dtype `dt` (DT_F32 / DT_BF16) as row-major (M, features) matrices, M = B * T rows.
// F is the feature count of the data windows, H the hidden width; supported: (F, H) in
// {(32, 100), (36, 100)} (mlp_supported).  `slab` arguments are per-wave partial sums
// (mlp_slab_rows(M) rows) reduced by launch_mlp_finish in a fixed order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hfrep {

bool mlp_supported(int F, int H);
// rows of every per-wave partial-sum slab a launch over M rows writes (grid x waves per block)
int mlp_slab_rows(int64_t M);

// G(noise): Dense(H, sigmoid) -> LReLU -> LN -> Dense(H, sigmoid) -> LReLU -> LN -> Dense(F)
struct MlpGen {
  const float *W1, *b1, *g1, *be1, *W2, *b2, *g2, *be2, *W3, *b3;
};
// critic / discriminator: Dense(H) -> Dense(H) -> head; head 0 = Flatten -> Dense(1) over T rows
// (w3: T*H), head 1 = per-row Dense(1, sigmoid) (w3: H)
struct MlpCritic {
  const float *W1, *b1, *W2, *b2, *w3, *b3;
};

void launch_mlp_gen_fwd(int dt, const void* noise, const MlpGen& g, void* out, int64_t M, int F, int H,
                        hipStream_t s);
// per-row squared norm of the linear critic's input gradient dD/dx (head 0): gsq (M) fp32
void launch_mlp_wgp_norm(int dt, const MlpCritic& c, float* gsq, int64_t M, int Tn, int F, int H, hipStream_t s);
// per-sample GP coefficient c_b = -(2 lam / B)(1 - |g_b|) / |g_b|, and e = per-block sums of (1 - |g_b|)^2
// (mlp_wgp_coef_parts(B) values)
int mlp_wgp_coef_parts(int64_t B);
void launch_mlp_wgp_coef(const float* gsq, int Tn, int64_t B, float lam, float* c, float* e, hipStream_t s);
// the WGAN-GP critic step of the linear critic on one row tile: W terms on real / fake and the
// reverse-over-tangent GP term, as combined wgrad operands (see mlp.hip)
void launch_mlp_wgp_critic(int dt, const void* real, const void* fake, const float* c, const MlpCritic& cr,
                           void* X2c, void* dY2, void* X1c, void* dY1, void* Y3c, float* slab, int64_t M, int Tn,
                           int F, int H, hipStream_t s);
// critic input gradient for the generator step: dx = dL/dx with the Wasserstein (head 0, label -1)
// or BCE (head 1, label `label`) loss; slab: loss partials
void launch_mlp_critic_dx(int dt, int head, const void* x, const MlpCritic& cr, float label, void* dx, float* slab,
                          int64_t M, int Tn, int F, int H, hipStream_t s);
// discriminator update of the vanilla GAN (head 1, BCE with label `label`): wgrad operands
// h1 (X of W2), dh2 (dY of W2), dh1 (dY of W1), h2 (X of w3), dz3 (dY of w3); slab: loss partials
void launch_mlp_gan_critic(int dt, const void* x, const MlpCritic& cr, float label, void* h1, void* dh2, void* dh1,
                           void* h2, void* dz3, float* slab, int64_t M, int F, int H, hipStream_t s);
// generator reverse pass from dfake: wgrad operands dz1 (dY of W1), u1 (X of W2), dz2 (dY of W2),
// u2 (X of W3); LayerNorm parameter partials lnslab (mlp_slab_rows(M) x 4H: dgamma1, dbeta1,
// dgamma2, dbeta2)
void launch_mlp_gen_bwd(int dt, const void* noise, const void* dfake, const MlpGen& g, void* dz1, void* u1,
                        void* dz2, void* u2, float* lnslab, int64_t M, int F, int H, hipStream_t s);
// fixed-order reduction of a loss slab (P rows x 2) and optional per-sample e (n_e values) into
// out[4]: mode 0 = WGAN-GP critic pack [w_real + w_fake + lam pen, w_real, w_fake, pen];
// mode 1 = generator loss [loss, 0, 0, 0] (W: -mean score; BCE: mean); mode 2 = BCE segment loss [loss, 0, 0, 0]
void launch_mlp_finish(const float* slab, int P, const float* e, int64_t n_e, int mode, float invB, const float* b3,
                       float lam, float* out, hipStream_t s);
// fixed-order column sums of a (P, L) slab added into out[L]; the 4-segment form adds segment k of
// every (P, 4 L) slab row into o_k (nullptr: skipped)
void launch_mlp_slab_sum(const float* slab, int P, int L, float* out, hipStream_t s);
void launch_mlp_slab_sum4(const float* slab, int P, int L, float* o0, float* o1, float* o2, float* o3, hipStream_t s);
// out[j] += sum_p slab[p * stride + col0 + j], j < L (fixed order)
void launch_mlp_slab_sum_cols(const float* slab, int P, int64_t stride, int col0, int L, float* out, hipStream_t s);

// The GP critic update with its three weight gradients accumulated in the kernel (bf16 only; the LDS
// plan must fit: T <= 34 at F = 32, T <= 18 at F = 36, mlp_wgpw_supported).  Launches mlp_wgpw_blocks(M) workgroups; gslab
// (blocks x (H + F + T) H fp32) gets each workgroup's partial [gW2 | gW1 | gw3], slab (4 blocks x 2)
// the per-wave W-loss partials of mlp_wgp_critic.  Every slab element is written.
// The generator reverse with its parameter gradients accumulated in the kernel (bf16, F in {32, 36}):
// mlp_gbw_blocks(M) workgroups; gslab rows (one per workgroup) = [W1 F x H][b1 H][W2 H x H][b2 H]
// [W3 H x F][b3 F] partials, lnslab (4 rows per workgroup, 4 H) = the LayerNorm partials of
// launch_mlp_gen_bwd.  Every slab element is written.
// The GAN discriminator update with its gradients in the kernel (fp32 / bf16): mlp_slab_rows(M) rows of
// gslab ([s1 F | s2 H | s3 H | S], the per-wave dz-weighted column sums of x, h1, h2 and dz) and of the
// loss slab (2 columns, as launch_mlp_gan_critic).  launch_mlp_gan_grad_finish adds the gradients
// gW1 = s1 (x) W2 w3, gb1 = S W2 w3, gW2 = s2 (x) w3, gb2 = S w3, gw3 = s3, gb3 = S from the REDUCED
// sums v (F + 2 H + 1 floats).
void launch_mlp_gan_critic_g(int dt, const void* x, const MlpCritic& cr, float label, float* gslab, float* slab,
                             int64_t M, int F, hipStream_t s);
void launch_mlp_gan_grad_finish(const float* v, const MlpCritic& cr, int F, int H, float* gW1, float* gb1, float* gW2,
                                float* gb2, float* gw3, float* gb3, hipStream_t s);
// The GP critic update with per-t column-sum weight gradients (fp32 / bf16): rows walked t-major, one t
// per wave (mlp_wgpt_waves_per_t(T) waves per t, mlp_wgpt_blocks(T) workgroups); tslab: 4 rows per
// workgroup of F + 2 H floats, tsum: mlp_wgpt_tsum_floats(F, T) floats (scratch), slab: the W-loss partials
// (4 rows per workgroup x 2); gW1 / gW2 / gw3 accumulate.  Bn = samples (rows = Bn T).
int mlp_wgpt_waves_per_t(int Tn);
int mlp_wgpt_blocks(int Tn);
size_t mlp_wgpt_tsum_floats(int F, int Tn);
void launch_mlp_wgp_critic_t(int dt, const void* real, const void* fake, const float* c, const MlpCritic& cr,
                             float* tslab, float* tsum, float* slab, int64_t Bn, int Tn, int F, float* gW1, float* gW2,
                             float* gw3, hipStream_t s);
// The affine critic's update from batch sums (both dtypes; csrc/mlp.hip mlp_wgp_affine_kernel): per-t
// column sums of real and fake -> one-workgroup fp32 finish; gW1 / gW2 / gw3 accumulate, slab (1 x 2) =
// the real / fake score sums, e (1) = B (1 - |g|)^2.  ws: mlp_affine_ws_floats floats of scratch.
// critic_dx_affine: the generator step's dfake (-g_t / B broadcast over the batch) and its score slab.
bool mlp_affine_supported(int F, int Tn);
size_t mlp_affine_ws_floats(int dt, int64_t Bn, int Tn, int F);
void launch_mlp_wgp_affine(int dt, const void* real, const void* fake, const MlpCritic& cr, int64_t Bn, int Tn, int F,
                           float lam, float* ws, float* slab, float* e, float* gW1, float* gW2, float* gw3, hipStream_t s);
void launch_mlp_critic_dx_affine(int dt, const void* fake, const MlpCritic& cr, int64_t Bn, int Tn, int F, float* ws,
                                 float* slab, void* dx, hipStream_t s);
int mlp_gbw_blocks(int64_t M);
void launch_mlp_gen_bwd_w(const void* noise, const void* dfake, const MlpGen& g, float* gslab, float* lnslab, int64_t M,
                          int F, hipStream_t s);
bool mlp_wgpw_supported(int F, int Tn);
int mlp_wgpw_blocks(int64_t M);
void launch_mlp_wgp_critic_w(const void* real, const void* fake, const float* c, const MlpCritic& cr, float* gslab,
                             float* slab, int64_t M, int Tn, int F, hipStream_t s);

}  // namespace hfrep
