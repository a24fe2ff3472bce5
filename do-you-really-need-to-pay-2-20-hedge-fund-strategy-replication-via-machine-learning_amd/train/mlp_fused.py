"""Fused MLP-GAN training steps (BASELINE configs 3 / 4) on the kernels of ``csrc/mlp.hip``.

The layer-by-layer engine (``Sequential.efwd / ebwd / etfwd / etbwd``) runs one kernel per layer and
pass and round-trips every (B*T, 100) activation and adjoint through HBM: 607 GB per bf16 MLP WGAN-GP
iteration (``profiles/r06_mlp/baseline``).  For the two MLP models of the BASELINE configs this module
replaces it with one kernel per pass that carries a 32-row tile through every layer in registers:

* ``mlp_gen_fwd``     G(z) (GAN/WGAN_GP.py:221-236, GAN/GAN.py:127-142);
* ``mlp_wgp_norm`` + ``mlp_wgp_coef``   the gradient penalty's first-order pass: |dD/dx_hat| per
  sample and the adjoint coefficient c_b (GAN/WGAN_GP.py:201-216);
* ``mlp_wgp_critic``  a whole WGAN-GP critic update of the linear critic (GAN/WGAN_GP.py:238-253):
  W terms on real / fake and the reverse-over-tangent of the penalty, as one combined weight-gradient
  operand per weight (see the kernel's comment); in bf16 ``mlp_wgp_critic_w`` also accumulates the
  three weight gradients in the kernel (128-row block tiles staged transposed in LDS), in fp32
  ``mlp_wgp_critic_t`` (rows walked t-major, per-t column sums in registers);
* ``mlp_gan_critic``  a vanilla-GAN discriminator update (GAN/GAN.py:144-158, 187-189);
  ``mlp_gan_critic_g`` takes its gradients in the kernel as dz-weighted column sums (the linear hidden
  layers make every adjoint of a row rank-1);
* ``mlp_critic_dx`` + ``mlp_gen_bwd``  the generator update through the frozen critic
  (GAN/WGAN_GP.py:178-189, GAN/GAN.py:195-198); in bf16 ``mlp_gen_bwd_w`` accumulates all ten
  generator parameter gradients in the kernel;

followed by the streaming weight-gradient kernels (``linear_wgrad_``) and the fused optimizer.  The
random draws are the engine path's, in its order (real, noise, alpha per critic update), so both paths
see the same batches; ``HFREP_MLP_FUSED=0`` selects the engine path (A/B, tests).

For the affine WGAN-GP critic the penalty's input gradient dD/dx_hat does not depend on x_hat, so
neither x_hat nor D(x_hat) is formed (alpha is still drawn: the RNG stream stays the engine's).  Going
one step further (``mlp_wgp_affine``, default): g_t = W1 W2 w3_t depends on t alone, so every sample has
the same penalty coefficient, and the W terms enter the weight gradients and the losses only through
per-t sums over the batch (sum_b (x_b W) = (sum_b x_b) W).  A critic update then reads real and fake
once (per-t column sums) and finishes in fp32 in one workgroup; the generator step's dfake is -g_t / B
for every row (``mlp_critic_dx_affine``).  ``HFREP_MLP_AFFINE=0`` keeps the per-row kernels above.
"""
from __future__ import annotations

import os

import torch

from ..models.layers import Dense, Flatten, LayerNormalization, LeakyReLU
from ..ops import _native
from ..ops import functional as Fn


def _ops():
    return _native.native()


def _views(model, layer, names, grad=False):
    get = model.gview if grad else model.view
    return [get(layer, n) for n in names]


def _gen_lists(G, grad=False):
    """[W1, b1, gamma1, beta1, W2, b2, gamma2, beta2, W3, b3] of the MLP generator, or None if G is
    not Dense(s) -> LReLU -> LN -> Dense(s) -> LReLU -> LN -> Dense."""
    L = G.layers
    kinds = [Dense, LeakyReLU, LayerNormalization, Dense, LeakyReLU, LayerNormalization, Dense]
    if len(L) != 7 or not all(isinstance(l, k) for l, k in zip(L, kinds)):
        return None
    if not (L[0].act_code == 1 and L[3].act_code == 1 and L[6].act_code == 0 and all(L[i].use_bias for i in (0, 3, 6))):
        return None
    if abs(L[1].alpha - 0.2) > 1e-6 or abs(L[4].alpha - 0.2) > 1e-6 or L[2].eps != 1e-3 or L[5].eps != 1e-3:
        return None
    out = []
    for d, ln in ((L[0], L[2]), (L[3], L[5])):
        out += _views(G, d, ["kernel", "bias"], grad) + _views(G, ln, ["gamma", "beta"], grad)
    return out + _views(G, L[6], ["kernel", "bias"], grad)


def _critic_lists(C, head: int, grad=False):
    """[W1, b1, W2, b2, w3, b3] of Dense -> Dense -> (Flatten ->) Dense(1) with linear hidden layers;
    head 0 = Flatten -> Dense(1) linear, head 1 = per-row Dense(1, sigmoid)."""
    L = C.layers
    if head == 0:
        ok = len(L) == 4 and isinstance(L[2], Flatten) and L[3].act_code == 0
        last = L[3] if ok else None
    else:
        ok = len(L) == 3 and L[2].act_code == 1
        last = L[2] if ok else None
    if not ok or not all(isinstance(l, Dense) and l.use_bias for l in (L[0], L[1], last)):
        return None
    if L[0].act_code != 0 or L[1].act_code != 0 or last.units != 1:
        return None
    return (_views(C, L[0], ["kernel", "bias"], grad) + _views(C, L[1], ["kernel", "bias"], grad)
            + _views(C, last, ["kernel", "bias"], grad))


class FusedMLP:
    """The MLP models' training step on the fused kernels (attached to a GANTrainer)."""

    def __init__(self, tr):
        self.tr = tr
        self.head = 0 if tr.cfg.loss == "wgan_gp" else 1
        self.gw, self.gg = _gen_lists(tr.generator), _gen_lists(tr.generator, grad=True)
        self.cw, self.cg = _critic_lists(tr.critic, self.head), _critic_lists(tr.critic, self.head, grad=True)
        self._ones = {}
        # GP critic update (both dtypes): rows walked t-major, the weight gradients as per-t column sums
        # in registers (mlp_wgp_critic_t) -- no per-row operands in HBM.  HFREP_MLP_WGRAD_TSUM=0 takes
        # the bf16 kernel that stages 128-row tiles transposed in LDS instead (mlp_wgp_critic_w, A/B:
        # 4 % slower on config 4, profiles/r06_wgpw/tsum); HFREP_MLP_WGRAD_INKERNEL=0 keeps the operand
        # path (mlp_wgp_critic + linear_wgrad_).  The generator reverse: mlp_gen_bwd_w (bf16).
        cfg = tr.cfg
        on = os.environ.get("HFREP_MLP_WGRAD_INKERNEL", "1") != "0"
        inkernel = tr.dtype == torch.bfloat16 and on
        self.wgrad_inkernel = (inkernel and self.head == 0 and os.environ.get("HFREP_MLP_WGRAD_TSUM", "1") == "0"
                               and bool(_ops().mlp_wgpw_supported(int(cfg.features), int(cfg.window))))
        self.wgrad_tsum = self.head == 0 and on and not self.wgrad_inkernel
        # affine critic: the update from per-t batch sums (mlp_wgp_affine / mlp_critic_dx_affine)
        self.affine = (self.head == 0 and os.environ.get("HFREP_MLP_AFFINE", "1") != "0"
                       and bool(_ops().mlp_affine_supported(int(cfg.features), int(cfg.window))))
        self.gen_wgrad_inkernel = inkernel
        # GAN discriminator: rank-1 adjoints per row -> gradients as dz-weighted column sums in the
        # kernel (mlp_gan_critic_g, both dtypes); HFREP_MLP_WGRAD_INKERNEL=0 keeps the operand path
        self.gan_colsum = self.head == 1 and os.environ.get("HFREP_MLP_WGRAD_INKERNEL", "1") != "0"

    @staticmethod
    def supported(tr) -> bool:
        cfg = tr.cfg
        if os.environ.get("HFREP_MLP_FUSED", "1") == "0":
            return False
        if cfg.arch != "mlp" or cfg.loss not in ("gan", "wgan_gp") or tr.device.type != "cuda":
            return False
        if tr.dtype not in (torch.float32, torch.bfloat16) or _native.fallback_allowed():
            return False
        if not _native.available() or not bool(_ops().mlp_supported(int(cfg.features), int(cfg.hidden))):
            return False
        head = 0 if cfg.loss == "wgan_gp" else 1
        return _gen_lists(tr.generator) is not None and _critic_lists(tr.critic, head) is not None

    def _ones_col(self, n, dtype):
        key = (n, dtype)
        t = self._ones.get(key)
        if t is None:
            t = self._ones[key] = torch.ones((n, 1), dtype=dtype, device=self.tr.device)
        return t

    # ---- generator update through the frozen critic ---------------------------------------------
    def _generator_grads(self, noise, fake):
        tr, ops = self.tr, _ops()
        B = noise.shape[0]
        if self.head == 0:
            if self.affine:
                dfake, slab = ops.mlp_critic_dx_affine(fake, self.cw)
            else:
                dfake, slab = ops.mlp_critic_dx(fake, self.cw, 0, -1.0)
            loss = ops.mlp_finish(slab, None, 1, 1.0 / B, self.cw[5], 0.0)
        else:
            dfake, slab = ops.mlp_critic_dx(fake, self.cw, 1, 1.0)
            loss = ops.mlp_finish(slab, None, 2, 1.0 / noise[..., 0].numel(), None, 0.0)
        if self.gen_wgrad_inkernel:
            ops.mlp_gen_bwd_w(noise, dfake, self.gw, self.gg)
            return loss[0:1]
        dz1, u1, dz2, u2, lnslab = ops.mlp_gen_bwd(noise, dfake, self.gw)
        gW1, gb1, gg1, gbe1, gW2, gb2, gg2, gbe2, gW3, gb3 = self.gg
        Fn.linear_wgrad_(noise, dz1, gW1, gb1)
        Fn.linear_wgrad_(u1, dz2, gW2, gb2)
        Fn.linear_wgrad_(u2, dfake, gW3, gb3)
        ops.mlp_slab_sum_(lnslab, int(gg1.numel()), gg1, gbe1, gg2, gbe2)
        return loss[0:1]

    # ---- WGAN-GP (config 4) -----------------------------------------------------------------------
    def _wgp_critic_grads(self, real, fake):
        tr, ops = self.tr, _ops()
        B, T = real.shape[0], real.shape[1]
        if self.affine:
            gW1, _gb1, gW2, _gb2, gw3, _gb3 = self.cg
            slab, e = ops.mlp_wgp_affine(real, fake, self.cw, float(tr.gp_weight), gW1, gW2, gw3)
            return ops.mlp_finish(slab, e, 0, 1.0 / B, self.cw[5], float(tr.gp_weight))
        gsq = ops.mlp_wgp_norm(real, self.cw)
        c, e = ops.mlp_wgp_coef(gsq, float(tr.gp_weight))
        gW1, _gb1, gW2, _gb2, gw3, _gb3 = self.cg
        if self.wgrad_inkernel or self.wgrad_tsum:
            op = ops.mlp_wgp_critic_w if self.wgrad_inkernel else ops.mlp_wgp_critic_t
            slab = op(real, fake, c, self.cw, gW1, gW2, gw3)
            return ops.mlp_finish(slab, e, 0, 1.0 / B, self.cw[5], float(tr.gp_weight))
        X2c, dY2, X1c, dY1, Y3c, slab = ops.mlp_wgp_critic(real, fake, c, self.cw)
        # the W terms' bias gradients cancel (-1/B and +1/B per row pair) and the tangent has none
        Fn.linear_wgrad_(X2c, dY2, gW2, None)
        Fn.linear_wgrad_(X1c, dY1, gW1, None)
        Fn.linear_wgrad_(Y3c.reshape(B, -1), self._ones_col(B, Y3c.dtype), gw3, None)
        return ops.mlp_finish(slab, e, 0, 1.0 / B, self.cw[5], float(tr.gp_weight))

    def _step_wgan_gp(self):
        tr, ops = self.tr, _ops()
        B = tr.cfg.batch_size
        for _ in range(tr.n_critic):
            real, noise = tr._batch(B)
            tr.rng.uniform((B,))  # alpha: drawn for RNG-stream parity (the affine critic needs no x_hat)
            fake = ops.mlp_gen_fwd(noise, self.gw)
            tr._d_acc = self._wgp_critic_grads(real, fake)
            tr._apply(tr.critic)
        # the generator step trains on the last critic update's noise (GAN/WGAN_GP.py:282) with the
        # same generator weights: its fake windows are that update's
        tr._g_acc = self._generator_grads(noise, fake).to(tr._acc)
        tr._apply(tr.generator)

    # ---- vanilla GAN (config 3) -------------------------------------------------------------------
    def _gan_d_grads(self, x, label: float):
        """Accumulate the discriminator gradient of BCE(D(x), label) (mean over the B*T rows); returns
        the loss."""
        ops = _ops()
        if self.gan_colsum:
            slab = ops.mlp_gan_critic_g(x, self.cw, float(label), self.cg)
            return ops.mlp_finish(slab, None, 2, 1.0 / x[..., 0].numel(), None, 0.0)[0]
        h1, dh2, dh1, h2, dz3, slab = ops.mlp_gan_critic(x, self.cw, float(label))
        gW1, gb1, gW2, gb2, gw3, gb3 = self.cg
        Fn.linear_wgrad_(h1, dh2, gW2, gb2)
        Fn.linear_wgrad_(x, dh1, gW1, gb1)
        Fn.linear_wgrad_(h2, dz3, gw3, gb3)
        return ops.mlp_finish(slab, None, 2, 1.0 / x[..., 0].numel(), None, 0.0)[0]

    def _gan_d_step(self, x, label: float):
        tr = self.tr
        loss = self._gan_d_grads(x, label)
        tr._apply(tr.critic)
        return loss.to(tr._acc)

    def _step_gan(self):
        tr, ops = self.tr, _ops()
        cfg, B = tr.cfg, tr.cfg.batch_size
        real, noise = tr._batch(B)
        fake = ops.mlp_gen_fwd(noise, self.gw)
        lr_ = self._gan_d_step(real, 1.0)
        lf_ = self._gan_d_step(fake, 0.0)
        d = 0.5 * (lr_ + lf_)
        tr._d_acc = torch.stack([d, lr_, lf_, torch.zeros_like(d)])
        noise2 = tr.rng.normal((B, cfg.window, cfg.features), dtype=tr.dtype)
        fake2 = ops.mlp_gen_fwd(noise2, self.gw)
        tr._g_acc = self._generator_grads(noise2, fake2).to(tr._acc)
        tr._apply(tr.generator)

    def train_step(self):
        if self.head == 0:
            self._step_wgan_gp()
        else:
            self._step_gan()
