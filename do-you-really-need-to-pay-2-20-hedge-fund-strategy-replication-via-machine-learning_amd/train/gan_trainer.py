"""One training loop for the whole GAN zoo, with the loss as a strategy.

Reference loops (all hand-rolled ``train_on_batch`` sequences):

* ``gan``     — GAN/GAN.py:160-204, GAN/MTSS_GAN.py:159-203: D on real (label 1), D on G(z)
  (label 0), then G through the frozen D (label 1); BCE; one Adam shared by both compiled models.
* ``wgan``    — GAN/WGAN.py:166-212, GAN/MTSS_WGAN.py:165-211: n_critic x [D on real (-1), D on
  G(z) (+1), clip every critic weight to +-c], then G on the LAST critic noise (label -1).
* ``wgan_gp`` — GAN/WGAN_GP.py:255-288, GAN/MTSS_WGAN_GP.py:254-287: n_critic x one critic
  update on [W(real,-1) + W(G(z),+1) + lambda * GP(x_hat)], then G on the last critic noise.

MI355X-first differences (semantics preserved):

* everything stays on the device: batches are gathered and noise is drawn by in-kernel Philox
  (no host RNG, no H2D copies, no ``generator.predict`` round trip — GAN/WGAN.py:188);
* gradients are produced by the explicit engine (``Sequential.efwd/ebwd/etfwd/etbwd``); the GP
  critic update is the reverse-over-tangent Hessian-vector product (no autograd graph);
* losses are accumulated on device and read back only at log intervals (the reference prints —
  and therefore syncs — every iteration, GAN/MTSS_WGAN_GP.py:284);
* small batches run independent chains side by side on HIP streams (``concurrent``): at the
  reference's batch of 32 one LSTM call occupies a single CU, so the W-terms chain and the gradient
  penalty's input-gradient chain of a critic update, and the next critic update's generator forward,
  overlap instead of queueing (same kernels, same inputs, same RNG draw order: bitwise the sequential
  result, tests/test_gpu_runtime.py);
* data parallel: each rank samples its own batch; the flat gradient buffer of each model is
  all-reduced (averaged) before the fused optimizer launch (``hfrep.parallel``).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..models import gan as zoo
from ..ops import functional as Fn
from ..utils.rng import DeviceRNG
from ..utils.trace import trange
from .optim import KerasOptimizer


@dataclass
class GANConfig:
    arch: str = "lstm"            # mlp | lstm | conv
    loss: str = "wgan_gp"         # gan | wgan | wgan_gp
    window: int = 48              # T
    features: int = 35            # F
    batch_size: int = 32          # per-rank batch
    epochs: int = 5000            # reference "epochs" = iterations
    n_critic: int | None = None   # default from the zoo entry
    lr: float | None = None
    clip: float | None = None
    gp_weight: float | None = None
    hidden: int = 100
    lrelu_after_first: bool = False   # production generator variant
    seed: int = 123
    dtype: str = "float32"        # compute dtype of activations: float32 | bfloat16
    log_every: int = 100
    concurrent: bool | None = None  # side-stream overlap of independent chains (None: auto, batch <= 2048)
    extra: dict = field(default_factory=dict)

    def entry(self) -> zoo.ZooEntry:
        return zoo.ZOO[(self.arch, self.loss)]


_DT = {"float32": torch.float32, "fp32": torch.float32, "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
       "float64": torch.float64}


class GANTrainer:
    # the generator step reuses the last critic step's generator forward (bitwise the same result as
    # recomputing it: tests/test_engine.py::test_generator_forward_reuse_is_exact)
    reuse_gen_forward = True

    def __init__(self, cfg: GANConfig, dataset, device="cpu", process_group=None, rank: int = 0, world: int = 1,
                 param_dtype=torch.float32):
        self.cfg = cfg
        e = cfg.entry()
        self.device = torch.device(device)
        self.dtype = _DT[cfg.dtype]
        self._acc = torch.float64 if self.dtype == torch.float64 else torch.float32
        self.n_critic = cfg.n_critic if cfg.n_critic is not None else e.n_critic
        self.lr = cfg.lr if cfg.lr is not None else e.lr
        self.clip = cfg.clip if cfg.clip is not None else e.clip
        self.gp_weight = cfg.gp_weight if cfg.gp_weight is not None else e.gp_weight
        T, F = cfg.window, cfg.features
        gkw = dict(seed=cfg.seed, dtype=param_dtype)
        if cfg.arch != "mlp":
            self.generator = e.generator(T, F, cfg.hidden, lrelu_after_first=cfg.lrelu_after_first, **gkw)
        else:
            self.generator = e.generator(T, F, cfg.hidden, **gkw)
        self.critic = e.critic(T, F, cfg.hidden, seed=cfg.seed + 1, dtype=param_dtype)
        self.generator.to(self.device)
        self.critic.to(self.device)
        # one optimizer instance shared by the critic and the combined model, as in the reference
        if e.optimizer == "adam":
            self.opt = KerasOptimizer.adam(self.lr, beta_1=0.5, device=self.device)
        else:
            self.opt = KerasOptimizer.rmsprop(self.lr, device=self.device)
        self.pg, self.rank, self.world = process_group, rank, world
        if isinstance(dataset, np.ndarray):
            dataset = torch.from_numpy(np.ascontiguousarray(dataset, dtype=np.float32))
        self.dataset = dataset.to(self.device, torch.float32).contiguous()
        assert self.dataset.shape[1:] == (T, F), f"dataset windows {tuple(self.dataset.shape[1:])} != {(T, F)}"
        self.rng = DeviceRNG(cfg.seed, self.device, stream=rank)
        self.iteration = 0
        self._d_acc = torch.zeros(4, device=self.device)  # last d_loss terms: total, real, fake, gp
        self._g_acc = torch.zeros(1, device=self.device)
        self._ones_cache = {}
        self.grad_sync = None  # set by hfrep.parallel.DataParallel
        self.concurrent = self._want_concurrent(cfg)
        self._streams = None
        if world > 1 and process_group is not None:
            from ..parallel.dp import GradSync

            self.grad_sync = GradSync(process_group, world)
            self.grad_sync.broadcast_params([self.generator, self.critic])
        # BASELINE configs 3 / 4 (MLP GAN, MLP WGAN-GP): one fused kernel per pass instead of the
        # layer-by-layer engine (train/mlp_fused.py; HFREP_MLP_FUSED=0 keeps the engine)
        self._fused = None
        if self.device.type == "cuda":
            from .mlp_fused import FusedMLP

            if FusedMLP.supported(self):
                self._fused = FusedMLP(self)

    # ------------------------------------------------------------------------------------
    def _want_concurrent(self, cfg) -> bool:
        """Side-stream overlap pays only where one chain leaves most CUs idle: the persistent LSTM kernels
        take one CU per 32-row tile, so up to ~2048 rows per call (HFREP_CONCURRENT=0 / 1 overrides)."""
        import os

        if self.device.type != "cuda":
            return False
        env = os.environ.get("HFREP_CONCURRENT")
        if env in ("0", "1"):
            return env == "1"
        if cfg.concurrent is not None:
            return bool(cfg.concurrent)
        return cfg.batch_size <= 2048

    def _side(self, i: int):
        """Side stream ``i`` (0: the gradient-penalty input-gradient chain, 1: the next generator forward,
        2: the layers' weight gradients, off the reverse pass's critical path), or None when running
        sequentially."""
        if not self.concurrent:
            return None
        if self._streams is None:
            self._streams = [torch.cuda.Stream(device=self.device) for _ in range(3)]
        return self._streams[i]

    def _wgrad_side(self, hook):
        """Stream for the layers' weight gradients (``Fn.wgrad_on``): side stream 2 when concurrent and no
        per-layer all-reduce hook needs final gradients layer by layer; ``HFREP_WGRAD_SIDE=0`` keeps
        them inline (A/B)."""
        if hook is not None or os.environ.get("HFREP_WGRAD_SIDE", "1") == "0":
            return None
        return self._side(2)

    def _batch(self, B, out=None):
        real = self.rng.sample_windows(self.dataset, B, out_dtype=self.dtype, out=out)
        noise = self.rng.normal((B, self.cfg.window, self.cfg.features), dtype=self.dtype)
        return real, noise

    def _hook(self, model):
        """Reverse-pass hook that launches each gradient bucket's all-reduce as soon as it is
        final (None when single-process): the reduction of the last layers overlaps the backward
        of the first ones."""
        if self.grad_sync is None or self.grad_sync.buckets <= 1:
            return None
        plan = {li: (a, b) for li, a, b in model.grad_buckets(self.grad_sync.buckets)}
        g = model.flat.grad

        def hook(i):
            if i in plan:
                a, b = plan[i]
                self.grad_sync.start_(g[a:b])
        return hook

    def _sync(self, model):
        if self.grad_sync is not None:
            with trange("allreduce"):
                if self.grad_sync.finish_() == 0:  # no overlapped buckets were launched
                    self.grad_sync.all_reduce_(model.flat.grad)

    def _apply(self, model, clip=0.0):
        self._sync(model)
        with trange("optimizer"):
            self.opt.apply(model.flat, clip=clip)
            model.zero_grad()

    # ---- critic losses --------------------------------------------------------------------
    def _bce_step(self, x, label: float):
        C = self.critic
        p, tape = C.efwd(x, save=True)
        out, dp = Fn.gan_loss(p, p.numel(), label, label, 1)  # K10: value + gradient, one pass
        C.ebwd(tape, dp, hook=self._hook(C))
        self._apply(C)
        return out[0].to(self._acc)

    def _wgan_step(self, x, label: float, clip: float):
        C = self.critic
        s, tape = C.efwd(x, save=True)
        out, ds = Fn.gan_loss(s, s.numel(), label, label, 0)
        C.ebwd(tape, ds, hook=self._hook(C))
        self._apply(C, clip=clip)
        return out[0].to(self._acc)

    def _gp_step(self, real, noise, xrf=None, keep_gen_tape=False):
        """One GP critic update.  ``keep_gen_tape``: run the generator forward with its tape and
        return (fake, tape) for the generator step that follows (see train_step)."""
        dst = None if xrf is None else xrf[real.shape[0]:]
        with trange("critic/generate"):
            if keep_gen_tape:
                fake, gtape = self.generator.efwd(noise, save=True, out=dst)
            else:
                fake, gtape = self.generator.predict(noise, out=dst), None
            alpha = self.rng.uniform((real.shape[0],))
        out = self.critic_gp_grads(real, fake, alpha, xrf=xrf)
        self._apply(self.critic)
        return out, ((fake, gtape) if keep_gen_tape else None)

    def _gp_critic_steps_overlapped(self, B):
        """The n_critic GP critic updates with the generator forward of update k + 1 on a side stream
        while update k's critic work runs (the critic updates never touch G).  The RNG draws keep the
        sequential order (real_k, noise_k, alpha_k, real_k+1, noise_k+1, ...), so every update sees the
        bits it would see sequentially.  Returns (noise, (fake, tape)) of the last update for the
        generator step."""
        cfg, G = self.cfg, self.generator
        side = self._side(1)
        cur = torch.cuda.current_stream(self.device)
        last = self.n_critic - 1

        def sample():
            with trange("critic/sample"):
                xrf = torch.empty((2 * B, cfg.window, cfg.features), dtype=self.dtype, device=self.device)
                real, noise = self._batch(B, out=xrf[:B])
            return xrf, real, noise

        def generate(noise, xrf, keep):
            with trange("critic/generate"):
                if keep:
                    return G.efwd(noise, save=True, out=xrf[B:])
                return G.predict(noise, out=xrf[B:]), None

        xrf, real, noise = sample()
        fake, gtape = generate(noise, xrf, self.reuse_gen_forward and last == 0)
        for k in range(self.n_critic):
            with trange("critic/generate"):
                alpha = self.rng.uniform((B,))
            if k < last:
                nxt = sample()
                side.wait_stream(cur)  # (after the sampling kernels of update k + 1)
                with torch.cuda.stream(side):
                    gnext = generate(nxt[2], nxt[0], self.reuse_gen_forward and k + 1 == last)
            self._d_acc = self.critic_gp_grads(real, fake, alpha, xrf=xrf)
            self._apply(self.critic)
            if k < last:
                cur.wait_stream(side)
                (xrf, real, noise), (fake, gtape) = nxt, gnext
        return noise, ((fake, gtape) if self.reuse_gen_forward else None)

    def critic_gp_grads(self, real, fake, alpha, xrf=None):
        """Accumulate d/dtheta_C of W(real,-1) + W(fake,+1) + lambda*GP(x_hat) into C.flat.grad.

        ``xrf``: the [real; fake] critic input when ``real`` / ``fake`` already are its two row
        halves (the sampler and the generator write straight into it: no concatenation copy)."""
        C = self.critic
        xh = Fn.interpolate(real, fake, alpha)
        if xrf is None:
            xrf = torch.cat([real, fake], 0)
        side = self._side(0)
        if side is not None:
            # the gradient penalty's input-gradient chain (forward on x_hat, backward with wgrad off) and
            # the tangent forward along v = dGP/dg write no gradient and share nothing with the W-terms
            # chain: they run on a side stream; only the tangent reverse (whose weight gradient
            # accumulates into C.flat.grad after the W terms') waits for the join.  Every tensor the side
            # chain allocates lives until after the join, and the side stream's next use starts with a
            # fork from this stream, so no allocator block is reused across the streams while in use.
            cur = torch.cuda.current_stream(self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side), trange("critic/gp_input_grad"):
                sh, tape_h = C.efwd(xh, save=True, head_out=False)  # D(x_hat) itself is never read
                g = C.ebwd(tape_h, self._ones(sh), need_dx=True, wgrad=False)
                pen, v = Fn.gp_coef(g, self.gp_weight)
                sd, ttape = C.etfwd(tape_h, v.to(xh.dtype), head_out=False)
        hook = self._hook(C)
        # (concurrent, no per-layer all-reduce hook: every layer's weight gradient runs on side stream
        # 2 beside the next layer's backward, in the sequential order; joined before the return)
        with Fn.wgrad_on(self._wgrad_side(hook)):
            # W terms on [real; fake]
            with trange("critic/w_terms"):
                # W(real, -1) and W(fake, +1): the score gradient of every row is the known constant
                # -1/B or +1/B, so the head's weight gradient rides along with the head forward
                n2 = xrf.shape[0] // 2
                hw = (n2, Fn.loss_grad_value(-1.0, n2, xrf.dtype), Fn.loss_grad_value(1.0, xrf.shape[0] - n2, xrf.dtype))
                s, tape = C.efwd(xrf, save=True, head_wgrad=hw)
                # both segment means and the score gradient in one launch
                w, ds = Fn.gan_loss(s, s.numel() // 2, -1.0, 1.0, 0)
                C.ebwd(tape, ds)
            if side is not None:
                cur.wait_stream(side)
            # gradient penalty: g = dD/dx_hat (input gradient only), v = dGP/dg, then the
            # theta-gradient of <v, g> as reverse-over-tangent
            if side is None:
                with trange("critic/gp_input_grad"):
                    sh, tape_h = C.efwd(xh, save=True, head_out=False)  # D(x_hat) itself is never read
                    g = C.ebwd(tape_h, self._ones(sh), need_dx=True, wgrad=False)
                    pack, v = Fn.gp_coef_pack(g, self.gp_weight, w)  # [total, W real, W fake, GP]
                with trange("critic/gp_second_order"):
                    sd, ttape = C.etfwd(tape_h, v.to(xh.dtype), head_out=False)
            else:
                pack = Fn.gp_pack(pen, self.gp_weight, w)
            with trange("critic/gp_second_order"):
                C.etbwd(tape_h, ttape, None, self._ones(sd), hook=hook)
        return pack.to(self._acc)

    def _ones(self, like):
        """A persistent all-ones seed shaped like ``like`` (allocated once per shape / dtype: no fill
        kernel on the step; read-only, so graph replays see the same tensor)."""
        key = (tuple(like.shape), like.dtype, like.device)
        t = self._ones_cache.get(key)
        if t is None:
            t = self._ones_cache[key] = torch.ones_like(like)
        return t

    # ---- generator ------------------------------------------------------------------------
    def _generator_step(self, noise, gen=None):
        with trange("generator"):
            loss = self.generator_grads(noise, gen=gen)
        self._apply(self.generator)
        return loss

    def generator_grads(self, noise, gen=None):
        """Accumulate d/dtheta_G of the generator loss through the frozen critic.

        ``gen``: (fake, tape) of G(noise) already computed with the CURRENT generator weights (the
        last critic step's forward of the same noise: the critic updates do not touch G), reused
        instead of a second identical forward."""
        G, C = self.generator, self.critic
        fake, tg = gen if gen is not None else G.efwd(noise, save=True)
        s, tc = C.efwd(fake, save=True)
        if self.cfg.loss == "gan":
            out, ds = Fn.gan_loss(s, s.numel(), 1.0, 1.0, 1)
        else:
            out, ds = Fn.gan_loss(s, s.numel(), -1.0, -1.0, 0)
        loss = out[0].to(self._acc)
        dfake = C.ebwd(tc, ds, need_dx=True, wgrad=False)
        hook = self._hook(G)
        with Fn.wgrad_on(self._wgrad_side(hook)):
            G.ebwd(tg, dfake, hook=hook)
        return loss

    # ---- one reference "epoch" (= iteration) ----------------------------------------------------
    @torch.no_grad()
    def train_step(self):
        cfg, B = self.cfg, self.cfg.batch_size
        if self._fused is not None:
            self._fused.train_step()
        elif cfg.loss == "gan":
            real, noise = self._batch(B)
            fake = self.generator.predict(noise)
            lr_ = self._bce_step(real, 1.0)
            lf_ = self._bce_step(fake, 0.0)
            d = 0.5 * (lr_ + lf_)
            self._d_acc = torch.stack([d, lr_, lf_, torch.zeros_like(d)])
            noise2 = self.rng.normal((B, cfg.window, cfg.features), dtype=self.dtype)
            self._g_acc = self._generator_step(noise2).reshape(1)
        elif cfg.loss == "wgan":
            gen = None
            for k in range(self.n_critic):
                real, noise = self._batch(B)
                if self.reuse_gen_forward and k == self.n_critic - 1:  # reused by the G step (same noise, same G)
                    gen = self.generator.efwd(noise, save=True)
                    fake = gen[0]
                else:
                    fake = self.generator.predict(noise)
                lr_ = self._wgan_step(real, -1.0, 0.0)
                lf_ = self._wgan_step(fake, 1.0, self.clip)
                self._d_acc = torch.stack([0.5 * (lr_ + lf_), lr_, lf_, torch.zeros_like(lr_)])
            self._g_acc = self._generator_step(noise, gen=gen).reshape(1)
        elif self._side(1) is not None:
            noise, gen = self._gp_critic_steps_overlapped(B)
            self._g_acc = self._generator_step(noise, gen=gen).reshape(1)
        else:
            gen = None
            for k in range(self.n_critic):
                with trange("critic/sample"):
                    xrf = torch.empty((2 * B, cfg.window, cfg.features), dtype=self.dtype, device=self.device)
                    real, noise = self._batch(B, out=xrf[:B])
                # the generator step trains on the LAST critic step's noise (GAN/MTSS_WGAN_GP.py:281)
                # with the same generator weights: that step keeps its generator tape for it
                self._d_acc, gen = self._gp_step(real, noise, xrf, keep_gen_tape=self.reuse_gen_forward and k == self.n_critic - 1)
            self._g_acc = self._generator_step(noise, gen=gen).reshape(1)
        self.iteration += 1

    def close(self) -> None:
        """Collective teardown of the data-parallel communicators this trainer owns (every rank, same
        point; a no-op for a single process)."""
        if self.grad_sync is not None:
            self.grad_sync.close()

    def losses(self) -> dict:
        d = self._d_acc.detach().float().cpu().numpy()
        return {"iteration": self.iteration, "d_loss": float(d[0]), "d_real": float(d[1]), "d_fake": float(d[2]),
                "gp": float(d[3]), "g_loss": float(self._g_acc.detach().float().cpu()[0])}

    def allreduce_floats_per_step(self) -> int:
        """Gradient floats one rank all-reduces per iteration under data parallelism: the critic's flat
        buffer once per critic update (2 for the BCE GAN, 2 n_critic for the clipped WGAN, n_critic
        with the gradient penalty) plus the generator's once."""
        loss = self.cfg.loss
        updates = 2 if loss == "gan" else 2 * self.n_critic if loss == "wgan" else self.n_critic
        return updates * self.critic.flat.numel() + self.generator.flat.numel()

    def windows_per_iteration(self) -> int:
        """Windows consumed per iteration on this rank (SURVEY §6 seq/s definition)."""
        B = self.cfg.batch_size
        nc = 2 if self.cfg.loss == "gan" else self.n_critic
        return nc * B + B

    def train(self, epochs: int | None = None, log=None, verbose: bool = True, graph: bool = False):
        """``epochs`` reference iterations.  ``graph=True`` replays the step from a captured hipGraph
        after two eager warmup steps (train/runner.py GraphedStep: bitwise identical to eager)."""
        epochs = self.cfg.epochs if epochs is None else epochs
        t0 = time.time()
        hist = []
        step = self.train_step
        if graph:
            from .runner import GraphedStep

            step = GraphedStep(self)
        for ep in range(epochs):
            step()
            if (ep + 1) % self.cfg.log_every == 0 or ep == epochs - 1:
                rec = self.losses()
                rec["elapsed_s"] = time.time() - t0
                hist.append(rec)
                if log is not None:
                    log(rec)
                elif verbose and self.rank == 0:
                    print("%d [D loss: %f] [G loss: %f]" % (ep, rec["d_loss"], rec["g_loss"]))
        return hist

    # ---- generation ---------------------------------------------------------------------------
    @torch.no_grad()
    def generate(self, n: int, window: int | None = None, batch: int = 4096, seed: int | None = None) -> np.ndarray:
        """N(0,1) noise -> generator windows; LSTM generators accept any window length."""
        T = window or self.cfg.window
        rng = DeviceRNG(self.cfg.seed if seed is None else seed, self.device, stream=10_000 + self.rank)
        out = []
        for s in range(0, n, batch):
            b = min(batch, n - s)
            z = rng.normal((b, T, self.cfg.features), dtype=self.dtype)
            out.append(self.generator.predict(z).float().cpu())
        return torch.cat(out).numpy()
