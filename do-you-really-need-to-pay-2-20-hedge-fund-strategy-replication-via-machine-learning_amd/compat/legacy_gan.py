"""Legacy GAN classes with the reference constructor/training API.

Each reference script defines one class taking the (N, T, F) window array and exposing
``train(epochs, batch_size, sample_interval)``, ``generator``, ``critic``/``discriminator`` and
``build_generator()/build_critic()`` (e.g. GAN/MTSS_WGAN_GP.py:115-287).  Here every class is a
thin wrapper around :class:`hfrep.train.gan_trainer.GANTrainer` keyed by (architecture, loss):

    GAN -> (mlp, gan)        WGAN -> (mlp, wgan)        MTTS_WGAN_GP -> (mlp, wgan_gp)
    MTTS_GAN -> (lstm, gan)  MTTS_WGAN -> (lstm, wgan)  WGAN_GP -> (lstm, wgan_gp)

At the end of ``train`` the generator is saved as ``./trained_generator/<Prefix><timestamp>.pkl``
(prefixes as in the reference, e.g. ``MTSS_GAN_GP``) plus an ``.npz`` twin.  Unlike the reference
the dataset prologue does NOT run at import: call :func:`reference_dataset` (or run the script).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..models import gan as zoo
from ..train.gan_trainer import GANConfig, GANTrainer
from ..utils import checkpoint


def reference_dataset(n_sample: int = 1000, window: int = 48, seed: int = 123, include_rf: bool = False):
    """The scripts' module prologue (GAN/MTSS_WGAN_GP.py:88-101): 1000 x 48 x 35 scaled windows."""
    from ..data.io import load_cleaned
    from ..data.windows import gan_dataset
    from ..utils.seed import set_seed

    set_seed(seed)
    wins, scaler, cols = gan_dataset(load_cleaned(), n_sample=n_sample, window=window, include_rf=include_rf,
                                     seed=seed)
    return wins


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class _LegacyGAN:
    KEY = ("mlp", "gan")

    def __init__(self, dataset, device=None, dtype: str = "float32", seed: int = 123, **cfg_overrides):
        assert isinstance(dataset, np.ndarray) and dataset.ndim == 3
        self.X_train = dataset
        self.ts_length, self.ts_feature = dataset.shape[1], dataset.shape[2]
        self.ts_shape = self.latent_shape = (self.ts_length, self.ts_feature)
        self._entry = zoo.ZOO[self.KEY]
        self.n_critic = self._entry.n_critic
        self.clip_value = self._entry.clip
        self.device = torch.device(device) if device is not None else _default_device()
        self._cfg_kw = dict(arch=self.KEY[0], loss=self.KEY[1], window=self.ts_length, features=self.ts_feature,
                            dtype=dtype, seed=seed, **cfg_overrides)
        self._trainer = None
        self._make(batch_size=32)

    def _make(self, batch_size):
        cfg = GANConfig(batch_size=batch_size, **self._cfg_kw)
        old = self._trainer
        self._trainer = GANTrainer(cfg, self.X_train, device=self.device)
        if old is not None:  # keep trained weights when only the batch size changes
            with torch.no_grad():
                self._trainer.generator.flat.copy_(old.generator.flat)
                self._trainer.critic.flat.copy_(old.critic.flat)
            self._trainer.opt = old.opt

    # reference attribute names
    @property
    def generator(self):
        return self._trainer.generator

    @property
    def critic(self):
        return self._trainer.critic

    discriminator = critic

    def build_generator(self):
        """A fresh generator of this model's architecture, honouring the ``hidden`` and (LSTM
        generators) ``lrelu_after_first`` overrides the instance was built with."""
        cfg = self._trainer.cfg
        if self.KEY[0] == "mlp":
            return self._entry.generator(self.ts_length, self.ts_feature, cfg.hidden)
        return self._entry.generator(self.ts_length, self.ts_feature, cfg.hidden,
                                     lrelu_after_first=cfg.lrelu_after_first)

    def build_critic(self):
        return self._entry.critic(self.ts_length, self.ts_feature)

    build_discriminator = build_critic

    def train(self, epochs, batch_size=128, sample_interval=50, save_dir: str | None = "./trained_generator",
              verbose: bool = True, log_every: int = 1, graph: bool | None = None):
        """The reference ``train``; on a GPU the step replays from a hipGraph unless ``graph=False``
        or HFREP_GRAPH=0 (at the reference's batch 32 the step is launch-bound: graph replay is what
        makes it fast, profiles/r01_parity)."""
        if batch_size != self._trainer.cfg.batch_size:
            self._make(batch_size)
        self._trainer.cfg.log_every = log_every
        if graph is None:
            graph = (self.device.type == "cuda" and os.environ.get("HFREP_GRAPH", "1") != "0"
                     and self._trainer.rng.native)
        hist = self._trainer.train(epochs, verbose=verbose, graph=graph)
        self.history = hist
        if save_dir:
            os.makedirs(save_dir, exist_ok=True)
            stem = os.path.join(save_dir, f"{self._entry.save_prefix}{checkpoint.timestamp()}")
            # the trainer's real architecture: a Q2-variant generator (LReLU after the first LSTM) or
            # a non-default width must be rebuilt as such by checkpoint.load_generator
            tc = self._trainer.cfg
            cfg = dict(self._cfg_kw, hidden=tc.hidden, lrelu_after_first=tc.lrelu_after_first)
            checkpoint.save_generator(stem + ".pkl", self.generator, cfg)
            checkpoint.save_generator(stem + ".npz", self.generator, cfg)
            self.saved_path = stem + ".pkl"
        return hist

    def generate(self, n: int, window: int | None = None, seed: int | None = None) -> np.ndarray:
        return self._trainer.generate(n, window=window, seed=seed)


class GAN(_LegacyGAN):
    KEY = ("mlp", "gan")


class WGAN(_LegacyGAN):
    KEY = ("mlp", "wgan")


class MTTS_WGAN_GP(_LegacyGAN):  # MLP + gradient penalty (GAN/WGAN_GP.py)
    KEY = ("mlp", "wgan_gp")


class MTTS_GAN(_LegacyGAN):
    KEY = ("lstm", "gan")


class MTTS_WGAN(_LegacyGAN):
    KEY = ("lstm", "wgan")


class WGAN_GP(_LegacyGAN):  # stacked LSTM + gradient penalty (GAN/MTSS_WGAN_GP.py)
    KEY = ("lstm", "wgan_gp")


def script_main(cls, epochs: int = 5000, batch_size: int = 32):
    """``python GAN/<Model>.py``: reference prologue + 5000 iterations at batch 32 + save."""
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=epochs)
    ap.add_argument("--batch-size", type=int, default=batch_size)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--save-dir", default="./trained_generator")
    ap.add_argument("--log-every", type=int, default=100)
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of hipGraph replay (GPU)")
    a = ap.parse_args()
    ds = reference_dataset()
    model = cls(ds, dtype=a.dtype)
    model.train(epochs=a.epochs, batch_size=a.batch_size, save_dir=a.save_dir, log_every=a.log_every,
                graph=False if a.no_graph else None)
    print(f"saved {model.saved_path}")
