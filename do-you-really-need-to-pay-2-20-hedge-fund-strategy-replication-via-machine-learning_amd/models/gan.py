"""The GAN model zoo: generators and critics/discriminators of the six reference scripts.

Registry key = (architecture, loss) with architecture in {mlp, lstm, conv} and loss in
{gan (BCE), wgan (weight clipping), wgan_gp (gradient penalty)}; the reference's class names
are kept as aliases (the GP file/class names are swapped upstream).

| key               | reference                                   | generator               | critic                                    |
|-------------------|---------------------------------------------|-------------------------|-------------------------------------------|
| (mlp, gan)        | GAN/GAN.py:127-158, class GAN               | MLP G                   | Dense(100)->Dense(100)->Dense(1,sigmoid)  |
| (mlp, wgan)       | GAN/WGAN.py:129-164, class WGAN             | MLP G                   | Dense->LReLU->LN->Dense->LReLU->LN->Dense(1) |
| (mlp, wgan_gp)    | GAN/WGAN_GP.py:221-253, class MTTS_WGAN_GP  | MLP G                   | Dense(100)->Dense(100)->Flatten->Dense(1) |
| (lstm, gan)       | GAN/MTSS_GAN.py:127-157, class MTTS_GAN     | LSTM G                  | LSTM(100)->LSTM(100)->Dense(1,sigmoid)    |
| (lstm, wgan)      | GAN/MTSS_WGAN.py:129-163, class MTTS_WGAN   | LSTM G                  | LSTM(lin)->LReLU->LN->LSTM(lin)->LReLU->LN->Dense(1) |
| (lstm, wgan_gp)   | GAN/MTSS_WGAN_GP.py:221-252, class WGAN_GP  | LSTM G                  | LSTM(100)->LSTM(100)->Flatten->Dense(1)   |
| (conv, wgan_gp)   | north-star K14 (not in the reference)       | LSTM G                  | Conv1D x2 -> Flatten -> Dense(1)          |

MLP G = Dense(100,sigmoid)->LReLU->LN->Dense(100,sigmoid)->LReLU->LN->Dense(F).
LSTM G = LSTM(100,act=sigmoid)->[LReLU]->LN->LSTM(100,sigmoid)->LReLU->LN->Dense(F); the
optional LReLU after the first LSTM reproduces the shipped production checkpoint
(``MTTS_GAN_GP20220621_02-49-32.h5``).
"""
from __future__ import annotations

from dataclasses import dataclass

from .layers import LSTM, Conv1D, Dense, Flatten, LayerNormalization, LeakyReLU, Sequential

HIDDEN = 100


def mlp_generator(T, F, hidden=HIDDEN, **kw):
    return Sequential([Dense(hidden, "sigmoid"), LeakyReLU(), LayerNormalization(),
                       Dense(hidden, "sigmoid"), LeakyReLU(), LayerNormalization(), Dense(F)], (T, F),
                      name="generator", **kw)


def lstm_generator(T, F, hidden=HIDDEN, lrelu_after_first: bool = False, **kw):
    layers = [LSTM(hidden, activation="sigmoid")]
    if lrelu_after_first:
        layers.append(LeakyReLU())
    layers += [LayerNormalization(), LSTM(hidden, activation="sigmoid"), LeakyReLU(), LayerNormalization(), Dense(F)]
    return Sequential(layers, (T, F), name="generator", **kw)


def mlp_discriminator(T, F, hidden=HIDDEN, **kw):
    return Sequential([Dense(hidden), Dense(hidden), Dense(1, "sigmoid")], (T, F), name="discriminator", **kw)


def mlp_critic_clip(T, F, hidden=HIDDEN, **kw):
    return Sequential([Dense(hidden), LeakyReLU(), LayerNormalization(), Dense(hidden), LeakyReLU(),
                       LayerNormalization(), Dense(1)], (T, F), name="critic", **kw)


def mlp_critic_gp(T, F, hidden=HIDDEN, **kw):
    return Sequential([Dense(hidden), Dense(hidden), Flatten(), Dense(1)], (T, F), name="critic", **kw)


def lstm_discriminator(T, F, hidden=HIDDEN, **kw):
    return Sequential([LSTM(hidden, "tanh"), LSTM(hidden, "tanh"), Dense(1, "sigmoid")], (T, F),
                      name="discriminator", **kw)


def lstm_critic_clip(T, F, hidden=HIDDEN, **kw):
    return Sequential([LSTM(hidden, None), LeakyReLU(), LayerNormalization(), LSTM(hidden, None), LeakyReLU(),
                       LayerNormalization(), Dense(1)], (T, F), name="critic", **kw)


def lstm_critic_gp(T, F, hidden=HIDDEN, **kw):
    return Sequential([LSTM(hidden, "tanh"), LSTM(hidden, "tanh"), Flatten(), Dense(1)], (T, F), name="critic", **kw)


def conv_critic_gp(T, F, hidden=HIDDEN, kernel_size=3, **kw):
    return Sequential([Conv1D(hidden, kernel_size, "leaky_relu"), Conv1D(hidden, kernel_size, "leaky_relu", dilation=2),
                       Flatten(), Dense(1)], (T, F), name="critic", **kw)


@dataclass(frozen=True)
class ZooEntry:
    generator: callable
    critic: callable
    loss: str           # gan | wgan | wgan_gp
    optimizer: str      # adam | rmsprop
    lr: float
    n_critic: int
    clip: float = 0.0
    gp_weight: float = 0.0
    save_prefix: str = ""
    legacy_class: str = ""


ZOO = {
    ("mlp", "gan"): ZooEntry(mlp_generator, mlp_discriminator, "gan", "adam", 2e-4, 1, save_prefix="GAN",
                             legacy_class="GAN"),
    ("mlp", "wgan"): ZooEntry(mlp_generator, mlp_critic_clip, "wgan", "rmsprop", 5e-5, 5, clip=0.01,
                              save_prefix="WGAN", legacy_class="WGAN"),
    ("mlp", "wgan_gp"): ZooEntry(mlp_generator, mlp_critic_gp, "wgan_gp", "rmsprop", 5e-5, 5, gp_weight=10.0,
                                 save_prefix="GAN_GP", legacy_class="MTTS_WGAN_GP"),
    ("lstm", "gan"): ZooEntry(lstm_generator, lstm_discriminator, "gan", "adam", 2e-4, 1, save_prefix="MTSS_GAN",
                              legacy_class="MTTS_GAN"),
    ("lstm", "wgan"): ZooEntry(lstm_generator, lstm_critic_clip, "wgan", "rmsprop", 5e-5, 5, clip=0.01,
                               save_prefix="MTSS_WGAN", legacy_class="MTTS_WGAN"),
    ("lstm", "wgan_gp"): ZooEntry(lstm_generator, lstm_critic_gp, "wgan_gp", "rmsprop", 5e-5, 5, gp_weight=10.0,
                                  save_prefix="MTSS_GAN_GP", legacy_class="WGAN_GP"),
    ("conv", "wgan_gp"): ZooEntry(lstm_generator, conv_critic_gp, "wgan_gp", "rmsprop", 5e-5, 5, gp_weight=10.0,
                                  save_prefix="CONV_GAN_GP", legacy_class="CONV_WGAN_GP"),
    # the MTSS-WGAN LayerNorm critic trained with the gradient penalty instead of clipping (a
    # framework variant: exercises the LayerNorm tangent kernels in the reverse-over-tangent critic step)
    ("lstm_ln", "wgan_gp"): ZooEntry(lstm_generator, lstm_critic_clip, "wgan_gp", "rmsprop", 5e-5, 5, gp_weight=10.0,
                                     save_prefix="MTSS_LN_GAN_GP", legacy_class="MTSS_LN_WGAN_GP"),
}

LEGACY = {e.legacy_class: k for k, e in ZOO.items()}
ALIASES = {
    "gan": ("mlp", "gan"), "wgan": ("mlp", "wgan"), "wgan_gp": ("mlp", "wgan_gp"),
    "mtss_gan": ("lstm", "gan"), "mtss_wgan": ("lstm", "wgan"), "mtss_wgan_gp": ("lstm", "wgan_gp"),
    "conv_wgan_gp": ("conv", "wgan_gp"), "mtss_ln_wgan_gp": ("lstm_ln", "wgan_gp"),
}


def resolve(name_or_key) -> tuple:
    if isinstance(name_or_key, tuple):
        return name_or_key
    if name_or_key in LEGACY:
        return LEGACY[name_or_key]
    return ALIASES[name_or_key.lower()]
