"""Window datasets: reference sampling, the GAN-script dataset and synthetic windows.

* :func:`random_sampling` — ``helper.random_sampling`` (helper.py:44-62): ``n_sample`` windows
  of length ``window`` drawn WITH replacement, start ``randint(0, N - window)`` inclusive.
* :func:`gan_dataset` — the module prologue of every GAN script (e.g. GAN/MTSS_WGAN_GP.py:88-101):
  join factor ETFs + HF indices (35 cols; +rf for the production 36-col variant), MinMax-scale on
  the full panel (Q11), sample 1000 windows of 48.
* :func:`synthetic_windows` — the benchmark's synthetic return windows (no network, no data):
  a correlated Gaussian factor model with fat-tailed shocks, MinMax-scaled to [0, 1] like the
  real pipeline, any (N, T, F).
"""
from __future__ import annotations

import random

import numpy as np

from .scaler import MinMaxScaler


def random_sampling(dataset: np.ndarray, n_sample: int, window: int, seed: int | None = None) -> np.ndarray:
    dataset = np.asarray(dataset)
    r = random.Random(seed) if seed is not None else random
    hi = dataset.shape[0] - window
    starts = [r.randint(0, hi) for _ in range(n_sample)]
    idx = np.asarray(starts)[:, None] + np.arange(window)[None, :]
    return dataset[idx]


def gan_dataset(cleaned: dict, n_sample: int = 1000, window: int = 48, include_rf: bool = False,
                seed: int | None = 123):
    """(windows (n, window, F) float32, fitted scaler, column names)."""
    panel = cleaned["factor_etf_data"].join(cleaned["hfd"])
    if include_rf:
        panel = panel.join(cleaned["rf"])
    scaler = MinMaxScaler()
    data = scaler.fit_transform(panel.to_numpy())
    wins = random_sampling(data, n_sample, window, seed=seed).astype(np.float32)
    return wins, scaler, list(panel.columns)


def synthetic_windows(n: int, window: int = 24, features: int = 32, seed: int = 0, factors: int = 4,
                      dtype=np.float32) -> np.ndarray:
    rs = np.random.RandomState(seed)
    L = rs.randn(features, factors) * 0.6
    idio = 0.3 + 0.2 * rs.rand(features)
    # latent AR(1) factors with Student-t shocks -> cross-sectionally correlated, autocorrelated returns
    T = window
    f = np.zeros((n, T, factors))
    shocks = rs.standard_t(5, size=(n, T, factors)) * 0.5
    for t in range(T):
        f[:, t] = (0.2 * f[:, t - 1] if t else 0) + shocks[:, t]
    eps = rs.standard_t(4, size=(n, T, features)) * idio
    x = f @ L.T + eps
    lo, hi = np.percentile(x, 0.5, axis=(0, 1)), np.percentile(x, 99.5, axis=(0, 1))
    x = np.clip((x - lo) / (hi - lo), 0.0, 1.0)
    return x.astype(dtype)
