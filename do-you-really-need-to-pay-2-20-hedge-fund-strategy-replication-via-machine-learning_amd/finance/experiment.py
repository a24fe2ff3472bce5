"""The notebook's autoencoder replication experiment as a library.

``autoencoder_v4.ipynb`` drives everything by hand: a 50/50 chronological split of the ETF
factor panel and the hedge-fund index panel (cell 112/159), one factor autoencoder per latent
size 1..21, in-sample / out-of-sample reconstruction metrics, ex-ante / ex-post clone returns and
turnover per latent size (cells 899-1000), the analytics table of each clone, and the best latent
size per strategy by ex-post Sharpe (``res_sort``, cell 958).  The same study is then repeated
with the training rows augmented by MTSS-WGAN-GP generated windows (cells 1277-1475:
generator -> N(0,1) noise -> inverse MinMax with the 36-column scaler -> ``factor_hf_split``
-> vstack with the real rows).

:func:`latent_sweep` and :func:`generated_augmentation` reproduce those two flows; both return
plain DataFrames / arrays so they can be scripted or run from the CLI
(``python -m hfrep replicate --method ae-sweep``).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import pandas as pd

from ..data.scaler import MinMaxScaler
from . import analytics
from .autoencoder_replication import AE
from .replication import factor_hf_split


@dataclass
class SweepResult:
    metrics: pd.DataFrame                         # latent x [IS_r2, IS_RMSE, OOS_r2, OOS_RMSE]
    sharpe_ante: pd.DataFrame                     # latent x strategy
    sharpe_post: pd.DataFrame                     # latent x strategy
    turnover: pd.DataFrame                        # latent x strategy
    best: pd.DataFrame                            # strategy -> best latent by ex-post Sharpe
    post_tables: list = field(default_factory=list)


def chronological_split(cleaned: dict, frac: float = 0.5):
    """(x_train, y_train, x_test, y_test) DataFrames: first / second part of the monthly panel."""
    etf, hfd = cleaned["factor_etf_data"], cleaned["hfd"]
    n = int(len(etf) * frac)
    return etf.iloc[:n], hfd.iloc[:n], etf.iloc[n:], hfd.iloc[n:]


def latent_sweep(cleaned: dict, latents=range(1, 22), window: int = 24, frac: float = 0.5,
                 x_extra: np.ndarray | None = None, y_extra: np.ndarray | None = None, seed: int = 123,
                 device="cpu", verbose: bool = False, dtype=None) -> SweepResult:
    """Train one autoencoder per latent size and evaluate it as a hedge-fund clone.

    ``x_extra`` / ``y_extra``: extra (generated) training rows appended to the real training rows
    (the augmented study); the test period is always real data.  ``device`` / ``dtype``: where and
    in which compute dtype the autoencoders train and predict (fp32 on the CPU by default; ``cuda``
    runs the engine's native Dense / optimizer kernels, BASELINE config 2).  On the GPU the sweep's
    fits train in one launch (``AE.train_many``).
    """
    return latent_sweep_many(cleaned, seeds=[seed], latents=latents, window=window, frac=frac,
                             x_extras=[x_extra], y_extras=[y_extra], device=device, verbose=verbose, dtype=dtype)[0]


def latent_sweep_many(cleaned: dict, seeds, latents=range(1, 22), window: int = 24, frac: float = 0.5,
                      x_extras=None, y_extras=None, device="cpu", verbose: bool = False, dtype=None) -> list:
    """``latent_sweep`` for several seeds (``x_extras[i]`` / ``y_extras[i]``: seed i's extra rows or None):
    every (seed, latent) autoencoder is built first and all of them train together (one csrc/ae.hip
    launch on a native GPU build), then each is evaluated.  Returns one SweepResult per seed."""
    seeds = list(seeds)
    latents = list(latents)
    x_extras = list(x_extras) if x_extras is not None else [None] * len(seeds)
    y_extras = list(y_extras) if y_extras is not None else [None] * len(seeds)
    x_tr, y_tr, x_te, y_te = chronological_split(cleaned, frac)
    rf = cleaned["rf"]
    names = cleaned.get("hfd_fullname", {c: c for c in y_te.columns})
    aes = []
    for s, xe, ye in zip(seeds, x_extras, y_extras):
        xtr, ytr = x_tr.to_numpy(), y_tr.to_numpy()
        if xe is not None:
            xtr = np.vstack([xtr, xe])
            ytr = np.vstack([ytr, ye])
        for k in latents:
            aes.append(AE(xtr, ytr, x_te, y_te, k, device=device, seed=s,
                          **({"dtype": dtype} if dtype is not None else {})))
    AE.train_many(aes)
    out = []
    for si in range(len(seeds)):
        rows, s_ante, s_post, turns, posts = [], [], [], [], []
        for ki, k in enumerate(latents):
            ae = aes[si * len(latents) + ki]
            oos_r2, oos_rmse = ae.model_OOS_r2(), ae.model_OOS_RMSE()
            rows.append({"latent": k, "IS_r2": float(ae.model_IS_r2()), "IS_RMSE": float(ae.model_IS_RMSE()),
                         "OOS_r2": float(np.mean(oos_r2)), "OOS_RMSE": float(np.mean(oos_rmse))})
            ante = ae.ante(rf.iloc[-len(y_te):], y_te, window=window)
            post = ae.post(cleaned["factor_etf_data"])
            to = ae.turnover(names)
            rf_slice = pd.DataFrame(np.asarray(rf.iloc[-len(post):], dtype=np.float64)[:, :1], index=post.index)
            s_ante.append({c: float(analytics.annualized_sharpe_ratio(ante[c], rf_slice)) for c in ante.columns})
            s_post.append({c: float(analytics.annualized_sharpe_ratio(post[c], rf_slice)) for c in post.columns})
            turns.append(dict(zip(post.columns, to["Turnover"].to_numpy())))
            posts.append(pd.DataFrame({"Annualized_Sharpe": [s_post[-1][c] for c in post.columns]},
                                      index=list(post.columns)))
            if verbose:
                print(f"seed {seeds[si]} latent {k}: {rows[-1]}")
        idx = pd.Index(latents, name="latent")
        best, bidx = analytics.res_sort(posts)
        best["latent"] = [b + 1 for b in bidx] if latents == list(range(1, len(posts) + 1)) else \
            [latents[b] for b in bidx]
        out.append(SweepResult(metrics=pd.DataFrame(rows).set_index("latent"),
                               sharpe_ante=pd.DataFrame(s_ante, index=idx), sharpe_post=pd.DataFrame(s_post, index=idx),
                               turnover=pd.DataFrame(turns, index=idx), best=best, post_tables=posts))
    return out


def generated_augmentation(generated: np.ndarray, cleaned: dict, split_pos: int = 22, include_rf: bool = True):
    """Generated windows -> extra (X, Y) training rows in return units (notebook cells 1277-1426).

    ``generated`` is (N, T, F) in the generator's MinMax-scaled space; F = 36 for the production
    generator (22 ETF factors + 13 HF indices + rf), 35 without rf.  The scaler is refit on the
    full cleaned panel exactly as the GAN scripts' prologue fitted it (GAN/MTSS_WGAN_GP.py:88-101).
    """
    panel = cleaned["factor_etf_data"].join(cleaned["hfd"])
    if include_rf:
        panel = panel.join(cleaned["rf"])
    if generated.shape[-1] != panel.shape[1]:
        raise ValueError(f"generated windows have {generated.shape[-1]} features, panel has {panel.shape[1]}")
    scaler = MinMaxScaler().fit(panel.to_numpy())
    flat = scaler.inverse_transform(generated.reshape(-1, generated.shape[-1]))
    x, y = factor_hf_split(flat.reshape(generated.shape), split_pos, reshape=True)
    y = y[:, : cleaned["hfd"].shape[1]]  # drop rf if present
    return x, y


def daily_factor_study(daily: pd.DataFrame, latents=range(1, 22), seeds=(123,), frac: float = 0.5, device="cpu",
                       dtype=None, oos_stride: int = 21) -> pd.DataFrame:
    """BASELINE config 2 on its stated data: the factor autoencoder (Autoencoder_encapsulate.py:39-105)
    fitted on the DAILY ETF excess-return matrix (``data.cleaning.build_factor_etf_daily``) instead of
    the 337-month panel.  Chronological ``frac`` split; the Keras fit (Nadam, batch 48, last 25 % of the
    training rows for validation, EarlyStopping(5)) of every (seed, latent) trains in one launch on a
    native GPU build (``AE.train_many``).  Returns one row per (seed, latent): in-sample R^2 / RMSE on
    the training days, the mean out-of-sample R^2 / RMSE over expanding test windows (one every
    ``oos_stride`` trading days, each with its own refit scaler, the reference's OOS procedure), the
    epochs run, and the wall time of the batched fit (``fit_s``, the same for every row)."""
    import time

    x = daily.to_numpy(np.float64)
    n = int(len(x) * frac)
    x_tr, x_te = x[:n], x[n:]
    aes = []
    for s in seeds:
        for k in latents:
            aes.append(AE(x_tr, x_tr, x_te, x_te, k, device=device, seed=s, oos_stride=oos_stride,
                          **({"dtype": dtype} if dtype is not None else {})))
    t0 = time.perf_counter()
    AE.train_many(aes)
    if str(device).startswith("cuda"):
        import torch

        torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    rows = []
    for i, ae in enumerate(aes):
        rows.append({"seed": seeds[i // len(list(latents))], "latent": ae._latent_dim,
                     "IS_r2": float(ae.model_IS_r2()), "IS_RMSE": float(ae.model_IS_RMSE()),
                     "OOS_r2": float(np.mean(ae.model_OOS_r2())), "OOS_RMSE": float(np.mean(ae.model_OOS_RMSE())),
                     "epochs": len(ae.history["loss"]), "fit_s": fit_s, "train_rows": n, "test_rows": len(x_te)})
    return pd.DataFrame(rows)
