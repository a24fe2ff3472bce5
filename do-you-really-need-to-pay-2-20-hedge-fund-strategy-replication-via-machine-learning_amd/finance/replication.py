"""Factor-replication math: clone weights, ex-ante/ex-post returns, costs, turnover.

Capabilities of the reference's ``helper.py`` (helper.py:10-153) and the replication half of
``Autoencoder_encapsulate.AE`` (Autoencoder_encapsulate.py:133-224), re-expressed as
vectorised numpy over (time, asset, strategy) arrays:

* :func:`normalization`         helper.py:10-17 (volatility-matching factor)
* :func:`transaction_cost`      helper.py:65-80  (0.5*dx^2*sqrt(diag S)*kappa)
* :func:`price_impact`          helper.py:83-92
* :func:`reshape_cab`           helper.py:94-110
* :func:`ex_post_return`        helper.py:112-131 (ex-ante + transaction penalty; Q10 sign kept)
* :func:`factor_hf_split`       helper.py:133-153
* :func:`rolling_ols`           statsmodels ``OLS(Y, X)`` (no intercept) on a sliding window
* :func:`clone_weights` / :func:`ex_ante_returns` / :func:`turnover`  (AE.ante/AE.turnover)
* :class:`LinearCloneBenchmark` the rolling-24-month OLS benchmark of the missing
  ``data_cleaning+benchmark.ipynb`` (referenced by Autoencoder_encapsulate.py:143).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import pandas as pd


# ----------------------------------------------------------------------------------------
# helper.py primitives
# ----------------------------------------------------------------------------------------
def normalization(Y, X, beta, window):
    """sqrt(var(Y)) / sqrt(var(X @ beta)) per column, with (window-1) denominators."""
    Y = np.asarray(Y, dtype=np.float64)
    X = np.asarray(X, dtype=np.float64)
    beta = np.asarray(beta, dtype=np.float64)
    r_hat = X @ beta
    den = np.sum((r_hat - r_hat.mean(axis=0)) ** 2 / (window - 1), axis=0)
    num = np.sum((Y - Y.mean(axis=0)) ** 2 / (window - 1), axis=0)
    return np.sqrt(num) / np.sqrt(den)


def _sigma_kappa(cov, param):
    cov = np.asarray(cov, dtype=np.float64)
    return np.sqrt(np.diag(cov)) * param


def transaction_cost(old_x, new_x, covMatrix, param=0.05):
    sk = _sigma_kappa(covMatrix, param)
    dx = np.asarray(old_x, dtype=np.float64) - np.asarray(new_x, dtype=np.float64)
    return 0.5 * dx ** 2 * sk


def price_impact(old_x, new_x, covMatrix, param=0.05, phi=0.5):
    sk = _sigma_kappa(covMatrix, param)
    old_x = np.asarray(old_x, dtype=np.float64)
    new_x = np.asarray(new_x, dtype=np.float64)
    dx = old_x - new_x
    return phi * new_x * sk * dx - old_x * sk * dx - 0.5 * dx ** 2 * sk


def reshape_cab(df_list):
    """list of T frames (A x B) -> list of B frames (T x A), as helper.py:94-110.

    Frame b has the A row labels of the inputs as columns and its own label repeated T times
    as index (what ``pd.DataFrame([df.iloc[:, b] for df in df_list])`` yields).
    """
    assert isinstance(df_list, list) and len(df_list) and isinstance(df_list[0], pd.DataFrame)
    cube = np.stack([d.to_numpy() for d in df_list])  # (T, A, B)
    cols = df_list[0].index
    return [pd.DataFrame(cube[:, :, b], index=[lab] * len(df_list), columns=cols)
            for b, lab in enumerate(df_list[0].columns)]


def rolling_cov(returns: np.ndarray, window: int) -> np.ndarray:
    """(T, A) -> (T-window+1, A, A) sample covariances (ddof=1), vectorised."""
    r = np.asarray(returns, dtype=np.float64)
    win = np.lib.stride_tricks.sliding_window_view(r, window, axis=0)  # (n, A, w)
    mu = win.mean(axis=2, keepdims=True)
    d = win - mu
    return np.einsum("naw,nbw->nab", d, d) / (window - 1)


def transaction_penalty(weights: np.ndarray, etf: np.ndarray, window: int, param=0.05, phi=0.5) -> np.ndarray:
    """Per-period penalty sum(tc + pi) for a weight path.

    weights: (T, A, S) clone weights over time; etf: (T_etf, A) returns where the window
    [i, i+window) gives the covariance used at rebalancing date i (helper.py:121).
    Returns (T-1, S) penalties for i = 1..T-1.
    """
    n = min(weights.shape[0], etf.shape[0] - window)
    covs = rolling_cov(etf, window)  # covs[i] = cov(etf[i:i+w])
    sk = np.sqrt(np.einsum("naa->na", covs[1:n])) * param  # (n-1, A)
    new = weights[1:n]
    old = weights[: n - 1]
    dx = old - new
    tc = 0.5 * dx ** 2 * sk[..., None]
    pi = phi * new * sk[..., None] * dx - old * sk[..., None] * dx - 0.5 * dx ** 2 * sk[..., None]
    return (tc + pi).sum(axis=1)  # (n-1, S)


def ex_post_return(ex_ante, window, strat_weight, factor_etf):
    """helper.py:112-131: ex-post = ex-ante + transaction penalty (penalty added, Q10).

    ``strat_weight`` is the list of per-strategy (T x A) frames produced by :func:`reshape_cab`.
    """
    assert isinstance(ex_ante, pd.DataFrame) and isinstance(factor_etf, pd.DataFrame)
    W = np.stack([np.asarray(w, dtype=np.float64) for w in strat_weight], axis=2)  # (T, A, S)
    pen = transaction_penalty(W, factor_etf.to_numpy(np.float64), window)  # (T-1, S)
    ante = ex_ante.to_numpy(np.float64)
    post = ante.copy()
    k = min(ante.shape[0] - 1, pen.shape[0])
    post[1 : 1 + k] = ante[1 : 1 + k] + pen[:k]
    return pd.DataFrame(post, index=ex_ante.index, columns=ex_ante.columns)


def factor_hf_split(arr, split_pos, reshape=True):
    assert isinstance(arr, np.ndarray) and arr.ndim == 3
    assert isinstance(split_pos, (int, np.integer)) and 0 < split_pos < arr.shape[2]
    factor, hf = arr[:, :, :split_pos], arr[:, :, split_pos:]
    if reshape:
        factor = factor.reshape(-1, factor.shape[2])
        hf = hf.reshape(-1, hf.shape[2])
    return np.ascontiguousarray(factor), np.ascontiguousarray(hf)


# ----------------------------------------------------------------------------------------
# rolling OLS + clone construction
# ----------------------------------------------------------------------------------------
def ols(Y: np.ndarray, X: np.ndarray, add_const: bool = False) -> np.ndarray:
    """Least-squares coefficients (statsmodels OLS semantics: pinv solution)."""
    X = np.asarray(X, dtype=np.float64)
    if add_const:
        X = np.column_stack([np.ones(len(X)), X])
    return np.linalg.pinv(X) @ np.asarray(Y, dtype=np.float64)


def rolling_ols(Y, X, window: int):
    """Betas (n, K, S) and normalisation factors (n, S) for windows [i, i+window), i < T-window."""
    Y = np.asarray(Y, dtype=np.float64)
    X = np.asarray(X, dtype=np.float64)
    n = len(X) - window
    betas, norms = [], []
    for i in range(n):
        xs, ys = X[i : i + window], Y[i : i + window]
        b = ols(ys, xs)
        betas.append(b)
        norms.append(normalization(ys, xs, b, window))
    return np.stack(betas), np.stack(norms)


def ex_ante_returns(weights: np.ndarray, etf: np.ndarray, rf: np.ndarray) -> np.ndarray:
    """weights (T, A, S), etf (T, A), rf (T,) -> (T, S): rf*(1-sum w) + sum(etf*w)."""
    rf_w = 1.0 - weights.sum(axis=1)  # (T, S)
    return rf_w * rf[:, None] + np.einsum("ta,tas->ts", etf, weights)


def turnover(weights: np.ndarray) -> np.ndarray:
    """Annualised turnover per strategy (Autoencoder_encapsulate.py:210-224)."""
    T = weights.shape[0]
    tot = np.abs(np.diff(weights, axis=0)).sum(axis=(0, 1))
    return tot / (T / 12.0)


@dataclass
class LinearCloneBenchmark:
    """Rolling-window OLS linear clone (the reference's benchmark).

    For each out-of-sample month t the clone holds ``w_t = beta_t * norm_t`` in the factor ETFs
    (``beta_t`` from an OLS of HF returns on ETF returns over the previous ``window`` months,
    no intercept, as in Autoencoder_encapsulate.py:148-156) and ``1 - sum(w_t)`` in the
    risk-free asset.  Ex-post returns add the transaction-cost / price-impact penalty.
    """

    window: int = 24

    def fit(self, factor_etf: pd.DataFrame, hfd: pd.DataFrame, rf: pd.DataFrame):
        X = factor_etf.to_numpy(np.float64)
        Y = hfd.to_numpy(np.float64)
        betas, norms = rolling_ols(Y, X, self.window)  # (n, A, S)
        self.weights_ = betas * norms[:, None, :]
        # weights estimated on [i, i+w) are applied to month i+w
        idx = factor_etf.index[self.window :]
        n = len(idx)
        W = self.weights_[:n]
        self.ante_ = pd.DataFrame(
            ex_ante_returns(W, X[self.window :], rf.to_numpy(np.float64).reshape(-1)[self.window :]),
            index=idx, columns=hfd.columns,
        )
        self.W_ = W
        self.etf_ = factor_etf
        return self

    def post(self) -> pd.DataFrame:
        W = self.W_
        etf = self.etf_.to_numpy(np.float64)
        # penalty at month i uses cov of the window preceding the rebalance (same convention as AE.post)
        pen = transaction_penalty(W, etf, self.window)
        post = self.ante_.to_numpy().copy()
        k = min(post.shape[0] - 1, pen.shape[0])
        post[1 : 1 + k] += pen[:k]
        return pd.DataFrame(post, index=self.ante_.index, columns=self.ante_.columns)

    def turnover(self) -> np.ndarray:
        return turnover(self.W_)
