"""Performance analytics and spanning tests (reference notebook cells 17-27).

numpy/scipy ports of the analytics the reference runs in ``autoencoder_v4.ipynb``:

* Omega ratio / curve, annualised Sharpe, historical VaR / CVaR, certainty equivalent (CEQ),
  Fama-French OLS alpha (cell 23, raw JSON line ~695-770);
* the Gibbons-Ross-Shanken F-test (R ``grstest``, cell 19, line ~510) and the
  Huberman-Kandel spanning test (R ``hktest``, cell 17, line ~401) — originally R code called
  through rpy2; here pure numpy with ``scipy.stats.f`` tails;
* :func:`data_analysis` (15-column statistics table) and :func:`res_sort` (best latent size
  per strategy by a chosen column).

Parity target: the notebook's published ``hfd_res`` table (cell 30) is reproduced from the
cleaned data (tests/test_finance.py).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
from scipy import stats

from .replication import ols


def omega_ratio(df, threshold=0.0) -> float:
    daily_threshold = (threshold + 1) ** np.sqrt(1 / 252) - 1  # (sic) as the reference
    r = np.asarray(df, dtype=np.float64)
    ex = r - daily_threshold
    return float(np.sum(ex[ex > 0]) / (-np.sum(ex[ex < 0])))


def omega_curve(df, thresholds=np.linspace(0, 0.2, 50)):
    return [omega_ratio(df, t) for t in thresholds]


def annualized_sharpe_ratio(ret, rf=0) -> float:
    ret = np.asarray(ret, dtype=np.float64)
    rf = np.asarray(rf, dtype=np.float64)
    return float((np.mean(ret) - np.mean(rf)) / np.std(ret) * np.sqrt(12))


def ols_alpha(ret, X) -> float:
    return float(ols(np.asarray(ret, dtype=np.float64), np.asarray(X, dtype=np.float64), add_const=True)[0])


def historical_var(returns, alpha=5):
    if isinstance(returns, pd.Series):
        return float(np.percentile(returns, alpha))
    if isinstance(returns, pd.DataFrame):
        return returns.aggregate(historical_var, alpha=alpha)
    raise TypeError("Expected returns to be dataframe or series")


def historical_cvar(returns, alpha=5):
    if isinstance(returns, pd.Series):
        below = returns <= historical_var(returns, alpha=alpha)
        return float(returns[below].mean())
    if isinstance(returns, pd.DataFrame):
        return returns.aggregate(historical_cvar, alpha=alpha)
    raise TypeError("Expected returns to be dataframe or series")


def ceq(ret, rf, gamma=2) -> float:
    """Certainty-equivalent return; rf and ret are aligned by index (DataFrame.join)."""
    assert gamma != 1
    assert len(ret) == len(rf)
    df = pd.DataFrame(rf).join(ret)
    mid = np.power((1 + df.iloc[:, 1]) / (1 + df.iloc[:, 0]), 1 - gamma)
    return float(np.log(np.mean(mid)) / ((1 - gamma) / 12))


def grs_test(ret_mat, factor_mat):
    """Gibbons-Ross-Shanken test: returns array [[F], [p]] (R grstest semantics)."""
    R = np.asarray(ret_mat, dtype=np.float64)
    if R.ndim == 1:
        R = R[:, None]
    Fm = np.asarray(factor_mat, dtype=np.float64)
    if Fm.ndim == 1:
        Fm = Fm[:, None]
    T, N = R.shape
    K = Fm.shape[1]
    D = np.column_stack([np.ones(T), Fm])
    B = np.linalg.solve(D.T @ D, D.T @ R)  # (K+1, N)
    E = R - D @ B
    sigma = E.T @ E / (T - K - 1)
    alpha = B[0][:, None]
    fmean = Fm.mean(axis=0)[None, :]
    omega = (Fm - fmean).T @ (Fm - fmean) / (T - 1)
    tem1 = alpha.T @ np.linalg.solve(sigma, alpha)
    tem2 = 1 + fmean @ np.linalg.solve(omega, fmean.T)
    F = (T / N) * ((T - N - K) / (T - K - 1)) * (tem1 / tem2)
    F = float(F.squeeze())
    p = float(stats.f.sf(F, N, T - N - K))
    return np.array([[F], [p]])


def hk_test(rt, rb):
    """Huberman-Kandel mean-variance spanning test: [[F], [p]] (R hktest semantics)."""
    rt = np.asarray(rt, dtype=np.float64)
    if rt.ndim == 1:
        rt = rt[:, None]
    rb = np.asarray(rb, dtype=np.float64)
    if rb.ndim == 1:
        rb = rb[:, None]
    Tn, N = rt.shape
    K = rb.shape[1]
    A = np.vstack([np.hstack([[1.0], np.zeros(K)]), np.hstack([[0.0], -np.ones(K)])])
    C = np.vstack([np.zeros((1, N)), -np.ones((1, N))])
    X = np.column_stack([np.ones(Tn), rb])
    B = np.linalg.lstsq(X, rt, rcond=None)[0]
    Theta = A @ B - C
    e = rt - X @ B
    Sigma = np.atleast_2d(np.cov(e, rowvar=False))
    H = Theta @ np.linalg.inv(Sigma) @ Theta.T
    mu1 = rb.mean(axis=0)[None, :]
    V11i = np.linalg.pinv(np.atleast_2d(np.cov(rb, rowvar=False)))
    a1 = float(mu1 @ V11i @ mu1.T)
    b1 = float(np.sum(V11i @ mu1.T))
    c1 = float(np.sum(V11i))
    G = np.array([[1 + a1, b1], [b1, c1]])
    lam = np.linalg.eigvals(H @ np.linalg.inv(G))
    Ui = float(np.real(np.prod(1 + lam)))
    if N == 1:
        F = (Tn - K - 1) * (Ui - 1) / 2
        p = stats.f.sf(F, 2, Tn - K - 1)
    else:
        F = (Tn - K - N) * (np.sqrt(Ui) - 1) / N
        p = stats.f.sf(F, 2 * N, 2 * (Tn - N - K))
    return np.array([[float(F)], [float(p)]])


COLUMNS_REAL = ["Skewness", "Kurtosis", "Omega_ratio(0%)", "Omega_ratio(10%)", "cVaR(95%)", "CEQ Gamma=2",
                "CEQ Gamma=5", "CEQ Gamma=10", "Annualized_Sharpe", "FF3F_alpha", "FF5F_alpha", "GRS_testF",
                "HK_testF", "GRS_test_pval", "HK_test_pval"]


def data_analysis(df: pd.DataFrame, name, rf=None, start=None, end=None, span=None, real_data=True,
                  three_factor: pd.DataFrame | None = None, five_factor: pd.DataFrame | None = None) -> pd.DataFrame:
    """15-column statistics table per strategy column of ``df`` (notebook ``data_analysis``).

    ``three_factor``/``five_factor`` are the monthly FF frames (:func:`hfrep.data.cleaning.fama_french_monthly`);
    they are only needed when ``real_data`` is true.
    """
    if rf is None:
        rf = pd.DataFrame(np.zeros(len(df)), index=df.index)
    rows = []
    for strat in df.columns:
        s = df[strat]
        row = {
            "Skewness": s.skew(),
            "Kurtosis": s.kurt(),
            "Omega_ratio(0%)": omega_ratio(s, 0),
            "Omega_ratio(10%)": omega_ratio(s, 0.1),
            "cVaR(95%)": historical_cvar(s),
            "CEQ Gamma=2": ceq(s, rf, 2),
            "CEQ Gamma=5": ceq(s, rf, 5),
            "CEQ Gamma=10": ceq(s, rf, 10),
            "Annualized_Sharpe": annualized_sharpe_ratio(s, rf),
        }
        if real_data:
            ff3 = three_factor.loc[start:end] if (start and end) else three_factor
            ff5 = five_factor.loc[start:end] if (start and end) else five_factor
            row["FF3F_alpha"] = ols_alpha(s, ff3)
            row["FF5F_alpha"] = ols_alpha(s, ff5)
            if span is not None:
                base = np.asarray(span.loc[start:end] if (start and end) else span)
            else:
                base = np.asarray(df.loc[:, df.columns != strat])
            hk = hk_test(np.asarray(s), base)
            grs = grs_test(np.asarray(s), base)
            row["GRS_testF"] = grs[0][0]
            row["HK_testF"] = hk[0][0]
            row["GRS_test_pval"] = round(grs[1][0], 6)
            row["HK_test_pval"] = round(hk[1][0], 6)
        rows.append(row)
    cols = COLUMNS_REAL if real_data else COLUMNS_REAL[:9]
    out = pd.DataFrame(rows)[cols]
    out.index = list(name)
    return out


def res_sort(post_res, item="Annualized_Sharpe"):
    """Best table row per strategy across latent sizes (notebook cell 27)."""
    best, names, idxs = [], [], []
    for si in range(len(post_res[0].index)):
        vals = [df[item].iloc[si] for df in post_res]
        bi = int(np.argmax(vals))
        best.append(post_res[bi].iloc[si])
        names.append(f"{post_res[0].index[si]} latent {bi + 1}")
        idxs.append(bi)
    return pd.DataFrame(best, index=names), idxs
