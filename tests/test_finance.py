"""Replication math, analytics and spanning tests.

The notebook's published HF-index statistics table (autoencoder_v4.ipynb cell 30, ``hfd_res``) depends
only on the cleaned data, so the numpy/scipy ports of the R GRS/HK tests and the analytics must
reproduce it (fixture extracted from the notebook output: tests/fixtures/hfd_res_golden.json).
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

from hfrep.data.cleaning import fama_french_monthly
from hfrep.finance import analytics as A
from hfrep.finance import replication as Rp

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "hfd_res_golden.json")


def test_hfd_res_table_matches_notebook(data_root, cleaned):
    ff3 = fama_french_monthly(f"{data_root}/data/F-F_Research_Data_Factors_daily.CSV")
    ff5 = fama_french_monthly(f"{data_root}/data/F-F_Research_Data_5_Factors_2x3_daily.CSV")
    hfd, etf, rf = cleaned["hfd"], cleaned["factor_etf_data"], cleaned["rf"]
    res = A.data_analysis(hfd[-144:], cleaned["hfd_fullname"].values(), rf=rf[-144:], span=etf, real_data=True,
                          start="2010-05-31", end="2022-04-30", three_factor=ff3, five_factor=ff5)
    gold = json.load(open(FIX))["table"]
    for name in res.index:
        for col in res.columns:
            a, b = res.loc[name, col], gold[name.strip()][col]
            # the notebook prints 6 significant digits
            assert abs(a - b) <= 5e-6 * max(1.0, abs(b)) + 1.2e-6, (name, col, a, b)


def _loop_ex_post(ex_ante, window, strat_weight, etf):
    """Direct transcription of the per-date loop semantics (helper.py:112-131) for cross-checking."""
    out = []
    for s in range(len(ex_ante.columns)):
        pen = []
        for i in range(1, len(etf) - window):
            cov = etf.iloc[i:i + window].cov().to_numpy()
            new, old = strat_weight[s].iloc[i].to_numpy(), strat_weight[s].iloc[i - 1].to_numpy()
            pen.append((Rp.transaction_cost(old, new, cov) + Rp.price_impact(old, new, cov)).sum())
        col = [ex_ante.iloc[0, s]] + [ex_ante.iloc[i, s] + pen[i - 1] for i in range(1, len(ex_ante))]
        out.append(col)
    return np.array(out).T


def test_ex_post_vectorised_equals_loop():
    rs = np.random.RandomState(0)
    T, A_, S, w = 30, 5, 3, 6
    etf = pd.DataFrame(rs.randn(T + w, A_) * 0.02)
    ante = pd.DataFrame(rs.randn(T, S) * 0.01)
    frames = [pd.DataFrame(rs.randn(A_, S)) for _ in range(T)]
    sw = Rp.reshape_cab(frames)
    assert len(sw) == S and sw[0].shape == (T, A_)
    got = Rp.ex_post_return(ante, w, sw, etf).to_numpy()
    np.testing.assert_allclose(got, _loop_ex_post(ante, w, sw, etf), rtol=1e-12, atol=1e-15)


def test_normalization_and_costs():
    rs = np.random.RandomState(1)
    X, Y = rs.randn(24, 4), rs.randn(24, 3)
    beta = np.linalg.lstsq(X, Y, rcond=None)[0]
    n = Rp.normalization(Y, X, beta, 24)
    np.testing.assert_allclose(n, Y.std(0, ddof=1) / (X @ beta).std(0, ddof=1))
    cov = np.cov(rs.randn(24, 4), rowvar=False)
    old, new = rs.randn(4), rs.randn(4)
    sk = np.sqrt(np.diag(cov)) * 0.05
    np.testing.assert_allclose(Rp.transaction_cost(old, new, cov), 0.5 * (old - new) ** 2 * sk)
    d = old - new
    np.testing.assert_allclose(Rp.price_impact(old, new, cov), 0.5 * new * sk * d - old * sk * d - 0.5 * d ** 2 * sk)


def test_factor_hf_split():
    arr = np.arange(2 * 3 * 5, dtype=float).reshape(2, 3, 5)
    f, h = Rp.factor_hf_split(arr, 2)
    assert f.shape == (6, 2) and h.shape == (6, 3)
    f3, h3 = Rp.factor_hf_split(arr, 2, reshape=False)
    np.testing.assert_array_equal(f3, arr[:, :, :2])


def test_linear_clone_benchmark(cleaned):
    hfd, etf, rf = cleaned["hfd"], cleaned["factor_etf_data"], cleaned["rf"]
    bm = Rp.LinearCloneBenchmark(window=24).fit(etf, hfd, rf)
    assert bm.ante_.shape == (len(etf) - 24, 13)
    post = bm.post()
    assert post.shape == bm.ante_.shape and np.isfinite(post.to_numpy()).all()
    # the out-of-sample rolling clone tracks its target: clearly positive correlation (0.44 here)
    corr = np.corrcoef(bm.ante_.iloc[:, 0], hfd.iloc[24:, 0])[0, 1]
    assert corr > 0.3
    assert (bm.turnover() > 0).all()


def test_omega_sharpe_ceq_cvar():
    rs = np.random.RandomState(2)
    idx = pd.date_range("2010-01-31", periods=60, freq="ME")
    r = pd.Series(rs.randn(60) * 0.02 + 0.005, index=idx, name="s")
    rf = pd.DataFrame({"RF": np.full(60, 0.001)}, index=idx)
    ex = r.to_numpy() - ((1 + 0.0) ** np.sqrt(1 / 252) - 1)
    assert np.isclose(A.omega_ratio(r, 0), ex[ex > 0].sum() / -ex[ex < 0].sum())
    assert np.isclose(A.annualized_sharpe_ratio(r, rf), (r.mean() - 0.001) / r.std(ddof=0) * np.sqrt(12))
    g = 5
    assert np.isclose(A.ceq(r, rf, g), np.log(np.mean(((1 + r) / (1 + 0.001)) ** (1 - g))) / ((1 - g) / 12))
    var = np.percentile(r, 5)
    assert np.isclose(A.historical_cvar(r), r[r <= var].mean())


def test_res_sort():
    a = pd.DataFrame({"Annualized_Sharpe": [0.1, 0.9]}, index=["x", "y"])
    b = pd.DataFrame({"Annualized_Sharpe": [0.5, 0.2]}, index=["x", "y"])
    best, idx = A.res_sort([a, b])
    assert idx == [1, 0] and list(best.index) == ["x latent 2", "y latent 1"]


def test_latent_sweep_and_augmentation(cleaned):
    """Notebook experiment driver (P31/P32): AE per latent size -> metrics, clone Sharpes, turnover,
    best latent per strategy; generated windows -> extra training rows in return units."""
    from hfrep.finance.experiment import generated_augmentation, latent_sweep

    res = latent_sweep(cleaned, latents=[1, 3])
    assert list(res.metrics.index) == [1, 3]
    assert (res.metrics["IS_r2"] <= 1).all() and np.isfinite(res.metrics.to_numpy()).all()
    assert res.sharpe_post.shape == (2, cleaned["hfd"].shape[1])
    assert np.isfinite(res.sharpe_post.to_numpy()).all() and (res.turnover.to_numpy() >= 0).all()
    assert set(res.best["latent"]) <= {1, 3} and len(res.best) == cleaned["hfd"].shape[1]

    gen = np.random.RandomState(0).rand(4, 10, 36).astype(np.float32)
    x, y = generated_augmentation(gen, cleaned)
    assert x.shape == (40, 22) and y.shape == (40, 13)
    panel = cleaned["factor_etf_data"].join(cleaned["hfd"]).join(cleaned["rf"]).to_numpy()
    lo, hi = panel.min(0), panel.max(0)
    assert (x >= lo[:22] - 1e-9).all() and (x <= hi[:22] + 1e-9).all()
    aug = latent_sweep(cleaned, latents=[2], x_extra=x, y_extra=y)
    assert np.isfinite(aug.metrics.to_numpy()).all()


def test_latent_sweep_many_equals_single_sweeps(cleaned):
    """latent_sweep_many (every (seed, latent) AE built first and trained together -- one launch on a GPU)
    gives each seed exactly the sweep latent_sweep gives it alone (here on the CPU, fits one by one)."""
    from hfrep.finance.experiment import generated_augmentation, latent_sweep, latent_sweep_many

    gen = np.random.RandomState(1).rand(3, 10, 36).astype(np.float32)
    x, y = generated_augmentation(gen, cleaned)
    many = latent_sweep_many(cleaned, seeds=[123, 7], latents=[2], x_extras=[None, x], y_extras=[None, y])
    one = [latent_sweep(cleaned, latents=[2], seed=123), latent_sweep(cleaned, latents=[2], seed=7, x_extra=x, y_extra=y)]
    for a, b in zip(many, one):
        pd.testing.assert_frame_equal(a.metrics, b.metrics)
        pd.testing.assert_frame_equal(a.sharpe_post, b.sharpe_post)
