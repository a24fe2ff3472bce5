"""Data pipeline goldens: regenerate cleaned_data from raw data/."""
import numpy as np
import pytest

from hfrep.data import cleaning
from hfrep.data.io import safe_pickle_load
from hfrep.data.scaler import MinMaxScaler
from hfrep.data.windows import random_sampling


def test_rf_hfd_reproduce(data_root, cleaned):
    res = cleaning.build_all(f"{data_root}/data")
    for k in ("rf", "hfd"):
        a, b = res[k], cleaned[k]
        assert a.shape == b.shape and (a.index == b.index).all()
        np.testing.assert_allclose(a[b.columns].values, b.values, atol=1e-14, rtol=0)


def test_etf_reproducible_columns(data_root, cleaned):
    res = cleaning.build_all(f"{data_root}/data")
    a, b = res["factor_etf_data"], cleaned["factor_etf_data"]
    assert a.shape == b.shape
    cols = cleaning.REPRODUCIBLE_ETF
    np.testing.assert_allclose(a[cols].values, b[cols].values, atol=1e-14, rtol=0)


def test_safe_pickle_names_and_array(data_root):
    d = safe_pickle_load(f"{data_root}/cleaned_data/hfd_fullname.pkl")
    assert d["HEDG"] == "Hedge Fund Index " and len(d) == 13
    arr = safe_pickle_load(f"{data_root}/GAN/generated_data2022-07-09.pkl")
    assert arr.shape == (10, 168, 36) and arr.dtype == np.float32


def test_safe_pickle_refuses_code(tmp_path):
    import pickle

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    p = tmp_path / "evil.pkl"
    p.write_bytes(pickle.dumps(Evil()))
    with pytest.raises(ValueError):
        safe_pickle_load(str(p))


def test_safe_pickle_roundtrip(tmp_path):
    import pickle

    obj = {"a": [1, 2.5, None, True], "b": ("x", b"yz"), "arr": np.arange(12, dtype=np.float64).reshape(3, 4)}
    p = tmp_path / "ok.pkl"
    p.write_bytes(pickle.dumps(obj, protocol=4))
    out = safe_pickle_load(str(p))
    assert out["a"] == obj["a"] and out["b"] == obj["b"]
    np.testing.assert_array_equal(out["arr"], obj["arr"])


def test_minmax_scaler_matches_sklearn():
    from sklearn.preprocessing import MinMaxScaler as SK

    x = np.random.RandomState(0).randn(100, 7)
    a, b = MinMaxScaler().fit(x), SK().fit(x)
    np.testing.assert_allclose(a.transform(x), b.transform(x), atol=1e-15)
    np.testing.assert_allclose(a.inverse_transform(a.transform(x)), x, atol=1e-12)


def test_random_sampling_shapes():
    data = np.arange(337 * 3, dtype=np.float64).reshape(337, 3)
    w = random_sampling(data, 50, 48, seed=1)
    assert w.shape == (50, 48, 3)
    # every window is a contiguous slice of the panel
    starts = w[:, 0, 0] / 3
    for s, win in zip(starts.astype(int), w):
        np.testing.assert_array_equal(win, data[s:s + 48])


def test_daily_etf_matrix_aggregates_to_monthly_panel(data_root):
    """BASELINE config 2's daily ETF excess-return matrix: summed over each month (price relatives) and
    net of the monthly rf it reproduces cleaned_data/factor_etf_data.csv for the 14 columns the shipped
    raw prices reproduce, to float rounding."""
    import os

    import numpy as np

    from hfrep.data.cleaning import REPRODUCIBLE_ETF, aggregate_daily_to_monthly, build_factor_etf_daily, build_rf
    from hfrep.data.io import load_cleaned

    ff = os.path.join(data_root, "data", "F-F_Research_Data_Factors_daily.CSV")
    ex, rfd = build_factor_etf_daily(os.path.join(data_root, "data", "ETF_data.csv"), ff, tickers=REPRODUCIBLE_ETF)
    assert list(ex.columns) == REPRODUCIBLE_ETF and not ex.isna().any().any()
    assert str(ex.index[0].date()) == "1994-04-01" and str(ex.index[-1].date()) == "2022-04-29"
    assert 7000 < len(ex) < 7400 and ex.index.is_monotonic_increasing
    assert (rfd >= 0).all() and rfd.max() < 1e-3
    m = aggregate_daily_to_monthly(ex, rfd, build_rf(ff))
    ref = load_cleaned(data_root)["factor_etf_data"]
    d = (m[REPRODUCIBLE_ETF].to_numpy() - ref[REPRODUCIBLE_ETF].to_numpy())
    assert m.shape[0] == ref.shape[0] == 337 and np.abs(d).max() < 1e-13


def test_daily_factor_study_cpu_smoke():
    """The daily study's pipeline on a small synthetic daily panel (CPU engine): one row per latent with
    reference-style metrics and the strided OOS windows."""
    import numpy as np
    import pandas as pd

    from hfrep.finance.experiment import daily_factor_study

    rs = np.random.RandomState(0)
    f = rs.randn(300, 3) * 0.01
    x = f @ rs.randn(3, 22) * 0.5 + rs.randn(300, 22) * 0.001
    daily = pd.DataFrame(x, index=pd.bdate_range("2000-01-03", periods=300))
    st = daily_factor_study(daily, latents=[1, 3], oos_stride=21)
    assert list(st["latent"]) == [1, 3] and (st["train_rows"] == 150).all()
    assert np.isfinite(st[["IS_r2", "OOS_r2", "IS_RMSE", "OOS_RMSE"]].to_numpy()).all()
    assert st["IS_r2"].iloc[1] > st["IS_r2"].iloc[0]
