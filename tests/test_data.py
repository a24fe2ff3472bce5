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
