"""Shared pytest setup.

* ``gpu`` marker: tests that need a real MI355X (run with ``-m gpu`` on the GPU box).
* ``data`` fixture: the reference dataset (cleaned_data + raw data/) if present; tests that
  need it skip when it is absent (e.g. on the GPU box, where only the repo snapshot exists).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import hfrep  # noqa: E402  (registers the package)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (gfx950) and the native kernel library")
    config.addinivalue_line("markers", "slow: long-running test")


def _first_root_with(sub):
    from hfrep.data.io import data_root as _dr

    for r in (os.environ.get("HFREP_DATA_ROOT"), "/root/reference", _dr()):
        if r and os.path.isdir(os.path.join(r, sub)):
            return r
    return None


@pytest.fixture(scope="session")
def data_root():
    """A root with the RAW reference data (data/) and cleaned_data/."""
    r = _first_root_with("data")
    if r is None or not os.path.isdir(os.path.join(r, "cleaned_data")):
        pytest.skip("reference dataset not available")
    return r


@pytest.fixture(scope="session")
def cleaned():
    """The cleaned panel only (cleaned_data/: also staged under assets/ for GPU runs)."""
    r = _first_root_with("cleaned_data")
    if r is None:
        pytest.skip("cleaned reference data not available")
    from hfrep.data.io import load_cleaned

    return load_cleaned(r)


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hfrep.ops import _native

    _native.native()  # must load on a GPU box
    return torch.device("cuda")


@pytest.fixture(scope="session")
def daily():
    """The daily ETF excess-return matrix (staged CSV on GPU boxes, else built from the raw data)."""
    r = _first_root_with("cleaned_data")
    if r is None:
        pytest.skip("reference dataset not available")
    staged = os.path.exists(os.path.join(r, "cleaned_data", "factor_etf_daily.csv"))
    if not staged and not os.path.isdir(os.path.join(r, "data")):
        r = _first_root_with("data")
        if r is None:
            pytest.skip("daily ETF prices not available")
    from hfrep.data.io import load_daily_etf

    return load_daily_etf(r)[0]
