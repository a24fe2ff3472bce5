"""MinMax scaling (sklearn ``MinMaxScaler`` semantics) for numpy and torch arrays.

The reference scales with sklearn's MinMaxScaler in three places: the GAN scripts fit it on the
whole 1994-2022 panel before sampling windows (GAN/GAN.py:82-86, look-ahead kept for parity,
SURVEY Q11); ``AE.__init__`` fits on x_train (Autoencoder_encapsulate.py:65); the notebook fits a
36-column scaler to invert generated windows (autoencoder_v4.ipynb:1370).  ``fit_range`` lets a
caller restrict the fit rows (e.g. train months only) without changing the transform.
"""
from __future__ import annotations

import numpy as np


class MinMaxScaler:
    def __init__(self, feature_range=(0.0, 1.0)):
        self.feature_range = feature_range

    def fit(self, X, fit_range: slice | None = None):
        X = np.asarray(X, dtype=np.float64)
        if fit_range is not None:
            X = X[fit_range]
        self.data_min_ = np.nanmin(X, axis=0)
        self.data_max_ = np.nanmax(X, axis=0)
        rng = self.data_max_ - self.data_min_
        rng = np.where(rng == 0.0, 1.0, rng)  # sklearn handles constant features this way
        lo, hi = self.feature_range
        self.scale_ = (hi - lo) / rng
        self.min_ = lo - self.data_min_ * self.scale_
        return self

    def transform(self, X):
        return np.asarray(X, dtype=np.float64) * self.scale_ + self.min_

    def fit_transform(self, X, fit_range: slice | None = None):
        return self.fit(X, fit_range).transform(X)

    def inverse_transform(self, X):
        return (np.asarray(X, dtype=np.float64) - self.min_) / self.scale_

    def state(self) -> dict:
        return {"data_min": self.data_min_.tolist(), "data_max": self.data_max_.tolist(),
                "feature_range": list(self.feature_range)}

    @classmethod
    def from_state(cls, st: dict) -> "MinMaxScaler":
        s = cls(tuple(st["feature_range"]))
        s.data_min_ = np.asarray(st["data_min"], dtype=np.float64)
        s.data_max_ = np.asarray(st["data_max"], dtype=np.float64)
        rng = np.where(s.data_max_ - s.data_min_ == 0, 1.0, s.data_max_ - s.data_min_)
        lo, hi = s.feature_range
        s.scale_ = (hi - lo) / rng
        s.min_ = lo - s.data_min_ * s.scale_
        return s
