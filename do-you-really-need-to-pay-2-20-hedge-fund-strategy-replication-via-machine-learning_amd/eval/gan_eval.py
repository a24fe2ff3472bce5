"""Distribution-similarity metrics for generated return windows (reference GAN/GAN_eval.py).

API-compatible with ``GAN_eval(real, fake, dataset, subplot_title, model_name)``
(GAN/GAN_eval.py:15-458): every metric takes optional ``real/fake/dataset`` overrides and the
same keyword defaults, and :meth:`run_all` returns a DataFrame (metric x model_name).

Differences by design:

* ``statsmodels`` is not a dependency: ``acf`` (unadjusted, demeaned; statsmodels default),
  ``ECDF`` and OLS are implemented here in numpy.
* :meth:`R2_relative_error` keeps the reference quirk (Q8: it compares ``real`` with ``real``
  and is therefore always 0) unless ``fixed=True``, which uses ``fake`` for the second term.
* :meth:`wasserstein` is the W-dist parity metric of the north star (GAN/GAN_eval.py:309-326).
* ``kl_div``/``js_div`` keep the reference label layout (Q9).
* ``GANEval(..., device='cuda')`` (keyword only) runs the large-N reductions of FID and the MMDs
  on the GPU: the (N*T, F) covariances through the native fp32 weight-gradient kernel (X^T X of the
  centred samples, one fixed-order reduction: deterministic) and the sample means on the device;
  the F x F matrix square root and the (T x T) Gram matrices stay on the CPU.  It is an fp32 path
  (relative difference ~1e-6 against the fp64 CPU path, tests/test_kernels_gpu.py); the default
  CPU path is numerically identical to the reference formulas.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
from scipy.linalg import sqrtm
from scipy.special import rel_entr
from scipy.stats import kstest, wasserstein_distance
from sklearn import metrics
from sklearn.metrics import r2_score
from sklearn.naive_bayes import GaussianNB

from ..finance.replication import ols


def acf(x, nlags: int = 17) -> np.ndarray:
    """Sample autocorrelation, lags 0..nlags (statsmodels ``acf`` defaults: demeaned, /n)."""
    x = np.asarray(x, dtype=np.float64)
    x = x - x.mean()
    n = len(x)
    denom = np.dot(x, x)
    out = np.empty(nlags + 1)
    for k in range(nlags + 1):
        out[k] = np.dot(x[: n - k], x[k:]) / denom if k < n else np.nan
    return out


def acf_batch(x: np.ndarray, nlags: int = 17) -> np.ndarray:
    """Vectorised :func:`acf` over the last-but-one axis: x (..., T) -> (..., nlags+1)."""
    x = np.asarray(x, dtype=np.float64)
    x = x - x.mean(axis=-1, keepdims=True)
    T = x.shape[-1]
    denom = np.sum(x * x, axis=-1)
    out = np.empty(x.shape[:-1] + (nlags + 1,))
    for k in range(nlags + 1):
        out[..., k] = np.sum(x[..., : T - k] * x[..., k:], axis=-1) / denom if k < T else np.nan
    return out


class ECDF:
    """Right-continuous empirical CDF (statsmodels ``ECDF`` semantics)."""

    def __init__(self, x):
        self.x = np.sort(np.asarray(x, dtype=np.float64))
        self.n = len(self.x)

    def __call__(self, t):
        return np.searchsorted(self.x, t, side="right") / self.n


def _device_moments(a: np.ndarray, device):
    """(mean, covariance (ddof 1)) of the rows of a 2-D array on the GPU: fp32, the covariance as
    X^T X of the centred rows through the native weight-gradient kernel (csrc/gemm.hip wgrad)."""
    import torch

    from ..ops import functional as Fn

    x = torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=device)
    mu = x.double().mean(dim=0)
    xc = (x - mu.to(torch.float32)).contiguous()
    cov = torch.zeros(x.shape[1], x.shape[1], dtype=torch.float32, device=device)
    Fn.linear_wgrad_(xc, xc, cov, None)
    return mu.cpu().numpy(), cov.double().cpu().numpy() / max(x.shape[0] - 1, 1)


class GANEval:
    def __init__(self, real, fake, dataset, subplot_title, model_name, *, device=None):
        assert isinstance(real, np.ndarray)
        assert isinstance(fake, np.ndarray)
        assert isinstance(dataset, np.ndarray)
        assert isinstance(subplot_title, list)
        assert isinstance(model_name, list)
        assert real.ndim == fake.ndim
        self.real = real
        self.fake = fake
        self.dataset = dataset
        self.subplot_title = subplot_title
        self.model_name = model_name
        self.device = device if device is None or str(device) != "cpu" else None

    # -- helpers -------------------------------------------------------------------------
    def _args(self, real, fake, dataset):
        return (self.real if real is None else real, self.fake if fake is None else fake,
                self.dataset if dataset is None else dataset)

    @staticmethod
    def _flat(a):
        return a.reshape(a.shape[0] * a.shape[1], a.shape[2]) if a.ndim == 3 else a

    # -- metrics ---------------------------------------------------------------------------
    def FID(self, real=None, fake=None, dataset=None):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape
        real, fake = self._flat(real), self._flat(fake)
        if self.device is not None:
            (mu1, s1), (mu2, s2) = _device_moments(real, self.device), _device_moments(fake, self.device)
        else:
            mu1, s1 = real.mean(axis=0), np.cov(real, rowvar=False)
            mu2, s2 = fake.mean(axis=0), np.cov(fake, rowvar=False)
        ssdiff = np.sum((mu1 - mu2) ** 2.0)
        covmean = sqrtm(s1.dot(s2))
        if np.iscomplexobj(covmean):
            covmean = covmean.real
        return float(ssdiff + np.trace(s1 + s2 - 2.0 * covmean))

    def _mean_over_samples(self, real, fake):
        if real.ndim > 2 or fake.ndim > 2:
            if self.device is not None:
                import torch

                return tuple(torch.as_tensor(a, device=self.device).double().mean(dim=0).cpu().numpy() for a in (real, fake))
            return np.mean(real, axis=0), np.mean(fake, axis=0)
        return real, fake

    def linear_MMD(self, real=None, fake=None, dataset=None):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape
        real, fake = self._mean_over_samples(real, fake)
        return float(np.dot(real, real.T).mean() + np.dot(fake, fake.T).mean() - 2 * np.dot(real, fake.T).mean())

    def gaussian_MMD(self, real=None, fake=None, dataset=None, gamma=1.0):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape
        real, fake = self._mean_over_samples(real, fake)
        k = metrics.pairwise.rbf_kernel
        return float(k(real, real, gamma).mean() + k(fake, fake, gamma).mean() - 2 * k(real, fake, gamma).mean())

    def poly_MMD(self, real=None, fake=None, dataset=None, degree=2, gamma=1, coef0=0):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape
        real, fake = self._mean_over_samples(real, fake)
        k = metrics.pairwise.polynomial_kernel
        return float(k(real, real, degree, gamma, coef0).mean() + k(fake, fake, degree, gamma, coef0).mean()
                     - 2 * k(real, fake, degree, gamma, coef0).mean())

    def _nb_probs(self, real, fake, dataset):
        assert real.ndim in (2, 3) and dataset.ndim == 3 and real.shape == fake.shape
        # one row per (sample, feature) series window; labels repeat feature ids (Q9 layout)
        Td = np.transpose(dataset, (0, 2, 1)).reshape(-1, dataset.shape[1])
        if real.ndim > 2:
            Tr = np.transpose(real, (0, 2, 1)).reshape(-1, real.shape[1])
            Tf = np.transpose(fake, (0, 2, 1)).reshape(-1, fake.shape[1])
        else:
            Tr, Tf = real.T, fake.T
        gnb = GaussianNB()
        gnb.fit(Td, np.repeat(np.arange(real.shape[2] if real.ndim == 3 else real.shape[1]), dataset.shape[0]))
        return gnb.predict_proba(Tr), gnb.predict_proba(Tf)

    def kl_div(self, real=None, fake=None, dataset=None, div_only=True):
        real, fake, dataset = self._args(real, fake, dataset)
        rp, fp = self._nb_probs(real, fake, dataset)
        res = rel_entr(fp, rp).sum(axis=1)
        if div_only:
            return float(np.mean(res))
        return float(np.mean(res)), float(np.mean(np.sqrt(res)))

    def js_div(self, real=None, fake=None, dataset=None, div_only=True):
        real, fake, dataset = self._args(real, fake, dataset)
        rp, fp = self._nb_probs(real, fake, dataset)
        m = 0.5 * (fp + rp)
        res = 0.5 * rel_entr(fp, m).sum(axis=1) + 0.5 * rel_entr(rp, m).sum(axis=1)
        if div_only:
            return float(np.mean(res))
        return float(np.mean(res)), float(np.mean(np.sqrt(res)))

    def Inception_score(self, real=None, fake=None, dataset=None):
        real, fake, dataset = self._args(real, fake, dataset)
        kld, _ = self.kl_div(real, fake, dataset, div_only=False)
        return float(np.exp(np.mean(kld)))

    def ks_test(self, real=None, fake=None, dataset=None, group=True, p_val_only=True):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape and real.ndim in (2, 3)
        real, fake = self._flat(real), self._flat(fake)
        res = []
        for i in range(real.shape[1]):
            st, pv = kstest(real[:, i], fake[:, i])
            res.append([st, pv])
        if group:
            return float(np.mean(res, axis=0)[1]) if p_val_only else np.mean(res, axis=0)
        return pd.DataFrame(res)

    def lp_dist(self, real=None, fake=None, dataset=None, ord=2, group=True):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape and real.ndim in (2, 3)
        real, fake = self._flat(real), self._flat(fake)
        res = [np.linalg.norm(real[:, i] - fake[:, i], ord=ord) / real.shape[0] for i in range(real.shape[1])]
        return float(np.mean(res)) if group else res

    def wasserstein(self, real=None, fake=None, dataset=None, group=True):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape and real.ndim in (2, 3)
        real, fake = self._flat(real), self._flat(fake)
        res = [wasserstein_distance(real[:, i], fake[:, i]) for i in range(real.shape[1])]
        return float(np.mean(res)) if group else res

    def ACF(self, real=None, fake=None, dataset=None, nlags=17, group=True):
        real, fake, _ = self._args(real, fake, dataset)
        assert real.shape == fake.shape and real.ndim in (2, 3)
        if real.ndim == 3:
            # (N, T, F) -> per sample/feature acf over T, averaged over samples -> (F, nlags+1)
            ra = acf_batch(np.transpose(real, (0, 2, 1)), nlags).mean(axis=0)
            fa = acf_batch(np.transpose(fake, (0, 2, 1)), nlags).mean(axis=0)
            res = [float(np.mean(np.abs(ra[i] - fa[i]))) for i in range(ra.shape[0])]
        else:
            res = [float(np.mean(np.abs(acf(real[:, i], nlags) - acf(fake[:, i], nlags)))) for i in range(real.shape[1])]
        return float(np.mean(res)) if group else res

    def R2_relative_error(self, real=None, fake=None, dataset=None, group=True, fixed=False):
        real, fake, dataset = self._args(real, fake, dataset)
        assert dataset.ndim == 3 and real.ndim == 3 and fake.ndim == 3

        def xy(a, col):
            a = a.reshape(-1, a.shape[2]).astype(np.float64)
            y = a[1:, col]
            x = np.delete(a[:-1], col, axis=1)
            return y, x

        res = []
        second = fake if fixed else real  # Q8: the reference compares real with real
        for col in range(dataset.shape[2]):
            y_tr, x_tr = xy(dataset, col)
            y_te, x_te = xy(real, col)
            y_in, x_in = xy(second, col)
            beta = ols(y_tr, x_tr)
            res.append(abs(r2_score(y_te, x_te @ beta) - r2_score(y_in, x_in @ beta)))
        return float(np.mean(res)) if group else res

    def eyeball(self, real=None, fake=None, dataset=None, subplot_title=None, show=True):
        import matplotlib

        if not show:
            matplotlib.use("Agg")
        from matplotlib import pyplot as plt

        real, fake, _ = self._args(real, fake, dataset)
        subplot_title = self.subplot_title if subplot_title is None else subplot_title
        assert real.ndim == 3 and fake.ndim == 3
        if not isinstance(subplot_title, list):
            raise TypeError
        assert len(subplot_title) == real.shape[2]
        real, fake = self._flat(real), self._flat(fake)
        nrow = int(np.ceil(real.shape[1] / 3))
        fig, ax = plt.subplots(max(nrow, 1), 3, figsize=(20, 2.5 * max(nrow, 1)), squeeze=False)
        for i in range(real.shape[1]):
            r, c = divmod(i, 3)
            x = np.linspace(real[:, i].min(), real[:, i].max())
            ax[r, c].step(x, ECDF(real[:, i])(x))
            ax[r, c].step(x, ECDF(fake[:, i])(x))
            ax[r, c].set_title(subplot_title[i])
            ax[r, c].legend(["True", "Generated"], loc="upper left")
        plt.suptitle(self.model_name[0], y=1, fontsize=24)
        fig.tight_layout()
        if show:
            plt.show()
        return fig

    METRICS = ("ACF", "FID", "Inception_score", "R2_relative_error", "gaussian_MMD", "js_div", "kl_div", "ks_test",
               "linear_MMD", "lp_dist", "poly_MMD", "wasserstein")

    def run_all(self, plot=True, verbose=True):
        """Every metric (alphabetical, like the reference's ``dir(self)`` walk)."""
        res, names = [], []
        for i, name in enumerate(self.METRICS):
            res.append(getattr(self, name)())
            names.append(name)
            if verbose:
                print(f"{i + 1} out of {len(self.METRICS)} done.")
        if plot:
            self.eyeball(show=False)
        return pd.DataFrame(res, index=names, columns=self.model_name)


GAN_eval = GANEval  # reference class name
