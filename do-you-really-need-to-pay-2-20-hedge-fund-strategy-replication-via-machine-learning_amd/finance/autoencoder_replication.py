"""Autoencoder factor replication (reference ``Autoencoder_encapsulate.AE``, :37-243).

Pipeline per latent size k (the notebook loops k = 1..21, autoencoder_v4.ipynb:159):

1. MinMax-scale x_train (22 ETF excess log returns), train the AE: Nadam, MSE, batch 48,
   ``validation_split=.25`` (the LAST 25% of rows, Keras semantics), EarlyStopping(val_loss,
   patience) — :class:`AETrainer` (explicit engine; native kernels on GPU, bf16 or fp32).
2. In/out-of-sample R^2 and RMSE (:meth:`AE.model_IS_r2` ...; OOS = expanding windows with a
   refit scaler, 167 values for 169 test rows).
3. ``ante``: encoder factors of the (unscaled, Q7) test returns -> rolling 24-month OLS of every HF
   index on the factors -> decoder-mapped ETF weights, LeakyReLU mask, volatility normalisation,
   residual in the risk-free asset -> 144 months of ex-ante clone returns.  The reference always
   uses the FIRST window's beta/normalisation (Q6); ``beta_index='rolling'`` uses the window's own.
4. ``post``: ex-post returns with transaction-cost / price-impact penalties; ``turnover``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from ..data.scaler import MinMaxScaler
from ..models.autoencoder import FactorAutoencoder
from ..ops import _native
from ..train.optim import KerasOptimizer
from .replication import ex_post_return, normalization, ols, reshape_cab


# ------------------------------------------------------------------------------------------
# metrics (sklearn semantics, multioutput='uniform_average')
# ------------------------------------------------------------------------------------------
def r2_score(y, p) -> float:
    y = np.asarray(y, dtype=np.float64)
    p = np.asarray(p, dtype=np.float64)
    ss_res = ((y - p) ** 2).sum(axis=0)
    ss_tot = ((y - y.mean(axis=0)) ** 2).sum(axis=0)
    with np.errstate(divide="ignore", invalid="ignore"):
        r2 = np.where(ss_tot != 0, 1 - ss_res / np.where(ss_tot == 0, 1, ss_tot), np.where(ss_res == 0, 1.0, 0.0))
    return float(r2.mean())


def rmse(y, p) -> float:
    y = np.asarray(y, dtype=np.float64)
    p = np.asarray(p, dtype=np.float64)
    return float(np.sqrt(((y - p) ** 2).mean(axis=0)).mean())


# ------------------------------------------------------------------------------------------
# training (Keras fit + EarlyStopping semantics)
# ------------------------------------------------------------------------------------------
class AETrainer:
    def __init__(self, model: FactorAutoencoder, lr: float = 1e-3, device="cpu"):
        self.model = model
        self.device = torch.device(device)
        self.opt = KerasOptimizer.nadam(lr, device=self.device)

    def fit(self, x: np.ndarray, epochs: int = 1000, batch_size: int = 48, validation_split: float = 0.25,
            patience: int = 5, shuffle: bool = True, seed: int = 123, dtype=torch.float32, verbose: int = 0,
            fused: bool | None = None):
        """Keras ``fit`` semantics: ``validation_split`` takes the LAST rows, one Nadam tick per batch,
        EarlyStopping(val_loss, patience) per epoch (weights of the last epoch are kept).

        On the GPU the whole fit is ONE launch of csrc/ae.hip (``fused``, default on a native GPU
        build): the batch permutations are drawn here up front from the same numpy stream, and the
        forward, the fused MSE value + gradient, the reverse pass, Nadam, the validation loss and the
        stopping decision all run inside one workgroup.  ``fused=False`` runs the explicit engine
        batch by batch (the CPU path)."""
        x = np.asarray(x, dtype=np.float64)
        n = len(x)
        split = int(n * (1.0 - validation_split)) if validation_split else n
        rs = np.random.RandomState(seed)
        enc, dec = self.model.parts()
        A, k = x.shape[1], self.model.latent_dim
        if fused is None:
            fused = (self.device.type == "cuda" and _native.use_native_for(enc.flat)
                     and dtype in (torch.float32, torch.bfloat16)
                     and bool(_native.native().ae_fit_supported(A, k, batch_size)))
        if fused:
            return self._fit_fused(x, split, epochs, batch_size, patience, shuffle, rs, dtype, verbose)
        xt = torch.as_tensor(x[:split], dtype=dtype, device=self.device)
        xv = torch.as_tensor(x[split:], dtype=dtype, device=self.device) if split < n else None
        hist = {"loss": [], "val_loss": []}
        best, wait = np.inf, 0
        # one host <-> device round trip per epoch: the epoch's batch order goes to the device in
        # one copy, the loss is accumulated there (float64, batch order: the same sum as the
        # host-side one), and the training and validation losses come back together for the
        # EarlyStopping decision (which is per epoch in Keras too)
        for ep in range(epochs):
            order = rs.permutation(split) if shuffle else np.arange(split)
            order_t = torch.as_tensor(order, device=self.device)
            tot = torch.zeros((), dtype=torch.float64, device=self.device)
            for s in range(0, split, batch_size):
                idx = order_t[s:s + batch_size]
                xb = xt.index_select(0, idx)
                loss = self.model.loss_and_grads(xb)
                # Keras applies ONE optimizer step per batch to all variables (one iteration tick)
                self.opt.apply_group([enc.flat, dec.flat])
                enc.zero_grad()
                dec.zero_grad()
                tot = tot + loss.double() * idx.numel()
            vl_t = None
            if xv is not None:
                with torch.no_grad():
                    pv = self.model.predict(xv)
                    vl_t = ((pv.double() - xv.double()) ** 2).mean()
            pair = torch.stack([tot, vl_t if vl_t is not None else tot]).cpu().tolist()
            hist["loss"].append(pair[0] / split)
            if xv is not None:
                vl = pair[1]
                hist["val_loss"].append(vl)
                if verbose:
                    print(f"epoch {ep + 1}: loss {hist['loss'][-1]:.6f} val_loss {vl:.6f}")
                if vl < best:
                    best, wait = vl, 0
                else:
                    wait += 1
                    if wait >= patience:
                        break
        return hist

    @torch.no_grad()
    def _fit_fused(self, x, split, epochs, batch_size, patience, shuffle, rs, dtype, verbose):
        return fit_fused_many([self._fused_job(x, split, epochs, patience, shuffle, rs)], batch_size, dtype,
                              verbose)[0]

    def _fused_job(self, x, split, epochs, patience, shuffle, rs):
        """One fit's operands for csrc/ae.hip: row-major fp32 train / validation rows, the epochs' batch
        permutations (drawn up front from the fit's numpy stream, the eager trainer's draws), the
        weights and Nadam slots (updated in place) and the shared counters."""
        n, A = x.shape
        enc, dec = self.model.parts()
        nw = A * self.model.latent_dim
        orders = np.stack([rs.permutation(split) if shuffle else np.arange(split) for _ in range(epochs)])
        dev = self.device
        # row-major copies: the scaler's output can be column-major (MinMaxScaler keeps Fortran order)
        xt = torch.as_tensor(np.ascontiguousarray(x[:split]), dtype=torch.float32, device=dev).contiguous()
        xv = torch.as_tensor(np.ascontiguousarray(x[split:]), dtype=torch.float32, device=dev).reshape(-1, A).contiguous()
        (mWe, vWe), (mWd, vWd) = self.opt._slots(enc.flat), self.opt._slots(dec.flat)
        return dict(trainer=self, Xt=xt, Xv=xv, order=torch.as_tensor(orders.astype(np.int32), device=dev),
                    We=enc.flat.data[:nw], Wd=dec.flat.data[:nw], mWe=mWe[:nw], vWe=vWe[:nw], mWd=mWd[:nw],
                    vWd=vWd[:nw], step=self.opt.iterations, m_cache=self.opt.m_cache,
                    patience=patience if split < n else epochs + 1, has_val=split < n)


@torch.no_grad()
def fit_fused_many(jobs: list, batch_size: int, dtype, verbose: int = 0) -> list:
    """Train every job (``AETrainer._fused_job`` records) in ONE launch of csrc/ae.hip: one workgroup per
    fit, so a latent sweep (21 fits) or a multi-seed study (hundreds) trains side by side across the
    CUs instead of one single-workgroup launch after another.  The fits share the input width, batch
    size, dtype and the Nadam hyper-parameters (every trainer's optimizer must agree).  Returns one
    Keras-style history dict per job."""
    if not jobs:
        return []
    o0 = jobs[0]["trainer"].opt
    for j in jobs:
        o = j["trainer"].opt
        if (o.lr, o.b1, o.b2, o.eps) != (o0.lr, o0.b1, o0.b2, o0.eps):
            raise ValueError("fit_fused_many: every fit must use the same Nadam hyper-parameters")
    L = lambda key: [j[key] for j in jobs]  # noqa: E731
    hist_t, nep_t = _native.native().ae_fit(
        L("Xt"), L("Xv"), L("order"), L("We"), L("Wd"), L("mWe"), L("vWe"), L("mWd"), L("vWd"), L("step"),
        L("m_cache"), [int(j["patience"]) for j in jobs], o0.lr, o0.b1, o0.b2, o0.eps, batch_size,
        dtype == torch.bfloat16)
    nep = nep_t.cpu().tolist()
    hall = hist_t.cpu().numpy()
    out = []
    for i, j in enumerate(jobs):
        h = hall[i, :nep[i]]
        hist = {"loss": h[:, 0].tolist(), "val_loss": h[:, 1].tolist() if j["has_val"] else []}
        if verbose:
            for ep in range(nep[i]):
                print(f"epoch {ep + 1}: loss {h[ep, 0]:.6f} val_loss {h[ep, 1]:.6f}")
        out.append(hist)
    return out


# ------------------------------------------------------------------------------------------
# the AE replication object (reference API)
# ------------------------------------------------------------------------------------------
class AE:
    """API-compatible re-design of ``Autoencoder_encapsulate.AE``.

    ``AE(x_train, y_train, x_test, y_test, latent_dim)``; data unscaled (DataFrames or arrays).
    Extra keyword options (defaults = reference semantics): ``device``, ``dtype``,
    ``scale_test`` (Q7 fix), ``beta_index`` ('first' = Q6 parity, 'rolling').
    """

    def __init__(self, x_train, y_train, x_test, y_test, latent_dim, device="cpu", dtype=torch.float32,
                 seed: int = 123, scale_test: bool = False, beta_index: str = "first", oos_stride: int = 1):
        assert len(x_train) == len(y_train) and len(y_test) == len(x_test)
        self.train_scale = MinMaxScaler()
        self._x_train = self.train_scale.fit_transform(np.asarray(x_train, dtype=np.float64))
        self._x_test = x_test
        self._y_train = y_train
        self._y_test = y_test
        self._latent_dim = latent_dim
        self.device, self.dtype, self.seed = torch.device(device), dtype, seed
        self.scale_test, self.beta_index = scale_test, beta_index
        # expanding OOS windows xt[:i] for i = 2, 2 + stride, ... (1 = the reference's every window; the
        # daily panel evaluates one window per ~month of trading days)
        self.oos_stride = int(oos_stride)
        self.autoencoder = None
        self.history = None
        self._ante = self._post = None

    # -- training ------------------------------------------------------------------------------
    def _new_trainer(self) -> AETrainer:
        self._oos_cache = None  # (predictions of the previous model)
        self.autoencoder = FactorAutoencoder(self._latent_dim, self._x_train.shape[1], seed=self.seed, dtype=torch.float32,
                                             device=self.device)
        return AETrainer(self.autoencoder, device=self.device)

    def train(self, patience=5, verbose=2, plot=True):
        tr = self._new_trainer()
        self.history = tr.fit(self._x_train, epochs=1000, batch_size=48, validation_split=0.25, patience=patience,
                              seed=self.seed, dtype=self.dtype, verbose=1 if verbose == 1 else 0)
        if plot:
            self.plot_history()
        return self.history

    def plot_history(self):
        import matplotlib.pyplot as plt

        print(self.autoencoder.encoder.summary())
        print(self.autoencoder.decoder.summary())
        plt.plot(self.history["loss"])
        plt.plot(self.history["val_loss"])
        plt.title("Model Loss")
        plt.ylabel("loss")
        plt.xlabel("epoch")
        plt.legend(["train", "val"], loc="upper left")
        plt.show()

    @staticmethod
    def train_many(aes: list, patience: int = 5) -> list:
        """``ae.train(patience, plot=False)`` for every AE, the same fits and results; on a native GPU
        build all of them (any latent sizes, seeds and panels with one input width and dtype) train in
        ONE launch, one workgroup per fit (``fit_fused_many``).  Otherwise they train one by one."""
        if not aes:
            return []
        a0 = aes[0]
        A = a0._x_train.shape[1]
        batched = (all(a.device.type == "cuda" and a.device == a0.device and a.dtype == a0.dtype
                       and a._x_train.shape[1] == A for a in aes)
                   and a0.dtype in (torch.float32, torch.bfloat16)
                   # use_native_for first: with HFREP_ALLOW_TORCH_FALLBACK=1 and no library it is False (the
                   # one-by-one fallback below), where native() would raise
                   and _native.use_native_for(torch.empty(0, device=a0.device))
                   and all(bool(_native.native().ae_fit_supported(A, a._latent_dim, 48)) for a in aes))
        if batched:
            jobs = []
            for a in aes:
                tr = a._new_trainer()
                if not _native.use_native_for(a.autoencoder.parts()[0].flat):
                    batched = False
                    break
                x = np.asarray(a._x_train, dtype=np.float64)
                split = int(len(x) * 0.75)
                jobs.append(tr._fused_job(x, split, 1000, patience, True, np.random.RandomState(a.seed)))
        if not batched:
            return [a.train(patience=patience, verbose=0, plot=False) for a in aes]
        for a, h in zip(aes, fit_fused_many(jobs, 48, a0.dtype)):
            a.history = h
        return [a.history for a in aes]

    def _predict(self, x) -> np.ndarray:
        xt = torch.as_tensor(np.asarray(x, dtype=np.float64), dtype=self.dtype, device=self.device)
        return self.autoencoder.predict(xt).double().cpu().numpy()

    def _encode(self, x) -> np.ndarray:
        xt = torch.as_tensor(np.asarray(x, dtype=np.float64), dtype=self.dtype, device=self.device)
        return self.autoencoder.encoder.predict(xt).double().cpu().numpy()

    # -- reconstruction metrics -------------------------------------------------------------------
    def model_IS_r2(self):
        return r2_score(self._x_train, self._predict(self._x_train))

    def model_IS_RMSE(self):
        return rmse(self._x_train, self._predict(self._x_train))

    def _oos_windows(self):
        """(scaled window, prediction) for every expanding window xt[:i], i = 2 .. len - 1, each scaled by its
        own refit MinMaxScaler (the reference's OOS loop).  The autoencoder is row-wise, so all windows'
        rows go through ONE batched prediction (one launch chain instead of one per window and metric);
        cached until the model is retrained."""
        if getattr(self, "_oos_cache", None) is None:
            xt = np.asarray(self._x_test, dtype=np.float64)
            xrs = [MinMaxScaler().fit_transform(xt[:i]) for i in range(2, len(xt), self.oos_stride)]
            pred = self._predict(np.concatenate(xrs, 0)) if xrs else np.zeros((0, xt.shape[1]))
            cuts = np.cumsum([len(x) for x in xrs])[:-1]
            self._oos_cache = list(zip(xrs, np.split(pred, cuts)))
        return self._oos_cache

    def _oos(self, metric):
        return [metric(xr, p) for xr, p in self._oos_windows()]

    def model_OOS_r2(self):
        return self._oos(r2_score)

    def model_OOS_RMSE(self):
        return self._oos(rmse)

    # -- replication ---------------------------------------------------------------------------------
    def ante(self, rf, hfd, window=24):
        assert isinstance(rf, pd.DataFrame)
        xt = np.asarray(self._x_test, dtype=np.float64)
        if self.scale_test:
            xt = self.train_scale.transform(xt)
        main_factor = self._encode(xt)
        Y = np.asarray(self._y_test, dtype=np.float64)
        n_win = len(xt) - window
        betas, norms = [], []
        for i in range(n_win):
            X, Yw = main_factor[i:i + window], Y[i:i + window]
            b = ols(Yw, X)
            betas.append(b)
            norms.append(normalization(Yw, X, b, window))
        Wd = self.autoencoder.decoder_kernel().astype(np.float64)  # (k, 22)
        weights, delta = [], []
        for i in range(n_win):
            lr_mask = np.where(main_factor[window + i] @ Wd < 0, 0.2, 1.0)
            j = 0 if self.beta_index == "first" else i
            sw = ((betas[j].T @ Wd) * lr_mask).T * norms[j]  # (22, 13)
            weights.append(sw)
            delta.append(1 - sw.sum(axis=0))
        weights.pop()
        delta.pop()
        T = len(weights)
        self.OOS_etf = np.asarray(self._x_test, dtype=np.float64)[-T:]
        self.OOS_hfd = self._y_test.iloc[-T:] if hasattr(self._y_test, "iloc") else np.asarray(self._y_test)[-T:]
        self.OOS_rf = np.asarray(rf.iloc[-T:], dtype=np.float64)
        rets = [delta[i] * self.OOS_rf[i] + np.sum(self.OOS_etf[i] * weights[i].T, axis=1) for i in range(T)]
        ante = pd.DataFrame(rets, columns=hfd.columns, index=hfd.index[-T:])
        cols = list(hfd.columns)
        self.strat_weight_on_etf = [pd.DataFrame(w, columns=cols) for w in weights]
        self.reshape_strat_weight_on_etf = reshape_cab(self.strat_weight_on_etf)
        self._ante, self.rf, self.hfd, self.window = ante, rf, hfd, window
        return ante

    def post(self, factor_etf_data):
        if self._ante is None:
            raise Exception("please execute ante before turnover")
        oos = factor_etf_data.iloc[-len(self.reshape_strat_weight_on_etf[0]) - self.window:]
        self._post = ex_post_return(self._ante, self.window, self.reshape_strat_weight_on_etf, oos)
        return self._post

    def turnover(self, hfd_fullname):
        if self._ante is None:
            raise Exception("please execute ante before turnover")
        W = np.stack([w.to_numpy() for w in self.strat_weight_on_etf])
        to = np.abs(np.diff(W, axis=0)).sum(axis=(0, 1)) / (len(W) / 12)
        out = pd.DataFrame({"Real_AE": list(hfd_fullname.values())[: len(to)], "Turnover": to}).set_index("Real_AE")
        self.hfd_fullname = hfd_fullname
        return out

    def plot(self, hfd_fullname, title=None, show=True):
        assert isinstance(title, str)
        import matplotlib

        if not show:
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        n = len(self._ante.columns)
        rows = int(np.ceil(n / 3))
        fig, ax = plt.subplots(rows, 3, figsize=(30, 4 * rows), squeeze=False)
        for idx, strat in enumerate(self._ante.columns):
            r, c = divmod(idx, 3)
            real = self.OOS_hfd.iloc[:, idx] if hasattr(self.OOS_hfd, "iloc") else self.OOS_hfd[:, idx]
            temp = pd.DataFrame([self._ante.iloc[:, idx].cumsum().values, self._post.iloc[:, idx].cumsum().values,
                                 np.cumsum(np.asarray(real))], index=["Ex-ante", "Ex_post", "Real"]).T
            for name in temp.columns:
                ax[r][c].plot(temp[name].values, label=name)
            ax[r][c].legend(loc="upper left")
            ax[r][c].set_title(hfd_fullname.get(strat, strat))
        plt.suptitle(title, y=0.93, fontsize=24)
        if show:
            plt.show()
        return fig
