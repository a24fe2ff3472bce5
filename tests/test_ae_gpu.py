"""Factor autoencoder (BASELINE config 2: AE on one MI355X) — the GPU engine vs the CPU fp64 engine.

On the GPU the whole fit (forward, fused MSE value + gradient, reverse pass, Keras Nadam, validation
loss, EarlyStopping) is ONE launch of csrc/ae.hip; ``fused=False`` runs the explicit engine batch by
batch (native Dense / LeakyReLU / Nadam kernels).  Same initial weights, same batch order, five
epochs: fp32 must track the fp64 CPU run tightly, bf16 (bf16 activations, fp32 master weights)
within bf16 noise (Autoencoder_encapsulate.py:23-30, :79-96).
"""
import numpy as np
import pytest
import torch

from hfrep.finance.autoencoder_replication import AE, AETrainer
from hfrep.models.autoencoder import FactorAutoencoder

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt,tol", [(torch.float32, 2e-4), (torch.bfloat16, 5e-2)])
@pytest.mark.parametrize("k", [1, 7, 21])
@pytest.mark.parametrize("fused", [True, False])
def test_ae_trainer_gpu_vs_cpu(cuda, dt, tol, k, fused):
    rs = np.random.RandomState(k)
    x = rs.rand(168, 22)
    mg = FactorAutoencoder(k, 22, seed=3, device=cuda)
    mc = FactorAutoencoder(k, 22, seed=3, dtype=torch.float64)
    with torch.no_grad():
        for a, b in zip(mg.parts(), mc.parts()):
            b.flat.copy_(a.flat.double().cpu())
    # column-major input, as MinMaxScaler returns it (the fused fit must take any layout)
    hg = AETrainer(mg, device=cuda).fit(np.asfortranarray(x), epochs=5, patience=100, seed=9, dtype=dt, fused=fused)
    hc = AETrainer(mc).fit(x, epochs=5, patience=100, seed=9, dtype=torch.float64)
    np.testing.assert_allclose(hg["loss"], hc["loss"], rtol=tol * 10, atol=1e-7)
    for a, b in zip(mg.parts(), mc.parts()):
        wa, wb = a.flat.detach().double().cpu(), b.flat.detach()
        rel = ((wa - wb).norm() / wb.norm()).item()
        assert rel < tol, f"k={k} {dt}: weight rel err {rel:.2e}"


def test_ae_replication_object_on_gpu(cuda, cleaned):
    """AE.train/metrics/ante/post on the GPU give finite reference-shaped outputs (167 OOS windows,
    144 clone months) at fp32 and bf16."""
    etf, hfd, rf = cleaned["factor_etf_data"], cleaned["hfd"], cleaned["rf"]
    half = len(hfd) // 2
    for dt in (torch.float32, torch.bfloat16):
        ae = AE(etf.iloc[:half].to_numpy(), hfd.iloc[:half].to_numpy(), etf.iloc[half:].to_numpy(), hfd.iloc[half:], 4,
                device=cuda, dtype=dt)
        ae.train(verbose=0, plot=False)
        assert 0 < ae.model_IS_r2() <= 1
        oos = ae.model_OOS_r2()
        assert len(oos) == 167 and np.isfinite(oos).all()
        ante = ae.ante(rf.iloc[half:], hfd.iloc[half:])
        post = ae.post(etf)
        assert ante.shape == (144, 13) and post.shape == (144, 13)
        assert np.isfinite(post.to_numpy()).all()


def test_ae_fused_fit_early_stopping(cuda):
    """The in-kernel EarlyStopping: the fused fit stops where the Keras rule says, given the history it
    returns (first epoch whose val_loss has not improved on the best for `patience` epochs), and its
    weights / optimizer counter equal an eager fp32 run of that many epochs within fp32 noise."""
    rs = np.random.RandomState(5)
    x = rs.rand(168, 22)
    m1 = FactorAutoencoder(3, 22, seed=4, device=cuda)
    m2 = FactorAutoencoder(3, 22, seed=4, device=cuda)
    t1 = AETrainer(m1, device=cuda)
    h1 = t1.fit(x, epochs=1000, patience=3, seed=2, fused=True)
    ne = len(h1["val_loss"])
    assert 3 < ne < 1000
    vl, best, wait, stop = h1["val_loss"], np.inf, 0, None
    for i, v in enumerate(vl):
        if v < best:
            best, wait = v, 0
        else:
            wait += 1
            if wait >= 3:
                stop = i + 1
                break
    assert stop == ne, (stop, ne)
    t2 = AETrainer(m2, device=cuda)
    h2 = t2.fit(x, epochs=ne, patience=10 ** 6, seed=2, fused=False)
    np.testing.assert_allclose(h1["loss"], h2["loss"], rtol=1e-4)
    assert float(t1.opt.iterations.item()) == float(t2.opt.iterations.item()) == ne * 3
    for a, b in zip(m1.parts(), m2.parts()):
        rel = ((a.flat - b.flat).norm() / b.flat.norm()).item()
        assert rel < 1e-4, rel


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_ae_train_many_matches_one_by_one(cuda, cleaned, dt):
    """AE.train_many trains every fit in ONE csrc/ae.hip launch (one workgroup per fit): for a mix of
    latent sizes, seeds and training panels (different row counts) the histories, epochs run and
    weights equal the one-launch-per-fit path bitwise (each workgroup runs the same fixed-order code)."""
    etf, hfd = cleaned["factor_etf_data"].to_numpy(), cleaned["hfd"].to_numpy()
    half = len(hfd) // 2
    rs = np.random.RandomState(0)
    xa = np.vstack([etf[:half], rs.rand(40, etf.shape[1]) * 0.1])  # an "augmented" panel: more rows
    ya = np.vstack([hfd[:half], rs.rand(40, hfd.shape[1]) * 0.1])
    specs = [(etf[:half], hfd[:half], 1, 3), (etf[:half], hfd[:half], 7, 3), (xa, ya, 4, 11), (etf[:half], hfd[:half], 21, 5)]

    def make():
        return [AE(x, y, etf[half:], hfd[half:], k, device=cuda, dtype=dt, seed=s) for x, y, k, s in specs]

    many, single = make(), make()
    AE.train_many(many)
    for a in single:
        a.train(verbose=0, plot=False)
    for a, b in zip(many, single):
        assert a.history["loss"] == b.history["loss"] and a.history["val_loss"] == b.history["val_loss"]
        for pa, pb in zip(a.autoencoder.parts(), b.autoencoder.parts()):
            assert torch.equal(pa.flat, pb.flat)


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-3), (torch.bfloat16, 5e-2)])
def test_ae_fit_daily_size_vs_cpu(cuda, daily, dt, tol):
    """BASELINE config 2 at its stated size: the fused Keras fit (csrc/ae.hip) on the DAILY ETF panel's
    training half (~3,660 days: ~57 batches per epoch, ~900 validation rows) tracks the CPU fp64 engine
    over 3 epochs (same weights, same batch order)."""
    from hfrep.data.scaler import MinMaxScaler

    x = daily.to_numpy(np.float64)
    x = MinMaxScaler().fit_transform(x[: len(x) // 2])
    k = 7
    mg = FactorAutoencoder(k, x.shape[1], seed=3, device=cuda)
    mc = FactorAutoencoder(k, x.shape[1], seed=3, dtype=torch.float64)
    with torch.no_grad():
        for a, b in zip(mg.parts(), mc.parts()):
            b.flat.copy_(a.flat.double().cpu())
    hg = AETrainer(mg, device=cuda).fit(x, epochs=3, patience=100, seed=9, dtype=dt, fused=True)
    hc = AETrainer(mc).fit(x, epochs=3, patience=100, seed=9, dtype=torch.float64)
    np.testing.assert_allclose(hg["loss"], hc["loss"], rtol=tol * 10, atol=1e-7)
    np.testing.assert_allclose(hg["val_loss"], hc["val_loss"], rtol=tol * 10, atol=1e-7)
    for a, b in zip(mg.parts(), mc.parts()):
        wa, wb = a.flat.detach().double().cpu(), b.flat.detach()
        rel = ((wa - wb).norm() / wb.norm()).item()
        assert rel < tol, f"{dt}: weight rel err {rel:.2e}"


def test_ae_daily_study_on_gpu(cuda, daily):
    """The daily factor study (finance.experiment.daily_factor_study): every (latent) fit of the daily
    panel in one launch, finite reference-style metrics at fp32 and bf16."""
    from hfrep.finance.experiment import daily_factor_study

    for dt in (torch.float32, torch.bfloat16):
        st = daily_factor_study(daily, latents=[1, 7, 21], device=cuda, dtype=dt)
        assert len(st) == 3 and np.isfinite(st[["IS_r2", "IS_RMSE", "OOS_r2", "OOS_RMSE"]].to_numpy()).all()
        assert (st["IS_r2"] <= 1).all() and st["IS_r2"].iloc[-1] > st["IS_r2"].iloc[0]
        assert (st["epochs"] >= 1).all() and st["train_rows"].iloc[0] == len(daily) // 2
