"""Factor autoencoder (BASELINE config 2: AE on one MI355X) — the GPU engine vs the CPU fp64 engine.

The AE trains through the explicit engine: native Dense (no bias, LeakyReLU epilogue) kernels,
the fused Keras-Nadam kernel and the MSE adjoint on the GPU (Autoencoder_encapsulate.py:23-30,
:79-96).  Same initial weights, same batch order, five epochs: fp32 must track the fp64 CPU run
tightly, bf16 (bf16 activations, fp32 master weights) within bf16 noise.
"""
import numpy as np
import pytest
import torch

from hfrep.finance.autoencoder_replication import AE, AETrainer
from hfrep.models.autoencoder import FactorAutoencoder

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt,tol", [(torch.float32, 2e-4), (torch.bfloat16, 5e-2)])
@pytest.mark.parametrize("k", [1, 7, 21])
def test_ae_trainer_gpu_vs_cpu(cuda, dt, tol, k):
    rs = np.random.RandomState(k)
    x = rs.rand(168, 22)
    mg = FactorAutoencoder(k, 22, seed=3, device=cuda)
    mc = FactorAutoencoder(k, 22, seed=3, dtype=torch.float64)
    with torch.no_grad():
        for a, b in zip(mg.parts(), mc.parts()):
            b.flat.copy_(a.flat.double().cpu())
    hg = AETrainer(mg, device=cuda).fit(x, epochs=5, patience=100, seed=9, dtype=dt)
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
