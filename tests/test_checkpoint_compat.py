"""Checkpoint IO, the Keras .h5 importer and the reference-API compatibility modules.

W-dist parity against the shipped artifacts: the production generator
(GAN/trained_generator/MTTS_GAN_GP20220621_02-49-32.h5) imported through hfrep.utils.h5lite and run
through the hfrep LSTM produces windows whose Wasserstein distance to the shipped generated sample
(GAN/generated_data2022-07-09.pkl, 10x168x36) is at the sampling-noise floor (the noise draws
differ: the notebook's RNG stream is not reproducible), while a different generator is far away.
"""
import glob
import os
import sys

import numpy as np
import pytest
import torch

from hfrep.data.io import safe_pickle_load
from hfrep.eval.gan_eval import GANEval
from hfrep.utils import checkpoint
from hfrep.utils.h5lite import read_keras_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_h5_importer_reads_every_shipped_generator(data_root):
    files = sorted(glob.glob(f"{data_root}/GAN/trained_generator/**/*.h5", recursive=True))
    assert len(files) == 8
    for p in files:
        m = read_keras_model(p)
        g, cfg = checkpoint.load_generator(p)
        assert g.count_params() == sum(w.size for w in m["weights"])
    m = read_keras_model(f"{data_root}/GAN/trained_generator/MTTS_GAN_GP20220621_02-49-32.h5")
    assert m["config"]["window"] == 168 and m["config"]["features"] == 36 and m["config"]["lrelu_after_first"]
    assert m["config"]["keras_version"] == "2.7.0"


def test_production_generator_wdist_parity(data_root):
    g, _ = checkpoint.load_generator(f"{data_root}/GAN/trained_generator/MTTS_GAN_GP20220621_02-49-32.h5")
    ref = safe_pickle_load(f"{data_root}/GAN/generated_data2022-07-09.pkl")
    gen = lambda s: g.predict(torch.tensor(np.random.RandomState(s).normal(0, 1, (10, 168, 36))).float()).numpy()
    a, b = gen(123), gen(456)
    ev = GANEval(a, ref, ref, [str(i) for i in range(36)], ["x"])
    w_ref, w_floor = ev.wasserstein(), ev.wasserstein(a, b)
    assert w_ref < 1.5 * w_floor, (w_ref, w_floor)
    assert abs(a.mean() - ref.mean()) < 2e-3 and abs(a.std() - ref.std()) < 2e-3
    other, _ = checkpoint.load_generator(f"{data_root}/GAN/trained_generator/temp/MTTS_GAN_GP20220621_04-28-13.h5")
    c = other.predict(torch.tensor(np.random.RandomState(1).normal(0, 1, (10, 168, 36))).float()).numpy()
    assert ev.wasserstein(c, ref) > 2 * w_floor


@pytest.mark.parametrize("ext", [".pkl", ".npz"])
def test_generator_roundtrip(tmp_path, ext):
    from hfrep.models import gan as zoo

    g = zoo.lstm_generator(12, 5, 16, lrelu_after_first=True)
    cfg = {"arch": "lstm", "window": 12, "features": 5, "hidden": 16, "lrelu_after_first": True}
    p = checkpoint.save_generator(str(tmp_path / f"g{ext}"), g, cfg)
    g2, cfg2 = checkpoint.load_generator(p)
    for a, b in zip(g.get_weights(), g2.get_weights()):
        np.testing.assert_array_equal(a, b)
    x = torch.randn(3, 12, 5)
    torch.testing.assert_close(g.predict(x), g2.predict(x))


def test_windows_npy_roundtrip(tmp_path):
    arr = np.random.rand(4, 24, 32).astype(np.float32)
    p = checkpoint.save_windows(str(tmp_path / "w.npy"), arr)
    np.testing.assert_array_equal(checkpoint.load_windows(p), arr)


def test_resume_is_bitwise(tmp_path):
    """Train 4 steps straight vs 2 + save/load + 2: identical parameters (fp32, CPU)."""
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    ds = np.random.RandomState(0).rand(30, 8, 4).astype(np.float32)
    cfg = GANConfig(arch="lstm", loss="wgan_gp", window=8, features=4, batch_size=6, hidden=8)
    a = GANTrainer(cfg, ds)
    a.train(4, verbose=False)
    b = GANTrainer(cfg, ds)
    b.train(2, verbose=False)
    p = checkpoint.save_training_state(str(tmp_path / "s.pt"), b)
    c = GANTrainer(cfg, ds)
    checkpoint.load_training_state(p, c)
    c.train(2, verbose=False)
    assert torch.equal(a.generator.flat, c.generator.flat) and torch.equal(a.critic.flat, c.critic.flat)
    assert c.iteration == 4


def test_helper_compat_module():
    sys.path.insert(0, ROOT)
    import helper

    for name in ["normalization", "read_csv", "dic_read", "set_seed", "random_sampling", "transaction_cost",
                 "price_impact", "reshape_cab", "ex_post_return", "factor_hf_split", "dic_save"]:
        assert callable(getattr(helper, name))
    helper.set_seed(1)
    w = helper.random_sampling(np.arange(100.0).reshape(50, 2), 7, 10)
    assert w.shape == (7, 10, 2)


def test_legacy_gan_classes_api(tmp_path):
    sys.path.insert(0, ROOT)
    from GAN.GAN import GAN
    from GAN.MTSS_WGAN_GP import WGAN_GP
    from GAN.WGAN_GP import MTTS_WGAN_GP

    ds = np.random.RandomState(0).rand(20, 6, 3).astype(np.float32)
    for cls in (GAN, MTTS_WGAN_GP, WGAN_GP):
        m = cls(ds, device="cpu")
        assert m.ts_shape == (6, 3) and m.generator is not None and m.critic is not None
        m.train(epochs=1, batch_size=4, save_dir=str(tmp_path), verbose=False)
        assert os.path.exists(m.saved_path)
        assert m.generate(5).shape == (5, 6, 3)


@pytest.mark.parametrize("kw", [dict(lrelu_after_first=True), dict(hidden=24), dict(lrelu_after_first=True, hidden=16)])
def test_legacy_checkpoint_roundtrip_keeps_architecture(tmp_path, kw):
    """A Q2-variant (LeakyReLU after the first LSTM, the production checkpoint's generator)
    or non-default-width generator trained through the legacy class API saves its real architecture:
    load_generator rebuilds it and predicts bitwise-identically; build_generator honours the flags."""
    sys.path.insert(0, ROOT)
    import torch

    from GAN.MTSS_WGAN_GP import WGAN_GP
    from hfrep.models.layers import LeakyReLU
    from hfrep.utils import checkpoint

    ds = np.random.RandomState(0).rand(20, 6, 3).astype(np.float32)
    m = WGAN_GP(ds, device="cpu", **kw)
    m.train(epochs=2, batch_size=4, save_dir=str(tmp_path), verbose=False)
    lrelu = kw.get("lrelu_after_first", False)
    assert isinstance(m.generator.layers[1], LeakyReLU) == lrelu
    fresh = m.build_generator()
    assert [type(l) for l in fresh.layers] == [type(l) for l in m.generator.layers]
    assert fresh.count_params() == m.generator.count_params()
    z = torch.randn(5, 6, 3, generator=torch.Generator().manual_seed(3))
    want = m.generator.predict(z)
    for path in (m.saved_path, m.saved_path[:-4] + ".npz"):
        g, cfg = checkpoint.load_generator(path)
        assert cfg["lrelu_after_first"] == lrelu and cfg["hidden"] == kw.get("hidden", 100)
        assert [type(l) for l in g.layers] == [type(l) for l in m.generator.layers]
        assert torch.equal(g.predict(z), want)


def test_autoencoder_compat(cleaned):
    sys.path.insert(0, ROOT)
    from Autoencoder_encapsulate import AE

    etf, hfd, rf = cleaned["factor_etf_data"], cleaned["hfd"], cleaned["rf"]
    n = len(etf)
    nt = int(np.ceil(n * 0.5))
    ae = AE(etf.iloc[:n - nt], hfd.iloc[:n - nt], etf.iloc[n - nt:], hfd.iloc[n - nt:], 4)
    ae.train(verbose=0, plot=False)
    assert 0 < ae.model_IS_r2() <= 1 and ae.model_IS_RMSE() > 0
    oos = ae.model_OOS_r2()
    assert len(oos) == nt - 2
    ante = ae.ante(rf, hfd)
    assert ante.shape == (144, 13)
    post = ae.post(etf)
    assert post.shape == (144, 13) and np.isfinite(post.to_numpy()).all()
    to = ae.turnover(cleaned["hfd_fullname"])
    assert to.shape == (13, 1) and (to["Turnover"] > 0).all()
