"""GAN_eval metric suite vs direct scipy/sklearn computations."""
import numpy as np
import pytest
from scipy.stats import kstest, wasserstein_distance
from sklearn import metrics

from hfrep.eval.gan_eval import ECDF, GANEval, acf

RS = np.random.RandomState(0)
REAL = RS.normal(size=(40, 24, 5))
FAKE = RS.normal(loc=0.1, size=(40, 24, 5))
DATA = RS.normal(size=(40, 24, 5))
EV = GANEval(REAL, FAKE, DATA, [f"f{i}" for i in range(5)], ["m"])


def test_wasserstein_is_per_feature_mean():
    r, f = REAL.reshape(-1, 5), FAKE.reshape(-1, 5)
    assert np.isclose(EV.wasserstein(), np.mean([wasserstein_distance(r[:, i], f[:, i]) for i in range(5)]))


def test_ks_lp_fid_mmd():
    r, f = REAL.reshape(-1, 5), FAKE.reshape(-1, 5)
    assert np.isclose(EV.ks_test(), np.mean([kstest(r[:, i], f[:, i])[1] for i in range(5)]))
    assert np.isclose(EV.lp_dist(), np.mean([np.linalg.norm(r[:, i] - f[:, i]) / len(r) for i in range(5)]))
    assert EV.FID() > 0 and EV.FID(REAL, REAL) < 1e-6
    rm, fm = REAL.mean(0), FAKE.mean(0)
    k = metrics.pairwise.rbf_kernel
    assert np.isclose(EV.gaussian_MMD(), k(rm, rm, 1.0).mean() + k(fm, fm, 1.0).mean() - 2 * k(rm, fm, 1.0).mean())
    assert np.isclose(EV.linear_MMD(), (rm @ rm.T).mean() + (fm @ fm.T).mean() - 2 * (rm @ fm.T).mean())


def test_acf_matches_definition():
    x = RS.randn(50)
    xc = x - x.mean()
    ref = [np.dot(xc[:50 - k], xc[k:]) / np.dot(xc, xc) for k in range(18)]
    np.testing.assert_allclose(acf(x, 17), ref)
    assert EV.ACF() >= 0


def test_divergences_and_is():
    assert EV.kl_div() >= 0 and EV.js_div() >= 0
    assert EV.Inception_score() >= 1.0


def test_r2_relative_error_quirk_and_fix():
    assert EV.R2_relative_error() == 0.0  # reference compares real with real (Q8)
    assert EV.R2_relative_error(fixed=True) > 0.0


def test_run_all_and_ecdf(tmp_path):
    df = EV.run_all(plot=False, verbose=False)
    assert list(df.columns) == ["m"] and len(df) == 12 and "wasserstein" in df.index
    e = ECDF([1, 2, 2, 3])
    assert e(2) == 0.75 and e(0) == 0 and e(3) == 1
