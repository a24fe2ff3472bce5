"""W-dist parity anchor: the reference's own trained MTSS-WGAN-GP generator
(GAN/trained_generator/old/MTSS_WGAN_GP20220613_20-40-15.h5, 48 x 35 LSTM G) under the parity
protocol of ``hfrep parity`` (1000 N(0,1) windows vs 1000 held-out real windows of the MinMax-scaled
cleaned panel, GAN_eval.wasserstein, GAN/GAN_eval.py:309-326).  Our own reference-preset training
runs are reported against this number (profiles/r02_parity/README.md)."""
import os

import pytest

from hfrep.cli import REFERENCE_GENERATOR, reference_anchor


def test_reference_generator_wdist_pinned(data_root):
    if not os.path.exists(os.path.join(data_root, REFERENCE_GENERATOR)):
        pytest.skip("reference generator .h5 not available")
    res = reference_anchor(h5=os.path.join(data_root, REFERENCE_GENERATOR), seed=123)
    assert res["n"] == 1000
    assert abs(res["w_fake_vs_real"] - 0.019319) < 2e-5, res
    # the protocol's own scale: real-vs-real floor << generator << uniform noise
    assert res["w_real_vs_real_floor"] < 0.002 and 0.19 < res["w_uniform_vs_real"] < 0.21
