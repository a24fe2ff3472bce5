"""Compatibility module: ``GAN_eval`` (GAN/GAN_eval.py:15-458) on hfrep.eval."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hfrep  # noqa: E402,F401
from hfrep.eval.gan_eval import ECDF, GAN_eval, GANEval, acf  # noqa: E402,F401

if __name__ == "__main__":
    # the reference's smoke: random N(0,1) windows through the metric suite
    import numpy as np

    real, fake, dataset = (np.random.normal(size=(500, 48, 35)) for _ in range(3))
    ev = GAN_eval(real, fake, dataset, [f"f{i}" for i in range(35)], ["Benchmark"])
    print(ev.run_all(plot=False))
