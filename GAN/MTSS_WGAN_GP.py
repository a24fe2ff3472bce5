"""Compatibility entry point for the reference script ``GAN/MTSS_WGAN_GP.py`` (training loop GAN/MTSS_WGAN_GP.py:254-287).

``python GAN/MTSS_WGAN_GP.py`` runs the reference prologue (cleaned data -> MinMax -> 1000 x 48 windows)
and trains class ``WGAN_GP`` for 5000 iterations at batch 32 on the MI355X (native kernels) or CPU.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hfrep  # noqa: E402,F401
from hfrep.compat.legacy_gan import WGAN_GP, reference_dataset, script_main  # noqa: E402,F401

if __name__ == "__main__":
    script_main(WGAN_GP)
