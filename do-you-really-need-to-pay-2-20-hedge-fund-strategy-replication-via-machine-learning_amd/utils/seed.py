"""Global seeding (``helper.set_seed``, helper.py:32-41).

Seeds PYTHONHASHSEED, ``random``, numpy and torch (CPU + all GPUs).  The reference also forced
single-threaded TF sessions for determinism; here determinism comes from counter-based Philox
streams on device and fixed reduction orders in the kernels (run-to-run bitwise equal on GPU
except for the LayerNorm-parameter gradient, which uses float atomics).
"""
import os
import random

import numpy as np


def set_seed(seed_value: int = 123) -> None:
    os.environ["PYTHONHASHSEED"] = str(seed_value)
    random.seed(seed_value)
    np.random.seed(seed_value)
    try:
        import torch

        torch.manual_seed(seed_value)
    except ImportError:  # pragma: no cover
        pass
