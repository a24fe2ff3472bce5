"""List the torch (aten) ops one training iteration dispatches on the device, with their call sites.

The headline step should launch only hand-written hfrep kernels; every aten op that reaches the
device (a fill, a cat, an elementwise add) shows up in the rocprof table as an ``at::native`` kernel.
This runs one warmed-up MTSS-WGAN-GP iteration under a TorchDispatchMode and prints, per (op, first
call site inside the package), how often it ran.  hfrep custom ops and metadata-only ops (views,
empty allocations) are skipped.

usage: python scripts/aten_audit.py [--batch 4096] [--dtype float32]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import hfrep  # noqa: E402,F401

SKIP = {"empty", "empty_strided", "view", "_unsafe_view", "as_strided", "reshape", "slice", "select", "t",
        "transpose", "permute", "unsqueeze", "squeeze", "expand", "detach", "alias", "split", "split_with_sizes",
        "_reshape_alias", "unbind", "lift_fresh", "new_empty", "new_empty_strided", "is_same_size", "_to_copy_meta",
        "set_", "resize_", "_local_scalar_dense", "result_type"}


class Audit(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        ns = func.namespace
        name = func.__name__.split(".")[0]
        if ns == "aten" and name not in SKIP:
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "hfrep" in fr.filename or "machine-learning_amd" in fr.filename:
                    site = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                    break
            self.hits[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", default="float32")
    a = ap.parse_args()
    from hfrep.data.windows import synthetic_windows
    from hfrep.models import gan as zoo
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    dev = torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
    arch, loss = zoo.resolve("mtss_wgan_gp")
    cfg = GANConfig(arch=arch, loss=loss, window=24, features=32, batch_size=a.batch,
                    dtype=a.dtype, seed=123)
    tr = GANTrainer(cfg, synthetic_windows(8192, 24, 32, seed=1234), device=dev)
    for _ in range(2):
        tr.train_step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    with Audit() as au:
        tr.train_step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    for (name, site), n in sorted(au.hits.items(), key=lambda x: -x[1]):
        print(f"{n:4d}  {name:28s} {site}")
    print(f"{sum(au.hits.values())} aten ops in one iteration ({dev.type}, {a.dtype}, B = {a.batch})")


if __name__ == "__main__":
    main()
