"""Reference-preset step time: MTSS-WGAN-GP at the reference's own shape (GAN/MTSS_WGAN_GP.py:292:
batch 32, 48-step windows, 35 features), the whole iteration replayed from one hipGraph.

    python scripts/bench_small.py [--batch 32] [--iters 200] [--dtypes float32,bfloat16]

Prints one JSON line per dtype: ms per iteration (5 critic updates with the gradient penalty + 1
generator update) and windows/s.  At this batch one 32-row tile per layer call occupies one CU, so
the number is the latency of the sequential LSTM chain, not throughput.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--window", type=int, default=48)
    ap.add_argument("--features", type=int, default=35)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--dtypes", default="float32,bfloat16")
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()

    import numpy as np
    import torch

    import hfrep  # noqa: F401
    from hfrep.data.windows import synthetic_windows
    from hfrep.train.gan_trainer import GANConfig, GANTrainer
    from hfrep.train.runner import GraphedStep

    dev = torch.device("cuda", 0)
    ds = synthetic_windows(1000, a.window, a.features, seed=7)
    for dt in a.dtypes.split(","):
        cfg = GANConfig(arch="lstm", loss="wgan_gp", window=a.window, features=a.features, batch_size=a.batch,
                        dtype=dt, seed=123)
        tr = GANTrainer(cfg, ds, device=dev)
        step = tr.train_step if a.no_graph else GraphedStep(tr, warmup=2)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.iters * 1e3
        rec = tr.losses()
        print(json.dumps({"dtype": dt, "batch": a.batch, "window": a.window, "features": a.features,
                          "graph": not a.no_graph, "ms_per_iter": round(ms, 3),
                          "windows_per_s": round(tr.windows_per_iteration() / ms * 1e3, 1),
                          "losses_finite": bool(all(np.isfinite(v) for v in rec.values()))}), flush=True)
        del tr, step
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
