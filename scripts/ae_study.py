"""Multi-seed autoencoder replication study in ONE process (BASELINE config 2 on the GPU).

For every seed S and compute dtype: the latent sweep k = 1..21 (finance/experiment.py latent_sweep) on
the real panel and on the panel augmented with the production generator's windows of seed S
(``--aug-dir``/aug_sS.npy, written by ``hfrep generate`` from the reference's .h5, autoencoder_v4.ipynb:1291).
Each sweep is written as the same JSON as ``hfrep replicate --method ae-sweep --out`` so
scripts/ae_summary.py tables it.  On a GPU every autoencoder fit is one launch of csrc/ae.hip.

    python scripts/ae_study.py --out DIR --seeds 1-30 --dtypes float32,bfloat16 --device cuda
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
    ap.add_argument("--out", required=True)
    ap.add_argument("--seeds", default="1-30")
    ap.add_argument("--dtypes", default="float32,bfloat16")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--aug-dir", default="assets/ae_aug")
    ap.add_argument("--latents", default="1-21")
    a = ap.parse_args()

    import numpy as np
    import torch

    import hfrep  # noqa: F401
    from hfrep.data.io import load_cleaned
    from hfrep.finance.experiment import generated_augmentation, latent_sweep_many

    lo, _, hi = a.seeds.partition("-")
    seeds = list(range(int(lo), int(hi or lo) + 1))
    klo, _, khi = a.latents.partition("-")
    latents = range(int(klo), int(khi or klo) + 1)
    os.makedirs(a.out, exist_ok=True)
    c = load_cleaned()
    dev = torch.device(a.device)
    t_all = time.perf_counter()
    for dt_name in a.dtypes.split(","):
        dt = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float64": torch.float64}[dt_name]
        for aug in (False, True):
            # every (seed, latent) fit of this dtype and panel trains in one launch (one workgroup per fit)
            xes, yes = [], []
            for s in seeds:
                xe = ye = None
                if aug:
                    xe, ye = generated_augmentation(np.load(os.path.join(a.aug_dir, f"aug_s{s}.npy"), allow_pickle=False), c)
                xes.append(xe)
                yes.append(ye)
            t0 = time.perf_counter()
            sws = latent_sweep_many(c, seeds, latents=latents, x_extras=xes, y_extras=yes, device=dev, dtype=dt)
            el = time.perf_counter() - t0
            panel = "augmented" if aug else "real"
            for s, sw in zip(seeds, sws):
                res = {"ae_sweep": {"device": str(dev), "dtype": dt_name, "seed": s, "augmented": aug,
                                    "elapsed_s": round(el / len(seeds), 3), "batch_elapsed_s": round(el, 3),
                                    "batch_seeds": len(seeds),
                                    "metrics": sw.metrics.to_dict(orient="index"),
                                    "sharpe_ante": sw.sharpe_ante.to_dict(orient="index"),
                                    "turnover": sw.turnover.to_dict(orient="index"),
                                    "sharpe_post": sw.sharpe_post.to_dict(orient="index"),
                                    "best": sw.best.to_dict(orient="index")}}
                path = os.path.join(a.out, f"sweep_{panel}_{dev.type}_{dt_name}_s{s}.json")
                with open(path, "w") as fh:
                    json.dump(res, fh, indent=1, default=float)
            is1 = sws[0].metrics["IS_r2"].iloc[0]
            print(f"[ae_study] {dt_name} {panel}: {len(seeds)} seeds x {len(latents)} latents in {el:.2f} s "
                  f"(seed {seeds[0]} IS R2 k={latents[0]} {is1:.3f})", flush=True)
    print(f"[ae_study] total {time.perf_counter() - t_all:.1f} s", flush=True)


if __name__ == "__main__":
    main()
