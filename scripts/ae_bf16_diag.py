"""Where does the bf16 autoencoder lose IS R^2 at small k?  (profiles/r04_ae/README.md)

For latent sizes k and seeds: fit the factor autoencoder (Keras semantics, EarlyStopping) in bf16 with
the fused GPU kernel, with the explicit engine on the GPU, with the explicit engine on the CPU, and in
fp32; report the epochs run, the last train / val loss and the IS R^2 of each fitted model evaluated
with bf16 AND with fp32 predictions -- separating the training dynamics from the evaluation precision.

    python scripts/ae_bf16_diag.py [--latents 1,2,4,8] [--seeds 1,2,3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--latents", default="1,2,4,8")
    ap.add_argument("--seeds", default="1,2,3")
    a = ap.parse_args()

    import numpy as np
    import torch

    import hfrep  # noqa: F401
    from hfrep.data.io import load_cleaned
    from hfrep.data.scaler import MinMaxScaler
    from hfrep.finance.autoencoder_replication import AETrainer, r2_score
    from hfrep.finance.experiment import chronological_split
    from hfrep.models.autoencoder import FactorAutoencoder

    xtr, _, _, _ = chronological_split(load_cleaned())
    x = MinMaxScaler().fit_transform(np.asarray(xtr, dtype=np.float64))
    A = x.shape[1]
    gpu = torch.device("cuda", 0) if torch.cuda.is_available() else None
    cfgs = [("fp32 fused", gpu, torch.float32, True), ("bf16 fused", gpu, torch.bfloat16, True),
            ("bf16 engine", gpu, torch.bfloat16, False), ("bf16 cpu", torch.device("cpu"), torch.bfloat16, False)]
    for k in (int(v) for v in a.latents.split(",")):
        for seed in (int(v) for v in a.seeds.split(",")):
            for name, dev, dt, fused in cfgs:
                if dev is None:
                    continue
                m = FactorAutoencoder(k, A, seed=seed, dtype=torch.float32, device=dev)
                h = AETrainer(m, device=dev).fit(x, epochs=1000, batch_size=48, validation_split=0.25, patience=5,
                                                 seed=seed, dtype=dt, fused=fused if dev.type == "cuda" else False)
                r2 = {}
                for ename, edt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
                    xt = torch.as_tensor(x, dtype=edt, device=dev)
                    r2[ename] = r2_score(x, m.predict(xt).double().cpu().numpy())
                print(json.dumps({"k": k, "seed": seed, "run": name, "epochs": len(h["loss"]),
                                  "loss": round(h["loss"][-1], 6), "val_loss": round(h["val_loss"][-1], 6),
                                  "IS_r2_bf16_eval": round(r2["bf16"], 4), "IS_r2_fp32_eval": round(r2["fp32"], 4)}),
                      flush=True)


if __name__ == "__main__":
    main()
