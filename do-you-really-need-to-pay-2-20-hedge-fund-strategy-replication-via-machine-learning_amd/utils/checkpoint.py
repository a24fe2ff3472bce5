"""Checkpoint IO: generator checkpoints (.pkl / .npz), generated windows (.npy), full resume state.

Reference artifacts: the scripts save only the final generator as a Keras ``.h5``
(GAN/MTSS_WGAN_GP.py:285-287) and generated windows as a pickled ndarray
(``helper.dic_save``, GAN/generated_data2022-07-09.pkl) or ``.npy``.  This framework writes:

* ``<prefix><YYYYmmdd_HH-MM-SS>.pkl`` — a plain-data dict: format tag, model config and the
  Keras-named weights (ndarray list in ``get_weights`` order).  Read back with the
  non-executing reader (:func:`hfrep.data.io.safe_pickle_load`);
* ``.npz`` — the same payload for numpy-only consumers (``allow_pickle=False``);
* ``.npy`` — generated windows (N, T, F) float32;
* ``.pt`` — full training state for bitwise resume (both models, optimizer slots + shared
  iteration counter, RNG counters, iteration), loaded with ``torch.load(weights_only=True)``;
* Keras ``.h5`` generators from the reference are IMPORTED via :mod:`hfrep.utils.h5lite`.
"""
from __future__ import annotations

import datetime
import json
import os
import pickle

import numpy as np
import torch

FORMAT = "hfrep-generator-v1"


def timestamp() -> str:
    return datetime.datetime.now().strftime("%Y%m%d_%H-%M-%S")


def _payload(model, config: dict) -> dict:
    return {"format": FORMAT, "config": dict(config),
            "weight_names": [n for n, _ in model.named_weights()],
            "weights": [np.ascontiguousarray(w, dtype=np.float32) for w in model.get_weights()]}


def save_generator(path: str, model, config: dict) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    p = _payload(model, config)
    if path.endswith(".npz"):
        arrays = {f"w{i:03d}": w for i, w in enumerate(p["weights"])}
        np.savez(path, __meta__=np.frombuffer(json.dumps({k: p[k] for k in ("format", "config", "weight_names")}).encode(),
                                                dtype=np.uint8), **arrays)
    else:
        with open(path, "wb") as fh:
            pickle.dump(p, fh, protocol=4)
    return path


def read_generator_payload(path: str) -> dict:
    if path.endswith(".npz"):
        z = np.load(path, allow_pickle=False)
        meta = json.loads(bytes(z["__meta__"]).decode())
        meta["weights"] = [z[f"w{i:03d}"] for i in range(len(meta["weight_names"]))]
        return meta
    if path.endswith(".h5"):
        from .h5lite import read_keras_model

        return read_keras_model(path)
    from ..data.io import safe_pickle_load

    p = safe_pickle_load(path)
    if not (isinstance(p, dict) and p.get("format") == FORMAT):
        raise ValueError(f"{path}: not an hfrep generator checkpoint")
    return p


def build_generator_from_config(cfg: dict, device="cpu"):
    from ..models import gan as zoo

    arch = cfg.get("arch", "lstm")
    T, F, H = cfg["window"], cfg["features"], cfg.get("hidden", 100)
    if arch == "mlp":
        return zoo.mlp_generator(T, F, H, device=device)
    return zoo.lstm_generator(T, F, H, lrelu_after_first=cfg.get("lrelu_after_first", False), device=device)


def load_generator(path: str, device="cpu"):
    """Rebuild a generator (any supported format incl. reference Keras .h5) and load its weights."""
    p = read_generator_payload(path)
    g = build_generator_from_config(p["config"], device=device)
    ws = p["weights"]
    mine = g.get_weights()
    if len(ws) != len(mine) or any(a.shape != b.shape for a, b in zip(ws, mine)):
        raise ValueError(f"{path}: weight shapes {[w.shape for w in ws]} do not match {[w.shape for w in mine]}")
    g.set_weights(ws)
    return g, p["config"]


def save_windows(path: str, arr: np.ndarray) -> str:
    np.save(path, np.ascontiguousarray(arr, dtype=np.float32))
    return path


def load_windows(path: str) -> np.ndarray:
    return np.load(path, allow_pickle=False)


# ---------------------------------------------------------------------------------------------
# full training state (resume)
# ---------------------------------------------------------------------------------------------
def save_training_state(path: str, trainer, rng_states_by_rank=None) -> str:
    """``rng_states_by_rank``: under data parallelism with the host (torch.Generator) RNG, every
    rank's generator state (gathered by the caller), so each rank resumes its OWN stream; the
    device Philox counter is identical on all ranks and needs no such list."""
    opt = trainer.opt
    st = {
        "format": "hfrep-train-state-v1",
        "iteration": torch.tensor(trainer.iteration),
        "generator": trainer.generator.flat.detach().cpu(),
        "critic": trainer.critic.flat.detach().cpu(),
        "opt_iterations": opt.iterations.detach().cpu(),
        "opt_m_cache": opt.m_cache.detach().cpu(),
        "opt_slots_generator": list(opt._slots(trainer.generator.flat)),
        "opt_slots_critic": list(opt._slots(trainer.critic.flat)),
        "rng_ctr": trainer.rng.ctr.detach().cpu() if trainer.rng.native else torch.zeros(1, dtype=torch.int64),
        "rng_gen_state": (trainer.rng.gen.get_state() if not trainer.rng.native else torch.zeros(0, dtype=torch.uint8)),
        "rng_gen_states_by_rank": list(rng_states_by_rank or []),
        "config_json": torch.tensor(list(json.dumps(trainer.cfg.__dict__, default=str).encode()), dtype=torch.uint8),
    }
    st["opt_slots_generator"] = [s.detach().cpu() for s in st["opt_slots_generator"]]
    st["opt_slots_critic"] = [s.detach().cpu() for s in st["opt_slots_critic"]]
    tmp = path + ".tmp"
    torch.save(st, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a truncated checkpoint
    return path


def read_training_state(path: str) -> dict:
    st = torch.load(path, weights_only=True, map_location="cpu")
    assert st["format"] == "hfrep-train-state-v1"
    return st


def load_training_state(path: str, trainer) -> None:
    apply_training_state(read_training_state(path), trainer)


def apply_training_state(st: dict, trainer) -> None:
    with torch.no_grad():
        trainer.generator.flat.copy_(st["generator"].to(trainer.generator.flat))
        trainer.critic.flat.copy_(st["critic"].to(trainer.critic.flat))
        opt = trainer.opt
        opt.iterations.copy_(st["opt_iterations"].to(opt.iterations))
        opt.m_cache.copy_(st["opt_m_cache"].to(opt.m_cache))
        opt.load_slots(trainer.generator.flat, st["opt_slots_generator"])
        opt.load_slots(trainer.critic.flat, st["opt_slots_critic"])
        if trainer.rng.native:
            trainer.rng.ctr.copy_(st["rng_ctr"].to(trainer.rng.ctr))
        else:
            by_rank = st.get("rng_gen_states_by_rank") or []
            gs = by_rank[trainer.rank] if trainer.rank < len(by_rank) else st["rng_gen_state"]
            if gs.numel():
                trainer.rng.gen.set_state(gs)
    trainer.iteration = int(st["iteration"])
