"""Summarise `hfrep latent-sweep` JSONs (one per seed) against the published notebook numbers.

usage: python scripts/ae_summary.py profiles/r02_ae/sweep_real_*.json -- profiles/r02_ae/sweep_augmented_*.json
Prints a markdown table per data set: mean / min / max over seeds of IS R2, OOS R2 and the HF
index clone's ex-ante / ex-post Sharpe, next to the reference values (BASELINE.md:30-45,
autoencoder_v4.ipynb:193,319,1039,1066,1497,1630,1836,1863).
"""
import json
import sys

import numpy as np

# autoencoder_v4.ipynb:193 (IS R2, real), :1497 (IS R2 augmented: only k=1 / k=21 published in BASELINE)
REF_IS_REAL = [0.138, 0.213, 0.197, 0.479, 0.382, 0.506, 0.505, 0.544, 0.554, 0.481, 0.731, 0.849, 0.659, 0.846,
               0.821, 0.855, 0.627, 0.817, 0.688, 0.785, 0.889]
REF = {
    False: {"IS_r2": dict(enumerate(REF_IS_REAL, 1)), "OOS_r2": {12: 0.581, 15: 0.622, 21: 0.681},
            "ante": {2: 0.693}, "post": {2: 0.688}},
    True: {"IS_r2": {1: 0.201, 21: 0.992}, "OOS_r2": {20: 0.955, 21: 0.941}, "ante": {8: 0.836}, "post": {8: 0.818}},
}


def _load(paths):
    runs = [json.load(open(p))["ae_sweep"] for p in paths]
    ks = sorted(int(k) for k in runs[0]["metrics"])
    return runs, ks


def _band(vals):
    v = np.asarray(vals, dtype=float)
    return f"{v.mean():.3f} [{v.min():.3f}, {v.max():.3f}]"


def table(paths):
    runs, ks = _load(paths)
    aug = bool(runs[0]["augmented"])
    ref = REF[aug]
    seeds = ", ".join(str(r["seed"]) for r in runs)
    out = [f"### {'augmented (real + generated)' if aug else 'real data'} — {runs[0]['device']} "
           f"{runs[0]['dtype']}, seeds {seeds}", "",
           "| k | IS R² ours | IS R² ref | OOS R² ours | OOS R² ref | HEDG ex-ante SR ours | ref | HEDG ex-post SR ours | ref |",
           "|---|---|---|---|---|---|---|---|---|"]
    f = lambda d, k: f"{d[k]:.3f}" if k in d else "—"
    for k in ks:
        s = str(k)
        out.append(" | ".join([
            f"| {k}", _band([r["metrics"][s]["IS_r2"] for r in runs]), f(ref["IS_r2"], k),
            _band([r["metrics"][s]["OOS_r2"] for r in runs]), f(ref["OOS_r2"], k),
            _band([r["sharpe_ante"][s]["HEDG"] for r in runs]), f(ref["ante"], k),
            _band([r["sharpe_post"][s]["HEDG"] for r in runs]), f(ref["post"], k)]) + " |")
    best_post = [max(r["sharpe_post"][str(k)]["HEDG"] for k in ks) for r in runs]
    out += ["", f"best-k HEDG ex-post Sharpe per seed: {', '.join(f'{v:.3f}' for v in best_post)} "
                f"(reference best: {max(ref['post'].values()):.3f})", ""]
    return "\n".join(out)


if __name__ == "__main__":
    args = sys.argv[1:]
    groups, cur = [], []
    for a in args:
        if a == "--":
            groups.append(cur)
            cur = []
        else:
            cur.append(a)
    groups.append(cur)
    print("\n".join(table(g) for g in groups if g))
