"""Per-k comparison of autoencoder sweeps across runs (device / dtype): mean and spread over seeds.

usage: python scripts/ae_compare.py LABEL=glob [LABEL=glob ...] [--panel real|augmented] [--metric IS_r2]

Each glob matches `ae_sweep` JSONs (scripts/ae_study.py / `hfrep replicate --method ae-sweep --out`);
prints one markdown table: k, then per label `mean (sd)` of the metric over its seeds, and the number of
epochs is not stored, so only the published metrics are compared.
"""
import glob
import json
import sys

import numpy as np


def load(pattern, metric):
    runs = [json.load(open(p))["ae_sweep"] for p in sorted(glob.glob(pattern))]
    if not runs:
        raise SystemExit(f"no files match {pattern}")
    ks = sorted(int(k) for k in runs[0]["metrics"])
    vals = np.array([[r["metrics"][str(k)][metric] for k in ks] for r in runs], dtype=float)
    return ks, vals


def main(argv):
    metric = "IS_r2"
    specs = []
    it = iter(argv)
    for a in it:
        if a == "--metric":
            metric = next(it)
        else:
            lab, _, pat = a.partition("=")
            specs.append((lab, pat))
    cols = [(lab,) + load(pat, metric) for lab, pat in specs]
    ks = cols[0][1]
    head = "| k | " + " | ".join(f"{lab} ({v.shape[0]} seeds)" for lab, _, v in cols) + " |"
    print(f"{metric}: mean (sd) over seeds\n")
    print(head)
    print("|---" * (len(cols) + 1) + "|")
    for i, k in enumerate(ks):
        print(f"| {k} | " + " | ".join(f"{v[:, i].mean():.3f} ({v[:, i].std():.3f})" for _, _, v in cols) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
