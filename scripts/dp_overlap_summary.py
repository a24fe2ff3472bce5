"""Summarise a rocprofv3 kernel trace of scripts/dp_overlap_trace.py: RCCL kernels vs compute kernels.

    python scripts/dp_overlap_summary.py OUT/.../kernel_trace.csv [--last-steps 1]

For every collective kernel (name contains "nccl" / "rccl", or the one-shot p2p_allreduce) of the traced window: its queue, start / end
relative to the first traced kernel, and the compute kernels on OTHER queues that ran during it (the
reduction overlapping the reverse pass).  The window is the last ``--last-steps`` training iterations,
found by the optimizer launches (rmsprop_kernel: 6 per iteration).
"""
from __future__ import annotations

import argparse
import csv
import re
import sys


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-steps", type=int, default=1)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = []
    for r in rows:
        name = _col(r, "Kernel_Name", "KernelName")
        q = _col(r, "Queue_Id", "Queue_ID", "queue_id")
        t0, t1 = int(_col(r, "Start_Timestamp", "BeginNs")), int(_col(r, "End_Timestamp", "EndNs"))
        ks.append((t0, t1, q, name))
    ks.sort()
    opt = [k for k in ks if "rmsprop_kernel" in k[3]]
    per_it = 6
    if len(opt) >= per_it * a.last_steps + 1:
        start = opt[-per_it * a.last_steps - 1][1]
        ks = [k for k in ks if k[0] >= start]
    base = ks[0][0]
    short = lambda n: re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("void ", "")[:70]
    coll = [k for k in ks if re.search(r"nccl|rccl|p2p_allreduce", k[3], re.I)]
    comp = [k for k in ks if k not in coll]
    print(f"# {len(ks)} kernels in the last {a.last_steps} iteration(s), {len(coll)} RCCL kernels; "
          f"queues: RCCL {sorted({k[2] for k in coll})}, compute {sorted({k[2] for k in comp})}")
    n_ov = 0
    for t0, t1, q, name in coll:
        ov = [c for c in comp if c[0] < t1 and c[1] > t0 and c[2] != q]
        n_ov += bool(ov)
        print(f"{short(name)}  queue {q}  {(t0 - base) / 1e6:9.3f} .. {(t1 - base) / 1e6:9.3f} ms "
              f"({(t1 - t0) / 1e3:7.1f} us); concurrent compute kernels on other queues: {len(ov)}")
        for c in ov[:4]:
            lo, hi = max(t0, c[0]), min(t1, c[1])
            print(f"      {short(c[3])}  queue {c[2]}  overlap {(hi - lo) / 1e3:.1f} us")
    print(f"# RCCL kernels with a concurrent compute kernel on another queue: {n_ov} / {len(coll)}")
    return 0 if coll else 1


if __name__ == "__main__":
    sys.exit(main())
