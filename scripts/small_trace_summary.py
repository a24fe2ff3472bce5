"""Kernel-trace summary of a small-batch run (rocprofv3 --kernel-trace rocpd database): per kernel name the
calls and GPU time per iteration, and over the trace's last N iterations the wall time, the time at least one
kernel runs (union of intervals) and the time two or more run at once (the stream overlap).

usage: python scripts/small_trace_summary.py RUN_results.db [--iter-kernel NAME] [--last 10]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--iter-kernel", default="step_advance_kernel", help="a kernel launched once per iteration")
    ap.add_argument("--last", type=int, default=10)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    marks = [r[1] for r in rows if a.iter_kernel in r[0]]
    if len(marks) < a.last + 1:
        raise SystemExit(f"only {len(marks)} '{a.iter_kernel}' launches")
    t0, t1 = marks[-a.last - 1], marks[-1]
    sel = [r for r in rows if t0 <= r[1] < t1]
    n = a.last
    per = defaultdict(lambda: [0, 0.0])
    for name, s, e, *_ in sel:
        k = name.split("(")[0]
        k = k if len(k) < 90 else k[:90]
        per[k][0] += 1
        per[k][1] += (e - s) / 1e6
    wall = (t1 - t0) / 1e6 / n
    ev = sorted([(s, 1) for _, s, e, *_ in sel] + [(e, -1) for _, s, e, *_ in sel])
    busy = multi = 0.0
    depth, last = 0, None
    for t, d in ev:
        if last is not None:
            if depth >= 1:
                busy += t - last
            if depth >= 2:
                multi += t - last
        depth += d
        last = t
    tot = sum(v[1] for v in per.values()) / n
    print(f"iterations {n}: wall {wall:.3f} ms / iteration, kernels busy (union) {busy / 1e6 / n:.3f} ms, "
          f">= 2 at once {multi / 1e6 / n:.3f} ms, sum of kernel times {tot:.3f} ms, launches {len(sel) / n:.1f}")
    print(f"{'kernel':92s} {'calls':>6s} {'ms/iter':>8s} {'us/call':>8s}")
    for k, (cnt, ms) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:92s} {cnt / n:6.1f} {ms / n:8.3f} {1e3 * ms / cnt:8.1f}")


if __name__ == "__main__":
    main()
