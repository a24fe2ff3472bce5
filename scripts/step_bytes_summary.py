"""Per-kernel and per-iteration HBM bytes from a rocprofv3 --pmc pass of TCC_EA0 request counters
(scripts/pmc_step_bytes.sh).  Read bytes = 128 B x (RDREQ - RDREQ_32B) + 32 B x RDREQ_32B; write bytes
= 64 B x WRREQ_64B + 32 B x (WRREQ - WRREQ_64B).  Kernel time from the same run's kernel trace when
present.  usage: python scripts/step_bytes_summary.py DIR ITERATIONS"""
import collections
import csv
import glob
import os
import sys


def main(d, iters):
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            dur[k] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-6
    rows = []
    for k, c in cnt.items():
        rd = 128 * (c["TCC_EA0_RDREQ_sum"] - c["TCC_EA0_RDREQ_32B_sum"]) + 32 * c["TCC_EA0_RDREQ_32B_sum"]
        wr = 64 * c["TCC_EA0_WRREQ_64B_sum"] + 32 * (c["TCC_EA0_WRREQ_sum"] - c["TCC_EA0_WRREQ_64B_sum"])
        rows.append((k, rd / iters / 1e9, wr / iters / 1e9, dur.get(k, 0.0) / iters))
    rows.sort(key=lambda r: -(r[1] + r[2]))
    trd, twr, tms = sum(r[1] for r in rows), sum(r[2] for r in rows), sum(r[3] for r in rows)
    print(f"per iteration (of {iters} profiled): read {trd:.1f} GB, write {twr:.1f} GB, total {trd + twr:.1f} GB; "
          f"kernel time {tms:.1f} ms (PMC-serialised) -> {(trd + twr) / max(tms, 1e-9):.2f} TB/s average")
    print(f"{'kernel':60s} {'read GB':>9s} {'write GB':>9s} {'ms':>8s} {'TB/s':>6s}")
    for k, rd, wr, ms in rows:
        print(f"{k:60s} {rd:9.2f} {wr:9.2f} {ms:8.2f} {(rd + wr) / ms if ms else 0:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
