"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {100 * float(r['TotalDurationNs']) / tot:5.1f}%  "
          f"n={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")
