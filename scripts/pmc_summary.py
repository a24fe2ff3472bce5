"""Summarise rocprofv3 --pmc csv passes: per kernel name, mean of each counter over dispatches."""
import collections
import csv
import glob
import os
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:72]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
