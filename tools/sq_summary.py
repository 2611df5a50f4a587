#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel (optionally filtered by a substring of the name).

    python tools/sq_summary.py DIR [name-substring]
"""
import collections
import csv
import glob
import sys


def main():
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                k = r["Kernel_Name"].split("(")[0][-60:]
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
        print(f)
        for k, c in acc.items():
            print(f"  {k}  ({len(disp[k])} dispatches)")
            for n, v in sorted(c.items()):
                print(f"    {n:30s} {v:.4g}")


if __name__ == "__main__":
    main()
