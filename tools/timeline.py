#!/usr/bin/env python3
"""Print one iteration of a rocprofv3 kernel trace: start offset, gap, duration per dispatch.

    python tools/timeline.py TRACE.csv [--anchor SUBSTRING] [--nth K]
The iteration is the span from the K-th dispatch whose name contains ANCHOR to the next one.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="mfma16r")
    ap.add_argument("--nth", type=int, default=10)
    a = ap.parse_args()
    r = sorted(csv.DictReader(open(a.trace)), key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(r) if a.anchor in x["Kernel_Name"]]
    lo, hi = idx[a.nth], idx[a.nth + 1]
    t0 = int(r[lo]["Start_Timestamp"])
    prev = None
    busy = 0
    for x in r[lo:hi + 1]:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        if x is not r[hi]:
            busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} gap {gap:6.1f} dur {(e - s) / 1e3:8.1f}  {x['Kernel_Name'][:72]}")
        prev = e
    span = int(r[hi]["Start_Timestamp"]) - t0
    print(f"iteration {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
