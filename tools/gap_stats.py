"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace, per transition (median, n).
Usage: python tools/gap_stats.py <kernel_trace.csv> [min_count]"""
import collections
import csv
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("void icp::(anonymous namespace)::", "").replace("icp::(anonymous namespace)::", "").split("(")[0][:30]  # noqa: E731
st = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    st[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for k, v in sorted(st.items(), key=lambda kv: -len(kv[1])):
    if len(v) >= lo:
        print(f"{k[0]:32s} -> {k[1]:32s} n={len(v):4d} median gap {np.median(v):6.2f} us")
