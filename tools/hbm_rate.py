#!/usr/bin/env python3
"""Per-kernel achieved HBM rate: PMC bytes per launch (tools/pmc_summary.py output) over the
mean launch time of the same workload's rocprofv3 kernel trace (--stats kernel_stats.csv).

    python tools/hbm_rate.py PMC_TRAFFIC.json KERNEL_STATS.csv [--peak 8000]
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("stats")
    ap.add_argument("--peak", type=float, default=8000.0, help="HBM peak, GB/s")
    a = ap.parse_args()
    traffic = json.load(open(a.pmc))["kernels"]
    rows = []
    for r in csv.DictReader(open(a.stats)):
        k = short(r["Name"])
        if k not in traffic:
            continue
        t_us = float(r["AverageNs"]) / 1e3
        b = traffic[k]["traffic_bytes_per_launch"]
        rows.append((float(r["TotalDurationNs"]), k, int(r["Calls"]), t_us, b / 1e6, b / (t_us * 1e3)))
    print(f"{'kernel':34s} {'calls':>5s} {'avg us':>9s} {'MB/launch':>10s} {'GB/s':>8s} {'of peak':>7s}")
    for _, k, n, t, mb, gbs in sorted(rows, reverse=True):
        print(f"{k:34s} {n:5d} {t:9.1f} {mb:10.2f} {gbs:8.0f} {gbs / a.peak:7.1%}")


if __name__ == "__main__":
    main()
