#!/usr/bin/env python3
"""Where the f16 filter's L2-miss traffic comes from (run under rocprofv3 --pmc FETCH_SIZE).

The C4 pair (2^20 points, seed 42), 3 fixed ICP iterations, with the scene in its own random
order (--order random, the bench) or sorted by a 2^10-cell-per-axis Morton code (--order morton).
Only the grouping of queries changes: each 32-query group of nn_mfma16r_kernel then holds
neighbours, whose winning 32-point blocks coincide, so the epilogue's index recovery (one
1 KiB model-block re-read per distinct winning block) touches a few blocks per group instead of
~32 random ones.  The model tiles stream identically in both runs.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o fetch -- python3 tools/recovery_traffic.py --order morton
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
import icp_amd  # noqa: E402


def morton_order(p):
    lo, hi = p.min(axis=0), p.max(axis=0)
    c = np.clip(((p - lo) / (hi - lo + 1e-300) * 1024).astype(np.int64), 0, 1023)
    key = np.zeros(len(p), dtype=np.int64)
    for bit in range(10):
        for a in range(3):
            key |= ((c[:, a] >> bit) & 1) << (3 * bit + a)
    return np.argsort(key, kind="stable")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", choices=["random", "morton"], default="random")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    m, p = icp_amd.synthetic_pair(a.n, seed=42)
    if a.order == "morton":
        p = np.ascontiguousarray(p[morton_order(p)])
    ctx = icp_amd.Context()
    ctx.set_model(m)
    ctx.set_scene(p)
    res, errs = ctx.run(a.iters, -1.0)
    print({"order": a.order, "iters": a.iters, "err": [float(e) for e in errs]})


if __name__ == "__main__":
    main()
