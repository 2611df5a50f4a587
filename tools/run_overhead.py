"""Fixed cost of one icp_run call at C4: wall time of run(K) for several K after a warm-up,
fitted as F + K * x (median of reps).  Usage: python tools/run_overhead.py [--reps 5]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
import icp_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--n", type=int, default=1 << 20)
args = ap.parse_args()
m, p = icp_amd.synthetic_pair(args.n, seed=42)
out = {}
with icp_amd.Context(0) as ctx:
    ctx.set_model(m)
    ctx.set_scene(p)
    ctx.run(5, -1.0)
    for k in (1, 2, 4, 8, 16, 30, 60, 120):
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            ctx.run(k, -1.0)
            ts.append(time.perf_counter() - t0)
        out[k] = float(np.median(ts)) * 1e3
ks = np.array(sorted(out))
ms = np.array([out[k] for k in ks])
x, f = np.polyfit(ks, ms, 1)
print(json.dumps({"ms_by_k": out, "fit_ms_per_iter": x, "fit_fixed_ms": f,
                  "per_iter_at_30": out[30] / 30, "per_iter_at_120": out[120] / 120}))
