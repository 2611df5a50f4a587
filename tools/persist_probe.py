"""Phase stamps of the one-launch registration (ICP_PERSIST_STAMPS=1 prints them per run).

usage: ICP_PERSIST_STAMPS=1 python tools/persist_probe.py [--reps 3]
Runs cow_ref/cow_tr1 (20 iterations, threshold 1e-5) and a 4096-point synthetic pair
(10 fixed iterations) in the one-launch mode, then times both modes over many registrations.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import icp_amd  # noqa: E402
import datasets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--time", type=float, default=0.5)
args = ap.parse_args()

m = icp_amd.load_matrix(datasets.path("cow_ref"))
p = icp_amd.load_matrix(datasets.path("cow_tr1"))
rng = np.random.default_rng(1)
m2 = rng.uniform(-1, 1, size=(4096, 3))
p2 = m2 + rng.normal(scale=0.02, size=(4096, 3))
for name, (mm, pp, it, thr) in {"cow": (m, p, 20, 1e-5), "synthetic4096": (m2, p2, 10, -1.0)}.items():
    for mode in (icp_amd.RUN_PERSISTENT, icp_amd.RUN_LAUNCHES):
        with icp_amd.Context(0) as ctx:
            ctx.set_run_mode(mode)
            ctx.set_model(mm)
            for _ in range(args.reps if mode == icp_amd.RUN_PERSISTENT else 1):
                ctx.set_scene(pp)
                res, _ = ctx.run(it, thr)
            stamps = os.environ.pop("ICP_PERSIST_STAMPS", None)
            n = 0
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < args.time:
                ctx.set_scene(pp)
                ctx.run(it, thr)
                n += 1
            dt = (time.perf_counter() - t0) / n
            if stamps:
                os.environ["ICP_PERSIST_STAMPS"] = stamps
            print(f"{name} mode {mode}: {res.iterations} iterations, {dt * 1e6:.1f} us per registration "
                  f"(incl. set_scene), persistent_runs {ctx.stats()['persistent_runs']}", flush=True)
