#!/usr/bin/env python3
"""Randomised bit-identity check of the one-launch registrations (icp_persistent_kernel,
icp_persistent_mid_kernel) against the launch loop: random scene/model sizes across both
kernels' ranges, model shapes (uniform, surface, clustered, lattice with exact ties,
duplicated points), random rigid motions (small to far), fixed or converging runs.  Every case
must agree bit for bit (error trace, final cloud, correspondences) and must actually take the
one launch.

    python tools/persist_fuzz.py --cases 200 --seed 1 [--max-seconds 400]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
import icp_amd  # noqa: E402


def model(rng, kind, nm):
    if kind == "uniform":
        return rng.uniform(-1, 1, size=(nm, 3))
    if kind == "surface":  # a wavy sheet: surface-like density, as the scanned clouds
        u, v = rng.uniform(-1, 1, size=(2, nm))
        return np.stack([u, v, 0.2 * np.sin(3 * u) * np.cos(2 * v)], axis=1)
    if kind == "clusters":
        c = rng.uniform(-5, 5, size=(8, 3))
        return c[rng.integers(0, 8, nm)] + rng.normal(scale=0.05, size=(nm, 3))
    if kind == "lattice":  # exact D64 ties for half-integer queries
        side = int(np.ceil(nm ** (1 / 3)))
        g = np.arange(side, dtype=float)
        m = np.stack(np.meshgrid(g, g, g, indexing="ij"), axis=-1).reshape(-1, 3)[:nm]
        return m[rng.permutation(m.shape[0])]
    base = rng.uniform(-1, 1, size=(max(1, nm // 3), 3))  # duplicates
    return np.concatenate([base, base, base, base])[:nm][rng.permutation(nm)]


def rigid(rng, p, scale):
    a = rng.uniform(0.01, 0.4) * scale
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    rot = np.eye(3) + np.sin(a) * k + (1 - np.cos(a)) * k @ k
    return p @ rot.T + rng.normal(scale=0.05 * scale, size=3)


def run(m, p, mode, iters, thr):
    with icp_amd.Context(0) as ctx:
        ctx.set_run_mode(mode)
        ctx.set_allow_unequal(m.shape[0] != p.shape[0])
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(iters, thr)
        return res.iterations, errs, ctx.get_scene(), ctx.get_indices(), ctx.stats()["persistent_runs"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-seconds", type=float, default=400.0)
    ap.add_argument("--only", type=int, default=-1, help="run just this case (the others' data is still drawn)")
    ap.add_argument("--dump", default="", help="with --only: save the case's clouds and both runs' indices (.npz)")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    t0 = time.time()
    done = fails = 0
    kinds = ["uniform", "surface", "clusters", "lattice", "duplicates"]
    for c in range(a.cases):
        if time.time() - t0 > a.max_seconds:
            break
        small = rng.random() < 0.35
        n = int(rng.integers(4, 4097)) if small else int(rng.integers(4097, 49153))
        nm = int(rng.integers(1, 6001)) if small else int(rng.integers(16, 65537))
        kind = kinds[int(rng.integers(0, len(kinds)))]
        m = model(rng, kind, nm)
        p = m[rng.integers(0, nm, n)] + rng.normal(scale=rng.choice([0.0, 1e-3, 0.02]), size=(n, 3))
        p = rigid(rng, p, rng.choice([0.2, 1.0, 10.0]))
        if kind == "lattice":
            p = np.round(p * 2) / 2 + 0.5 * (rng.random() < 0.5)  # many exact half-integer ties
        iters = int(rng.integers(1, 12))
        thr = -1.0 if rng.random() < 0.5 else 1e-6
        if a.only >= 0 and c != a.only:
            continue
        one = run(m, p, icp_amd.RUN_PERSISTENT, iters, thr)
        loop = run(m, p, icp_amd.RUN_LAUNCHES, iters, thr)
        ok = (one[4] == 1 and loop[4] == 0 and one[0] == loop[0] and np.array_equal(one[1], loop[1], equal_nan=True)
              and np.array_equal(one[2], loop[2], equal_nan=True) and np.array_equal(one[3], loop[3]))
        done += 1
        fails += not ok
        if a.dump:
            np.savez(a.dump, m=m, p=p, iters=iters, thr=thr, one_err=one[1], loop_err=loop[1], one_idx=one[3],
                     loop_idx=loop[3], one_p=one[2], loop_p=loop[2])
        rec = {"case": c, "n": n, "nm": nm, "kind": kind, "iters": iters, "thr": thr, "ran": one[0],
               "one_launch": one[4], "bitwise": ok}
        print(json.dumps(rec), flush=True)
    print(json.dumps({"cases": done, "failures": fails, "seconds": round(time.time() - t0, 1)}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
