#!/usr/bin/env python3
"""Randomised bit-identity check of the default NN cascade at scale (f16 MFMA filter + fp64
certificate + grid resolver + fp64 fallback, the launch loop that C4 runs) against the fp64
brute force (ICP_NN_FP64) (--variant: another level-1 filter): random model / scene sizes from 2^15 to 2^19 points, the model shapes
of persist_fuzz.py, coordinate scales 10^-3 .. 10^3 with far offsets, small to far rigid motions.
Each case runs a fixed number of ICP iterations (the first unseeded, the rest seeded) in both
modes and must agree bit for bit: error trace, final cloud and every iteration's
correspondence digest.

    python tools/scale_fuzz.py --cases 40 --seed 1 [--max-seconds 400] [--log2 15 19]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import icp_amd  # noqa: E402
from persist_fuzz import model, rigid  # noqa: E402


def run(m, p, nn_mode, iters, variant=0):
    with icp_amd.Context(0, nn_mode) as ctx:
        ctx.set_run_mode(icp_amd.RUN_LAUNCHES)
        ctx.set_nn_variant(variant)
        ctx.set_allow_unequal(m.shape[0] != p.shape[0])
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.set_index_digest(iters)
        res, errs = ctx.run(iters, -1.0)
        return res.iterations, errs, ctx.get_scene(), ctx.index_digest(iters), ctx.stats()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=40)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-seconds", type=float, default=400.0)
    ap.add_argument("--log2", type=float, nargs=2, default=[15.0, 19.0], metavar=("LO", "HI"),
                    help="cloud sizes 2^U(LO, HI) (20 20: C4-size clouds)")
    ap.add_argument("--variant", choices=["auto", "mfma16", "bundle"], default="auto",
                    help="level-1 filter of the certified run (auto: the default)")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    t0 = time.time()
    done = fails = 0
    kinds = ["uniform", "surface", "clusters", "lattice", "duplicates"]
    for c in range(a.cases):
        if time.time() - t0 > a.max_seconds:
            break
        n = int(2 ** rng.uniform(*a.log2))
        nm = int(2 ** rng.uniform(*a.log2))
        kind = kinds[int(rng.integers(0, len(kinds)))]
        m = model(rng, kind, nm)
        p = m[rng.integers(0, nm, n)] + rng.normal(scale=rng.choice([0.0, 1e-3, 0.02]), size=(n, 3))
        p = rigid(rng, p, rng.choice([0.2, 1.0, 10.0]))
        if kind == "lattice":
            p = np.round(p * 2) / 2 + 0.5 * (rng.random() < 0.5)  # many exact half-integer ties
        else:  # (lattice ties need exact coordinates: no rescaling there)
            sc = 10.0 ** rng.uniform(-3, 3)
            off = rng.normal(size=3) * sc * rng.choice([0.0, 10.0, 1e3])
            m, p = m * sc + off, p * sc + off
        iters = int(rng.integers(2, 6))
        var = {"auto": icp_amd.VARIANT_AUTO, "mfma16": icp_amd.VARIANT_MFMA16,
               "bundle": icp_amd.VARIANT_BUNDLE}[a.variant]
        cert = run(m, p, icp_amd.NN_CERTIFIED, iters, var)
        ref = run(m, p, icp_amd.NN_FP64, iters)
        ok = (cert[0] == ref[0] and np.array_equal(cert[1], ref[1], equal_nan=True)
              and np.array_equal(cert[2], ref[2], equal_nan=True) and np.array_equal(cert[3], ref[3]))
        done += 1
        fails += not ok
        st = cert[4]
        rec = {"case": c, "n": n, "nm": nm, "kind": kind, "iters": iters, "ran": cert[0],
               "level1_queued": st.get("level1_queued"), "grid_fallback": st.get("grid_fallback"),
               "bitwise": ok}
        print(json.dumps(rec), flush=True)
    print(json.dumps({"cases": done, "failures": fails, "seconds": round(time.time() - t0, 1)}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
