#!/usr/bin/env python3
"""BASELINE.json configs C2 (bun000 vs bun045, 50 iterations) and C3 (horse_ref vs horse_tr1,
50 iterations) on one GPU: complete registrations (reference semantics, threshold 1e-5) per
NN variant, with the NN filter's mean launch time.

    python tools/configs_probe.py [--reps 5] [--variants auto valu mfma16 grid]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import icp_amd  # noqa: E402
import datasets  # noqa: E402

CONFIGS = {"C2_bunny": ("bun000", "bun045", True), "C3_horse": ("horse_ref", "horse_tr1", False),
           "C1_cow_gpu": ("cow_ref", "cow_tr1", False)}
VARIANTS = {"auto": 0, "valu": 1, "mfma": 2, "mfma16": 3, "grid": 4,
            "loop": 0}  # loop: the default NN cascade in the launch loop (icp_set_run_mode LAUNCHES)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", nargs="+", default=["auto", "valu", "mfma16", "grid"])
    ap.add_argument("--configs", nargs="+", default=list(CONFIGS),
                    help="names of CONFIGS, or synN for a synthetic N-point pair")
    a = ap.parse_args()
    for name in a.configs:
        if name.startswith("syn"):  # synthetic pair of n points (fixed iterations: threshold off)
            n = int(name[3:])
            m, p = icp_amd.synthetic_pair(n, seed=42)
            unequal, thr = False, -1.0
        else:
            ref, scene, unequal = CONFIGS[name]
            m = icp_amd.load_matrix(datasets.path(ref))
            p = icp_amd.load_matrix(datasets.path(scene))
            thr = 1e-5
        for v in a.variants:
            with icp_amd.Context(0, icp_amd.NN_CERTIFIED) as ctx:
                ctx.set_nn_variant(VARIANTS[v])
                if v == "loop":
                    ctx.set_run_mode(icp_amd.RUN_LAUNCHES)
                ctx.set_allow_unequal(unequal)
                ctx.set_model(m)
                ctx.set_scene(p)
                ctx.run(50, thr)  # warm
                ctx.reset_stats()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    ctx.set_scene(p)
                    res, errs = ctx.run(50, thr)
                dt = (time.perf_counter() - t0) / a.reps
                st = ctx.stats()
            print(json.dumps({"config": name, "variant": v, "n_model": m.shape[0], "n_scene": p.shape[0],
                              "iterations": res.iterations, "ms_per_registration": dt * 1e3,
                              "iterations_per_s": res.iterations / dt,
                              "nn_kernel_ms": st["nn_ms"] / max(st["nn_launches"], 1),
                              "queued_per_iter": st["level1_queued"] / max(st["iterations"], 1),
                              "fallback_per_iter": st["grid_fallback"] / max(st["iterations"], 1),
                              "persistent_runs": st["persistent_runs"],
                              "final_err": float(errs[res.iterations - 1])}), flush=True)


if __name__ == "__main__":
    main()
