#!/usr/bin/env python3
"""The bundle-bound filter against the full N x M f16 filter on one workload: ICP iterations/s,
the level-1 kernel's mean launch time, the bundle filter's executed work (icp_set_bundle_counters)
and bitwise equality of the two runs (error trace, final cloud, per-iteration index digests).

    python tools/bundle_probe.py [--n 1048576] [--steps 10] [--variants mfma16 bundle]
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

VAR = {"auto": 0, "mfma16": 3, "bundle": 5, "grid": 4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--nm", type=int, default=0, help="model points (default: n)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--variants", nargs="+", default=["mfma16", "bundle"])
    ap.add_argument("--shard", type=int, default=1, help="rank 0's shard of a W-way job (queries n/W)")
    a = ap.parse_args()
    m, p = icp_amd.synthetic_pair(a.n, seed=42)
    if a.shard > 1:
        b, c = icp_amd.shard_range(a.n, 0, a.shard)
        p = np.ascontiguousarray(p[b:b + c])
    runs = {}
    for v in a.variants:
        with icp_amd.Context(0) as ctx:
            ctx.set_nn_variant(VAR[v])
            ctx.set_allow_unequal(True)
            t0 = time.perf_counter()
            ctx.set_model(m)
            t_model = time.perf_counter() - t0
            ctx.set_scene(p, np_total=p.shape[0])
            ctx.run(a.warmup, -1.0)
            ctx.reset_stats()
            t0 = time.perf_counter()
            _, errs = ctx.run(a.steps, -1.0)
            dt = time.perf_counter() - t0
            st = ctx.stats()
            out = ctx.get_scene()
            # untimed: the same run again with digests and (bundle) work counters
            ctx.set_scene(p, np_total=p.shape[0])
            ctx.set_index_digest(a.steps + a.warmup)
            if v == "bundle":
                ctx.set_bundle_counters(True)
            _, errs2 = ctx.run(a.steps + a.warmup, -1.0)
            dig = ctx.index_digest(a.steps + a.warmup)
            cnt = ctx.bundle_counters() if v == "bundle" else None
            out2 = ctx.get_scene()
        runs[v] = (errs2, out2, dig)
        rec = {"variant": v, "n_scene": p.shape[0], "n_model": m.shape[0], "it_per_s": a.steps / dt,
               "ms_per_it": dt * 1e3 / a.steps, "nn_kernel_ms": st["nn_ms"] / max(st["nn_launches"], 1),
               "queued_per_it": st["level1_queued"] / max(st["iterations"], 1),
               "fallback_per_it": st["grid_fallback"] / max(st["iterations"], 1),
               "set_model_s": t_model, "final_err": float(errs[-1])}
        if cnt:
            it = a.steps + a.warmup
            nb = (m.shape[0] + 31) // 32
            rec["per_iteration"] = {k: v_ / it for k, v_ in cnt.items() if not isinstance(v_, dict)}
            rec["us_per_wave_task"] = cnt["us_per_wave_task"]
            rec["deferred_us_per_wave_task"] = cnt.get("deferred_us_per_wave_task")
            rec["slowest_task_us"] = cnt["slowest_task_us_total"] / it
            pi = rec["per_iteration"]
            # (v1 re-issued each fired block's stream test; v2 does not)
            reissued = pi["block_triggers"] if os.environ.get("ICP_BUNDLE_KERNEL") == "1" else 0.0
            rec["executed_mfma_per_it"] = pi["stream_mfma"] + reissued + pi["group_tests"] + pi["pair_tests"]
            rec["executed_tflops"] = 32768.0 * rec["executed_mfma_per_it"] / (rec["nn_kernel_ms"] * 1e-3) / 1e12
        print(json.dumps(rec), flush=True)
    names = list(runs)
    for v in names[1:]:
        same = all(np.array_equal(x, y) for x, y in zip(runs[names[0]], runs[v]))
        print(json.dumps({"bitwise_equal": [names[0], v], "ok": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
