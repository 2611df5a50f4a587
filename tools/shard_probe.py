#!/usr/bin/env python3
"""Per-rank cost of a W-way sharded C4 job, measured on ONE GPU.

Rank 0 of a W-rank job holds ceil(N/W) scene points against the whole (replicated) model.
This runs exactly that shard through a context with a 1-rank RCCL communicator (so every
per-iteration sum still goes through ncclAllReduce on the engine stream) and reports the
per-iteration time.  The only thing missing against the real W-GPU run is the cross-GPU
latency of the one 18-double all-reduce per iteration (xGMI).  The shard is registered on its
own (np_total = its own size, allow_unequal): its sums are a random sample's, so it follows
the whole cloud's trajectory closely, where np_total = N with one shard's sums would centre it
on an eighth of its centroid.

    python tools/shard_probe.py [--n 1048576] [--worlds 1 2 4 8] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
import icp_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-rccl", action="store_true")
    ap.add_argument("--variant", choices=["auto", "grid"], default="auto")
    a = ap.parse_args()
    m, p = icp_amd.synthetic_pair(a.n, seed=42)
    rows = []
    base = None
    for w in a.worlds:
        b, c = icp_amd.shard_range(a.n, 0, w)
        uid = None if a.no_rccl else icp_amd.rccl_unique_id()
        with icp_amd.Context(0, icp_amd.NN_CERTIFIED, rank=0, world_size=1, rccl_id=uid) as ctx:
            if a.variant == "grid":
                ctx.set_nn_variant(icp_amd.VARIANT_GRID)
            ctx.set_allow_unequal(True)
            ctx.set_model(m)
            ctx.set_scene(p[b:b + c], np_total=c)
            if m.shape[0] >= 2 * c and a.variant != "grid":  # (the bundle images, as bench.py: untimed)
                ctx.model_order(m.shape[0])
            ctx.run(a.warmup, -1.0)
            ctx.reset_stats()
            t0 = time.perf_counter()
            ctx.run(a.steps, -1.0)
            dt = (time.perf_counter() - t0) / a.steps
            st = ctx.stats()
        nn = st["nn_ms"] / max(st["nn_launches"], 1)
        if base is None and w == 1:
            base = dt
        row = {"world": w, "shard_points": c, "ms_per_iter": dt * 1e3, "filter_ms": nn,
               "other_ms": dt * 1e3 - nn, "grid_fallback_per_iter": st["grid_fallback"] / a.steps,
               "level1_queued_per_iter": st["level1_queued"] / a.steps,
               "last_filter": icp_amd.FILTER_NAMES.get(st["last_filter"]),
               "projected_efficiency": (base / (w * dt)) if base else None}
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
