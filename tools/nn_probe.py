#!/usr/bin/env python3
"""NN-only probe for profiling: repeated icp_closest_matrix on the C4 synthetic pair.

    python tools/nn_probe.py --variant mfma|valu|fp64 [--n 1048576] [--reps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
import icp_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="mfma", choices=["valu", "mfma", "mfma16", "fp64"])
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--icp", type=int, default=0,
                    help="run this many ICP iterations instead (iterations >= 2 use the seeded filter)")
    a = ap.parse_args()
    mode = icp_amd.NN_FP64 if a.variant == "fp64" else icp_amd.NN_CERTIFIED
    with icp_amd.Context(0, mode) as ctx:
        ctx.set_nn_variant({"valu": 1, "mfma": 2, "mfma16": 3, "fp64": 0}[a.variant])
        m, p = icp_amd.synthetic_pair(a.n, seed=42)
        ctx.set_model(m)
        if a.icp:
            ctx.set_scene(p, np_total=a.n)
            ctx.reset_stats()
            t0 = time.perf_counter()
            per = []
            for _ in range(a.icp):  # one iteration per call: the scene (and the seeds) carry over
                ctx.reset_stats()
                _, errs = ctx.run(1, -1.0)
                st = ctx.stats()
                per.append((st["nn_ms"], st["level1_queued"], float(errs[0])))
            dt = (time.perf_counter() - t0) / a.icp
            for i, (ms, qd, e) in enumerate(per):
                print(f"  it {i:2d}: filter {ms:7.2f} ms  queued {qd:7d}  err {e:.4e}")
            print(f"icp: {dt * 1e3:.2f} ms/iteration, filter {sum(x[0] for x in per) / a.icp:.2f} ms avg")
            return
        ctx.closest_matrix(p)
        ctx.reset_stats()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ctx.closest_matrix(p)
        dt = (time.perf_counter() - t0) / a.reps
        st = ctx.stats()
    ms = st["nn_ms"] / max(st["nn_launches"], 1)
    print(f"level1 queued {st['level1_queued'] / max(st['nn_launches'], 1):.0f} "
          f"(no candidate {st['level1_unrecovered'] / max(st['nn_launches'], 1):.0f}), fp64 {st['ambiguous']}")
    print(f"{a.variant}: wall {dt * 1e3:.2f} ms/search, filter kernel {ms:.2f} ms, "
          f"{8.0 * a.n * a.n / (ms * 1e-3) / 1e12:.1f} TF(8 flop/pair)")


if __name__ == "__main__":
    main()
