#!/usr/bin/env python3
"""Registration cost probe (SURVEY §8d's clock): set_model / set_scene / first iteration /
seeded iterations for one rank's shard of a synthetic pair, through bench.registration.

    python tools/registration_probe.py [--points N] [--world W --rank R] [--reps K]

Prints one JSON line per configuration.  Environment A/B switches pass through (e.g.
ICP_MODEL_HOST=1: the host model preparation)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))

import bench  # noqa: E402
import icp_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    m, p = icp_amd.synthetic_pair(a.points, seed=42)
    b, c = icp_amd.shard_range(a.points, a.rank, a.world)
    with icp_amd.Context(0) as ctx:
        # (a shard alone is registered on its own sums: np_total = its size, as tools/shard_probe.py)
        ctx.set_allow_unequal(True)
        r = bench.registration(ctx, m, p[b:b + c], c, a.iters, a.reps)
    r.update({"points": a.points, "shard": [a.rank, a.world], "n_local": c, "tag": a.tag,
              "env": {k: v for k, v in os.environ.items() if k.startswith("ICP_")}})
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
