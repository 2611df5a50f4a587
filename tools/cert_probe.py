#!/usr/bin/env python3
"""The exclusion certificate on a C4 registration (icp_grid.hip): per run, the queries certified
and walked (icp_stats run_certified / run_walked), the wall time of the run, and the index
digest of the last iteration -- printed for the certificate on and off (ICP_CERT is read once per
process, so each setting is its own process: `--child`).

    python tools/cert_probe.py [--n 1048576] [--iters 30] [--runs 3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))


def child(a):
    import numpy as np
    import icp_amd
    m, p = icp_amd.synthetic_pair(a.n, seed=42)
    out = []
    with icp_amd.Context(0, icp_amd.NN_CERTIFIED) as ctx:
        ctx.set_index_digest(a.iters)
        ctx.set_model(m)
        for r in range(a.runs):
            ctx.set_scene(p)
            ctx.reset_stats()
            t0 = time.perf_counter()
            res, errs = ctx.run(a.iters, -1.0)
            dt = time.perf_counter() - t0
            st = ctx.stats()
            dg = ctx.index_digest()
            out.append({"run": r, "ms": dt * 1e3, "iterations": res.iterations, "err_last": float(errs[-1]),
                        "certified": st["run_certified"], "walked": st["run_walked"],
                        "grid_searches": st["run_grid_searches"], "bundle_searches": st["run_bundle_searches"],
                        "digest_last": [int(x) for x in np.asarray(dg[-1]).ravel()],
                        "digest_sum": int(np.asarray(dg, dtype=np.uint64).sum(dtype=np.uint64))})
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--envs", nargs="+", default=["ICP_CERT=1", "ICP_CERT=0"])
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    res = {}
    for e in a.envs:
        env = dict(os.environ)
        for kv in e.split("+"):
            k, v = kv.split("=")
            env[k] = v
        r = subprocess.run([sys.executable, __file__, "--child", "--n", str(a.n), "--iters", str(a.iters),
                            "--runs", str(a.runs)], env=env, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stdout, r.stderr)
            sys.exit(r.returncode)
        res[e] = json.loads(r.stdout.strip().splitlines()[-1])
        for row in res[e]:
            print(e, json.dumps(row), flush=True)
    ks = list(res)
    same = all(res[k][-1]["digest_sum"] == res[ks[0]][-1]["digest_sum"] and
               res[k][-1]["err_last"] == res[ks[0]][-1]["err_last"] for k in ks)
    print("digests and last err equal across settings:", same)


if __name__ == "__main__":
    main()
