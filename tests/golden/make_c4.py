"""Generate tests/golden/c4_oracle.json: the oracle's trajectory on the bench workload (C4).

    python tests/golden/make_c4.py [--n 1048576] [--iters 30] [--threads 8]

The workload is exactly bench.py's (BASELINE.json configs[3]): the
2^20-point synthetic pair from icp_synthetic_pair (mt19937_64 seed 42, uniform [-1,1]^3
rounded to fp32; scene = R(5 deg about (1,2,3)) model + (0.05,-0.03,0.02)), 30 fixed
iterations (threshold disabled).  The inputs come from the product's host-side generator
(deterministic host code, no device work); their SHA-256 is stored so the GPU test first
proves it regenerated the same clouds.

Each iteration runs the oracle's own steps, exactly as oracle_icp (oracle/icp_oracle.c,
restating src/cpu.cc:55-79) sequences them: brute-force closest (squared-distance rule,
first minimum; split over threads by query range, every query still scans all M model
points; oracle_closest_range_blocked, the SIMD form of the same loop, checked index for index
against the scalar oracle in tests/test_oracle.py), find_alignment (cpu.cc:105-175), err_compute (cpu.cc:29-40),
err = (e_align + e_apply) / np.  Recorded per iteration: err, s, R, t, the Horn matrix,
and a digest of the NN index array.  Final cloud: SHA-256 of its bytes, per-axis sums and
sampled rows.  Runtime: ~30 x 1.1e12 pairs; about half an hour on 7 cores.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))

import oracle_py as O  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def idx_digest(idx: np.ndarray) -> dict:
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    i64 = idx.astype(np.uint64)
    w = np.arange(1, idx.size + 1, dtype=np.uint64)
    return {"crc32": zlib.crc32(idx.tobytes()), "sum": int(i64.sum()),
            "wsum": int((i64 * w).sum()),  # sum of (j+1)*idx[j] mod 2^64 (computed on the device too)
            "identity": int((idx == np.arange(idx.size)).sum())}


def sample_rows(n: int, k: int = 64, seed: int = 7) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([np.arange(8), np.arange(n - 8, n), rng.choice(n, k, replace=False)]))


def threaded_closest(p, m, threads):
    n = p.shape[0]
    bounds = np.linspace(0, n, 8 * threads + 1).astype(int)
    idx = np.empty(n, dtype=np.int32)
    y = np.empty_like(p)

    def work(k):
        yk, ik = O.closest_blocked(p, m, int(bounds[k]), int(bounds[k + 1]))
        y[bounds[k]:bounds[k + 1]] = yk
        idx[bounds[k]:bounds[k + 1]] = ik

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(len(bounds) - 1)))
    return y, idx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--out", default=os.path.join(HERE, "c4_oracle.json"))
    args = ap.parse_args()

    import icp_amd
    m, p = icp_amd.synthetic_pair(args.n, seed=42)
    out = {"n": args.n, "seed": 42, "iters": args.iters, "threshold": -1.0,
           "model_sha256": sha(m), "scene_sha256": sha(p),
           "nn_rule": "oracle NN_SQUARED: first minimum of ((dx*dx+dy*dy)+dz*dz), compute.cu:112-117,137",
           "err": [], "s": [], "R": [], "t": [], "Nm": [], "evals": [], "idx": []}
    rows = sample_rows(args.n)
    p = p.copy()
    for i in range(args.iters):
        t0 = time.time()
        y, idx = threaded_closest(p, m, args.threads)
        al = O.find_alignment(p, y)
        e_apply, p = O.err_compute(p, y, al.s, np.array(al.R), np.array(al.t))
        err = (al.err + e_apply) / args.n
        out["err"].append(err)
        out["s"].append(al.s)
        out["R"].append(list(al.R))
        out["t"].append(list(al.t))
        out["Nm"].append(list(al.Nm))
        out["evals"].append(list(al.evals))
        out["idx"].append(idx_digest(idx))
        print(f"iter {i}: err {err:.17g} s {al.s:.17g} identity {out['idx'][-1]['identity']} "
              f"({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    out["final"] = {"sha256": sha(p), "sum": p.sum(axis=0).tolist(),
                    "rows": rows.tolist(), "sample": p[rows].tolist()}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
