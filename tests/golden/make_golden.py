"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py      (run in the build container; ~3 min on 8 cores)

The oracle (oracle/icp_oracle.c) restates the reference's CPU path (src/cpu.cc); it is
itself pinned by the reference's known answers (7 iterations on cow_ref/cow_tr1, see
tests/test_oracle.py).  Fixtures are DATA only: inputs (the bundled CSVs, a seeded small
synthetic pair) and the oracle's outputs (per-iteration err / s / R / t, NN indices of
iteration 0, final clouds).
"""
from __future__ import annotations

import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_py as O  # noqa: E402
import datasets  # noqa: E402

CONFIGS = {
    # name: (model, scene, max_iter, allow_unequal, threshold)
    "cow_tr1": ("cow_ref", "cow_tr1", 20, False, 1e-5),   # BASELINE config 1 (C1)
    "cow_tr2": ("cow_ref", "cow_tr2", 20, False, 1e-5),
    "horse_tr2": ("horse_ref", "horse_tr2", 20, False, 1e-5),
    "horse_tr1": ("horse_ref", "horse_tr1", 50, False, 1e-5),  # C3
    "bunny": ("bun000", "bun045", 50, True, 1e-5),          # C2 (reference refuses np != nm)
}


def synthetic_small(n=4096, seed=1234, angle_deg=20.0, axis=(1.0, -2.0, 0.5), t=(0.1, -0.05, 0.2)):
    rng = np.random.default_rng(seed)
    m = rng.uniform(-1.0, 1.0, size=(n, 3)).astype(np.float32).astype(np.float64)
    ax = np.asarray(axis) / np.linalg.norm(axis)
    th = np.deg2rad(angle_deg)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    p = (m @ R.T + np.asarray(t)).astype(np.float32).astype(np.float64)
    return m, p


def run_config(name):
    mname, pname, iters, unequal, thr = CONFIGS[name]
    m = O.load_matrix(datasets.path(mname))
    p = O.load_matrix(datasets.path(pname))
    r = O.icp(m, p, iters, thr, allow_unequal=unequal, want_idx0=True)
    _, idx_sqrt = O.closest(p, m, O.NN_CPU_SQRT)
    return name, m.shape[0], p.shape[0], r, int((idx_sqrt != r["idx0"]).sum())


def summary(new_p):
    return dict(sum=new_p.sum(axis=0).tolist(), abs_sum=float(np.abs(new_p).sum()),
                head=new_p[:8].tolist(), tail=new_p[-8:].tolist())


def main():
    out = {}
    with ProcessPoolExecutor(max_workers=len(CONFIGS)) as ex:
        for name, nm, np_, r, sqrt_diff in ex.map(run_config, CONFIGS):
            mname, pname, iters, unequal, thr = CONFIGS[name]
            out[name] = dict(model=mname, scene=pname, max_iter=iters, allow_unequal=unequal,
                             threshold=thr, nm=nm, np=np_, iterations=r["iterations"],
                             err=r["err"].tolist(), s=r["s"].tolist(), R=r["R"].tolist(),
                             t=r["t"].tolist(), final=summary(r["new_p"]),
                             idx0_sqrt_vs_squared_mismatches=sqrt_diff)
            np.savez_compressed(os.path.join(HERE, f"{name}_oracle.npz"), idx0=r["idx0"],
                                new_p=r["new_p"])
            print(name, r["iterations"], r["err"][-1], file=sys.stderr)
    # small synthetic pair, fixed 30 iterations (threshold disabled)
    m, p = synthetic_small()
    r = O.icp(m, p, 30, -1.0, want_idx0=True)
    np.savez_compressed(os.path.join(HERE, "synthetic4096.npz"), model=m, scene=p, idx0=r["idx0"],
                        new_p=r["new_p"])
    out["synthetic4096"] = dict(model="synthetic4096.npz:model", scene="synthetic4096.npz:scene",
                                max_iter=30, allow_unequal=False, threshold=-1.0, nm=m.shape[0],
                                np=p.shape[0], iterations=r["iterations"], err=r["err"].tolist(),
                                s=r["s"].tolist(), R=r["R"].tolist(), t=r["t"].tolist(),
                                final=summary(r["new_p"]))
    with open(os.path.join(HERE, "traces.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
