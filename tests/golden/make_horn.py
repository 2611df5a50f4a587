"""Generate tests/golden/horn_matrices.json: Horn's 4x4 matrix N (src/cpu.cc:121-126) at every
iteration of every fixture trajectory (the configs of make_golden.py + synthetic4096).

    python tests/golden/make_horn.py          (about two minutes on one core)

Each trajectory is re-run step by step with the oracle's own pieces in oracle_icp's order
(closest -> find_alignment -> err_compute, src/cpu.cc:55-79); the per-iteration err is
checked against traces.json (identical) before N is recorded.  tests/test_eigen_order.py
feeds these matrices to the EigenSolver order emulation (tests/eigen_order.py).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_py as O  # noqa: E402
import datasets  # noqa: E402
from make_golden import CONFIGS  # noqa: E402


def trajectory(m, p, iters, thr):
    p = p.copy()
    errs, Ns = [], []
    for _ in range(iters):
        y, _ = O.closest_blocked(p, m)
        al = O.find_alignment(p, y)
        e2, p = O.err_compute(p, y, al.s, np.array(al.R), np.array(al.t))
        err = (al.err + e2) / p.shape[0]
        errs.append(err)
        Ns.append(list(al.Nm))
        if err < thr:
            break
    return errs, Ns


def main():
    traces = json.load(open(os.path.join(HERE, "traces.json")))
    out = {}
    for name, (mname, pname, iters, _unequal, thr) in CONFIGS.items():
        m = O.load_matrix(datasets.path(mname))
        p = O.load_matrix(datasets.path(pname))
        errs, Ns = trajectory(m, p, iters, thr)
        assert errs == traces[name]["err"], name
        out[name] = Ns
        print(name, len(Ns), file=sys.stderr)
    z = np.load(os.path.join(HERE, "synthetic4096.npz"))
    errs, Ns = trajectory(z["model"], z["scene"], 30, -1.0)
    assert errs == traces["synthetic4096"]["err"]
    out["synthetic4096"] = Ns
    with open(os.path.join(HERE, "horn_matrices.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
