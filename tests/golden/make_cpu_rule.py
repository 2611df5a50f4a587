"""Golden trajectories under the reference CPU path's NN rule (src/cpu.cc:17-22: first minimum of
sqrt((pow(dx,2) + pow(dy,2)) + pow(dz,2)), libm pow -- the oracle is built with
-fno-builtin-pow so that gcc does not fold pow(x, 2.0) into x*x).

Test infrastructure: the oracle's ICP loop of cpu.cc:55-79 (oracle_icp) with its O(N*M) search
split over processes (the per-query answers do not depend on the split); checked bit for bit
against oracle_icp itself on cow before the long bunny run.  Writes tests/golden/cpu_rule.json
and tests/golden/bun045_cpu_rule_idx0.npz.

    python tests/golden/make_cpu_rule.py        (~15 min on 8 cores)
"""
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

_M = None


def _init(m):
    global _M
    _M = m


def _part(args):
    p, = args
    return O.closest(p, _M, O.NN_CPU_SQRT)


def icp_cpu_rule(m, p, max_iter, threshold, pool):
    p = p.copy()
    n = p.shape[0]
    chunks = [(i, min(n, i + 1024)) for i in range(0, n, 1024)]
    out = dict(err=[], s=[], R=[], t=[])
    idx0 = None
    for i in range(max_iter):
        parts = list(pool.map(_part, [(p[a:b],) for a, b in chunks]))
        Y = np.concatenate([y for y, _ in parts])
        idx = np.concatenate([k for _, k in parts])
        if i == 0:
            idx0 = idx
        al = O.find_alignment(p, Y)                     # cpu.cc:65
        R = np.array(al.R).reshape(3, 3)
        e2, p = O.err_compute(p, Y, al.s, R, np.array(al.t))  # cpu.cc:67-71 (in place)
        err = (al.err + e2) / n                         # cpu.cc:73
        out["err"].append(err)
        out["s"].append(al.s)
        out["R"].append(R.tolist())
        out["t"].append(list(al.t))
        if err < threshold:                             # cpu.cc:76-77
            break
    out["iterations"] = len(out["err"])
    return out, p, idx0


def main():
    res = {}
    m = O.load_matrix(datasets.path("cow_ref"))
    p = O.load_matrix(datasets.path("cow_tr1"))
    with ProcessPoolExecutor(8, initializer=_init, initargs=(m,)) as pool:
        mine, fin, _ = icp_cpu_rule(m, p, 20, 1e-5, pool)
    ref = O.icp(m, p, 20, 1e-5, nn_mode=O.NN_CPU_SQRT)
    assert mine["iterations"] == ref["iterations"] and np.array_equal(mine["err"], ref["err"])
    assert np.array_equal(fin, ref["new_p"]), "the split loop must equal oracle_icp bit for bit"
    res["cow_tr1"] = dict(model="cow_ref", scene="cow_tr1", max_iter=20, threshold=1e-5, **mine,
                          final_sum=fin.sum(axis=0).tolist(), final_head=fin[:4].tolist())
    m = O.load_matrix(datasets.path("bun000"))
    p = O.load_matrix(datasets.path("bun045"))
    with ProcessPoolExecutor(8, initializer=_init, initargs=(m,)) as pool:
        mine, fin, idx0 = icp_cpu_rule(m, p, 50, -1.0, pool)  # BASELINE C2: 50 iterations
    _, sq0 = O.closest_blocked(p, m)
    res["bunny"] = dict(model="bun000", scene="bun045", max_iter=50, threshold=-1.0, allow_unequal=True, **mine,
                        final_sum=fin.sum(axis=0).tolist(), final_head=fin[:4].tolist(),
                        final_tail=fin[-4:].tolist(),
                        idx0_differs_from_squared=np.nonzero(idx0 != sq0)[0].tolist())
    np.savez_compressed(os.path.join(HERE, "bun045_cpu_rule_idx0.npz"), idx0=idx0)
    with open(os.path.join(HERE, "cpu_rule.json"), "w") as f:
        json.dump(res, f)
    print("bunny idx0 differs from the squared rule at", res["bunny"]["idx0_differs_from_squared"])


if __name__ == "__main__":
    main()
